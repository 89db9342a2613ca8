#!/bin/bash
# Round-6 GPU calls: bash scripts/gpu_r6.sh TAG step [step ...]
#   steps: sweep (HBM copy sweep), pytest (-m gpu suite), smoke, bench (default line), prof (rocprof stats of
#   the default bench), c3 / c2 / c5 (bench lines of the other workloads), mfma_c4 / mfma_c3 / mfma_c2 (MFMA
#   counters of an eager run against bench.py's issued-cycle model, scripts/mfma_check.py), stall_c4 / stall_c3
#   (per-kernel wave-cycle / wait / LDS counters of an eager run)
# Each GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
ok() { echo "== $1 rc=$2" | tee -a $O/status; [ "$2" -eq 0 ] || exit "$2"; }
for st in "$@"; do
  case $st in
    sweep) timeout -k 10 120 ./scripts/copy_sweep > $O/copy_sweep.txt 2>&1; ok sweep $? ;;
    pytest) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread -rf > $O/pytest.log 2>&1; ok pytest $? ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; ok smoke $? ;;
    bench) timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1; ok bench $?; tail -c 600 $O/bench.log ;;
    prof) (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o c4 -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 --copy-peak 0 --secondary none > "$GRAFT_REPO_ROOT/$O/bench_prof.log" 2>&1); ok prof $? ;;
    mfma_c4|mfma_c3|mfma_c2) w=${st#mfma_}; (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/mfma_$w" -o mfma -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload $w --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3 --copy-peak 0 --secondary none --median-windows 3 --stamp-windows 0 --env-groups 1 > "$GRAFT_REPO_ROOT/$O/mfma_$w.log" 2>&1); ok $st $?; python scripts/mfma_check.py $O/mfma_$w --workload $w --json $O/mfma_$w.json > $O/mfma_$w.txt 2>&1; cat $O/mfma_$w.txt ;;
    stall_c4|stall_c3) w=${st#stall_}; (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/stall_$w" -o stall -- python3 "$GRAFT_REPO_ROOT/bench.py" --workload $w --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3 --copy-peak 0 --secondary none --median-windows 3 --stamp-windows 0 --env-groups 1 > "$GRAFT_REPO_ROOT/$O/stall_$w.log" 2>&1); ok $st $?; python scripts/pmc_summary.py $O/stall_$w/*counter_collection.csv > $O/stall_$w.txt 2>&1; rm -rf $O/stall_$w ;;
    l2_c4) (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/l2_c4" -o l2 -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3 --copy-peak 0 --secondary none --median-windows 3 --stamp-windows 0 > "$GRAFT_REPO_ROOT/$O/l2_c4.log" 2>&1); ok $st $?; python scripts/pmc_summary.py $O/l2_c4/*counter_collection.csv > $O/l2_c4.txt 2>&1; rm -rf $O/l2_c4 ;;
    diag) timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --timed-diag 6 > $O/bench_diag.log 2>&1; ok diag $?; tail -c 300 $O/bench_diag.log ;;
    rms) timeout -k 10 180 python -u scripts/rms_sweep.py $O/rms_sweep.json > $O/rms_sweep.log 2>&1; ok rms $?; cat $O/rms_sweep.log ;;
    coh) timeout -k 10 300 python -u -m pytest tests/test_gpu_coherence.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $O/pytest_coh.log 2>&1; ok coh $? ;;
    c2|c3|c5) timeout -k 10 400 python -u bench.py --workload $st --cpu-seconds 0 --secondary none > $O/bench_$st.log 2>&1; ok $st $? ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
exit 0
