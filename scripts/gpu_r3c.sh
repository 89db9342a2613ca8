# Round 3: GPU suite, bench lines (C4 default with both CPU legs, C2, C3), the C3 A/B of the
# dedicated LSTM gate kernel vs the round-2 generic GEMM, and rocprof stats of C3.
#   gpurun --timeout 1200 -- bash scripts/gpu_r3c.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3c}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 280 --timeout-method thread -rf > $O/pytest.log 2>&1
step pytest $?
tail -n 2 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 12 > $O/bench_c4.log 2>&1
step bench_c4 $?
tail -n 1 $O/bench_c4.log | cut -c1-700
for w in c2 c3; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 100 --warmup 10 --cpu-seconds 0 --copy-peak 0 > $O/bench_$w.log 2>&1
  step bench_$w $?
  tail -n 1 $O/bench_$w.log | cut -c1-300
done
for r in 1 2; do
  for v in generic new; do
    ARL_LSTM_GEMM=$v timeout -k 10 300 python -u bench.py --workload c3 --steps 100 --warmup 10 --cpu-seconds 0 --copy-peak 0 --median-windows 0 --kernel-reps 5 > $O/c3_$v$r.log 2>&1
    step c3_$v $?
    echo "$v $(tail -n 1 $O/c3_$v$r.log | cut -c1-200)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python bench.py --workload c3 --steps 10 --warmup 3 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0 --median-windows 0 > $O/prof_c3.log 2>&1
step prof_c3 $?
exit 0
