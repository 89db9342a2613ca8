# BASELINE.json configs other than the default bench line: C3 (LSTM 1024
# envs), C4 (FF 512 envs/GPU, the per-GPU share of 4096 over 8), C5 (phi
# stress); bench line + rocprof kernel stats + FETCH/WRITE passes for each (the profiled runs without the
# C4 line's secondary C3 leg, so each kernel's per-dispatch average is that workload's own).
#   gpurun --timeout 1200 -- bash scripts/gpu_configs.sh [tag] [workloads...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cfg}
shift
WL=${@:-c3 c4 c5}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
for w in $WL; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 30 --warmup 5 --cpu-seconds 0 > $O/bench_$w.log 2>&1
  step bench_$w $?
  tail -n 1 $O/bench_$w.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python bench.py --workload $w --steps 10 --warmup 3 --cpu-seconds 0 --kernel-reps 10 --secondary none > $O/prof_$w.log 2>&1
  step prof_$w $?
  B="python bench.py --workload $w --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3 --secondary none"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_$w -o fetch -- $B > $O/pmc_fetch_$w.log 2>&1
  step fetch_$w $?
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_$w -o write -- $B > $O/pmc_write_$w.log 2>&1
  step write_$w $?
done
exit 0
