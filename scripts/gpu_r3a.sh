# Round 3, first GPU call: box probe (CPU share), the new bench / RCCL tests,
# the default bench line (C4 per-GPU leg) with both CPU legs, C2 / C3 lines.
#   gpurun --timeout 900 -- bash scripts/gpu_r3a.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3a}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
{ echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "nproc: $(nproc)";
  python -c "import os, psutil; print('affinity', len(os.sched_getaffinity(0)), 'physical', psutil.cpu_count(logical=False), 'logical', os.cpu_count())";
  lscpu | grep -E "Model name|Socket|Core|Thread" ; } > $O/probe.txt 2>&1
cat $O/probe.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench.py -x -v -p no:cacheprovider --timeout 280 --timeout-method thread -rf > $O/pytest_bench.log 2>&1
step pytest_bench $?
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 12 > $O/bench_c4.log 2>&1
step bench_c4 $?
tail -n 1 $O/bench_c4.log
for w in c2 c3; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 100 --warmup 10 --cpu-seconds 0 --copy-peak 0 > $O/bench_$w.log 2>&1
  step bench_$w $?
  tail -n 1 $O/bench_$w.log | cut -c1-400
done
exit 0
