# Round 3: the whole GPU suite, then the default bench line (C4 per-GPU leg) with both CPU
# legs, and C2 / C3 lines.
#   gpurun --timeout 900 -- bash scripts/gpu_r3b.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3b}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 280 --timeout-method thread -rf > $O/pytest.log 2>&1
step pytest $?
tail -n 2 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 12 > $O/bench_c4.log 2>&1
step bench_c4 $?
tail -n 1 $O/bench_c4.log | cut -c1-600
for w in c2 c3; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 100 --warmup 10 --cpu-seconds 0 --copy-peak 0 > $O/bench_$w.log 2>&1
  step bench_$w $?
  tail -n 1 $O/bench_$w.log | cut -c1-300
done
exit 0
