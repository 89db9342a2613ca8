# One GPU call: parity tests, smoke, bench, rocprof kernel stats, PMC traffic.
# Every GPU step has its own time limit; the first failure ends the call.
#   gpurun --timeout 1200 -- bash scripts/gpu_round.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-cur}
O=gpurun_out/$TAG
mkdir -p $O/pmc
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
step pytest $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step smoke $?
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 12 > $O/bench.log 2>&1
step bench $?
tail -n 1 $O/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --cpu-seconds 0 > $O/prof.log 2>&1
step prof $?
B="python bench.py --steps 4 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 5"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc -o fetch -- $B > $O/pmc/fetch.log 2>&1
step fetch $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc -o write -- $B > $O/pmc/write.log 2>&1
step write $?
find $O -name "*.csv" | head -20
exit 0
