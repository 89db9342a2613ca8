# Quick GPU check: the GPU test suite (optionally filtered) + one bench line.
#   gpurun -- bash scripts/gpu_quick.sh <tag> "<pytest -k expr or empty>" "<bench args>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
K=${2:-}
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf -k "$K" > $O/pytest.log 2>&1
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
fi
rc=$?; tail -n 5 $O/pytest.log; step pytest $rc
if [ -n "$3" ]; then
  timeout -k 10 300 python -u bench.py $3 > $O/bench.log 2>&1
  rc=$?; tail -n 3 $O/bench.log; step bench $rc
fi
exit 0
