# final check of the round's tree: GPU tests, smoke, default bench line, 2-rank gloo bench on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3an
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
step pytest $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
step smoke $?
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1
step bench $?
tail -n 1 $O/bench.log | cut -c1-400
ARL_BENCH_DIST_BACKEND=gloo ARL_BENCH_SHARE_GPU=1 timeout -k 10 300 python -u bench.py --gpus 2 --steps 20 --warmup 3 --cpu-seconds 0 --copy-peak 0 > $O/bench_g2.log 2>&1
step bench_g2 $?
tail -n 1 $O/bench_g2.log | cut -c1-400
