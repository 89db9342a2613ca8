# GPU tests, then interleaved bench windows of two environment settings of the in-tree build
#   gpurun -- bash scripts/gpu_env_ab.sh "<env A>" "<env B>" ["<bench args>"] [reps] [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/envab; mkdir -p $O
if [ -z "${5:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1
  rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${4:-3}); do
  for v in A B; do
    e="$1"; [ $v = B ] && e="$2"
    env $e timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --kernel-reps 20 --cpu-seconds 0 ${3:-} > $O/$v$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -n 5 $O/$v$r.log; exit $rc; }
    python -c "import json; d=json.loads(open('$O/$v$r.log').read().strip().splitlines()[-1]); print('$v$r [$e]', d['ms_per_step'], d['kernels']['fc_bwd']['avg_launch_us'])"
  done
done
