# GPU parity / identity tests, then a quick interleaved A/B of ARL_FUSE_OBS=0 vs 1
#   gpurun -- bash scripts/gpu_fuse.sh ["<bench args>"]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fuse
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; tail -n 4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab_quick.sh "${1:-}"
