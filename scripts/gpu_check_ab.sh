# GPU tests, then an interleaved A/B of a baseline package build (arg 1, a pkg
# root) against the in-tree one at C2 (and optionally more bench args)
#   gpurun -- bash scripts/gpu_check_ab.sh async-rl_amd/csrc/build_var_base ["<bench args>"] [reps]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/chk
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab.sh $1 async-rl_amd "--steps 100 --warmup 10 --kernel-reps 20 ${2:-}" ${3:-3}
