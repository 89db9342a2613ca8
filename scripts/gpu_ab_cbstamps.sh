# conv_bwd phase stamps of the stamp build, then GPU tests + A/B of the baseline vs the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ASYNCRL_HIP_LIB=$PWD/async-rl_amd/csrc/build_var_stamp/libasyncrl_hip.so timeout -k 10 200 python scripts/cb_stamps.py > gpurun_out/stamps.txt 2>&1
rc=$?; tail -n 4 gpurun_out/stamps.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_check_ab.sh ${1:-async-rl_amd/csrc/build_var_base}
