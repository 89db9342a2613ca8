# GPU tests, conv_fwd phase stamps of the cfstamp build, then the A/B of the baseline vs the in-tree build
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ASYNCRL_HIP_LIB=$PWD/async-rl_amd/csrc/build_var_cfstamp/libasyncrl_hip.so timeout -k 10 200 python scripts/cf_stamps.py > gpurun_out/cfstamps.txt 2>&1
rc=$?; tail -n 9 gpurun_out/cfstamps.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_check_ab.sh ${1:-async-rl_amd/csrc/build_var_base}
