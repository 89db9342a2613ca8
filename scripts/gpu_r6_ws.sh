# Round 6: conv_bwd wave-specialised form (ARL_CB_WS=1): its bitwise arm, then interleaved A/Bs at C4 / C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r6f}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread -k "two_envs_identical" > gpurun_out/$T/pytest.log 2>&1
rc=$?; tail -n 12 gpurun_out/$T/pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/env_ab.sh ARL_CB_WS=0 ARL_CB_WS=1 "--workload c4 --secondary none" 2 ws || exit $?
bash scripts/env_ab.sh ARL_CB_WS=0 ARL_CB_WS=1 "--workload c2 --secondary none" 1 ws || exit $?
exit 0
