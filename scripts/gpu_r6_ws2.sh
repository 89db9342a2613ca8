# Round 6: conv_bwd_ws_kernel phase stamps (diagnostic build) at C4 and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r6g}
mkdir -p gpurun_out/$T
timeout -k 10 200 python -u scripts/cb_ws_stamps.py > gpurun_out/$T/stamps_c4.txt 2>&1; rc=$?; cat gpurun_out/$T/stamps_c4.txt; [ $rc -ne 0 ] && exit $rc
N=256 timeout -k 10 200 python -u scripts/cb_ws_stamps.py > gpurun_out/$T/stamps_c2.txt 2>&1; rc=$?; cat gpurun_out/$T/stamps_c2.txt; exit $rc
