# Round 6: RMSProp form A/B (ARL_RMS_U 1 / 2 / 4, interleaved, C4 in-window times) + the size sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_r6.sh ${1:-r6c} rms || exit $?
bash scripts/env_ab.sh ARL_RMS_U=1 ARL_RMS_U=2 "--workload c4 --secondary none" 2 rmsu2 || exit $?
bash scripts/env_ab.sh ARL_RMS_U=1 ARL_RMS_U=4 "--workload c4 --secondary none" 2 rmsu4 || exit $?
exit 0
