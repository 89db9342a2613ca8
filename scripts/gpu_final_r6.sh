# Round-6 end-of-round evidence, part 1: GPU tests, smoke, default bench (+ CPU baseline legs, C3 secondary),
# the driver's own command with the timed-region diagnostic, rocprof stats, PMC FETCH / WRITE traffic (C4),
# MFMA busy and stall counters (C4)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r6final}
bash scripts/gpu_round.sh $T || exit $?
bash scripts/gpu_r6.sh $T diag mfma_c4 stall_c4 || exit $?
exit 0
