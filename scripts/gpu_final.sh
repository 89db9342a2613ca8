# End-of-round evidence in one call: GPU tests, smoke, C2 bench (+ CPU baseline legs), rocprof
# stats, PMC FETCH / WRITE traffic, then C3 / C4 / C5 bench + rocprof + traffic, then MFMA busy
#   gpurun --timeout 1200 -- bash scripts/gpu_final.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-final}
bash scripts/gpu_round.sh $TAG || exit $?
bash scripts/gpu_configs.sh ${TAG}_cfg c3 c4 c5 || exit $?
bash scripts/gpu_mfma_pmc.sh ${TAG}_mfma c2 c3 || exit $?
exit 0
