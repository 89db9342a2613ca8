# Round 3: r3h (LSTM parity + C3 bench) then r3i (learner-kernel time vs samples per workgroup)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r3h.sh ${1:-r3h} && bash scripts/gpu_r3i.sh ${2:-r3i}
