# fc_bwd_kernel ablations per job (timing only): full / no MFMA / no staging
set -o pipefail
cd $GRAFT_REPO_ROOT
for j in a b; do for ab in ${ABLS:-0 1 2}; do
  ARL_FC_BWD_JOBS=$j ARL_FC_BWD_ABL=$ab timeout -k 10 60 python -u scripts/fc_bwd_bench.py ${FCB_N:-256} 200 | sed "s/\$/ abl=$ab/" || exit 1
done; done
