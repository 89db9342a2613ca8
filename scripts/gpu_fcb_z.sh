# fc_bwd_kernel job A range count sweep (timing only): ARL_FC_BWD_Z=1..6
set -o pipefail
cd $GRAFT_REPO_ROOT
for z in ${ZS:-1 2 3 4 6}; do
  ARL_FC_BWD_Z=$z timeout -k 10 60 python -u scripts/fc_bwd_bench.py ${N:-256} 200 | sed "s/\$/ Z=$z/" || exit 1
  ARL_FC_BWD_Z=$z ARL_FC_BWD_JOBS=a timeout -k 10 60 python -u scripts/fc_bwd_bench.py ${N:-256} 200 | sed "s/\$/ Z=$z/" || exit 1
done
