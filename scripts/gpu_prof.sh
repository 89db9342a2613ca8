# rocprof kernel stats of one bench configuration: gpurun -- bash scripts/gpu_prof.sh <tag> "<bench args>"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py $2 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -n 1 $O/prof.log | cut -c1-300
exit $rc
