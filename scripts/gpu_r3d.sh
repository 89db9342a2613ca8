# fc_bwd XCD-aware job order A/B (ARL_FC_BWD_XCD=0 / 1): interleaved C2 / C4 bench lines,
# then FETCH / WRITE PMC passes of both arms at C2.
#   gpurun --timeout 900 -- bash scripts/gpu_r3d.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3d}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
for r in 1 2; do
  for w in c2 c4; do
    for x in 0 1; do
      ARL_FC_BWD_XCD=$x timeout -k 10 300 python -u bench.py --workload $w --steps 200 --warmup 10 --cpu-seconds 0 --copy-peak 0 --median-windows 0 --kernel-reps 20 > $O/${w}_x$x$r.log 2>&1
      step ${w}_x$x $?
      python -c "import json; d=json.loads(open('$O/${w}_x$x$r.log').read().strip().splitlines()[-1]); print('$w xcd=$x', d['ms_per_step'], 'fc_bwd', d['kernels']['fc_bwd']['avg_launch_us'], 'conv_bwd', d['kernels']['conv_bwd']['avg_launch_us'])"
    done
  done
done
B="python bench.py --workload c2 --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3 --copy-peak 0 --median-windows 0"
for x in 0 1; do
  ARL_FC_BWD_XCD=$x timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc$x -o fetch -- $B > $O/fetch$x.log 2>&1
  step fetch$x $?
  ARL_FC_BWD_XCD=$x timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc$x -o write -- $B > $O/write$x.log 2>&1
  step write$x $?
done
exit 0
