# Round 3 A/Bs: fc_bwd XCD-aware job order (ARL_FC_BWD_XCD=0 / 1) at C2 and C4, C4 with 2 vs 3
# env groups, PMC FETCH / WRITE of both fc_bwd arms at C2, and a rocprof kernel trace of the
# default bench (C4) for the in-graph window timeline.
#   gpurun --timeout 1200 -- bash scripts/gpu_r3d.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3d}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
Q="--steps 200 --warmup 10 --cpu-seconds 0 --copy-peak 0 --median-windows 0 --kernel-reps 20"
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']; print(sys.argv[2], d['ms_per_step'], 'fc_bwd', k['fc_bwd']['avg_launch_us'], 'conv_bwd', k['conv_bwd']['avg_launch_us'])" $1 "$2"; }
for r in 1 2; do
  for w in c2 c4; do
    for x in 0 1; do
      ARL_FC_BWD_XCD=$x timeout -k 10 300 python -u bench.py --workload $w $Q > $O/${w}_x$x$r.log 2>&1
      step ${w}_x$x $?
      show $O/${w}_x$x$r.log "$w xcd=$x"
    done
  done
  for g in 2 3; do
    timeout -k 10 300 python -u bench.py --env-groups $g $Q > $O/c4_g$g$r.log 2>&1
    step c4_g$g $?
    show $O/c4_g$g$r.log "c4 groups=$g"
  done
done
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 3 --cpu-seconds 0 > $O/c5.log 2>&1
step c5 $?
python -c "import json; d=json.loads(open('$O/c5.log').read().strip().splitlines()[-1]); print('c5', d['ms_per_step'], d['roofline']['achieved'], d['hbm_copy_peak'])"
B="python bench.py --workload c2 --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3 --copy-peak 0 --median-windows 0"
for x in 0 1; do
  ARL_FC_BWD_XCD=$x timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc$x -o fetch -- $B > $O/fetch$x.log 2>&1
  step fetch$x $?
  ARL_FC_BWD_XCD=$x timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc$x -o write -- $B > $O/write$x.log 2>&1
  step write$x $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4 -o run -- python bench.py --steps 30 --warmup 5 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0 --median-windows 0 > $O/prof_c4.log 2>&1
step prof_c4 $?
exit 0
