# Env-group A/B (A3C.run_window env_groups): ms/window per workload and group
# count, staggered (default) and unstaggered (ARL_GROUP_STAGGER=0), interleaved.
#   gpurun -- bash scripts/groups_ab.sh [reps] [workloads...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/groups
mkdir -p $O
run() {  # tag, env, args
  env $2 timeout -k 10 200 python -u bench.py $3 --steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 5 > $O/$1.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -n 5 $O/$1.log; exit $rc; }
  python -c "import json; d=json.loads(open('$O/$1.log').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['value'])"
}
REPS=${1:-1}
shift
WL=${@:-c2 c3 c4}
for r in $(seq 1 $REPS); do
  for w in $WL; do
    run ${w}_g1_$r "X=1" "--workload $w --env-groups 1"
    run ${w}_g2_$r "X=1" "--workload $w --env-groups 2"
    run ${w}_g2ns_$r "ARL_GROUP_STAGGER=0" "--workload $w --env-groups 2"
    run ${w}_g4ns_$r "ARL_GROUP_STAGGER=0" "--workload $w --env-groups 4"
  done
done
