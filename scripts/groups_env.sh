# Env-group window under HIP runtime graph settings (packet capture, graph queues).
#   gpurun -- bash scripts/groups_env.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/genv
mkdir -p $O
run() {  # tag, env, args
  env $2 timeout -k 10 200 python -u bench.py $3 --steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 5 > $O/$1.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { tail -n 5 $O/$1.log; exit $rc; }
  python -c "import json; d=json.loads(open('$O/$1.log').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['value'])"
}
run g1 "X=1" "--env-groups 1"
run g2 "X=1" "--env-groups 2"
run g1_nopc "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "--env-groups 1"
run g2_nopc "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "--env-groups 2"
run g2_fq1 "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "--env-groups 2"
run g2_fq4 "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "--env-groups 2"
run g2_nopc_fq4 "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4" "--env-groups 2"
