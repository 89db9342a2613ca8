# Round 3: HIP graph submission knobs vs env-group overlap (one multi-stream window graph; C3 at two
# chains of 512, C4 at two of 256) and a C3 timeline under the best-looking knob
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3n}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
summ() {
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); w=d['windows']
print(sys.argv[2], d['ms_per_step'], w['median_ms'])" $1 "$2"
}
i=0
for knob in "X=0" "DEBUG_HIP_FORCE_GRAPH_QUEUES=1" "DEBUG_HIP_FORCE_GRAPH_QUEUES=2" "DEBUG_HIP_FORCE_GRAPH_QUEUES=4" \
            "DEBUG_HIP_GRAPH_BATCH_SIZE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=4" "DEBUG_HIP_GRAPH_BATCH_SIZE=64" \
            "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0"; do
  for cfg in "c3 2" "c4 2"; do
    set -- $cfg
    i=$((i+1))
    env $knob timeout -k 10 200 python -u bench.py --workload $1 --env-groups $2 --single-graph --steps 100 --warmup 10 \
      --cpu-seconds 0 --copy-peak 0 --median-windows 100 --kernel-reps 1 > $O/run$i.log 2>&1
    step "$knob $1 g$2" $?
    summ $O/run$i.log "[$knob] $1 groups=$2"
  done
done
exit 0
