# Round 3: hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4) vs env-group overlap, for the
# one multi-stream window graph and the per-chain graphs (A3C.capture_window)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3p}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
summ() {
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); w=d['windows']
print(sys.argv[2], d['ms_per_step'], w['median_ms'], w['p10_ms'], w['p90_ms'])" $1 "$2"
}
i=0
for q in 8 16 4; do
  for cfg in "c3 2 per" "c3 2 single" "c4 2 per" "c4 2 single" "c4 1 single"; do
    set -- $cfg
    i=$((i+1))
    x=""; [ $3 = single ] && x="--single-graph"
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u bench.py --workload $1 --env-groups $2 $x --steps 100 --warmup 10 \
      --cpu-seconds 0 --copy-peak 0 --median-windows 100 --kernel-reps 1 > $O/run$i.log 2>&1
    step "q$q $cfg" $?
    summ $O/run$i.log "hwq=$q $1 groups=$2 $3"
  done
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c3 -o run -- python bench.py --workload c3 --steps 10 --warmup 3 --cpu-seconds 0 --kernel-reps 1 --copy-peak 0 --median-windows 0 > $O/prof_c3.log 2>&1
step prof_c3 $?
python scripts/window_timeline.py $(find $O/prof_c3 -name '*kernel_trace.csv' | head -1) > $O/c3_timeline.txt
tail -3 $O/c3_timeline.txt
exit 0
