# Round 3: per-chain window graphs (A3C.capture_window) -- identity tests, then A/B against the one
# multi-stream window graph (--single-graph) at C3 / C4, and a C3 window timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3o}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "capture_window or env_groups" > $O/pytest.log 2>&1
step pytest $?
tail -2 $O/pytest.log
summ() {
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); w=d['windows']
print(sys.argv[2], d['ms_per_step'], w['median_ms'], w['p10_ms'], w['p90_ms'])" $1 "$2"
}
i=0
for r in 1 2; do
  for cfg in "c3 2 per" "c3 2 single" "c3 3 per" "c4 2 per" "c4 1 per" "c4 2 single"; do
    set -- $cfg
    i=$((i+1))
    x=""; [ $3 = single ] && x="--single-graph"
    timeout -k 10 200 python -u bench.py --workload $1 --env-groups $2 $x --steps 100 --warmup 10 --cpu-seconds 0 \
      --copy-peak 0 --median-windows 100 --kernel-reps 1 > $O/run$i.log 2>&1
    step "$cfg" $?
    summ $O/run$i.log "$1 groups=$2 $3"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c3 -o run -- python bench.py --workload c3 --steps 10 --warmup 3 --cpu-seconds 0 --kernel-reps 1 --copy-peak 0 --median-windows 0 > $O/prof_c3.log 2>&1
step prof_c3 $?
python scripts/window_timeline.py $(find $O/prof_c3 -name '*kernel_trace.csv' | head -1) > $O/c3_timeline.txt
tail -3 $O/c3_timeline.txt
exit 0
