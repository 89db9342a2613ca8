# eager vs window graph, 3 interleaved reps: C2, C4 (1 group), C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ag
for r in 1 2 3; do
  for a in "c4 g" "c4 e" "c2 g" "c2 e" "c5 g" "c5 e"; do
    set -- $a
    x=""; [ $2 = e ] && x="--no-graph"
    timeout -k 10 200 python -u bench.py --workload $1 $x --steps 100 --warmup 10 --copy-peak 0 --cpu-seconds 0 --kernel-reps 5 > gpurun_out/r3ag/$1_$2.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/r3ag/$1_$2.log').read().strip().splitlines()[-1]); print('$a', d['ms_per_step'], d['windows']['median_ms'] if d.get('windows') else '')"
  done
done
# kernel traces of both forms at C4 (window timelines: per-kernel durations and gaps)
for m in g e; do
  x=""; [ $m = e ] && x="--no-graph"
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/r3ag/prof_$m -o run -- python3 bench.py $x --steps 30 --warmup 5 --copy-peak 0 --cpu-seconds 0 --kernel-reps 2 --median-windows 0 > gpurun_out/r3ag/prof_$m.log 2>&1 || exit $?
done
