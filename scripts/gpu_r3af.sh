# eager (no window graph) env-group chains vs the graph: C4 at 1 / 2 groups, C3 at 2 groups
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3af
for r in 1 2; do
  for a in "c4 1 g" "c4 1 e" "c4 2 e" "c3 2 g" "c3 2 e"; do
    set -- $a
    x=""; [ $3 = e ] && x="--no-graph"
    timeout -k 10 200 python -u bench.py --workload $1 --env-groups $2 $x --steps 60 --warmup 10 --copy-peak 0 --cpu-seconds 0 --kernel-reps 5 > gpurun_out/r3af/$1_$2_$3.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/r3af/$1_$2_$3.log').read().strip().splitlines()[-1]); print('$a', d['ms_per_step'], d['windows']['median_ms'])"
  done
done
