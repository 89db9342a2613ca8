# A/B of one build under two environment settings, interleaved:
#   gpurun -- bash scripts/env_ab.sh "<env A>" "<env B>" "<bench args>" [reps] [tag]
# e.g. bash scripts/env_ab.sh ARL_LEARN_FORK=0 ARL_LEARN_FORK=1 "--workload c2" 3
# prints ms/window (K-step wall), the median window and each stage's in-window us per launch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/envab${5:+_$5}
mkdir -p $O
tag=$(echo "$3" | tr -dc 'a-z0-9')
for r in $(seq 1 ${4:-3}); do
  for v in A B; do
    e=$1; [ $v = B ] && e=$2
    env $e timeout -k 10 200 python -u bench.py $3 --steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0 > $O/$tag$v$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -n 5 $O/$tag$v$r.log; exit $rc; }
    python -c "
import json; d=json.loads(open('$O/$tag$v$r.log').read().strip().splitlines()[-1])
print('$3', '$v$r', '$e', d['ms_per_step'], 'median', d['windows']['median_ms'], {k: v['avg_launch_us'] for k, v in d['kernels'].items() if v.get('time_source') == 'window'})"
  done
done
