# Round 3: learner-kernel time vs samples per workgroup (fixed cost vs per-sample cost)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3i}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
for n in 50 100 256 512 1024; do
  timeout -k 10 200 python -u bench.py --workload c2 --envs-per-gpu $n --steps 10 --warmup 3 --cpu-seconds 0 \
    --copy-peak 0 --median-windows 0 --kernel-reps 20 --env-groups 1 > $O/n$n.log 2>&1
  step n$n $?
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']
print('N', sys.argv[2], 'S', 5*int(sys.argv[2]), 'ms', d['ms_per_step'], ' '.join('%s=%.2f' % (n, k[n]['avg_launch_us']) for n in ('phi','conv_fwd','fc_fwd','policy','returns','fc_bwd','conv_bwd','conv_reduce','rmsprop')))" $O/n$n.log $n
done
exit 0
