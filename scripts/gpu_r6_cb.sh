# Round 6: conv_bwd merged-phase form: GPU tests, then A/Bs (interleaved) of the step order
# (ARL_CB_ORDER 0 / 1) and of the whole build against the previous commit's package (build_var_old)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r6d}
bash scripts/gpu_r6.sh $T pytest || exit $?
bash scripts/env_ab.sh ARL_CB_ORDER=0 ARL_CB_ORDER=1 "--workload c4 --secondary none" 2 cborder || exit $?
mkdir -p gpurun_out/$T
for r in 1 2; do
  for v in old new; do
    root=async-rl_amd/csrc/build_var_old; [ $v = new ] && root=async-rl_amd
    ASYNCRL_PKG_ROOT=$PWD/$root timeout -k 10 200 python -u bench.py --workload c4 --secondary none --steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0 > gpurun_out/$T/ab_$v$r.log 2>&1 || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/$T/ab_$v$r.log').read().strip().splitlines()[-1])
print('$v$r', d['ms_per_step'], 'median', d['windows']['median_ms'], {k: v['avg_launch_us'] for k, v in d['kernels'].items() if v.get('time_source') == 'window'})"
  done
done
exit 0
