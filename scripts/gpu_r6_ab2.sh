# Round 6: A/Bs (interleaved, C4 in-window times): the split residuals as scalar subs (build_var_ss,
# -DARL_SPLIT_SCALAR) against the tree's build; RMSProp ARL_RMS_U 1 / 2 / 4; then the RMSProp size sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r6e}
mkdir -p gpurun_out/$T
B="--workload c4 --secondary none --steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0"
for r in 1 2; do
  for v in base ss; do
    root=async-rl_amd; [ $v = ss ] && root=async-rl_amd/csrc/build_var_ss
    ASYNCRL_PKG_ROOT=$PWD/$root timeout -k 10 200 python -u bench.py $B > gpurun_out/$T/ab_$v$r.log 2>&1 || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/$T/ab_$v$r.log').read().strip().splitlines()[-1])
print('$v$r', d['ms_per_step'], 'median', d['windows']['median_ms'], {k: v['avg_launch_us'] for k, v in d['kernels'].items() if v.get('time_source') == 'window'})"
  done
done
for r in 1 2; do
  for u in 1 2 4; do
    ARL_RMS_U=$u timeout -k 10 200 python -u bench.py $B > gpurun_out/$T/rms_u$u$r.log 2>&1 || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/$T/rms_u$u$r.log').read().strip().splitlines()[-1])
k=d['kernels']['rmsprop']; print('rms_u$u$r', d['ms_per_step'], 'median', d['windows']['median_ms'], 'rmsprop', k['avg_launch_us'], 'alone', k['standalone_us'])"
  done
done
timeout -k 10 180 python -u scripts/rms_sweep.py gpurun_out/$T/rms_sweep.json > gpurun_out/$T/rms_sweep.log 2>&1 || exit $?
cat gpurun_out/$T/rms_sweep.log
bash scripts/gpu_r6_phi.sh ${T}_phi || exit $?
exit 0
