# Round 6: conv_bwd_ws_kernel with the screens committed after conv2 dW in the Y waves: bitwise arms, stamps,
# interleaved C4 A/B: ARL_CB_WS=0, the tree, prev (screens committed before conv2 dW)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r6r}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "two_envs_identical" > gpurun_out/$T/pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/$T/pytest.log; [ $rc -ne 0 ] && exit $rc
ARL_CB_WS=1 VAR=st timeout -k 10 200 python -u scripts/cb_ws_stamps.py > gpurun_out/$T/stamps_st.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/$T/stamps_st.txt | head -5; [ $rc -ne 0 ] && exit $rc
B="--workload c4 --secondary none --steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0"
for r in 1 2; do
  for v in old tree prev; do
    root=async-rl_amd; ws=1; [ $v = old ] && ws=0; [ $v = prev ] && root=async-rl_amd/csrc/build_var_prev
    ARL_CB_WS=$ws ASYNCRL_PKG_ROOT=$PWD/$root timeout -k 10 200 python -u bench.py $B > gpurun_out/$T/ab_$v$r.log 2>&1 || { tail -5 gpurun_out/$T/ab_$v$r.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/$T/ab_$v$r.log').read().strip().splitlines()[-1])
print('$v$r', d['ms_per_step'], 'median', d['windows']['median_ms'], {k: v['avg_launch_us'] for k, v in d['kernels'].items() if v.get('time_source') == 'window'})"
  done
done
exit 0
