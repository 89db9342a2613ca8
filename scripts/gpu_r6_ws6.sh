# Round 6: conv_bwd_ws2_kernel, a1 through the X waves' registers (CB_A1_REG) with the screens commit on Y / X /
# split: bitwise arms, stamps, interleaved C4 A/B: ws0, ws2 (DMA in Q), ar, arx0, arx2
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r6k}
mkdir -p gpurun_out/$T
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "two_envs_identical" > gpurun_out/$T/pytest.log 2>&1
rc=$?; tail -n 3 gpurun_out/$T/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in star:2 starx2:2; do
  var=${v%:*}; ws=${v#*:}
  ARL_CB_WS=$ws VAR=$var timeout -k 10 200 python -u scripts/cb_ws_stamps.py > gpurun_out/$T/stamps_${var}_$ws.txt 2>&1; rc=$?; echo "== $var ws=$ws"; grep -v amdgpu.ids gpurun_out/$T/stamps_${var}_$ws.txt | head -5; [ $rc -ne 0 ] && exit $rc
done
B="--workload c4 --secondary none --steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0"
for r in 1 2; do
  for v in ws0 ws2 ar:2 arx0:2 arx2:2; do
    root=async-rl_amd; ws=${v#ws}
    case $v in *:*) root=async-rl_amd/csrc/build_var_${v%:*}; ws=${v#*:};; esac
    tag=${v%:*}
    ARL_CB_WS=$ws ASYNCRL_PKG_ROOT=$PWD/$root timeout -k 10 200 python -u bench.py $B > gpurun_out/$T/ab_$tag$r.log 2>&1 || { tail -5 gpurun_out/$T/ab_$tag$r.log; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/$T/ab_$tag$r.log').read().strip().splitlines()[-1])
print('$tag$r', d['ms_per_step'], 'median', d['windows']['median_ms'], {k: v['avg_launch_us'] for k, v in d['kernels'].items() if v.get('time_source') == 'window'})"
  done
done
exit 0
