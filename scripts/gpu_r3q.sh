# Round 3: conv_bwd LDS read-ahead (steps 2 / 3) -- conv parity tests, then variants interleaved with the
# in-tree library at C2 / C4 (conv_bwd launch time + window)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3q}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "conv or c2 or c4 or window" > $O/pytest.log 2>&1
step pytest $?
tail -2 $O/pytest.log
for r in 1 2; do
  for wl in c2 c4; do
    for lib in async-rl_amd/asyncrl_amd/libasyncrl_hip.so async-rl_amd/csrc/build_var_*/libasyncrl_hip.so; do
      name=$(basename $(dirname $lib))
      ASYNCRL_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload $wl --steps 100 --warmup 10 --cpu-seconds 0 \
        --copy-peak 0 --median-windows 100 --kernel-reps 20 > $O/${wl}_${name}_$r.log 2>&1
      step "$wl $name" $?
      python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']
print(sys.argv[2], d['ms_per_step'], d['windows']['median_ms'], 'conv_bwd', k['conv_bwd']['avg_launch_us'], 'fc_bwd', k['fc_bwd']['avg_launch_us'])" $O/${wl}_${name}_$r.log "$wl $name"
    done
  done
done
exit 0
