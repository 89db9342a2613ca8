set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abl2
for b in 0 128 256 512 896; do
  lib=async-rl_amd/csrc/build_abl$b/libasyncrl_hip.so
  [ "$b" = 0 ] && lib=async-rl_amd/asyncrl_amd/libasyncrl_hip.so
  ASYNCRL_HIP_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --kernel-reps 30 > gpurun_out/abl2/b$b.log 2>&1 || exit $?
  python -c "
import json; d=json.loads(open('gpurun_out/abl2/b$b.log').read().strip().splitlines()[-1]); k=d['kernels']
print('abl $b', 'conv_fwd', k['conv_fwd']['avg_launch_us'], 'fc_fwd', k['fc_fwd']['avg_launch_us'], 'phi', k['phi']['avg_launch_us'])"
done
