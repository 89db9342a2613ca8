# Timing ablations: kernel times with parts of the fused conv kernels removed
# (results are wrong by construction; only rocprof durations are read).
# Build first (in the container): for b in 1 2 4 8 16 32 64; do make -C async-rl_amd/csrc ablate ABL=$b; done
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/abl
for b in 0 ${ABL_BITS:-1 2 4 8 16 32 64}; do
  lib=async-rl_amd/csrc/build_abl$b/libasyncrl_hip.so
  [ "$b" = 0 ] && lib=async-rl_amd/asyncrl_amd/libasyncrl_hip.so
  ASYNCRL_HIP_LIB=$PWD/$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
    -d gpurun_out/abl -o abl$b -- python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --kernel-reps 5 \
    > gpurun_out/abl/abl$b.log 2>&1
  rc=$?; echo "ablate $b rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
