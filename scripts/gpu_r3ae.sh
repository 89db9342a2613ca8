# fused FF heads in fc_fwd_big_kernel's ticket tail: bitwise identity test, then A/B at C4 (3 interleaved reps)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ae
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu \
  -k "two_envs_identical or a2_mask_bits" > gpurun_out/r3ae/pytest.log 2>&1
rc=$?; tail -n 8 gpurun_out/r3ae/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_variants.sh "--steps 100 --warmup 10 --copy-peak 0" 3
