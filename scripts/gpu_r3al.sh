# LDS-only barriers in conv_fwd (ARL_CF_LDSBAR) and the policy heads (ARL_POL_LDSBAR): C4 and C2, 3 / 2 interleaved reps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_variants.sh "--steps 100 --warmup 10 --copy-peak 0 --kernel-reps 20" 3 || exit $?
bash scripts/gpu_variants.sh "--workload c2 --steps 100 --warmup 10 --copy-peak 0 --kernel-reps 20" 2
