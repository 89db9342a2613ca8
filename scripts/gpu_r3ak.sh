# conv_bwd unroll variants (ARL_S2_UNROLL=2, ARL_S3_UNROLL=1) at C4 and C2, 2 interleaved reps each
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_variants.sh "--steps 100 --warmup 10 --copy-peak 0 --kernel-reps 20" 2 || exit $?
bash scripts/gpu_variants.sh "--workload c2 --steps 100 --warmup 10 --copy-peak 0 --kernel-reps 20" 2
