# phi fused into the conv forward (ARL_FUSE_OBS=1) vs separate launches, eager windows at C4 / C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3aj
run() {  # tag workload env...
  local tag=$1 w=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --workload $w --steps 100 --warmup 10 --copy-peak 0 --cpu-seconds 0 --kernel-reps 3 > gpurun_out/r3aj/$tag.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/r3aj/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['windows']['median_ms'])"
}
for r in 1 2 3; do
  run c4_sep c4 ARL_FUSE_OBS=0
  run c4_fused c4 ARL_FUSE_OBS=1
  run c2_sep c2 ARL_FUSE_OBS=0
  run c2_fused c2 ARL_FUSE_OBS=1
done
