# C2 on the eager window: the 512-env launch forms forced at 256 envs (ARL_CONV_EPW=2, ARL_FC_BIG=1), 2 interleaved reps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ap
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python -u bench.py --workload c2 --steps 100 --warmup 10 --copy-peak 0 --cpu-seconds 0 --kernel-reps 3 > gpurun_out/r3ap/$tag.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/r3ap/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['windows']['median_ms'])"
}
for r in 1 2; do
  run base A=1
  run epw2 ARL_CONV_EPW=2
  run fcbig ARL_FC_BIG=1
  run both ARL_CONV_EPW=2 ARL_FC_BIG=1
done
