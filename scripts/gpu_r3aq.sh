# C3: two chains on one stream (ARL_GROUP_STREAMS=1, eager and graph) vs the two-stream graph, 2 interleaved reps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3aq
run() {  # tag graph env...
  local tag=$1 g=$2; shift 2
  env "$@" timeout -k 10 200 python -u bench.py --workload c3 --graph $g --steps 60 --warmup 10 --copy-peak 0 --cpu-seconds 0 --kernel-reps 3 > gpurun_out/r3aq/$tag.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/r3aq/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['windows']['median_ms'])"
}
for r in 1 2; do
  run base auto A=1
  run one_e off ARL_GROUP_STREAMS=1
  run one_g on ARL_GROUP_STREAMS=1
done
