# the N > 1 window (one-rank RCCL group, ARL_BENCH_FORCE_DIST=1): window graph vs eager launches, 3 interleaved reps
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3am
for r in 1 2 3; do
  for g in on off; do
    ARL_BENCH_FORCE_DIST=1 timeout -k 10 200 python -u bench.py --gpus 1 --graph $g --steps 100 --warmup 10 --copy-peak 0 --cpu-seconds 0 --kernel-reps 3 > gpurun_out/r3am/$g.log 2>&1 || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/r3am/$g.log').read().strip().splitlines()[-1]); print('$g', d['ms_per_step'], d['windows']['median_ms'], d.get('collectives'), d['config']['graph'])"
  done
done
