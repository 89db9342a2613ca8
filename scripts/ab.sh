# A/B timing of two package builds, interleaved:
#   bash scripts/ab.sh <pkg root A> <pkg root B> "<bench args>" [reps]
# (a pkg root holds an asyncrl_amd/ package with its libasyncrl_hip.so, e.g.
# async-rl_amd or a copy of an older commit's build under async-rl_amd/csrc/build_abl_*)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in $(seq 1 ${4:-3}); do
  for v in A B; do
    root=$1; [ $v = B ] && root=$2
    ASYNCRL_PKG_ROOT=$PWD/$root timeout -k 10 200 python -u bench.py $3 --cpu-seconds 0 > gpurun_out/ab/$v$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -n 5 gpurun_out/ab/$v$r.log; exit $rc; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab/$v$r.log').read().strip().splitlines()[-1]); print('$v$r', d['ms_per_step'], {k: v['avg_launch_us'] for k, v in d['kernels'].items()})"
  done
done
