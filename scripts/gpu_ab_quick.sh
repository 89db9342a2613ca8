# quick interleaved A/B of ARL_FUSE_OBS=0 vs 1 at C2 (+ kernel stage times)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/abq
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    ARL_FUSE_OBS=$v timeout -k 10 200 python -u bench.py ${1:-} --steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 20 > $O/f$v$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -n 5 $O/f$v$r.log; exit $rc; }
    python -c "import json; d=json.loads(open('$O/f$v$r.log').read().strip().splitlines()[-1]); print('fuse=$v', d['ms_per_step'], {k: v['avg_launch_us'] for k, v in d['kernels'].items()})"
  done
done
