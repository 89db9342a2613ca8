# Round 6: phi_ring persistent streaming form: the bitwise arm test, then ARL_PHI_PERSIST 0 / 2 / 4
# interleaved (C4 in-window times) and C2 (256 envs) 0 / 4
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r6f}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "two_envs_identical" -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_bitwise.log 2>&1 || { tail -20 gpurun_out/$T/pytest_bitwise.log; exit 1; }
tail -2 gpurun_out/$T/pytest_bitwise.log
for w in c4 c2; do
for r in 1 2; do
  for u in 0 2 4; do
    [ $w = c2 ] && [ $u = 2 ] && continue
    ARL_PHI_PERSIST=$u timeout -k 10 200 python -u bench.py --workload $w --secondary none --steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0 > gpurun_out/$T/phi_${w}_$u$r.log 2>&1 || exit $?
    python -c "
import json; d=json.loads(open('gpurun_out/$T/phi_${w}_$u$r.log').read().strip().splitlines()[-1])
k=d['kernels']['phi']; print('$w phi_persist=$u r$r', d['ms_per_step'], 'median', d['windows']['median_ms'], 'phi', k['avg_launch_us'], 'alone', k['standalone_us'])"
  done
done
done
exit 0
