# Round 3: conv_fwd two envs a workgroup (ARL_CONV_EPW) -- bitwise test, LSTM tests (worker fix),
# C4 / C3 A/B of EPW x env groups
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3k}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "two_envs or lstm" > $O/pytest.log 2>&1
step pytest $?
tail -2 $O/pytest.log
summ() {
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); w=d['windows']; k=d['kernels']
print(sys.argv[2], d['ms_per_step'], w['median_ms'], ' '.join('%s=%.2f' % (n, v['avg_launch_us']) for n, v in k.items()))" $1 "$2"
}
for r in 1 2; do
  for wl in c4 c3; do
    for arm in "1 2" "1 1" "2 1" "2 2"; do
      set -- $arm
      ARL_CONV_EPW=$1 timeout -k 10 200 python -u bench.py --workload $wl --env-groups $2 --steps 100 --warmup 10 --cpu-seconds 0 \
        --copy-peak 0 --median-windows 100 --kernel-reps 20 > $O/${wl}_e$1g$2_$r.log 2>&1
      step ${wl}_e$1g$2_$r $?
      summ $O/${wl}_e$1g$2_$r.log "$wl epw=$1 groups=$2"
    done
  done
done
exit 0
