# Round 3: LSTM FC forward as fc_fwd_big_kernel + last-arriver ticket reduce (ARL_LSTM_XRED=0) vs the reduce
# in the gate kernel's staging (default) -- LSTM tests, then C3 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3aa}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "lstm or c3" > $O/pytest.log 2>&1
step pytest $?
tail -2 $O/pytest.log
for r in 1 2; do
  for x in 1 0; do
    ARL_LSTM_XRED=$x timeout -k 10 200 python -u bench.py --workload c3 --steps 100 --warmup 10 --cpu-seconds 0 \
      --copy-peak 0 --median-windows 100 --kernel-reps 20 > $O/c3_x${x}_$r.log 2>&1
    step "c3 xred=$x" $?
    python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']
print(sys.argv[2], d['ms_per_step'], d['windows']['median_ms'], ' '.join('%s=%.2f' % (n, v['avg_launch_us']) for n, v in k.items() if n in ('fc_fwd', 'lstm_gates', 'policy')))" $O/c3_x${x}_$r.log "c3 xred=$x"
  done
done
exit 0
