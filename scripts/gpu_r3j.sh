# Round 3: LSTM wgrad on fc_bwd.hip's ShapeLSTM kernel -- LSTM parity, C3 A/B vs ARL_LSTM_WGRAD=gemm,
# then learner-kernel time vs samples per workgroup (r3i)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3j}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "lstm or c3" > $O/pytest.log 2>&1
step pytest $?
tail -2 $O/pytest.log
for r in 1 2; do
  for arm in new gemm; do
    if [ $arm = gemm ]; then export ARL_LSTM_WGRAD=gemm; else unset ARL_LSTM_WGRAD; fi
    timeout -k 10 300 python -u bench.py --workload c3 --steps 100 --warmup 10 --cpu-seconds 0 --copy-peak 0 \
      --median-windows 100 --kernel-reps 20 > $O/c3_${arm}_$r.log 2>&1
    step c3_${arm}_$r $?
    python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); w=d['windows']; k=d['kernels']
print('c3', sys.argv[2], d['ms_per_step'], w['median_ms'], ' '.join('%s=%.2f' % (n, v['avg_launch_us']) for n, v in k.items()))" $O/c3_${arm}_$r.log $arm
  done
done
unset ARL_LSTM_WGRAD
bash scripts/gpu_r3i.sh ${2:-r3i}
