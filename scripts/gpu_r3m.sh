# Round 3: C4 / C3 window timelines under rocprofv3 (env-group overlap), LSTM gate weight-gradient
# A/B (fc_bwd ShapeLSTM vs the round-2 generic GEMM)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3m}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
for wl in c4 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- python bench.py --workload $wl --steps 10 --warmup 3 --cpu-seconds 0 --kernel-reps 2 --copy-peak 0 --median-windows 0 > $O/prof_$wl.log 2>&1
  step prof_$wl $?
  f=$(find $O/prof_$wl -name '*kernel_trace.csv' | head -1)
  python scripts/window_timeline.py $f > $O/${wl}_timeline.txt
  head -3 $O/${wl}_timeline.txt; tail -3 $O/${wl}_timeline.txt
done
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
exit 0
