# Round 3: LSTM parity + C3 bench with the LSTM kernel table (gates / BPTT / wgrad stages)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3h}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "lstm or c3" > $O/pytest.log 2>&1
step pytest $?
tail -2 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c3 --steps 100 --warmup 10 --cpu-seconds 0 --copy-peak 0 --median-windows 100 --kernel-reps 20 > $O/c3_$r.log 2>&1
  step c3_$r $?
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); w=d['windows']
print('c3', d['ms_per_step'], w['median_ms'], w['p10_ms'], w['p90_ms'])
for k,v in d['kernels'].items(): print('   ', k, v['avg_launch_us'], v['launches_per_window'], v['achieved'], v['frac'])" $O/c3_$r.log
done
exit 0
