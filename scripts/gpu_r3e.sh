# Round 3: LSTM parity with the fused BPTT kernel (lstm.hip lstm_bptt_kernel), then
# C3 A/B of ARL_LSTM_BPTT=generic vs fused, with a kernel trace of the fused arm.
#   gpurun --timeout 900 -- bash scripts/gpu_r3e.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3e}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "lstm" tests/test_gpu_configs.py tests/test_gpu_dropin.py > $O/pytest.log 2>&1
step pytest $?
tail -3 $O/pytest.log
Q="--workload c3 --steps 100 --warmup 10 --cpu-seconds 0 --copy-peak 0 --median-windows 100 --kernel-reps 20"
for r in 1 2; do
  for a in generic fused; do
    ARL_LSTM_BPTT=$a timeout -k 10 300 python -u bench.py $Q > $O/c3_$a$r.log 2>&1
    step c3_$a $?
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d.get('windows'))" $O/c3_$a$r.log "c3 $a"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python bench.py --workload c3 --steps 20 --warmup 5 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0 --median-windows 0 > $O/prof_c3.log 2>&1
step prof_c3 $?
exit 0
