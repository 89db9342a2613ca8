# Round 3: LSTM parity with the fused BPTT kernel (lstm_bptt_kernel) and the FC reduce in
# the gate kernel's staging (lstm_gates_kernel<true>); A/Bs: env-group issue order at C4
# and C3 (ARL_GROUP_ORDER=chain / interleave, stagger off), ARL_LSTM_BPTT=generic,
# ARL_LSTM_XRED=0, one env group; kernel traces of C4 / C3.
#   gpurun --timeout 900 -- bash scripts/gpu_r3e.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3e}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); w=d.get('windows') or {}; print(sys.argv[2], d['ms_per_step'], w.get('median_ms'), w.get('p10_ms'), w.get('p90_ms'))" $1 "$2"; }
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "lstm" tests/test_gpu_configs.py tests/test_gpu_dropin.py > $O/pytest.log 2>&1
step pytest $?
tail -2 $O/pytest.log
Q="--steps 100 --warmup 10 --cpu-seconds 0 --copy-peak 0 --median-windows 100 --kernel-reps 5"
for r in 1 2; do
  for v in "X=1" "ARL_GROUP_ORDER=chain" "ARL_GROUP_STAGGER=0"; do
    tag=$(echo $v | tr -d ' =_' | tr 'A-Z' 'a-z')
    env $v timeout -k 10 300 python -u bench.py --workload c4 $Q > $O/c4_$tag$r.log 2>&1
    step c4_$tag $?
    show $O/c4_$tag$r.log "c4 $v"
  done
  for v in "X=1" "ARL_GROUP_ORDER=chain" "ARL_LSTM_BPTT=generic" "ARL_LSTM_XRED=0" "ARL_GROUP_STAGGER=0"; do
    tag=$(echo $v | tr -d ' =_' | tr 'A-Z' 'a-z')
    env $v timeout -k 10 300 python -u bench.py --workload c3 $Q > $O/c3_$tag$r.log 2>&1
    step c3_$tag $?
    show $O/c3_$tag$r.log "c3 $v"
  done
  timeout -k 10 300 python -u bench.py --workload c3 $Q --env-groups 1 > $O/c3_g1$r.log 2>&1
  step c3_g1 $?
  show $O/c3_g1$r.log "c3 groups=1"
done
for w in c4 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python bench.py --workload $w --steps 20 --warmup 5 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0 --median-windows 0 > $O/prof_$w.log 2>&1
  step prof_$w $?
done
exit 0
