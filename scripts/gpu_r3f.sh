# Round 3: LSTM parity (fused BPTT step, FC reduce in the gate kernel's staging), the host
# cost of a window graph replay (scripts/replay_host.py), C3 A/B of ARL_LSTM_XRED, and
# C4 eager (no graph) vs graph kernel traces for the env-group overlap.
#   gpurun --timeout 900 -- bash scripts/gpu_r3f.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3f}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
show() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); w=d.get('windows') or {}; print(sys.argv[2], d['ms_per_step'], w.get('median_ms'), w.get('p10_ms'), w.get('p90_ms'))" $1 "$2"; }
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "lstm" tests/test_gpu_configs.py -k "lstm or c3" > $O/pytest.log 2>&1
step pytest $?
tail -2 $O/pytest.log
for args in "c4 2" "c4 1" "c2 1" "c3 2"; do
  timeout -k 10 200 python -u scripts/replay_host.py $args >> $O/replay_host.txt 2>&1
  step "replay_host $args" $?
done
cat $O/replay_host.txt
Q="--workload c3 --steps 100 --warmup 10 --cpu-seconds 0 --copy-peak 0 --median-windows 100 --kernel-reps 5"
for r in 1 2; do
  for x in 0 1; do
    ARL_LSTM_XRED=$x timeout -k 10 300 python -u bench.py $Q > $O/c3_xred$x$r.log 2>&1
    step c3_xred$x $?
    show $O/c3_xred$x$r.log "c3 xred=$x"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4_eager -o run -- python bench.py --no-graph --steps 20 --warmup 5 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0 --median-windows 0 > $O/prof_c4_eager.log 2>&1
step prof_c4_eager $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python bench.py --workload c3 --steps 20 --warmup 5 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0 --median-windows 0 > $O/prof_c3.log 2>&1
step prof_c3 $?
exit 0
