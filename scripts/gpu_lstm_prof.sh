# rocprof kernel stats of the C3 bench with the LSTM cell fused (ARL_LSTM_SPLIT=0) and split (1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lstmprof
mkdir -p $O
for v in 0 1; do
  ARL_LSTM_SPLIT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s$v -o run -- python bench.py --workload c3 --steps 20 --warmup 5 --cpu-seconds 0 --kernel-reps 3 > $O/s$v.log 2>&1
  rc=$?; echo "== split=$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  tail -n 1 $O/s$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms', d['ms_per_step'])"
done
