# GPU tests, then an interleaved A/B of the LSTM cell fused (ARL_LSTM_SPLIT=0)
# vs separate launches at C3, then the MFMA-utilisation PMC pass at C2 / C3
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lstm
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; tail -n 4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 1 0; do
    ARL_LSTM_SPLIT=$v timeout -k 10 200 python -u bench.py --workload c3 --steps 40 --warmup 5 --cpu-seconds 0 --kernel-reps 10 > $O/c3_split$v$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -n 5 $O/c3_split$v$r.log; exit $rc; }
    python -c "import json; d=json.loads(open('$O/c3_split$v$r.log').read().strip().splitlines()[-1]); print('c3 split=$v', d['ms_per_step'], d['value'])"
  done
done
bash scripts/gpu_mfma_pmc.sh mfma_r02 c2 c3
