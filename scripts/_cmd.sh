set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/doom
for cfg in "--arch doom_ff --doom-width 640" "--arch doom_ff --doom-width 160" "--arch doom_lstm --envs-per-gpu 1024 --doom-width 640"; do
  timeout -k 10 200 python -u bench.py $cfg --steps 100 --warmup 10 --cpu-seconds 0 > gpurun_out/doom/b.log 2>&1 || { tail -n 20 gpurun_out/doom/b.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/doom/b.log').read().strip().splitlines()[-1]); print('$cfg', d['ms_per_step'], d['value'], {k: (v['avg_launch_us'], v['frac']) for k, v in d['kernels'].items()})"
done
