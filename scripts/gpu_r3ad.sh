# A/B: LSTM policy rows per workgroup (ARL_POL_ROWS variants) at C3, and C3 at one env group
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_variants.sh "--workload c3 --steps 60 --warmup 5 --copy-peak 0" 2 || exit $?
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --workload c3 --steps 60 --warmup 5 --copy-peak 0 --cpu-seconds 0 --env-groups 1 > gpurun_out/var/g1.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/var/g1.log').read().strip().splitlines()[-1]); print('g1', d['ms_per_step'], {k: v['avg_launch_us'] for k, v in d['kernels'].items()})"
done
