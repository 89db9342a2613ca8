set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for i in 1 2; do
for v in 0 1; do
ARL_SERIAL_BACKWARD=$v timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 5 > gpurun_out/ab/c2_$v.log 2>&1 || exit $?
ARL_SERIAL_BACKWARD=$v timeout -k 10 300 python -u bench.py --workload c3 --steps 40 --warmup 5 --cpu-seconds 0 --kernel-reps 3 > gpurun_out/ab/c3_$v.log 2>&1 || exit $?
python -c "
import json
for w in ['c2','c3']:
    d=json.loads(open('gpurun_out/ab/%s_$v.log'%w).read().strip().splitlines()[-1]); print('serial=$v', w, d['value'], d['ms_per_step'])"
done
done
