# Round 3: the FC backward's ReLU mask as a2 > 0 bits written by conv_fwd -- tests, C2 / C4 A/B against
# job B reading a2 (ARL_FC_BWD_MASK=f32), and fc_bwd PMC FETCH / WRITE per arm at C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3u}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "mask or two_envs or window_match or c2 or c4 or fc_bwd or doom" > $O/pytest.log 2>&1
step pytest $?
tail -2 $O/pytest.log
for r in 1 2; do
  for wl in c2 c4; do
    for arm in bits f32; do
      m=""; [ $arm = f32 ] && m=f32
      ARL_FC_BWD_MASK=$m timeout -k 10 200 python -u bench.py --workload $wl --steps 100 --warmup 10 --cpu-seconds 0 \
        --copy-peak 0 --median-windows 100 --kernel-reps 20 > $O/${wl}_${arm}_$r.log 2>&1
      step "$wl $arm" $?
      python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['kernels']
print(sys.argv[2], d['ms_per_step'], d['windows']['median_ms'], 'fc_bwd', k['fc_bwd']['avg_launch_us'], 'conv_fwd', k['conv_fwd']['avg_launch_us'])" $O/${wl}_${arm}_$r.log "$wl $arm"
    done
  done
done
for arm in bits f32; do
  m=""; [ $arm = f32 ] && m=f32
  B="python bench.py --workload c2 --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3 --median-windows 0 --copy-peak 0"
  ARL_FC_BWD_MASK=$m timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_$arm -o fetch -- $B > $O/pmc_fetch_$arm.log 2>&1
  step fetch_$arm $?
  ARL_FC_BWD_MASK=$m timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_$arm -o write -- $B > $O/pmc_write_$arm.log 2>&1
  step write_$arm $?
  python scripts/traffic.py $O/pmc_$arm --envs 256 > $O/traffic_$arm.json
  python -c "
import json; d=json.load(open('$O/traffic_$arm.json')); r=d['raw']
print('$arm', {k: v for k, v in r.items() if 'fc_bwd' in k or 'conv_fwd' in k})"
done
exit 0
