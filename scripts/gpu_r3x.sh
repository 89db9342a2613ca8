# Round 3: non-temporal frame-pair loads in phi (ARL_PHI_NT) -- phi parity tests, then the in-tree library
# interleaved with the -DARL_PHI_NT=0 variant at C2 / C4 / C3 / C5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3x}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "phi or observe or ring or c5 or c2" > $O/pytest.log 2>&1
step pytest $?
tail -2 $O/pytest.log
for r in 1 2; do
  for wl in c2 c4 c3 c5; do
    for lib in async-rl_amd/asyncrl_amd/libasyncrl_hip.so async-rl_amd/csrc/build_var_*/libasyncrl_hip.so; do
      name=$(basename $(dirname $lib))
      ASYNCRL_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload $wl --steps 100 --warmup 10 --cpu-seconds 0 \
        --copy-peak 0 --median-windows 100 --kernel-reps 20 > $O/${wl}_${name}_$r.log 2>&1
      step "$wl $name" $?
      python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d.get('kernels') or {}
w=d.get('windows') or {}
print(sys.argv[2], d['ms_per_step'], w.get('median_ms'), 'phi', (k.get('phi') or {}).get('avg_launch_us'), d['roofline'].get('avg_launch_us'))" $O/${wl}_${name}_$r.log "$wl $name"
    done
  done
done
exit 0
