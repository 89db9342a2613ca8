# Bench every variant library under async-rl_amd/csrc/build_var_*/ (make variant NAME=.. DEFS=..)
# interleaved with the in-tree library, printing ms/window and per-stage launch times.
#   gpurun -- bash scripts/gpu_variants.sh "<bench args>" [reps] [variant names, default: every one except
#   the *stamp timing builds]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/var
ARGS=${1:-"--steps 30 --warmup 5"}
for r in $(seq 1 ${2:-1}); do
  LIBS="async-rl_amd/asyncrl_amd/libasyncrl_hip.so"
  if [ -n "$3" ]; then
    for v in $3; do LIBS="$LIBS async-rl_amd/csrc/build_var_$v/libasyncrl_hip.so"; done
  else
    for l in async-rl_amd/csrc/build_var_*/libasyncrl_hip.so; do case $l in *stamp/*) ;; *) LIBS="$LIBS $l" ;; esac; done
  fi
  for lib in $LIBS; do
    name=$(basename $(dirname $lib))
    ASYNCRL_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py $ARGS --cpu-seconds 0 > gpurun_out/var/$name.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -n 5 gpurun_out/var/$name.log; exit $rc; }
    python -c "import json; d=json.loads(open('gpurun_out/var/$name.log').read().strip().splitlines()[-1]); print('$name', d['ms_per_step'], d['windows']['median_ms'], {k: (v['avg_launch_us'], v.get('standalone_us')) for k, v in d['kernels'].items()})"
  done
done
exit 0
