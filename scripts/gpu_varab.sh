#!/bin/bash
# Interleaved A/B of variant libraries (make variant NAME=.. DEFS=..) against the in-tree build:
#   bash scripts/gpu_varab.sh TAG "<bench args>" REPS name [name ...]
# prints per run: ms/window, median window, each stage's in-window us per launch and standalone us
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; ARGS=$2; REPS=$3; shift 3
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $REPS); do
  for v in base "$@"; do
    lib=async-rl_amd/asyncrl_amd/libasyncrl_hip.so
    [ $v = base ] || lib=async-rl_amd/csrc/build_var_$v/libasyncrl_hip.so
    ASYNCRL_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py $ARGS > $O/$v.$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -n 5 $O/$v.$r.log; exit $rc; }
    python -c "
import json; d=json.loads([l for l in open('$O/$v.$r.log') if l.startswith('{')][-1])
print('$v.$r', d['ms_per_step'], d['windows']['median_ms'], {k: (v['avg_launch_us'], v.get('standalone_us')) for k, v in d['kernels'].items()})" | tee -a $O/summary.txt
  done
done
exit 0
