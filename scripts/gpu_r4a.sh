#!/bin/bash
# round 4 GPU check: the -m gpu suite, the default bench line (window timeline), rocprof stats of it
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4a}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread ${PYTEST_ARGS} > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" > $O/status
# test failures (1) still measure; a timeout / abort / crash ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || exit $?
echo "bench ok" >> $O/status
# conv_fwd phase stamps (ARL_CF_STAMP build) at 512 envs (two envs a workgroup) and 256
if [ -f async-rl_amd/csrc/build_var_cfstamp/libasyncrl_hip.so ]; then
  for n in 512 256; do
    ASYNCRL_HIP_LIB=$PWD/async-rl_amd/csrc/build_var_cfstamp/libasyncrl_hip.so timeout -k 10 200 python scripts/cf_stamps.py $n > $O/cfstamps$n.txt 2>&1 || exit $?
  done
fi
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o c4 -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 --copy-peak 0 > "$GRAFT_REPO_ROOT/$O/bench_prof.log" 2>&1 || exit $?
echo "prof ok" >> "$GRAFT_REPO_ROOT/$O/status"
