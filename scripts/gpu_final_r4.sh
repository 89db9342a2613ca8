#!/bin/bash
# Round-4 measurement of the final tree, in two gpurun calls:
#   gpurun --timeout 1200 -- bash scripts/gpu_final_r4.sh suite     # -m gpu suite, smoke, bench line, rocprof
#   gpurun --timeout 1200 -- bash scripts/gpu_final_r4.sh configs   # C4 / C3 / C2 / C5 lines + stats + PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${FTAG:-final4}
mkdir -p $O
case $1 in
  suite)
    timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
    echo "pytest rc=$rc" > $O/status
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
    echo "smoke ok" >> $O/status
    timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || exit $?
    echo "bench ok" >> $O/status
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o c4 -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 --copy-peak 0 > "$GRAFT_REPO_ROOT/$O/bench_prof.log" 2>&1) || exit $?
    echo "prof ok" >> $O/status ;;
  configs)
    bash scripts/gpu_configs.sh ${FTAG:-final4}cfg ${WL:-c4 c3 c2 c5} > $O/configs.log 2>&1 || exit $?
    echo "configs ok" >> $O/status ;;
esac
