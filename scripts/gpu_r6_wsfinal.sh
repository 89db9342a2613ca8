# Round 6: the wave-specialised conv_bwd as the default: full GPU suite, smoke, interleaved A/B against the
# 512-thread kernel (ARL_CB_WS=0) at C4, C2 and C3 (secondary off)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r6n}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
bash scripts/env_ab.sh ARL_CB_WS=0 ARL_CB_WS=1 "--workload c4 --secondary none" 2 wsfinal || exit $?
bash scripts/env_ab.sh ARL_CB_WS=0 ARL_CB_WS=1 "--workload c2 --secondary none" 1 wsfinal || exit $?
bash scripts/env_ab.sh ARL_CB_WS=0 ARL_CB_WS=1 "--workload c3 --secondary none" 1 wsfinal || exit $?
exit 0
