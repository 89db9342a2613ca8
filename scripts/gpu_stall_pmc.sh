# Round-4 per-kernel MFMA busy and LDS / wait counters (one --pmc pass per counter set, kernel-trace
# only, eager window so every dispatch is attributed):
#   gpurun -- bash scripts/gpu_stall_pmc.sh [tag] [workloads...]
#   python scripts/mfma_util.py gpurun_out/<tag>/mfma_<w>/*counter_collection.csv
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-stall}
shift
WL=${@:-c4}
O=gpurun_out/$TAG
mkdir -p $O
timeout -s KILL 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || echo "list-avail rc=$?" >> $O/status
for w in $WL; do
  B="python bench.py --workload $w --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3 --secondary none"
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/mfma_$w -o mfma -- $B > $O/mfma_$w.log 2>&1
  rc=$?; echo "== mfma $w rc=$rc" >> $O/status; [ $rc -eq 0 ] || exit $rc
  python scripts/mfma_util.py $O/mfma_$w/*counter_collection.csv --json $O/mfma_util_$w.json > $O/mfma_util_$w.txt 2>&1
  rm -rf $O/mfma_$w   # the per-dispatch CSVs run to tens of MB; only the summary comes back
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/lds_$w -o lds -- $B > $O/lds_$w.log 2>&1
  rc=$?; echo "== lds $w rc=$rc" >> $O/status; [ $rc -eq 0 ] || exit $rc
  python scripts/lds_util.py $O/lds_$w/*counter_collection.csv --json $O/lds_util_$w.json > $O/lds_util_$w.txt 2>&1
  rm -rf $O/lds_$w
done
exit 0
