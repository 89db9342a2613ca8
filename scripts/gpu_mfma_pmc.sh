# MFMA utilisation per kernel (north-star evidence for the conv / FC / LSTM
# contractions): one --pmc pass (SQ + GRBM counters only) per workload, with
# kernel-trace for durations, eager (--no-graph) so every dispatch is attributed.
#   gpurun -- bash scripts/gpu_mfma_pmc.sh [tag] [workloads...]
#   python scripts/mfma_util.py gpurun_out/<tag>/mfma_<w>/*counter_collection.csv
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-mfma}
shift
WL=${@:-c2 c3}
O=gpurun_out/$TAG
mkdir -p $O
for w in $WL; do
  B="python bench.py --workload $w --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3"
  timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/mfma_$w -o mfma -- $B > $O/mfma_$w.log 2>&1
  rc=$?; echo "== $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
