# SQ counter passes (two, each within the per-block limits) for the in-tree library
# and each given variant library, eager launches so every dispatch is attributed.
#   gpurun -- bash scripts/gpu_pmc_lib.sh <tag> [build_var_x ...]
#   python scripts/pmc_summary.py gpurun_out/<tag>/<lib>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=$1
shift
B="python bench.py --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3"
for v in asyncrl_amd "$@"; do
  lib=$PWD/async-rl_amd/csrc/$v/libasyncrl_hip.so
  [ "$v" = asyncrl_amd ] && lib=$PWD/async-rl_amd/asyncrl_amd/libasyncrl_hip.so
  O=gpurun_out/$TAG/$v
  mkdir -p $O
  ASYNCRL_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $O -o sq1 -- $B > $O/sq1.log 2>&1
  rc=$?; echo "$v sq1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
  ASYNCRL_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O -o sq2 -- $B > $O/sq2.log 2>&1
  rc=$?; echo "$v sq2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
exit 0
