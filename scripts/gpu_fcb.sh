# FC backward A/B (fc_bwd_kernel vs ARL_FC_BWD=gemm, each job alone) + one PMC pass.
#   gpurun -- bash scripts/gpu_fcb.sh [n_envs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
N=${1:-256}
O=gpurun_out/fcb; mkdir -p $O
for v in "" "ARL_FC_BWD=gemm" "ARL_FC_BWD_JOBS=a" "ARL_FC_BWD_JOBS=b"; do
  env $v timeout -k 10 60 python -u scripts/fc_bwd_bench.py $N 200 || exit 1
done
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/pmc -o p -- python scripts/fc_bwd_bench.py $N 20 > $O/pmc.log 2>&1 || exit 1
python scripts/pmc_one.py $O/pmc fc_bwd
