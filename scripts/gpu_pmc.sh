# PMC passes (counters only with kernel-trace; separate passes per TCC counter).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
B="python bench.py --steps 4 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 5"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d gpurun_out/pmc -o sq1 -- $B > gpurun_out/pmc/sq1.log 2>&1
echo "sq1 rc=$?"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc -o sq2 -- $B > gpurun_out/pmc/sq2.log 2>&1
echo "sq2 rc=$?"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc -o fetch -- $B > gpurun_out/pmc/fetch.log 2>&1
echo "fetch rc=$?"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc -o write -- $B > gpurun_out/pmc/write.log 2>&1
echo "write rc=$?"
ls -la gpurun_out/pmc
