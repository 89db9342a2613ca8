set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gp
timeout -k 10 120 ./scripts/gemm_planes_bench > gpurun_out/gp/planes.log 2>&1; rc=$?; cat gpurun_out/gp/planes.log; exit $rc
