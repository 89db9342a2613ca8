# HIP runtime kernarg knobs on the window graph (C4 --graph on, C3) against the eager C4 window
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r3ai
run() {  # tag workload graph env...
  local tag=$1 w=$2 g=$3; shift 3
  env "$@" timeout -k 10 200 python -u bench.py --workload $w --graph $g --steps 100 --warmup 10 --copy-peak 0 --cpu-seconds 0 --kernel-reps 3 > gpurun_out/r3ai/$tag.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/r3ai/$tag.log').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['windows']['median_ms'])"
}
for r in 1 2; do
  run c4_eager c4 off A=1
  run c4_graph c4 on A=1
  run c4_g_devka1 c4 on HIP_FORCE_DEV_KERNARG=1
  run c4_g_devka0 c4 on HIP_FORCE_DEV_KERNARG=0
  run c4_g_hdp0 c4 on DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0
  run c4_g_copyopt0 c4 on DEBUG_HIP_KERNARG_COPY_OPT=0
  run c4_g_fgs0 c4 on ROC_USE_FGS_KERNARG=0
  run c4_e_devka0 c4 off HIP_FORCE_DEV_KERNARG=0
  run c3_graph c3 auto A=1
  run c3_g_hdp0 c3 auto DEBUG_CLR_KERNARG_HDP_FLUSH_WA=0
  run c3_g_copyopt0 c3 auto DEBUG_HIP_KERNARG_COPY_OPT=0
done
