# fc_bwd bf16-split MFMA steps vs the exact-f32 16x16x4 steps (ARL_FC_BWD_F32=1):
# GPU tests, the stage alone per variant, then interleaved C2 bench windows.
#   gpurun -- bash scripts/gpu_fcb_split.sh [n_envs]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
N=${1:-256}
O=gpurun_out/fcbs; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in "ARL_FC_BWD_F32=1" "ARL_FC_BWD_F32=0" "ARL_FC_BWD_F32=1 ARL_FC_BWD_BM=64" \
         "ARL_FC_BWD_F32=1 ARL_FC_BWD_JOBS=a" "ARL_FC_BWD_F32=0 ARL_FC_BWD_JOBS=a" \
         "ARL_FC_BWD_F32=1 ARL_FC_BWD_JOBS=b" "ARL_FC_BWD_F32=0 ARL_FC_BWD_JOBS=b"; do
  env $v timeout -k 10 60 python -u scripts/fc_bwd_bench.py $N 200 | sed "s/\$/ [$v]/" || exit 1
done
for r in 1 2 3; do
  for f in 1 0; do
    ARL_FC_BWD_F32=$f timeout -k 10 200 python -u bench.py --steps 100 --warmup 10 --kernel-reps 20 --cpu-seconds 0 > $O/b$f$r.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -n 5 $O/b$f$r.log; exit $rc; }
    python -c "import json; d=json.loads(open('$O/b$f$r.log').read().strip().splitlines()[-1]); print('F32=$f r$r', d['ms_per_step'], d['kernels']['fc_bwd']['avg_launch_us'])"
  done
done
