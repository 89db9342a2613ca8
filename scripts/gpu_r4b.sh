#!/bin/bash
# round 4: bench tests, the default bench line + conv_fwd stamps + rocprof stats, then A/Bs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r4b}; mkdir -p $O
export TMPDIR=/tmp
# PYTEST_K: the -k expression (default "bench"; ALL: the whole -m gpu suite)
K=${PYTEST_K:-bench}
if [ "$K" = ALL ]; then KA=(); else KA=(-k "$K"); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "${KA[@]}" > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc" > $O/status
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > $O/bench.log 2>&1 || exit $?
echo "bench ok" >> $O/status
if [ "${CFSTAMP:-0}" = 1 ] && [ -f async-rl_amd/csrc/build_var_cfstamp/libasyncrl_hip.so ]; then
  for n in 512 256; do
    ASYNCRL_HIP_LIB=$PWD/async-rl_amd/csrc/build_var_cfstamp/libasyncrl_hip.so timeout -k 10 200 python scripts/cf_stamps.py $n > $O/cfstamps$n.txt 2>&1 || exit $?
  done
fi
if [ "${CBSTAMP:-0}" = 1 ] && [ -f async-rl_amd/csrc/build_var_cbstamp/libasyncrl_hip.so ]; then
  for n in 512 256; do
    ASYNCRL_HIP_LIB=$PWD/async-rl_amd/csrc/build_var_cbstamp/libasyncrl_hip.so timeout -k 10 200 python scripts/cb_stamps.py $n > $O/cbstamps$n.txt 2>&1 || exit $?
  done
fi
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o c4 -- python3 "$GRAFT_REPO_ROOT/bench.py" --cpu-seconds 0 --copy-peak 0 > "$GRAFT_REPO_ROOT/$O/bench_prof.log" 2>&1) || exit $?
echo "prof ok" >> $O/status
for ab in $AB; do
  case $ab in
    phidma) bash scripts/env_ab.sh ARL_PHI_DMA=0 ARL_PHI_DMA=1 "" 2 phidma || exit $? ;;
    variants) for w in ${VARWL:-c4 c2}; do
                bash scripts/gpu_variants.sh "--workload $w --steps 100 --warmup 10 --kernel-reps 3 --copy-peak 0 --secondary none" 2 "$VARIANTS" > $O/variants_$w.txt 2>&1 || exit $?
              done ;;
    varparity) for v in $VARIANTS; do
                 ASYNCRL_HIP_LIB=$PWD/async-rl_amd/csrc/build_var_$v/libasyncrl_hip.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "configs or window_matches or norm_fold" > $O/varparity_$v.log 2>&1 || exit $?
               done ;;
    norm) bash scripts/env_ab.sh ARL_NORM_TICKET=1 ARL_NORM_TICKET=0 "" 2 norm || exit $?
          bash scripts/env_ab.sh ARL_NORM_TICKET=1 ARL_NORM_TICKET=0 "--workload c2" 2 normc2 || exit $? ;;
    c3g) for r in 1 2; do for g in 1 2; do
           timeout -k 10 200 python -u bench.py --workload c3 --env-groups $g --steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 5 --copy-peak 0 --secondary none > $O/c3g$g.$r.log 2>&1 || exit $?
           python -c "import json; d=json.loads(open('$O/c3g$g.$r.log').read().strip().splitlines()[-1]); print('c3 env_groups $g', d['ms_per_step'], d['windows']['median_ms'], d['config'].get('graph'))"
         done; done ;;
    fcbabl) FCB_N=512 ABLS="0 1 2 3 4" bash scripts/gpu_fcb_abl.sh > $O/fcbabl512.txt 2>&1 || exit $?
            timeout -k 10 60 python -u scripts/fc_bwd_bench.py 512 200 >> $O/fcbabl512.txt 2>&1 || exit $? ;;
    fcbpmc) for v in default $VARIANTS; do
              L=$PWD/async-rl_amd/asyncrl_amd/libasyncrl_hip.so; [ $v = default ] || L=$PWD/async-rl_amd/csrc/build_var_$v/libasyncrl_hip.so
              for j in a b x; do for c in FETCH_SIZE WRITE_SIZE; do
                (cd /tmp && ASYNCRL_HIP_LIB=$L ARL_FC_BWD_JOBS=$j timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/fcbpmc_${v}_${j}_$c" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/fc_bwd_bench.py" 512 20 > "$GRAFT_REPO_ROOT/$O/fcbpmc_${v}_${j}_$c.log" 2>&1) || exit $?
                echo "$v jobs=$j $(python scripts/pmc_one.py $O/fcbpmc_${v}_${j}_$c fc_bwd_kernel 2>&1)" >> $O/fcbpmc.txt
              done; done
              for j in a b x; do echo "$v jobs=$j $(ASYNCRL_HIP_LIB=$L ARL_FC_BWD_JOBS=$j timeout -k 10 60 python -u scripts/fc_bwd_bench.py 512 200 2>&1 | tail -1)" >> $O/fcbpmc.txt; done
            done ;;
    rmsu) bash scripts/env_ab.sh ARL_RMS_U=1 ARL_RMS_U=2 "" 2 rmsu || exit $? ;;
    fcbz) for z in 2 4 5; do bash scripts/env_ab.sh ARL_FC_BWD_Z=3 ARL_FC_BWD_Z=$z "" 1 fcbz$z || exit $?; done ;;
  esac
  echo "ab $ab ok" >> $O/status
done
