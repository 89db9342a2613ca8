# Round 3 final: C2 / C3 / C5 bench lines + rocprof stats (PMC traffic for C2 and C5; C3's eager PMC pass
# runs past its limit), MFMA busy for C4 and C2
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3ac}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
for w in c2 c3 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --steps 100 --warmup 10 --cpu-seconds 0 > $O/bench_$w.log 2>&1
  step bench_$w $?
  tail -n 1 $O/bench_$w.log | cut -c1-300
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python bench.py --workload $w --steps 10 --warmup 3 --cpu-seconds 0 --kernel-reps 10 --median-windows 0 --copy-peak 0 > $O/prof_$w.log 2>&1
  step prof_$w $?
done
for w in c2 c5; do
  B="python bench.py --workload $w --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3 --median-windows 0 --copy-peak 0"
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_$w -o fetch -- $B > $O/pmc_fetch_$w.log 2>&1
  step fetch_$w $?
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_$w -o write -- $B > $O/pmc_write_$w.log 2>&1
  step write_$w $?
done
for w in c4 c2; do
  B="python bench.py --workload $w --steps 3 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 3 --median-windows 0 --copy-peak 0"
  timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/mfma_$w -o mfma -- $B > $O/mfma_$w.log 2>&1
  step mfma_$w $?
done
exit 0
