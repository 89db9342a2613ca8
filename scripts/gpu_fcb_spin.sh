# fc_bwd job A reduce: ticket-first (ARL_FC_BWD_SPIN=1) vs publish-then-ticket.
# GPU tests under the variant, interleaved C2 windows, then one WRITE_SIZE pass per arm.
#   gpurun -- bash scripts/gpu_fcb_spin.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/spin; mkdir -p $O
ARL_FC_BWD_SPIN=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -rf > $O/pytest_spin.log 2>&1
rc=$?; tail -n 3 $O/pytest_spin.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_env_ab.sh "ARL_FC_BWD_SPIN=0" "ARL_FC_BWD_SPIN=1" "" 3 skip || exit 1
B="python bench.py --steps 4 --warmup 2 --cpu-seconds 0 --no-graph --kernel-reps 5"
for v in 0 1; do
  export ARL_FC_BWD_SPIN=$v
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc$v -o write -- $B > $O/write$v.log 2>&1 || exit 1
done
python - <<'EOF'
import csv, glob
for v in (0, 1):
    f = glob.glob(f"gpurun_out/spin/pmc{v}/**/write_counter_collection.csv", recursive=True)[0]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "fc_bwd" in r["Kernel_Name"]]
    print(f"SPIN={v} fc_bwd WRITE_SIZE KiB per dispatch: mean {sum(vals) / len(vals):.1f} over {len(vals)}")
EOF
