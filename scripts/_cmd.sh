set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_quick.sh f1 "" "--steps 100 --warmup 10 --cpu-seconds 0 --kernel-reps 20" || exit $?
for i in 1 2; do
timeout -k 10 300 python -u bench.py --workload c3 --steps 40 --warmup 5 --cpu-seconds 0 --kernel-reps 3 > gpurun_out/f1/bench_c3_$i.log 2>&1 || exit $?
done
bash scripts/gpu_prof.sh f1 "--workload c3 --steps 10 --warmup 3 --cpu-seconds 0 --kernel-reps 3"
