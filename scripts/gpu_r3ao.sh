# default bench line (C4) and C2 with the PMC traffic files shipped
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3ao
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit $?
tail -n 1 $O/bench.log | cut -c1-200
timeout -k 10 300 python -u bench.py --workload c2 --cpu-seconds 0 > $O/bench_c2.log 2>&1 || exit $?
tail -n 1 $O/bench_c2.log | cut -c1-200
