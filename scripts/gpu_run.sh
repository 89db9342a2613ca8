set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 -rf > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/prof.log 2>&1
echo "prof rc=$?"
