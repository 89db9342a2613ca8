# Run one gpurun call, retrying only when the pool reports no free slot / box
# (status=transient: nothing ran, nothing was charged).  A call that ran is
# never repeated.  usage: bash scripts/gpurun_retry.sh <timeout_s> <script> [args...]
T=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout $T -- bash "$@" > /tmp/gpurun_last.out 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/gpurun_last.out; then
    echo "attempt $i: transient ($(grep -o 'all .* busy\|stopped responding[^;]*\|backing off[^;]*' /tmp/gpurun_last.out | head -1)); waiting"
    sleep 90
    continue
  fi
  cat /tmp/gpurun_last.out | tail -c 4000
  exit $rc
done
echo "gave up after 12 transient attempts"
exit 3
