# Run one gpurun command, retrying only while the pool reports no box / a transient
# infrastructure failure (gpurun exit code 3); any other outcome ends it.
#   bash scripts/gpurun_wait.sh <timeout_s> <attempts> '<command>'
for i in $(seq 1 $2); do
  /usr/local/graft/bin/gpurun --timeout $1 -- "$3"
  rc=$?
  echo "== attempt $i rc=$rc"
  [ $rc -ne 3 ] && exit $rc
  sleep 240
done
exit 3
