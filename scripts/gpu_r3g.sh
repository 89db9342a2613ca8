# Round 3: env-group chains as one graph per chain (single-stream graphs replayed on
# their own streams) vs the one multi-stream window graph (scripts/multigraph.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3g}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
for args in "c4 2" "c3 2" "c4 3"; do
  timeout -k 10 200 python -u scripts/multigraph.py $args >> $O/multigraph.txt 2>&1
  step "multigraph $args" $?
done
grep -v amdgpu.ids $O/multigraph.txt
exit 0
