# Round 3: large-launch forward forms (conv_fwd EPW 2, fc_fwd 64-row tiles) -- bitwise + full-size
# parity, then C4 / C3 A/B against the 256-env forms, per env-group count
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-r3l}
mkdir -p $O
step() { echo "== $1 rc=$2"; [ "$2" -eq 0 ] || exit "$2"; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_configs.py -k "two_envs or lstm or c3 or c4 or env_groups" > $O/pytest.log 2>&1
step pytest $?
tail -2 $O/pytest.log
summ() {
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); w=d['windows']; k=d['kernels']
print(sys.argv[2], d['ms_per_step'], w['median_ms'], ' '.join('%s=%.2f' % (n, v['avg_launch_us']) for n, v in k.items()))" $1 "$2"
}
for r in 1 2; do
  for cfg in "c4 new 2" "c4 nofc 2" "c4 old 2" "c4 new 1" "c3 new 2" "c3 nofc 2" "c3 old 2" "c2 new 1" "c2 forced 1"; do
    set -- $cfg
    unset ARL_CONV_EPW ARL_FC_BIG
    case $2 in
      nofc) export ARL_FC_BIG=0 ;;
      old) export ARL_CONV_EPW=1 ARL_FC_BIG=0 ;;
      forced) export ARL_CONV_EPW=2 ARL_FC_BIG=1 ;;
    esac
    timeout -k 10 200 python -u bench.py --workload $1 --env-groups $3 --steps 100 --warmup 10 --cpu-seconds 0 \
      --copy-peak 0 --median-windows 100 --kernel-reps 20 > $O/$1_$2_g$3_$r.log 2>&1
    step $1_$2_g$3_$r $?
    summ $O/$1_$2_g$3_$r.log "$1 $2 groups=$3"
  done
done
unset ARL_CONV_EPW ARL_FC_BIG
exit 0
