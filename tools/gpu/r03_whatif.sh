# what-if A/B of the round-3 additions (timing only; self-collision off in every run, like round 2's step), plus the
# product with self-collision on
set -e
t=${1:-r03t}
o=$GRAFT_REPO_ROOT/gpurun_out/$t
mkdir -p $o
cd $GRAFT_REPO_ROOT
V=ti5_isaacgym_amd/_lib/var
run() {  # name, lib, extra
  T1ENV_LIB=$2 timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 $3 > $o/bench_$1.json 2>> $o/err.log
  python -c "import json; d=json.load(open('$o/bench_$1.json')); print('$1', d['value'], d['ms_per_step'])" | tee -a $o/summary.txt
}
for r in 1 2; do
  run product_off ti5_isaacgym_amd/_lib/libt1env_hip.so --no-self-collision
  run nolog $V/libt1env_nolog.so --no-self-collision
  run noself $V/libt1env_noself.so --no-self-collision
  run norest $V/libt1env_norest.so --no-self-collision
  run none3 $V/libt1env_none3.so --no-self-collision
  run product_on ti5_isaacgym_amd/_lib/libt1env_hip.so ""
done
