# what-if A/B (timing only), self-collision ON (the default config): no shank terrain contact, no restitution set
# point, vs the product; and the product with self-collision off
set -e
t=${1:-r03af}
o=$GRAFT_REPO_ROOT/gpurun_out/$t
mkdir -p $o
cd $GRAFT_REPO_ROOT
V=ti5_isaacgym_amd/_lib/var
run() {  # name, lib, extra
  T1ENV_LIB=$2 timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 $3 > $o/bench_$1.json 2>> $o/err.log
  python -c "import json; d=json.load(open('$o/bench_$1.json')); print('$1', d['value'], d['ms_per_step'])" | tee -a $o/summary.txt
}
for r in 1 2; do
  run product ti5_isaacgym_amd/_lib/libt1env_hip.so ""
  run noshank $V/libt1env_noshank.so ""
  run norest $V/libt1env_norest.so ""
done
