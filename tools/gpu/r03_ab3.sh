# interleaved A/B: the tree's library (shift delay default), the late-staging variant, and the tree at delay 0
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03h}
mkdir -p $out
cd $GRAFT_REPO_ROOT
run() {  # name, env...
  n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/bench_${n}_$rep.json 2>> $out/err.log
  python -c "import json; d=json.load(open('$out/bench_${n}_$rep.json')); print('$n rep $rep', d['value'], d['ms_per_step'])" | tee -a $out/summary.txt
}
for rep in 1 2 3; do
  run default T1ENV_LIB=
  run stage_late T1ENV_LIB=$GRAFT_REPO_ROOT/ti5_isaacgym_amd/_lib/var/stage_late.so
  run delay0 T1ENV_SHIFT_DELAY=0
done
