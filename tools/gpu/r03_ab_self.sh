# A/B of the self-collision cost: the default bench vs asset.self_collisions = 1 (not the metric's config)
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03i}
mkdir -p $out
cd $GRAFT_REPO_ROOT
for v in on off on off; do
  extra=""; [ $v = off ] && extra="--no-self-collision"
  timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 $extra > $out/bench_$v.json 2>> $out/err.log
  python -c "import json; d=json.load(open('$out/bench_$v.json')); print('$v', d['value'], d['ms_per_step'])" | tee -a $out/summary.txt
done
