# A/B of the in-launch shift's delayed start (T1ENV_SHIFT_DELAY, 100 MHz ticks), interleaved, 8192 trimesh default bench
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03d2}
mkdir -p $out
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for d in 0 1500 3000 5000; do
    T1ENV_SHIFT_DELAY=$d timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/bench_d${d}_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/bench_d${d}_$rep.json')); print('delay $d rep $rep', d['value'], d['ms_per_step'])" | tee -a $out/summary.txt
  done
done
