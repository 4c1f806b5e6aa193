# A/B grid of the in-launch shift: workgroup count (T1ENV_SHIFT_BLOCKS; default = the 128 CUs the dynamics leave at
# 8192 envs) x delayed start (T1ENV_SHIFT_DELAY, 100 MHz ticks), interleaved twice, 8192 trimesh default bench
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03g}
mkdir -p $out
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for cfg in 128:0 128:2000 96:0 96:2000 112:1000 128:4000; do
    sb=${cfg%%:*}; d=${cfg##*:}
    T1ENV_SHIFT_BLOCKS=$sb T1ENV_SHIFT_DELAY=$d timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/bench_${sb}_${d}_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/bench_${sb}_${d}_$rep.json')); print('blocks $sb delay $d rep $rep', d['value'], d['ms_per_step'])" | tee -a $out/summary.txt
  done
done
