set -e
mkdir -p gpurun_out/r1e
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r1e/tests.log 2>&1
for sb in 0 128 256 512; do
  if [ $sb -gt 0 ]; then export T1ENV_SHIFT_BLOCKS=$sb; fi
  timeout -k 10 180 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/r1e/bench_sb$sb.json 2> gpurun_out/r1e/bench_sb$sb.err
  timeout -k 10 180 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > gpurun_out/r1e/bench0_sb$sb.json 2>> gpurun_out/r1e/bench_sb$sb.err
done
