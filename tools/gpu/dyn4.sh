# 4-wave dynamics: GPU tests, bench (4 vs 2 waves), phase profile
set -e
tag=${1:-dyn4}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/$tag/tests.log 2>&1
timeout -k 10 180 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > gpurun_out/$tag/bench0_w4.json 2> gpurun_out/$tag/bench.err
T1ENV_DYN_WAVES=2 timeout -k 10 180 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > gpurun_out/$tag/bench0_w2.json 2>> gpurun_out/$tag/bench.err
timeout -k 10 180 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/$tag/bench_w4.json 2>> gpurun_out/$tag/bench.err
timeout -k 10 300 python tools/prof_dynamics_phases.py > gpurun_out/$tag/phases.txt 2>&1
