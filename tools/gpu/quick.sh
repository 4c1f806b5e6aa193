# quick GPU iteration: GPU tests, uninstrumented + sampled bench, phase profile
#   bash tools/gpu/quick.sh <tag>
set -e
tag=${1:-quick}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 180 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/bench0.json 2> $out/bench.err
timeout -k 10 180 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > $out/bench.json 2>> $out/bench.err
timeout -k 10 300 python tools/prof_dynamics_phases.py > $out/phases.txt 2>&1
