# GPU check: pytest -m gpu, then bench.py sampled (--time-every 8) and uninstrumented (--time-every 0).
#   bash tools/gpu/check.sh <tag>   -> gpurun_out/<tag>/{tests.log,bench.json,bench0.json}
set -e
tag=${1:-check}
mkdir -p gpurun_out/$tag
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/$tag/tests.log 2>&1
timeout -k 10 180 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err
timeout -k 10 180 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > gpurun_out/$tag/bench0.json 2>> gpurun_out/$tag/bench.err
