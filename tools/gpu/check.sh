# GPU check: pytest -m gpu, then bench.py at the metric's config and at config 5 (uninstrumented timing for value).
#   bash tools/gpu/check.sh <tag> [pytest -k expr]  -> gpurun_out/<tag>/{tests.log,bench.json,cfg5.json}
set -e
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p $out
export T1_TEST_REPORT_DIR=$out
if [ -n "$2" ]; then sel=(-k "$2"); else sel=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread "${sel[@]}" > $out/tests.log 2>&1
timeout -k 10 180 python bench.py --steps 480 --warmup 48 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
timeout -k 10 180 python bench.py --steps 480 --warmup 48 --no-cpu-baseline --num-envs 32768 --mesh heightfield \
    --state-dtype fp16 --push > $out/cfg5.json 2>> $out/bench.err
