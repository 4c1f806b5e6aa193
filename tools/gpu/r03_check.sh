# round-3 GPU check: every -m gpu test (parity report of the worst per-field errors), then the default bench line.
#   bash tools/gpu/r03_check.sh <tag>  -> gpurun_out/<tag>/{tests.log,parity_report.json,bench.json}
set -e
tag=${1:-r03}
out=gpurun_out/$tag
mkdir -p $out
T1_PARITY_REPORT=$out/parity_report.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python bench.py --steps 300 --warmup 50 > $out/bench.json 2> $out/bench.err
