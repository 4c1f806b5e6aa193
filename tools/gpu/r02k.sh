# r02k: packed-f32 issue microbench (one wave alone), GPU tests, default bench.   bash tools/gpu/r02k.sh <tag>
set -e
tag=${1:-r02k}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 60 ./tools/pk_issue_bench > $out/pk_issue.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
