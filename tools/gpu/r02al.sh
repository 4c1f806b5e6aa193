# r02al: full GPU suite, default bench, 5-repeat median bench, rocprof kernel stats, SQ counters of the product
set -e
tag=${1:-r02al}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python bench.py --steps 480 --warmup 50 --repeats 5 --no-cpu-baseline > $out/bench_median5.json 2> $out/bench_median5.err
bash tools/gpu/profile.sh $tag
bash tools/gpu/pmc_sq.sh $tag
