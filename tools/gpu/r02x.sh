# r02x: full GPU test suite, default bench, rocprof kernel stats, PMC traffic, SQ counters of the product
set -e
tag=${1:-r02x}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
bash tools/gpu/profile.sh $tag
bash tools/gpu/pmc_sq.sh $tag
