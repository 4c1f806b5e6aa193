# Round-end evidence, part A: the whole GPU suite, smoke, the default bench (with the CPU baseline), the median of five
# 480-step runs, and the BASELINE configs.   bash tools/gpu/final_a.sh <tag>
set -e
tag=${1:-final}
out=gpurun_out/$tag
mkdir -p $out
export T1_TEST_REPORT_DIR=$out T1_PARITY_REPORT=$out/parity_report.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
tail -1 $out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err
timeout -k 10 300 python bench.py --steps 480 --warmup 48 --repeats 5 --no-cpu-baseline > $out/bench_median5.json 2>> $out/bench_default.err
bash tools/gpu/configs.sh $tag
