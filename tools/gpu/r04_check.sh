# round-4 GPU check: the dynamics tests first (k_dyn5 is the default kernel), then every -m gpu test, then the bench
# line and a k_dyn4 A/B line.
#   bash tools/gpu/r04_check.sh <tag> [pytest -k expr]  -> gpurun_out/<tag>/{tests.log,parity_report.json,bench*.json}
set -e
tag=${1:-r04}
kexpr=${2:-}
out=gpurun_out/$tag
# (the dynamics kernel: the default, k_dyn5; the tests parametrize both)
mkdir -p $out
if [ -n "$kexpr" ]; then
  T1_PARITY_REPORT=$out/parity_report.json timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 200 \
      --timeout-method thread -k "$kexpr" > $out/tests.log 2>&1 || echo "TESTS FAILED rc=$?" >> $out/tests.log
else
  T1_PARITY_REPORT=$out/parity_report.json timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 \
      --timeout-method thread > $out/tests.log 2>&1 || echo "TESTS FAILED rc=$?" >> $out/tests.log
fi
grep -q "Fatal\|core dumped\|Aborted\|Segmentation" $out/tests.log && exit 3
timeout -k 10 300 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
T1ENV_DYN_KERNEL=4 timeout -k 10 300 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > $out/bench_dyn4.json 2>> $out/bench.err
tail -3 $out/tests.log
cat $out/bench.json $out/bench_dyn4.json
