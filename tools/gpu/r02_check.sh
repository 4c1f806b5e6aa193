# GPU tests (all), the product-parity mutation check (a capture-substep mutant must FAIL the product parity test),
# and the default bench.   bash tools/gpu/r02_check.sh <tag>
set -e
tag=${1:-check}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
if T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/mutant_capture.so timeout -k 10 300 python -u -m pytest \
    tests/test_gpu_product_parity.py -x -q --timeout 200 --timeout-method thread -k config3 > $out/mutant.log 2>&1; then
  echo "MUTANT SURVIVED" >> $out/mutant.log; exit 3
fi
grep -q "dof_lag_sample\|obs" $out/mutant.log && echo "mutant killed" >> $out/mutant.log
timeout -k 10 300 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
