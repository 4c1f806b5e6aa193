# fp16 histories: GPU tests (fp16 == rounded fp32, plus the product parity and step tests as regressions), then
# config 5 benches fp32 vs fp16 (32768 envs, height field, pushes) and the default bench.
#   bash tools/gpu/r02_fp16.sh <tag>
set -e
tag=${1:-fp16}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_fp16.py tests/test_gpu_product_parity.py tests/test_gpu_step.py \
  tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread > $out/tests.log 2>&1
for dt in fp32 fp16; do
  timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --num-envs 32768 --mesh heightfield \
    --push --state-dtype $dt > $out/cfg5_$dt.json 2>> $out/bench.err
done
timeout -k 10 300 python bench.py --steps 200 --warmup 50 --no-cpu-baseline > $out/bench_default.json 2>> $out/bench.err
timeout -k 10 300 python bench.py --steps 200 --warmup 50 --no-cpu-baseline --state-dtype fp16 > $out/bench_default_fp16.json 2>> $out/bench.err
