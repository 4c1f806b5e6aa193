# r02m: correctness of the bodyc variant (dynamics/fused/parity/product tests), then interleaved A/B base/tleg/bodyc
set -e
tag=${1:-r02m}
out=gpurun_out/$tag
mkdir -p $out
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/bodyc.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dynamics.py \
  tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_gpu_product_parity.py -x -q --timeout 300 \
  --timeout-method thread > $out/bodyc.tests.log 2>&1
bash tools/gpu/ab.sh $tag base tleg bodyc
