# r02ao: actor-frame noise drawn by the helpers into LDS (hnoise): tests + A/B
set -e
out=gpurun_out/r02ao
mkdir -p $out
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/hnoise.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py \
  tests/test_gpu_product_parity.py tests/test_gpu_step.py tests/test_gpu_fp16.py -x -q --timeout 300 \
  --timeout-method thread > $out/hnoise.tests.log 2>&1
bash tools/gpu/ab.sh r02ao base hnoise
