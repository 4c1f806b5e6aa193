# r02s: in-launch history shift MLP: per-unit loop with deeper unroll (sh_u*) and contiguous ranges (shc_u*)
set -e
out=gpurun_out/r02s
mkdir -p $out
for v in shc_u16 shc_u8; do
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py \
  tests/test_gpu_step.py tests/test_gpu_product_parity.py tests/test_gpu_reset_idx.py -x -q --timeout 300 \
  --timeout-method thread > $out/$v.tests.log 2>&1
done
bash tools/gpu/ab.sh r02s base sh_u8 sh_u16 shc_u4 shc_u8 shc_u16
