# r02u: 32-bit row-local in-launch shift (shl_u*): tests, decimation split, A/B against the contiguous 64-bit shift
set -e
out=gpurun_out/r02u
mkdir -p $out
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/shl_u16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py \
  tests/test_gpu_step.py tests/test_gpu_product_parity.py tests/test_gpu_reset_idx.py tests/test_gpu_fp16.py -x -q \
  --timeout 300 --timeout-method thread > $out/shl_u16.tests.log 2>&1
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/shl_u16.so timeout -k 10 300 python tools/decimation_timing.py > $out/dec_shl_u16.json 2> $out/err.log
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/shl_u8.so timeout -k 10 300 python tools/decimation_timing.py > $out/dec_shl_u8.json 2>> $out/err.log
bash tools/gpu/ab.sh r02u shc_u16 shl_u8 shl_u16
