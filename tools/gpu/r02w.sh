# r02w: merged foot+shank terrain queries on the helper (pkm) vs packed contact (pk) vs base
set -e
out=gpurun_out/r02w
mkdir -p $out
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/pkm.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dynamics.py \
  tests/test_gpu_fused.py tests/test_gpu_product_parity.py -x -q --timeout 300 \
  --timeout-method thread > $out/pkm.tests.log 2>&1
bash tools/gpu/ab.sh r02w base pk pkm
