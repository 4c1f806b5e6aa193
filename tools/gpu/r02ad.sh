# r02ad: PD torques on the contact helper (hpd): correctness + A/B
set -e
out=gpurun_out/r02ad
mkdir -p $out
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/hpd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dynamics.py \
  tests/test_gpu_fused.py tests/test_gpu_product_parity.py tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread > $out/hpd.tests.log 2>&1
bash tools/gpu/ab.sh r02ad base hpd
