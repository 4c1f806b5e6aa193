# r02ak: forward-pass poses kept for the backward pass (kpose): tests + A/B
set -e
out=gpurun_out/r02ak
mkdir -p $out
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/kpose.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dynamics.py \
  tests/test_gpu_fused.py tests/test_gpu_product_parity.py -x -q --timeout 300 --timeout-method thread > $out/kpose.tests.log 2>&1
bash tools/gpu/ab.sh r02ak base kpose
