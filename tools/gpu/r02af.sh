# r02af: contact-force report from the helpers' own kinematics beside the leg's rigid report (rep): tests + A/B
set -e
out=gpurun_out/r02af
mkdir -p $out
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/rep.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dynamics.py \
  tests/test_gpu_fused.py tests/test_gpu_product_parity.py tests/test_gpu_parity.py tests/test_gpu_step.py -x -q \
  --timeout 300 --timeout-method thread > $out/rep.tests.log 2>&1
bash tools/gpu/ab.sh r02af base rep
