# the k_dyn6 shift rewrite: A/B vs the previous kernel, then the parity tests that read the histories
set -e
cd $GRAFT_REPO_ROOT
bash tools/gpu/r05_ab.sh r05ab_shift 2 k6 ti5_isaacgym_amd/_lib/var/libd6_head.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fused.py tests/test_gpu_product_parity.py tests/test_gpu_sharding.py tests/test_gpu_kernel_agreement.py > gpurun_out/r05ab_shift/tests.log 2>&1
tail -3 gpurun_out/r05ab_shift/tests.log
