# Product-kernel parity (substep log replayed through the oracle) + golden parity incl. push16.
#   bash tools/gpu/r02_product.sh <tag> -> gpurun_out/<tag>/tests.log
set -e
tag=${1:-product}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python -u -m pytest tests/test_gpu_product_parity.py tests/test_gpu_parity.py -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/$tag/tests.log 2>&1
