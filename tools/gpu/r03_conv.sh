# policy conv: GPU tests + kernel timing (old tap-major vs packed-fragment kernel)
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03c}
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_policy_conv.py > $out/tests.log 2>&1
timeout -k 10 120 python tools/conv_bench.py --out $out/conv_bench.json > $out/conv_bench.log 2>&1
