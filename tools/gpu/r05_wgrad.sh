# round-5: the bf16 update's HIP Linear weight-gradient kernel -- its GPU tests, per-layer timing against the split-K
# path, the PPO GPU tests and the PPO iteration timing (bf16 update)
set -e
tag=${1:-r05wg}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_linear_wgrad.py > $out/tests_wgrad.log 2>&1
tail -2 $out/tests_wgrad.log
timeout -k 10 300 python tools/wgrad_bench.py > $out/wgrad_bench.json 2> $out/wgrad_bench.err
cat $out/wgrad_bench.json
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ppo.py tests/test_gpu_ppo_distributed.py tests/test_ppo_golden.py tests/test_gpu_conv1_train.py > $out/tests_ppo.log 2>&1
tail -2 $out/tests_ppo.log
timeout -k 10 300 python tools/bench_ppo.py --iters 3 --bf16 > $out/ppo_bf16.json 2> $out/ppo_bf16.err
cat $out/ppo_bf16.json
