# round-5: graphed GAE -- PPO GPU tests and the PPO iteration timing; then the epilogue what-ifs (r05_epi2.sh)
set -e
tag=${1:-r05ppo2}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ppo.py tests/test_gpu_ppo_distributed.py tests/test_gpu_runner_contract.py tests/test_ppo_golden.py > $out/tests.log 2>&1
tail -2 $out/tests.log
timeout -k 10 300 python tools/bench_ppo.py --iters 3 --bf16 > $out/ppo_bf16.json 2> $out/ppo_bf16.err
cat $out/ppo_bf16.json
bash tools/gpu/r05_epi2.sh r05epi2
