# round-5: the rollout with the graphed process_env_step -- PPO GPU tests, rollout profile, PPO iteration timing
#   bash tools/gpu/r05_ppo.sh <tag>
set -e
tag=${1:-r05ppo}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_ppo.py tests/test_gpu_ppo_distributed.py tests/test_gpu_runner_contract.py tests/test_ppo_golden.py > $out/tests.log 2>&1
tail -2 $out/tests.log
timeout -k 10 300 python tools/prof_rollout.py > $out/prof_rollout.txt 2> $out/prof_rollout.err
head -c 400 $out/prof_rollout.txt; echo
timeout -k 10 300 python tools/bench_ppo.py --iters 3 --bf16 > $out/ppo_bf16.json 2> $out/ppo_bf16.err
timeout -k 10 300 python tools/bench_ppo.py --iters 3 > $out/ppo_fp32.json 2> $out/ppo_fp32.err
cat $out/ppo_bf16.json $out/ppo_fp32.json
