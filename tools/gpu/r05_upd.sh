# round-5: wgrad tests, PPO GPU tests, the PPO iteration timing and an eager update profile (bf16 update)
set -e
tag=${1:-r05upd}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_linear_wgrad.py tests/test_gpu_ppo.py tests/test_gpu_ppo_distributed.py tests/test_ppo_golden.py tests/test_gpu_conv1_train.py tests/test_gpu_policy_heads.py tests/test_gpu_history_rows.py tests/test_gpu_fold_rows.py > $out/tests.log 2>&1
tail -1 $out/tests.log
timeout -k 10 300 python tools/bench_ppo.py --iters 3 --bf16 > $out/ppo_bf16.json 2> $out/ppo_bf16.err
cat $out/ppo_bf16.json
timeout -k 10 300 python tools/ppo_update_profile.py --bf16 --eager --rows 40 > $out/upd_prof.txt 2> $out/upd_prof.err
echo profiled
