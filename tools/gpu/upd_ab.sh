# Dev: fp32 update -- kernel numerics tests, the PPO tests (golden replay, graphed == eager, DP), the PPO iteration
# (twice) and the eager update profile
set -e
out=gpurun_out/${1:-r06u}; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linear_wgrad.py tests/test_gpu_conv1_train.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_ppo.py tests/test_ppo_golden.py tests/test_gpu_ppo_distributed.py tests/test_runner_golden.py > $out/tests_ppo.log 2>&1 || { tail -30 $out/tests_ppo.log; exit 1; }
tail -1 $out/tests_ppo.log
for i in 1 2; do timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32_$i.json 2>> $out/ppo.err; grep -o '"update": [0-9.]*' $out/ppo_fp32_$i.json; done
timeout -k 10 300 python tools/ppo_update_profile.py --eager --rows 60 > $out/upd_prof_fp32_eager.txt 2>> $out/ppo.err
grep -h "Self CUDA time total" $out/upd_prof_fp32_eager.txt
