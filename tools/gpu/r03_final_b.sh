# round-3 policy-side evidence: conv kernel timing, PPO tests, PPO iteration bf16 (fp32-output split-K A/B) and fp32,
# the rollout profile
set -e
t=${1:-r03fb}
o=$GRAFT_REPO_ROOT/gpurun_out/$t
mkdir -p $o
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/conv_bench.py --out $o/conv_bench.json > $o/conv_bench.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ppo.py tests/test_gpu_policy_conv.py > $o/tests.log 2>&1
timeout -k 10 300 python tools/bench_ppo.py --bf16 --iters 6 > $o/ppo_bf16.json 2> $o/ppo_bf16.err
T1_WGRAD_OUT_F32=0 timeout -k 10 300 python tools/bench_ppo.py --bf16 --iters 6 > $o/ppo_bf16_widen.json 2> $o/ppo_bf16_widen.err
timeout -k 10 300 python tools/bench_ppo.py --iters 6 > $o/ppo_fp32.json 2> $o/ppo_fp32.err
timeout -k 10 300 python tools/prof_rollout.py > $o/rollout_profile.txt 2>&1
