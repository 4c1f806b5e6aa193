# history-row gather kernel + fused Adam: GPU tests, PPO benches, update profile
set -e
t=${1:-r03y}
o=$GRAFT_REPO_ROOT/gpurun_out/$t
mkdir -p $o
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -s tests/test_gpu_history_rows.py tests/test_gpu_ppo.py > $o/tests.log 2>&1
timeout -k 10 300 python tools/bench_ppo.py --bf16 --iters 6 > $o/ppo_bf16.json 2> $o/ppo_bf16.err
timeout -k 10 300 python tools/bench_ppo.py --iters 6 > $o/ppo_fp32.json 2> $o/ppo_fp32.err
bash tools/gpu/r03_w.sh $t
