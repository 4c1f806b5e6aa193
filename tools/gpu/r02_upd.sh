# PPO update phase timing + iteration bench + PPO GPU tests
set -e
tag=${1:-upd}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_ppo_golden.py tests/test_gpu_ppo.py -m gpu -x -v --timeout 200 \
  --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python tools/prof_ppo_update.py > $out/upd_phases.json 2> $out/upd.err
timeout -k 10 400 python tools/bench_ppo.py --num-envs 8192 --iters 3 > $out/ppo_8192.json 2> $out/ppo.err
