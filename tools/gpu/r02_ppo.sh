# PPO: update parity vs the reference on the GPU, single-GPU iteration bench, and a 2-rank gloo data-parallel
# rehearsal of tools/bench_ppo.py with both ranks on cuda:0 (the one-GPU box; not a scaling number).
#   bash tools/gpu/r02_ppo.sh <tag>
set -e
tag=${1:-ppo}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_ppo_golden.py tests/test_gpu_ppo.py -m gpu -x -v --timeout 200 \
  --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 400 python tools/bench_ppo.py --num-envs 8192 --iters 3 > $out/ppo_8192.json 2> $out/ppo.err
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 tools/bench_ppo.py --num-envs 4096 --iters 2 --backend gloo --one-gpu \
  > $out/ppo_2rank_gloo.json 2> $out/ppo_2rank.err
