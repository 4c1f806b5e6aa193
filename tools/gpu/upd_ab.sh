# Dev: fp32 update kernels -- numerics tests, layer timings with the staged wgrad on / off, the PPO iteration (fp32,
# and with the fused MLP node)
set -e
out=gpurun_out/${1:-r06p}; mkdir -p $out
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linear_wgrad.py tests/test_gpu_conv1_train.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for w in 1 0; do T1_WGRAD_STAGED=$w timeout -k 10 240 python -u tools/wgrad_bench.py --f32 --reps 30 > $out/wgrad_bench_f32_staged$w.json; done
timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32.json 2> $out/ppo.err
T1_MLP_F32=1 timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32_mlp.json 2>> $out/ppo.err
timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32_b.json 2>> $out/ppo.err
grep -h -o '"update": [0-9.]*' $out/ppo_fp32.json $out/ppo_fp32_mlp.json $out/ppo_fp32_b.json
