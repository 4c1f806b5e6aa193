set -e
out=gpurun_out/r06f; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear_wgrad.py tests/test_ppo_golden.py tests/test_gpu_ppo.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python tools/wgrad_bench.py --f32 > $out/wgrad_f32.json 2>> $out/err.log
timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32.json 2> $out/ppo.err
bash tools/gpu/clock_modes.sh r06f 4 clk_o1=ti5_isaacgym_amd/_lib/var/clk_o1.so clk_o2=ti5_isaacgym_amd/_lib/var/clk_o2.so
