set -e
out=gpurun_out/r06h; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear_wgrad.py tests/test_ppo_golden.py tests/test_gpu_ppo.py tests/test_gpu_ppo_distributed.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32.json 2> $out/ppo.err
for rep in 1 2; do
  for n in clk_o1 clk_o1_preA clk_o1_preC clk_o2 clk_o2_preA clk_o2_preC; do
    T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/$n.so timeout -k 10 200 python tools/clock_probe.py | sed "s/^/$n $rep /" | tee -a $out/clock.txt
  done
done
