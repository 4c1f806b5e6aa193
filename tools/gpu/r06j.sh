set -e
out=gpurun_out/r06j; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear_wgrad.py tests/test_ppo_golden.py tests/test_gpu_ppo.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $out/tests.log 2>&1
tail -1 $out/tests.log
T1_GEMM_STAGED_SPLIT=0 T1_WGRAD_STAGED_SPLIT=0 timeout -k 10 300 python tools/wgrad_bench.py --f32 > $out/wgrad_f32_old.json 2>> $out/err.log
timeout -k 10 300 python tools/wgrad_bench.py --f32 > $out/wgrad_f32_staged.json 2>> $out/err.log
timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32.json 2> $out/ppo.err
timeout -k 10 300 python tools/ppo_update_profile.py --eager --rows 45 > $out/upd_fp32_eager.txt 2>> $out/ppo.err
