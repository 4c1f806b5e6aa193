set -e
out=gpurun_out/r06e; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_linear_wgrad.py tests/test_gpu_conv1_train.py tests/test_ppo_golden.py tests/test_gpu_ppo.py tests/test_gpu_ppo_distributed.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32.json 2> $out/ppo.err
timeout -k 10 300 python tools/ppo_update_profile.py --eager --rows 45 > $out/upd_fp32_eager.txt 2>> $out/ppo.err
bash tools/gpu/clock_modes.sh r06e 4 clk_o1=ti5_isaacgym_amd/_lib/var/clk_o1.so clk_o2=ti5_isaacgym_amd/_lib/var/clk_o2.so
bash tools/gpu/ab_env.sh r06e 2 "--steps 300 --warmup 50 --time-every 8" trimesh=T1ENV_D4_SHIFT=1 o2=T1ENV_LIB=ti5_isaacgym_amd/_lib/var/o2.so
bash tools/gpu/ab_env.sh r06e_plane 2 "--steps 300 --warmup 50 --time-every 8 --mesh plane" plane=T1ENV_D4_SHIFT=1
