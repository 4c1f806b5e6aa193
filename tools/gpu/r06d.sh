set -e
out=gpurun_out/r06d; mkdir -p $out
bash tools/gpu/modes.sh r06d 5 o1=default o2=ti5_isaacgym_amd/_lib/var/o2.so o2ns=ti5_isaacgym_amd/_lib/var/o2_noshift.so o1ns=ti5_isaacgym_amd/_lib/var/o1_noshift.so
bash tools/gpu/ab_env.sh r06d 2 "--steps 300 --warmup 50 --time-every 8 --num-envs 32768 --mesh heightfield --state-dtype fp16 --push" u3=T1ENV_D4_SHIFT=1 u2=T1ENV_LIB=ti5_isaacgym_amd/_lib/var/c5u2.so u4=T1ENV_LIB=ti5_isaacgym_amd/_lib/var/c5u4.so
timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32.json 2> $out/ppo.err
timeout -k 10 300 python tools/bench_ppo.py --iters 4 --bf16 > $out/ppo_bf16.json 2>> $out/ppo.err
timeout -k 10 300 python tools/ppo_update_profile.py --eager --rows 45 > $out/upd_fp32_eager.txt 2>> $out/ppo.err
