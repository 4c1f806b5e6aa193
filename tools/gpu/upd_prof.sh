# Dev: where the fp32 update's time goes (torch profiler, eager minibatch step), layer by layer and with the fused MLPs
set -e
out=gpurun_out/${1:-r06q}; mkdir -p $out
timeout -k 10 300 python tools/ppo_update_profile.py --eager --rows 60 > $out/upd_prof_fp32_eager.txt 2> $out/upd_prof.err
T1_MLP_F32=1 timeout -k 10 300 python tools/ppo_update_profile.py --eager --rows 60 > $out/upd_prof_fp32_mlp_eager.txt 2>> $out/upd_prof.err
grep -h "Self CUDA time total" $out/upd_prof_fp32_eager.txt $out/upd_prof_fp32_mlp_eager.txt
