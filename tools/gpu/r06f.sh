set -e
out=gpurun_out/r06f; mkdir -p $out
bash tools/gpu/clock_modes.sh r06f 4 clk_o1=ti5_isaacgym_amd/_lib/var/clk_o1.so clk_o2=ti5_isaacgym_amd/_lib/var/clk_o2.so
for w in 1 2 3; do T1_WGRAD_WG_PER_CU=$w timeout -k 10 200 python tools/wgrad_bench.py --f32 > $out/wgrad_f32_wg$w.json 2>> $out/err.log; done
timeout -k 10 200 python tools/wgrad_bench.py > $out/wgrad_bf16.json 2>> $out/err.log
