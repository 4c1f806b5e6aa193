set -e
out=gpurun_out/r06i; mkdir -p $out
for v in flag_o1 flag_o2; do
  T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_product_parity.py tests/test_gpu_fused.py tests/test_gpu_dynamics.py tests/test_gpu_kernel_agreement.py tests/test_gpu_substep_log_identity.py -m gpu -x -q -k "dyn6 or not dyn" --timeout 300 --timeout-method thread > $out/tests_$v.log 2>&1
  tail -1 $out/tests_$v.log
done
for rep in 1 2; do
  for n in clk_o1 clk_o1_flag clk_o2 clk_o2_flag; do
    T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/$n.so timeout -k 10 200 python tools/clock_probe.py | sed "s/^/$n $rep /" | tee -a $out/clock.txt
  done
done
bash tools/gpu/modes.sh r06i 3 o1=default flag_o1=ti5_isaacgym_amd/_lib/var/flag_o1.so flag_o2=ti5_isaacgym_amd/_lib/var/flag_o2.so
timeout -k 10 300 python tools/ppo_update_profile.py --eager --rows 45 > $out/upd_fp32_eager.txt 2>> $out/ppo.err
