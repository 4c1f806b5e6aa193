set -e
out=gpurun_out/r06k; mkdir -p $out
timeout -k 10 60 ./tools/probes/unaligned_x4 | tee $out/probe.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_product_parity.py tests/test_gpu_fused.py tests/test_gpu_step.py tests/test_gpu_fp16.py tests/test_gpu_substep_log_identity.py tests/test_gpu_sharding.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
tail -1 $out/tests.log
bash tools/gpu/modes.sh r06k 3 o1x=default o1a2=ti5_isaacgym_amd/_lib/var/o1a2.so o2x=ti5_isaacgym_amd/_lib/var/o2x.so
for rep in 1 2; do
  for n in clk_o1x clk_o2x; do
    T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/$n.so timeout -k 10 200 python tools/clock_probe.py | sed "s/^/$n $rep /" | tee -a $out/clock.txt
  done
done
