set -e
out=gpurun_out/r06l; mkdir -p $out
for rep in 1 2 3 4; do
  T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/clk_o1x.so timeout -k 10 200 python tools/clock_probe.py --steps 201 | sed "s/^/clk_o1x $rep /" | tee -a $out/clock.txt
done
