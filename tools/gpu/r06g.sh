set -e
out=gpurun_out/r06g; mkdir -p $out
for rep in 1 2; do
  for n in clk_o1 clk_o2; do
    T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/$n.so timeout -k 10 200 python tools/clock_probe.py --dump $out/${n}_$rep.npy | sed "s/^/$n $rep /" | tee -a $out/clock.txt
  done
done
