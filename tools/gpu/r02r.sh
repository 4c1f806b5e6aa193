# r02r: is the in-launch history shift the fused step's critical path?  wall ms/step at decimation 10/5/2/1 for
# the product, the forced stand-alone shift (T1ENV_SHIFT_BLOCKS=-1) and the no-shift timing build
set -e
out=gpurun_out/r02r
mkdir -p $out
timeout -k 10 300 python tools/decimation_timing.py > $out/product.json 2> $out/err.log
T1ENV_SHIFT_BLOCKS=-1 timeout -k 10 300 python tools/decimation_timing.py > $out/prelaunch.json 2>> $out/err.log
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/wi_noshift.so timeout -k 10 300 python tools/decimation_timing.py > $out/noshift.json 2>> $out/err.log
T1ENV_SHIFT_BLOCKS=-1 timeout -k 10 300 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > $out/bench_prelaunch.json 2>> $out/err.log
