# r02t: decimation split of the contiguous-shift build; what-ifs on the dynamics with the shift removed
set -e
out=gpurun_out/r02t
mkdir -p $out
T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/shc_u16.so timeout -k 10 300 python tools/decimation_timing.py > $out/dec_shc_u16.json 2> $out/err.log
bash tools/gpu/ab.sh r02t ns ns_both ns_nohc ns_all
