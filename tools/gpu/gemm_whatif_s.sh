# Dev: timing-only what-if builds of the staged-split GEMM (T1_GEMM_S_WHATIF bits, tools/probes/gemm_whatif.hip)
set -e
out=gpurun_out/${1:-r06m}; mkdir -p $out
for w in 0 2 8 16 0; do
  b=./tools/probes/gemm_whatif_s$w; [ $w = 0 ] && b=./tools/probes/gemm_whatif_0
  timeout -k 5 60 $b | sed "s/^/s$w /" | tee -a $out/gemm_whatif_s.txt
done
