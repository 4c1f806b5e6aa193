# round-5: the hardware SIMD of each k_dyn6 wave vs the step time, 4 processes
set -e
cd $GRAFT_REPO_ROOT
for rep in 1 2 3 4; do
  T1ENV_LIB=$GRAFT_REPO_ROOT/ti5_isaacgym_amd/_lib/var/libd6_simd.so timeout -k 10 200 python tools/simd_probe.py 2>/dev/null | tee -a gpurun_out/r05simd.txt
done
