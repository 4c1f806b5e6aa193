# -O1/-O2/-O3 of the dynamics unit: current code (guard) and the 62e0912 tree where -O2/-O3 first gave wrong dynamics.
#   bash tools/gpu/r02_opt.sh <tag>
tag=${1:-opt}
out=$PWD/gpurun_out/$tag
mkdir -p $out
for v in o3 o2; do
  T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dynamics.py \
    tests/test_gpu_product_parity.py -x -q --timeout 200 --timeout-method thread > $out/cur_$v.log 2>&1
  rc=$?; echo "cur $v rc=$rc" >> $out/summary.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
done
cd _old62
for v in o1 o3; do
  T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_dynamics.py -x -q \
    --timeout 200 --timeout-method thread > $out/old_$v.log 2>&1
  rc=$?; echo "old $v rc=$rc" >> $out/summary.txt
  if [ $rc -ge 124 ]; then exit $rc; fi
done
exit 0
