# round-5 A/B: the fused heads kernel at 8 waves (two per SIMD, -DT1_HEADS_WAVES=8) against the product's 4 --
# heads tests on the variant, then act() timing alternated
set -e
tag=${1:-r05h8}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/ti5_isaacgym_amd/_lib/var/libheads8.so
T1ENV_LIB=$V timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_policy_heads.py > $out/tests_heads8.log 2>&1
tail -1 $out/tests_heads8.log
for rep in 1 2 3; do
  timeout -k 10 120 python tools/act_bench.py --iters 300 > $out/act_base_$rep.json 2>> $out/err.log
  T1ENV_LIB=$V timeout -k 10 120 python tools/act_bench.py --iters 300 > $out/act_h8_$rep.json 2>> $out/err.log
  echo "rep $rep base $(cat $out/act_base_$rep.json) h8 $(cat $out/act_h8_$rep.json)"
done
