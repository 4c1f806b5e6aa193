# round-5 A/B: the rollout history conv's pairs per CU (T1POLICY_CONV_PAIRS 4 = default, 5, 6), act() timing alternated
set -e
tag=${1:-r05cp}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
for rep in 1 2 3; do
  for p in 4 5 6 3; do
    T1POLICY_CONV_PAIRS=$p timeout -k 10 120 python tools/act_bench.py --iters 300 > $out/act_p${p}_$rep.json 2>> $out/err.log
    echo "rep $rep pairs $p $(cat $out/act_p${p}_$rep.json)"
  done
done
T1POLICY_CONV_PAIRS=6 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_policy_conv.py > $out/tests_p6.log 2>&1
tail -1 $out/tests_p6.log
