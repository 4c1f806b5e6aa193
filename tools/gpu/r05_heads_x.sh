# round-5 A/B: the heads launch's role placement (T1POLICY_HEADS_XCD: 1 = actor XCDs 0-3 / critic 4-7, 2 = both roles
# on every XCD alternating, 0 = alternating workgroups), heads tests under mode 2, act() timing alternated
set -e
tag=${1:-r05hx}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
T1POLICY_HEADS_XCD=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_policy_heads.py > $out/tests_x2.log 2>&1
tail -1 $out/tests_x2.log
for rep in 1 2 3; do
  for x in 1 2 0; do
    T1POLICY_HEADS_XCD=$x timeout -k 10 120 python tools/act_bench.py --iters 300 > $out/act_x${x}_$rep.json 2>> $out/err.log
    echo "rep $rep xcd $x $(cat $out/act_x${x}_$rep.json)"
  done
done
