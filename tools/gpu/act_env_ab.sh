# Interleaved A/B of an environment switch on the rollout's act() (tools/act_bench.py, 8192 envs) after the heads
# tests under both settings.   bash tools/gpu/act_env_ab.sh <tag> <reps> <VAR> <value_b>   (A: VAR unset)
set -e
tag=$1; reps=$2; var=$3; vb=$4
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy_heads.py tests/test_gpu_policy_conv.py -x -q --timeout 120 \
  --timeout-method thread > $out/a.tests.log 2>&1 || { echo "TESTS FAILED a"; tail -30 $out/a.tests.log; exit 1; }
tail -1 $out/a.tests.log | sed "s/^/a tests: /" | tee -a $out/summary.txt
env $var=$vb timeout -k 10 300 python -u -m pytest tests/test_gpu_policy_heads.py -x -q --timeout 120 \
  --timeout-method thread > $out/b.tests.log 2>&1 || { echo "TESTS FAILED b"; tail -30 $out/b.tests.log; exit 1; }
tail -1 $out/b.tests.log | sed "s/^/b tests: /" | tee -a $out/summary.txt
for rep in $(seq $reps); do
  timeout -k 10 200 python tools/act_bench.py --iters 400 > $out/act_a_$rep.json 2>> $out/err.log
  echo "a rep $rep $(cat $out/act_a_$rep.json)" | tee -a $out/summary.txt
  env $var=$vb timeout -k 10 200 python tools/act_bench.py --iters 400 > $out/act_b_$rep.json 2>> $out/err.log
  echo "b($var=$vb) rep $rep $(cat $out/act_b_$rep.json)" | tee -a $out/summary.txt
done
