# round-5 GPU check: k_dyn6's step tests, the new agreement / DP tests, then an interleaved k_dyn5 / k_dyn6 bench
#   bash tools/gpu/r05_b.sh <tag>
set -e
tag=${1:-r05b}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
run() { timeout -k 10 $1 python -u -m pytest "${@:2}" -x -v --timeout 300 --timeout-method thread; }
run 500 tests/test_gpu_dynamics.py tests/test_gpu_product_parity.py tests/test_gpu_fused.py -k dyn6 > $out/t1_dyn6.log 2>&1 || { tail -60 $out/t1_dyn6.log; exit 1; }
tail -3 $out/t1_dyn6.log
for rep in 1 2; do
  for k in 5 6; do
    T1ENV_DYN_KERNEL=$k timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/bench_k${k}_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/bench_k${k}_$rep.json')); print('k_dyn$k rep $rep', d['value'], d['ms_per_step'])" | tee -a $out/summary.txt
  done
done
run 400 tests/test_gpu_kernel_agreement.py -s > $out/t2_agree.log 2>&1 || { tail -40 $out/t2_agree.log; exit 1; }
tail -3 $out/t2_agree.log
run 300 tests/test_gpu_ppo_distributed.py tests/test_gpu_ppo.py > $out/t3_ppo.log 2>&1 || { tail -40 $out/t3_ppo.log; exit 1; }
tail -3 $out/t3_ppo.log
