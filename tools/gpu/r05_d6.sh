# k_dyn6 first light: its step tests, then an interleaved k_dyn5 / k_dyn6 bench (8192 trimesh, 300 steps, 3 reps)
#   bash tools/gpu/r05_d6.sh <tag> [pytest -k expr]
set -e
tag=${1:-r05a}; kexpr=${2:-dyn6}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_dynamics.py tests/test_gpu_product_parity.py tests/test_gpu_fused.py \
  -k "$kexpr" -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -5 $out/tests.log
for rep in 1 2 3; do
  for k in 5 6; do
    T1ENV_DYN_KERNEL=$k timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/bench_k${k}_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/bench_k${k}_$rep.json')); print('k_dyn$k rep $rep', d['value'], d['ms_per_step'])" | tee -a $out/summary.txt
  done
done
