# k_dyn6 diagnosis: phase profiles of k_dyn6 / k_dyn5, interleaved bench of k_dyn6, k_dyn6 without shift, k_dyn5; DP test
set -e
tag=${1:-r05c}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/prof_dynamics_phases.py --kernel 6 > $out/phases6.txt 2>&1
timeout -k 10 200 python tools/prof_dynamics_phases.py --kernel 5 > $out/phases5.txt 2>&1
head -3 $out/phases6.txt
for rep in 1 2; do
  for v in k6 k6noshift k5; do
    case $v in k6) lib=""; k=6;; k6noshift) lib=$GRAFT_REPO_ROOT/ti5_isaacgym_amd/_lib/var/libd6_noshift.so; k=6;; k5) lib=""; k=5;; esac
    T1ENV_LIB=$lib T1ENV_DYN_KERNEL=$k timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/bench_${v}_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/bench_${v}_$rep.json')); print('$v rep $rep', d['value'], d['ms_per_step'])" | tee -a $out/summary.txt
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ppo_distributed.py -x -v --timeout 250 --timeout-method thread > $out/t_dp.log 2>&1 || { tail -30 $out/t_dp.log; exit 1; }
tail -3 $out/t_dp.log
