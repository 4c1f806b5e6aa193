# Dev A/B of the fp32 GEMM forms (T1_GEMM_STAGED 0 / 1 through tools/probes/gemm_whatif_0), the numerics tests on the
# default form, the layer timings and the fp32 PPO iteration.
set -e
out=gpurun_out/${1:-r06o}; mkdir -p $out
for p in 0 1 0 1; do T1_GEMM_STAGED=$p timeout -k 5 60 ./tools/probes/gemm_whatif_0 | sed "s/^/staged$p /" | tee -a $out/gemm_ab.txt; done
timeout -k 10 240 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_linear_wgrad.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 240 python -u tools/wgrad_bench.py --f32 --reps 30 > $out/wgrad_bench_f32.json
timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32.json 2> $out/ppo.err
cat $out/ppo_fp32.json
