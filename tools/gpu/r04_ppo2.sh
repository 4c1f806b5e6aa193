# round-4 PPO update A/B: the HIP slice sum for the split-K weight gradients (T1_SLICE_SUM=1, default) against torch's
# dim-0 sum, after the conv1 / slice-sum kernel tests and the PPO GPU tests; then the epilogue split timing and the
# step kernel choice at 16384 envs.   bash tools/gpu/r04_ppo2.sh <tag> -> gpurun_out/<tag>/
set -e
tag=${1:-r04p3}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv1_train.py tests/test_gpu_ppo.py tests/test_ppo_golden.py -m gpu -v \
    --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
  timeout -k 10 300 python tools/bench_ppo.py --bf16 --iters 6 > $out/ppo_bf16_slicesum_$rep.json 2>> $out/err.log
  T1_SLICE_SUM=0 timeout -k 10 300 python tools/bench_ppo.py --bf16 --iters 6 > $out/ppo_bf16_torchsum_$rep.json 2>> $out/err.log
done
timeout -k 10 300 python tools/bench_ppo.py --iters 6 > $out/ppo_fp32_slicesum.json 2>> $out/err.log
for f in $out/ppo_*.json; do python -c "import json; d=json.load(open('$f')); print('$f', d['env_steps_per_s_incl_update'], d['phases_s_per_iter'])"; done
timeout -k 10 120 python tools/split_timing.py > $out/split_timing.json 2>> $out/err.log
cat $out/split_timing.json
for k in 5 4; do
  T1ENV_DYN_KERNEL=$k timeout -k 10 120 python bench.py --num-envs 16384 --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/n16384_k$k.json 2>> $out/err.log
  python -c "import json; d=json.load(open('$out/n16384_k$k.json')); print('k_dyn$k 16384', d['ms_per_step'])"
done
