# round-4 PPO check: the bf16 conv1 kernels' tests and the PPO GPU tests, then PPO iterations bf16 (HIP conv1 and
# the unfold + GEMM A/B) and fp32, and the bf16 update profile by op and shape.
#   bash tools/gpu/r04_ppo.sh <tag> -> gpurun_out/<tag>/
set -e
tag=${1:-r04q}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv1_train.py tests/test_gpu_ppo.py -m gpu -v --timeout 300 \
    --timeout-method thread > $out/tests.log 2>&1 || echo "TESTS FAILED rc=$?" >> $out/tests.log
grep -q "Fatal\|core dumped\|Aborted\|Segmentation" $out/tests.log && exit 3
timeout -k 10 300 python tools/bench_ppo.py --bf16 --iters 6 > $out/ppo_bf16.json 2> $out/ppo_bf16.err
T1_CONV1_TRAIN=0 timeout -k 10 300 python tools/bench_ppo.py --bf16 --iters 6 > $out/ppo_bf16_unfold.json 2> $out/ppo_bf16_unfold.err
timeout -k 10 300 python tools/bench_ppo.py --iters 6 > $out/ppo_fp32.json 2> $out/ppo_fp32.err
timeout -k 10 400 python tools/ppo_update_profile.py --bf16 --eager --rows 30 > $out/upd_prof_bf16_eager.txt 2>&1
tail -3 $out/tests.log
cat $out/ppo_bf16.json $out/ppo_bf16_unfold.json $out/ppo_fp32.json
