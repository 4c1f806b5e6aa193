# round-4 policy check: the fused heads' parity tests, the act() graphs' tests, then act() timings (fused, torch) and
# a rocprofv3 kernel summary of the fused act() loop.
#   bash tools/gpu/r04_policy.sh <tag>  -> gpurun_out/<tag>/{tests.log,act*.json,prof/}
set -e
tag=${1:-r04p}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_policy_heads.py tests/test_gpu_policy_conv.py tests/test_gpu_ppo.py \
    -m gpu -v --timeout 200 --timeout-method thread -k "${KEXPR:-heads or conv or act}" > $out/tests.log 2>&1 \
    || echo "TESTS FAILED rc=$?" >> $out/tests.log
grep -q "Fatal\|core dumped\|Aborted\|Segmentation" $out/tests.log && exit 3
timeout -k 10 200 python tools/act_bench.py > $out/act_fused.json
timeout -k 10 200 python tools/act_bench.py --torch > $out/act_torch.json
T1POLICY_HEADS_XCD=0 timeout -k 10 200 python tools/act_bench.py > $out/act_fused_noxcd.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o act -- python tools/act_bench.py --iters 100 > $out/prof.log 2>&1
tail -3 $out/tests.log
cat $out/act_fused.json $out/act_torch.json $out/act_fused_noxcd.json
timeout -k 10 400 python tools/ppo_update_profile.py --bf16 --eager --rows 30 > $out/upd_prof_bf16_eager.txt 2>&1
