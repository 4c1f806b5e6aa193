# act() change check: the PPO / heads GPU tests, act_bench x3, one rocprofv3 kernel trace of act_bench.
#   bash tools/gpu/act_check.sh <tag>
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-actcheck}; mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo.py tests/test_gpu_policy_heads.py tests/test_ppo_golden.py tests/test_gpu_runner_contract.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for i in 1 2 3; do timeout -k 10 200 python tools/act_bench.py --iters 400 >> $out/act.jsonl 2>> $out/act.err; done
cat $out/act.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out -o act -- python3 $GRAFT_REPO_ROOT/tools/act_bench.py --iters 200 > $out/act_prof.json 2> $out/act_prof.err
