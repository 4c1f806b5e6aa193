# Round-end evidence refresh after a policy-side change: smoke, the rollout's act(), the PPO iteration (fp32 and bf16)
# and the default bench line.   bash tools/gpu/final_c.sh <tag>
set -e
tag=${1:-final_c}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 300 python tools/act_bench.py > $out/act.json 2> $out/act.err
cat $out/act.json
timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32.json 2> $out/ppo.err
timeout -k 10 300 python tools/bench_ppo.py --iters 4 --bf16 > $out/ppo_bf16.json 2>> $out/ppo.err
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err
