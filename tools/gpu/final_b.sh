# Round-end evidence, part B: rocprofv3 kernel statistics of config 3 (the metric) and config 5, the HBM traffic (PMC
# FETCH_SIZE / WRITE_SIZE, one pass each) and the SQ counters of config 3, the rollout's act() and the PPO iteration.
#   bash tools/gpu/final_b.sh <tag>
set -e
tag=${1:-final}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy_heads.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/heads_tests.log 2>&1
tail -1 $out/heads_tests.log
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run -- python3 $B --steps 100 --warmup 20 > $out/bench_prof.json 2> $out/prof.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o cfg5 -- python3 $B --steps 100 --warmup 20 --num-envs 32768 --mesh heightfield --state-dtype fp16 --push > $out/bench_prof_cfg5.json 2> $out/prof_cfg5.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out -o fetch -- python3 $B --steps 20 --warmup 5 --time-every 0 > /dev/null 2> $out/pmc_fetch.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out -o write -- python3 $B --steps 20 --warmup 5 --time-every 0 > /dev/null 2> $out/pmc_write.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out -o fetch5 -- python3 $B --steps 20 --warmup 5 --time-every 0 --num-envs 32768 --mesh heightfield --state-dtype fp16 --push > /dev/null 2> $out/pmc_fetch5.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out -o write5 -- python3 $B --steps 20 --warmup 5 --time-every 0 --num-envs 32768 --mesh heightfield --state-dtype fp16 --push > /dev/null 2> $out/pmc_write5.log
cd $GRAFT_REPO_ROOT
bash tools/gpu/pmc_sq.sh $tag
timeout -k 10 300 python tools/act_bench.py > $out/act.json 2> $out/act.err
timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32.json 2> $out/ppo.err
timeout -k 10 300 python tools/bench_ppo.py --iters 4 --bf16 > $out/ppo_bf16.json 2>> $out/ppo.err
