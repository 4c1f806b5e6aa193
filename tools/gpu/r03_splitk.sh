# A/B of the split-K slice height of the PPO weight gradients (bf16 update, 8192 envs, 6 iterations each)
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03k}
mkdir -p $out
cd $GRAFT_REPO_ROOT
for rows in 2048 8192 4096 1024; do
  T1_SPLITK_ROWS=$rows timeout -k 10 300 python tools/bench_ppo.py --bf16 --iters 6 > $out/ppo_bf16_$rows.json 2> $out/err_$rows.log
  python -c "import json; d=json.load(open('$out/ppo_bf16_$rows.json')); print('rows $rows', d['env_steps_per_s_incl_update'], d['phases_s_per_iter'])" | tee -a $out/summary.txt
done
