# rocprofv3 kernel stats of the PPO iteration bench (rollout + update), to find where the update's time goes.
#   bash tools/gpu/r02_ppo_prof.sh <tag>
set -e
tag=${1:-ppoprof}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out -o ppo -- python3 $GRAFT_REPO_ROOT/tools/bench_ppo.py \
  --num-envs 8192 --iters 1 > $out/ppo.json 2> $out/prof.log
cd $GRAFT_REPO_ROOT
python3 tools/rocpd_stats.py $out/ppo_results.db -o $out/ppo_kernel_stats.csv --top 40 > $out/ppo_top.txt
rm -f $out/*.db
