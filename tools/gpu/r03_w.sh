# PPO update: wall time graphed vs eager, and the eager device profile (bf16)
set -e
t=${1:-r03w}
o=$GRAFT_REPO_ROOT/gpurun_out/$t
mkdir -p $o
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/ppo_update_profile.py --bf16 > $o/ppo_update_graphed_bf16.txt 2>&1
timeout -k 10 300 python tools/ppo_update_profile.py --bf16 --eager --rows 40 > $o/ppo_update_eager_bf16.txt 2>&1
