# rocprofv3 kernel stats of tools/prof_ppo_update.py (two DH-PPO updates on a synthetic 8192-env rollout)
set -e
tag=${1:-updprof}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o upd -- python3 $GRAFT_REPO_ROOT/tools/prof_ppo_update.py \
  > $out/prof.json 2> $out/prof.log
cd $GRAFT_REPO_ROOT
python3 tools/rocpd_stats.py $out/upd_results.db -o $out/upd_kernel_stats.csv --top 40 > $out/upd_top.txt
rm -f $out/*.db
