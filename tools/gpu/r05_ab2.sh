# round-5: k_dyn6 variants (W0 lane/leg launder, extras fast path, -O2) + the PPO rollout / update breakdown
#   bash tools/gpu/r05_ab2.sh <tag>
set -e
tag=${1:-r05ab2}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
bash tools/gpu/r05_ab.sh $tag 2 ti5_isaacgym_amd/_lib/var/libd6_base.so ti5_isaacgym_amd/_lib/var/libd6_w0l.so ti5_isaacgym_amd/_lib/var/libd6_w0lb.so ti5_isaacgym_amd/_lib/var/libd6_o2.so
timeout -k 10 300 python tools/prof_rollout.py > $out/prof_rollout.txt 2> $out/prof_rollout.err
timeout -k 10 300 python tools/bench_ppo.py --iters 3 --bf16 > $out/ppo_bf16.json 2> $out/ppo_bf16.err
head -c 1500 $out/ppo_bf16.json
