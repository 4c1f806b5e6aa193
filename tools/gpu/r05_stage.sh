# round-5: k_dyn6 epilogue staging placement A/B (before the loop on W4-W7 vs W4 after the first S2) + split timing
set -e
tag=${1:-r05stage}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/ti5_isaacgym_amd/_lib/var
for l in $V/libd6_early.so $V/libd6_late.so; do
  T1ENV_LIB=$l timeout -k 10 200 python tools/split_timing.py --steps 200 >> $out/split.jsonl 2>> $out/err.log
done
cat $out/split.jsonl
bash tools/gpu/r05_ab.sh $tag 3 ti5_isaacgym_amd/_lib/var/libd6_early.so ti5_isaacgym_amd/_lib/var/libd6_late.so
