# round-5: what the fused epilogue costs k_dyn6 (fused - split HIP-event times) and timing-only what-ifs of its parts
#   bash tools/gpu/r05_epi.sh <tag>
set -e
tag=${1:-r05epi}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/ti5_isaacgym_amd/_lib/var
for l in "" $V/libd6_noposta.so $V/libd6_nonoise.so; do
  T1ENV_LIB=$l timeout -k 10 200 python tools/split_timing.py --steps 200 >> $out/split.jsonl 2>> $out/err.log
done
cat $out/split.jsonl
bash tools/gpu/r05_ab.sh $tag 2 k6 ti5_isaacgym_amd/_lib/var/libd6_noposta.so ti5_isaacgym_amd/_lib/var/libd6_nonoise.so
