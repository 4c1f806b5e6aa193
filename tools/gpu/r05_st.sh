# round-5: W4's prologue loads before its first store (the staging loads first) vs after; no-finalize what-if
set -e
tag=${1:-r05st}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/ti5_isaacgym_amd/_lib/var
for l in $V/libd6_stafter.so $V/libd6_stpre.so $V/libd6_nofin.so; do
  T1ENV_LIB=$l timeout -k 10 200 python tools/split_timing.py --steps 200 >> $out/split.jsonl 2>> $out/err.log
done
python -c "
import json
for l in open('$out/split.jsonl'):
    d = json.loads(l); print(d['lib'][-20:] or 'product', d['fused']['k_dynamics'], d['split']['k_dynamics'])
"
bash tools/gpu/r05_ab.sh $tag 3 ti5_isaacgym_amd/_lib/var/libd6_stafter.so ti5_isaacgym_amd/_lib/var/libd6_stpre.so ti5_isaacgym_amd/_lib/var/libd6_nofin.so
