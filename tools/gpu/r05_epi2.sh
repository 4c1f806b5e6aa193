# round-5: which epilogue part of k_dyn6 binds -- timing-only builds skipping W1 (state), W2 (priv frame), W3 (actor
# frame), W2 + W3 (fused - split HIP-event times and interleaved bench)
set -e
tag=${1:-r05epi2}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/ti5_isaacgym_amd/_lib/var
for l in "" $V/libd6_skip1.so $V/libd6_skip2.so $V/libd6_skip3.so $V/libd6_skip23.so; do
  T1ENV_LIB=$l timeout -k 10 200 python tools/split_timing.py --steps 200 >> $out/split.jsonl 2>> $out/err.log
done
python -c "
import json
for l in open('$out/split.jsonl'):
    d = json.loads(l); print(d['lib'][-20:] or 'product', d['fused']['k_dynamics'], d['split']['k_dynamics'])
"
