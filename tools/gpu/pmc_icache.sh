# instruction-cache counters of the fused step kernel, one rocprofv3 pass per counter.
#   bash tools/gpu/pmc_icache.sh <tag> -> gpurun_out/<tag>/ic_*_results.db
set -e
tag=${1:-ic}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --time-every 0"
for c in SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c -d $out -o ic_$c -- python3 $B > /dev/null 2> $out/ic_$c.log
done
