# instruction-cache and SQ counters of the step kernel for k_dyn5 and k_dyn6, one rocprofv3 pass per counter group
#   bash tools/gpu/r05_pmc.sh <tag> [lib]
set -e
tag=${1:-r05pmc}; lib=${2:-}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --time-every 0"
for k in 5 6; do
  export T1ENV_DYN_KERNEL=$k T1ENV_LIB=$lib
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS -d $out -o ic$k -- python3 $B > /dev/null 2> $out/ic$k.log
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU -d $out -o sq$k -- python3 $B > /dev/null 2> $out/sq$k.log
  python3 $GRAFT_REPO_ROOT/tools/pmc_sq_summary.py $out/ic${k}_results.db $out/sq${k}_results.db --kernel k_dyn$k -o $out/summary_k$k.json > /dev/null
  python3 -c "import json; d=json.load(open('$out/summary_k$k.json')); print('k_dyn$k', json.dumps(d['derived']))"
done
