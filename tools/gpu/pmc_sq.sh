# SQ instruction-mix counters for the fused step kernel, one rocprofv3 pass per counter group.
#   bash tools/gpu/pmc_sq.sh <tag> -> gpurun_out/<tag>/sq{1,2}_results.db
set -e
tag=${1:-sq}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --time-every 0"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $out -o sq1 -- python3 $B > /dev/null 2> $out/sq1.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU -d $out -o sq2 -- python3 $B > /dev/null 2> $out/sq2.log
