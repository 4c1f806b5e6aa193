# SQ counters of the rollout's act() kernels (tools/act_bench.py, 8192 envs), one rocprofv3 pass per counter group.
#   bash tools/gpu/act_pmc.sh <tag> -> gpurun_out/<tag>/aq{1,2}_results.db
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-actpmc}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/tools/act_bench.py --iters 20"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $out -o aq1 -- python3 $B > /dev/null 2> $out/aq1.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_WR SQ_VALU_MFMA_BUSY_CYCLES -d $out -o aq2 -- python3 $B > /dev/null 2> $out/aq2.log
