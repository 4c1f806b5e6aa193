# Dev: SQ / LDS counters of the fp32 GEMM (tools/probes/gemm_whatif_0, one shape), one rocprofv3 pass per group.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-r06j}; mkdir -p $out
P=$GRAFT_REPO_ROOT/tools/probes/gemm_whatif_0
cd /tmp && export TMPDIR=/tmp
export GEMM_SHAPE=0
for pipe in 1 0; do
  export T1_GEMM_STAGED=$pipe
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU -d $out -o p1_$pipe -- $P > $out/p1_$pipe.log 2>&1
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_VMEM_RD SQ_WAVES -d $out -o p2_$pipe -- $P > $out/p2_$pipe.log 2>&1
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d $out -o p3_$pipe -- $P > $out/p3_$pipe.log 2>&1
done
cd $GRAFT_REPO_ROOT
for pipe in 1 0; do python tools/pmc_kernel_counters.py $out/p1_${pipe}_results.db $out/p2_${pipe}_results.db $out/p3_${pipe}_results.db --kernel k_gemm > $out/counters_$pipe.json; done
cat $out/counters_1.json $out/counters_0.json
