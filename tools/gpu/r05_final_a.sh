# round-5 measurement set A (the metric's config, k_dyn6 product build): bench default line (with the CPU baseline at
# the metric's 8192 envs), median of 5 x 480 steps, rocprofv3 kernel stats, PMC HBM traffic (FETCH_SIZE, WRITE_SIZE
# passes) and the SQ instruction counters (two passes), each pass its own run.
#   bash tools/gpu/r05_final_a.sh <tag> -> gpurun_out/<tag>/
set -e
tag=${1:-r05fa}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err
timeout -k 10 300 python bench.py --steps 480 --warmup 48 --repeats 5 --no-cpu-baseline > $out/bench_median5.json 2> $out/bench_median5.err
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/run -o run -- python3 $B --steps 100 --warmup 20 > $out/bench_prof.json 2> $out/prof.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/fetch -o fetch -- python3 $B --steps 20 --warmup 5 --time-every 0 > /dev/null 2> $out/pmc_fetch.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/write -o write -- python3 $B --steps 20 --warmup 5 --time-every 0 > /dev/null 2> $out/pmc_write.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $out/sq1 -o sq1 -- python3 $B --steps 20 --warmup 5 --time-every 0 > /dev/null 2> $out/sq1.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU -d $out/sq2 -o sq2 -- python3 $B --steps 20 --warmup 5 --time-every 0 > /dev/null 2> $out/sq2.log
cd $GRAFT_REPO_ROOT
find $out -name "*.db" | head -20
echo done
