# round-3 evidence set: every -m gpu test (+ parity report), smoke(), the default bench line, median of 5, a rocprof
# kernel trace of the bench, and the PMC passes (HBM traffic; SQ counters) bench.py's roofline reads.
#   bash tools/gpu/r03_full.sh <tag>  -> gpurun_out/<tag>/...
set -e
tag=${1:-r03z}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
T1_PARITY_REPORT=$out/parity_report.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 \
    --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
timeout -k 10 300 python bench.py --steps 300 --warmup 50 > $out/bench.json 2> $out/bench.err
timeout -k 10 300 python bench.py --steps 480 --warmup 48 --repeats 5 --no-cpu-baseline > $out/bench_median5.json 2>> $out/bench.err
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --time-every 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 --no-cpu-baseline --time-every 0 > $out/prof.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out -o fetch -- python3 $B > /dev/null 2> $out/pmc_fetch.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out -o write -- python3 $B > /dev/null 2> $out/pmc_write.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $out -o sq1 -- python3 $B > /dev/null 2> $out/sq1.log
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU -d $out -o sq2 -- python3 $B > /dev/null 2> $out/sq2.log
