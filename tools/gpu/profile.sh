# rocprofv3 kernel-trace stats of the default bench command + two PMC passes (HBM traffic), under gpurun.
#   bash tools/gpu/profile.sh <tag>  -> gpurun_out/<tag>/{run,fetch,write}_results.db, bench logs
# then here: python tools/rocpd_stats.py gpurun_out/<tag>/run_results.db -o profiles/<tag>_kernel_stats.csv
#            python tools/pmc_traffic.py gpurun_out/<tag>/fetch_results.db gpurun_out/<tag>/write_results.db \
#                --num-envs 8192 --mesh trimesh -o profiles/traffic_r01.json
set -e
tag=${1:-prof}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 200 --warmup 50 > $out/bench_default.json 2> $out/bench_default.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 --no-cpu-baseline > $out/bench_prof.json 2> $out/prof.log
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out -o fetch -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --time-every 0 > /dev/null 2> $out/pmc_fetch.log
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out -o write -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline --time-every 0 > /dev/null 2> $out/pmc_write.log
