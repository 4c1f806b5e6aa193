# round-3 bench set: default bench line, median of 5, and a rocprof kernel-trace of the same command.
#   bash tools/gpu/r03_bench.sh <tag>  -> gpurun_out/<tag>/{bench.json,bench_median5.json,prof/...}
set -e
tag=${1:-r03b}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 300 --warmup 50 > $out/bench.json 2> $out/bench.err
timeout -k 10 300 python bench.py --steps 480 --warmup 48 --repeats 5 --no-cpu-baseline > $out/bench_median5.json 2>> $out/bench.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 --no-cpu-baseline --time-every 0 > $out/prof.log 2>&1
