# round-5: kernel-level timing of the wgrad kernel (rocprof stats over tools/wgrad_bench.py), then the heads 8-wave A/B
set -e
tag=${1:-r05wp}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o wg -- python tools/wgrad_bench.py --reps 10 > $out/wgrad_bench.json 2> $out/prof.err
find $out/prof -name "*kernel_stats.csv" -exec cp {} $out/wgrad_kernel_stats.csv \;
head -30 $out/wgrad_kernel_stats.csv | cut -c1-200
bash tools/gpu/r05_heads8.sh r05h8
