# round-5: the wgrad kernel's GPU tests, then its kernel-level timing (rocprof kernel trace over tools/wgrad_bench.py;
# summarised here with tools/rocpd_stats.py) at each slicing target (T1_WGRAD_WG_PER_CU)
set -e
tag=${1:-r05wp}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_linear_wgrad.py > $out/tests_wgrad.log 2>&1
tail -1 $out/tests_wgrad.log
for k in ${WGPC:-2 1 3}; do
  T1_WGRAD_WG_PER_CU=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof$k -o wg -- python tools/wgrad_bench.py --reps 10 > $out/wgrad_bench$k.json 2> $out/prof$k.err
  echo profiled $k
done
