# kernel trace of the concurrent-shift step (k_dyn5 + k_shift5 on two streams) and of the in-workgroup shift
set -e
tag=${1:-r04s}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
T1ENV_D5_SHIFT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/conc -o step -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 --no-cpu-baseline --time-every 0 > $out/bench_conc.json 2> $out/conc.log
T1ENV_D5_SHIFT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/inwg -o step -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 --no-cpu-baseline --time-every 0 > $out/bench_inwg.json 2> $out/inwg.log
