# round-4 what-ifs: act() with the heads what-if libraries, and a kernel trace of the concurrent-shift step.
#   bash tools/gpu/r04_whatif.sh <tag> -> gpurun_out/<tag>/
set -e
tag=${1:-r04w}
out=gpurun_out/$tag
mkdir -p $out
for v in base h_noload h_nomfma h_noelu; do
  if [ $v = base ]; then lib=; else lib=$PWD/ti5_isaacgym_amd/_lib/var/$v.so; fi
  T1ENV_LIB=$lib timeout -k 10 120 python tools/act_bench.py > $out/act_$v.json 2> $out/act_$v.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o step -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 --no-cpu-baseline --time-every 0 > $GRAFT_REPO_ROOT/$out/bench_prof.json 2> $GRAFT_REPO_ROOT/$out/prof.log
cd $GRAFT_REPO_ROOT
cat $out/act_*.json
