# interleaved A/B of the tree's library against variant builds (T1ENV_LIB), 8192 trimesh default bench, 2 reps
#   bash tools/gpu/r03_libab.sh <tag> <variant.so>...
set -e
tag=${1:-r05}; shift
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in default "$@"; do
    n=$(basename $v .so)
    if [ $v = default ]; then lib=""; else lib=$GRAFT_REPO_ROOT/$v; fi
    T1ENV_LIB=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/bench_${n}_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/bench_${n}_$rep.json')); print('$n rep $rep', d['value'], d['ms_per_step'])" | tee -a $out/summary.txt
  done
done
