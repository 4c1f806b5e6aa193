# interleaved A/B of k_dyn6 variants (T1ENV_LIB) against k_dyn5, 8192 trimesh default bench
#   bash tools/gpu/r05_ab.sh <tag> <reps> <variant.so|k5|k6>...
set -e
tag=$1; reps=$2; shift 2
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
for rep in $(seq 1 $reps); do
  for v in "$@"; do
    case $v in k5) lib=""; k=5; n=k5;; k6) lib=""; k=6; n=k6;; *) lib=$GRAFT_REPO_ROOT/$v; k=6; n=$(basename $v .so);; esac
    T1ENV_LIB=$lib T1ENV_DYN_KERNEL=$k timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/bench_${n}_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/bench_${n}_$rep.json')); print('$n rep $rep', d['value'], d['ms_per_step'])" | tee -a $out/summary.txt
  done
done
