# Interleaved A/B of library builds (T1ENV_LIB) on the metric's workload (8192 trimesh, 300 steps, uninstrumented),
# after the step kernel's parity tests on every candidate that is not a timing-only what-if (name whatif*).
#   bash tools/gpu/ab.sh <tag> <reps> <name>=<lib.so> ...   -> gpurun_out/<tag>/{summary.txt,*.json,*.tests.log}
set -e
tag=$1; reps=$2; shift 2
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
for nv in "$@"; do
  n=${nv%%=*}; lib=$GRAFT_REPO_ROOT/${nv#*=}
  case $n in whatif*) continue;; esac
  T1ENV_LIB=$lib timeout -k 10 400 python -u -m pytest tests/test_gpu_product_parity.py tests/test_gpu_fused.py \
    tests/test_gpu_dynamics.py tests/test_gpu_dynamics_contact.py -x -q --timeout 200 --timeout-method thread \
    > $out/$n.tests.log 2>&1 || { echo "TESTS FAILED $n"; tail -30 $out/$n.tests.log; exit 1; }
  tail -1 $out/$n.tests.log | sed "s/^/$n tests: /" | tee -a $out/summary.txt
done
for rep in $(seq $reps); do
  for nv in default "$@"; do
    n=${nv%%=*}
    if [ $n = default ]; then lib=""; else lib=$GRAFT_REPO_ROOT/${nv#*=}; fi
    T1ENV_LIB=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/bench_${n}_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/bench_${n}_$rep.json')); print('$n rep $rep', round(d['value']/1e6,2), 'M', d['ms_per_step'])" | tee -a $out/summary.txt
  done
done
