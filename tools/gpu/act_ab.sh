# Interleaved A/B of library builds on the rollout's act() (tools/act_bench.py, 8192 envs), after the heads tests on
# every candidate that is not a timing-only what-if (name whatif*).
#   bash tools/gpu/act_ab.sh <tag> <reps> <name>=<lib.so> ...   -> gpurun_out/<tag>/summary.txt
set -e
tag=$1; reps=$2; shift 2
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
for nv in "$@"; do
  n=${nv%%=*}; lib=$GRAFT_REPO_ROOT/${nv#*=}
  case $n in whatif*) continue;; esac
  T1ENV_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_policy_heads.py -x -q --timeout 120 \
    --timeout-method thread > $out/$n.tests.log 2>&1 || { echo "TESTS FAILED $n"; tail -30 $out/$n.tests.log; exit 1; }
  tail -1 $out/$n.tests.log | sed "s/^/$n tests: /" | tee -a $out/summary.txt
done
for rep in $(seq $reps); do
  for nv in default "$@"; do
    n=${nv%%=*}
    if [ $n = default ]; then lib=""; else lib=$GRAFT_REPO_ROOT/${nv#*=}; fi
    T1ENV_LIB=$lib timeout -k 10 200 python tools/act_bench.py --iters 400 > $out/act_${n}_$rep.json 2>> $out/err.log
    echo "$n rep $rep $(cat $out/act_${n}_$rep.json)" | tee -a $out/summary.txt
  done
done
