# round-5: the kernel choice above 32 envs per CU (k_dyn6 in two rounds vs k_dyn4), then the whole GPU suite
#   bash tools/gpu/r05_full.sh <tag>
set -e
tag=${1:-r05full}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
for n in 16384 32768; do
  for k in 4 6; do
    T1ENV_DYN_KERNEL=$k timeout -k 10 200 python bench.py --num-envs $n --steps 200 --warmup 30 --no-cpu-baseline --time-every 0 > $out/n${n}_k$k.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/n${n}_k$k.json')); print('$n k$k', d['value'], d['ms_per_step'])" | tee -a $out/summary.txt
  done
done
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $out/tests.log 2>&1
tail -3 $out/tests.log
