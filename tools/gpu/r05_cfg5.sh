# round-5: config 5 (32768 envs, height field, pushes, fp16 histories) on k_dyn6 vs k_dyn4, and 16384 fp16
set -e
tag=${1:-r05cfg5}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for k in 4 6; do
    for n in 32768 16384; do
      T1ENV_DYN_KERNEL=$k timeout -k 10 200 python bench.py --num-envs $n --mesh heightfield --push --state-dtype fp16 --steps 200 --warmup 30 --no-cpu-baseline --time-every 0 > $out/n${n}_k${k}_$rep.json 2>> $out/err.log
      python -c "import json; d=json.load(open('$out/n${n}_k${k}_$rep.json')); print('$n fp16 k$k rep $rep', d['value'], d['ms_per_step'])" | tee -a $out/summary.txt
    done
  done
done
