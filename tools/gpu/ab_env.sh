# Interleaved A/B of environment settings (T1ENV_* switches read when an env is created) on one bench workload.
#   bash tools/gpu/ab_env.sh <tag> <reps> "<bench.py args>" <name>=<VAR=VAL[,VAR=VAL...]> ...
#   -> gpurun_out/<tag>/{summary.txt,bench_<name>_<rep>.json}
set -e
tag=$1; reps=$2; args=$3; shift 3
out=gpurun_out/$tag
mkdir -p $out
for rep in $(seq $reps); do
  for nv in "$@"; do
    n=${nv%%=*}; kv=${nv#*=}
    envs=(); IFS=',' read -ra pairs <<< "$kv"; for p in "${pairs[@]}"; do envs+=("$p"); done
    env "${envs[@]}" timeout -k 10 200 python bench.py $args --no-cpu-baseline > $out/bench_${n}_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/bench_${n}_$rep.json')); k=d['roofline']['kernels']; print('$n rep $rep', round(d['value']/1e6,2), 'M', d['ms_per_step'], {a: b['avg_ms'] for a, b in k.items()}, d['roofline'].get('step_span_ms_timed'))" | tee -a $out/summary.txt
  done
done
