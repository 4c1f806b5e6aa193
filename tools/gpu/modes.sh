# Step-time modes across processes: each library build (name=path, "default" = the product) benched in <reps> fresh
# processes, interleaved (8192 trimesh, 300 steps, sampled HIP events), with the history buffers' addresses.
#   bash tools/gpu/modes.sh <tag> <reps> <name>=<lib.so|default> ... -> gpurun_out/<tag>/{modes.txt,*.json}
set -e
tag=$1; reps=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for rep in $(seq $reps); do
  for nv in "$@"; do
    n=${nv%%=*}; lib=${nv#*=}
    if [ "$lib" = default ]; then lib=""; else lib=$PWD/$lib; fi
    T1ENV_LIB=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > $out/${n}_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/${n}_$rep.json')); k=d['roofline']['kernels']; print('$n', $rep, d['ms_per_step'], {a: b['avg_ms'] for a, b in k.items()}, d['buffers'])" | tee -a $out/modes.txt
  done
done
