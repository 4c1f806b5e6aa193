# round-4 A/B over environment settings of the product library: each argument is NAME=ENV[|BENCH ARGS] (ENV:
# space-separated VAR=value pairs, quoted), two interleaved rounds of bench.py, then optionally the k_dyn5 phase
# profile.
#   bash tools/gpu/r04_ab2.sh <tag> <phases 0|1> 'conc=T1ENV_DYN_KERNEL=5' 'inwg=T1ENV_DYN_KERNEL=5 T1ENV_D5_SHIFT=0' ...
set -e
tag=$1; shift
ph=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for r in 1 2; do
  for v in "$@"; do
    name=${v%%=*}; rest=${v#*=}
    envs=${rest%%|*}; args=; [ "$rest" != "$envs" ] && args=${rest#*|}
    env $envs timeout -k 10 120 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 $args \
      > $out/$name.$r.json 2> $out/$name.$r.err
  done
done
if [ "$ph" = "1" ]; then
  T1ENV_DYN_KERNEL=5 timeout -k 10 200 python tools/prof_dynamics_phases.py --kernel 5 > $out/phases5.txt 2>&1
fi
python - <<PY
import json, glob, os
for f in sorted(glob.glob("$out/*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), d["ms_per_step"], round(d["value"] / 1e6, 2), "M")
PY
