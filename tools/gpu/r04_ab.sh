# round-4 A/B: interleaved uninstrumented benches of the product library (k_dyn5 / k_dyn4 by T1ENV_DYN_KERNEL) and
# variant builds under _lib/var, then (optional) the k_dyn5 phase profile.
#   bash tools/gpu/r04_ab.sh <tag> <phases 0|1> [variant ...]  -> gpurun_out/<tag>/*.json
set -e
tag=$1; shift
ph=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for r in 1 2; do
  T1ENV_DYN_KERNEL=5 timeout -k 10 120 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 \
    > $out/dyn5.$r.json 2> $out/dyn5.$r.err
  T1ENV_DYN_KERNEL=4 timeout -k 10 120 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 \
    > $out/dyn4.$r.json 2> $out/dyn4.$r.err
  for v in "$@"; do
    T1ENV_DYN_KERNEL=5 T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/$v.so timeout -k 10 120 python bench.py --steps 300 --warmup 50 \
      --no-cpu-baseline --time-every 0 > $out/$v.$r.json 2> $out/$v.$r.err
  done
done
if [ "$ph" = "1" ]; then
  timeout -k 10 200 python tools/prof_dynamics_phases.py --kernel 5 > $out/phases5.txt 2>&1
fi
python - <<PY
import json, glob, os
for f in sorted(glob.glob("$out/*.json")):
    d = json.load(open(f))
    print(os.path.basename(f), d["ms_per_step"], round(d["value"] / 1e6, 2), "M")
PY
