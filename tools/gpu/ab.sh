# A/B bench of library builds under ti5_isaacgym_amd/_lib/var/*.so, interleaved (2 rounds), uninstrumented.
#   bash tools/gpu/ab.sh <tag> name...  -> gpurun_out/<tag>/<name>.<round>.json
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
for r in 1 2; do
  for v in "$@"; do
    T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/$v.so timeout -k 10 120 python bench.py --steps 300 --warmup 50 \
      --no-cpu-baseline --time-every 0 > $out/$v.$r.json 2> $out/$v.$r.err || exit 1
  done
done
