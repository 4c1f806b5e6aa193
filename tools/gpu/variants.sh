# A/B the library builds under ti5_isaacgym_amd/_lib/var/*.so: GPU dynamics/fused tests + uninstrumented bench each.
#   bash tools/gpu/variants.sh <tag> [names...]  -> gpurun_out/<tag>/<name>.{tests.log,bench.json}
tag=${1:-var}; shift
out=gpurun_out/$tag
mkdir -p $out
names=${@:-$(cd ti5_isaacgym_amd/_lib/var && ls *.so | sed 's/\.so$//')}
timeout -k 10 120 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/base.bench.json 2> $out/base.err || exit 1
for v in $names; do
  export T1ENV_LIB=$PWD/ti5_isaacgym_amd/_lib/var/$v.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_dynamics.py tests/test_gpu_fused.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $out/$v.tests.log 2>&1
  rc=$?
  if [ $rc -ge 124 ]; then echo "stop: $v tests rc=$rc"; exit $rc; fi
  timeout -k 10 120 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/$v.bench.json 2> $out/$v.err || exit 1
done
unset T1ENV_LIB
timeout -k 10 120 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0 > $out/base2.bench.json 2>> $out/base.err
