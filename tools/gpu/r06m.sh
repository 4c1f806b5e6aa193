set -e
out=gpurun_out/r06m; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_product_parity.py tests/test_gpu_fused.py tests/test_gpu_step.py tests/test_gpu_fp16.py tests/test_gpu_reset_idx.py tests/test_gpu_parity.py tests/test_gpu_sharding.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1
tail -1 $out/tests.log
for rep in 1 2 3 4; do
  for nv in new=default old=ti5_isaacgym_amd/_lib/var/zero_old.so; do
    n=${nv%%=*}; lib=${nv#*=}; if [ "$lib" = default ]; then lib=""; else lib=$PWD/$lib; fi
    T1ENV_SKIP_STAMP=1 T1ENV_LIB=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline > $out/${n}_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/${n}_$rep.json')); print('$n', $rep, d['ms_per_step'], d['roofline']['kernels'][d['roofline']['kernel']]['avg_ms'])" | tee -a $out/modes.txt
    T1ENV_SKIP_STAMP=1 T1ENV_LIB=$lib timeout -k 10 200 python bench.py --steps 300 --warmup 50 --no-cpu-baseline --num-envs 32768 --mesh heightfield --state-dtype fp16 --push > $out/${n}_c5_$rep.json 2>> $out/err.log
    python -c "import json; d=json.load(open('$out/${n}_c5_$rep.json')); print('$n cfg5', $rep, d['ms_per_step'])" | tee -a $out/modes.txt
  done
done
