# round-5 final tree after the update / act kernels: the GPU suite, smoke(), the default bench line, the median of 5,
# the PPO iteration (bf16 and fp32 updates) and act() timing
#   bash tools/gpu/r05_final_d.sh <tag>
set -e
tag=${1:-r05fd}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $out/gpu_tests.log 2>&1
tail -2 $out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err
timeout -k 10 300 python bench.py --steps 480 --warmup 48 --repeats 5 --no-cpu-baseline > $out/bench_median5.json 2> $out/bench_median5.err
python -c "import json; d=json.load(open('$out/bench_default.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['bound'], d['cpu_baseline']['value'])"
python -c "import json; d=json.load(open('$out/bench_median5.json')); print(d['value'], d['ms_per_step'], d.get('repeat_values'))"
timeout -k 10 300 python tools/bench_ppo.py --iters 4 --bf16 > $out/ppo_bf16.json 2> $out/ppo_bf16.err
timeout -k 10 300 python tools/bench_ppo.py --iters 4 > $out/ppo_fp32.json 2> $out/ppo_fp32.err
cat $out/ppo_bf16.json $out/ppo_fp32.json
timeout -k 10 120 python tools/act_bench.py --iters 300 > $out/act.json 2> $out/act.err
cat $out/act.json
