# round-5 end of session: the GPU suite and smoke() on the final tree
set -e
tag=${1:-r05fg}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $out/gpu_tests.log 2>&1
tail -1 $out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench_default.json 2> $out/bench_default.err
python -c "import json; d=json.load(open('$out/bench_default.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
