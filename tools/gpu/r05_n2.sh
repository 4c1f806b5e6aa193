# round-5: contact_pair's vectors by reference (less -O2 scratch): -O1 / -O2 vs the product build, 4 reps
set -e
tag=${1:-r05n2}
cd $GRAFT_REPO_ROOT
V=ti5_isaacgym_amd/_lib/var
bash tools/gpu/r05_ab.sh $tag 4 $V/libd6_base.so $V/libd6_n1b.so $V/libd6_n2b.so
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fp16.py > gpurun_out/$tag/fp16_tests.log 2>&1
tail -2 gpurun_out/$tag/fp16_tests.log
timeout -k 10 200 python bench.py --num-envs 32768 --mesh heightfield --push --state-dtype fp16 --steps 480 --warmup 48 --repeats 5 --no-cpu-baseline > gpurun_out/$tag/cfg5_fp16_default.json 2> gpurun_out/$tag/cfg5.err
python -c "import json; d=json.load(open('gpurun_out/$tag/cfg5_fp16_default.json')); print('cfg5 fp16 default', d['value'], d['ms_per_step'], list(d['roofline']['kernels']))"
bash tools/gpu/r05_ab.sh ${tag}_scr 3 ti5_isaacgym_amd/_lib/var/libd6_base.so ti5_isaacgym_amd/_lib/var/libd6_scr64.so
