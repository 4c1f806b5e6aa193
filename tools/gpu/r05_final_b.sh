# round-5 measurement set B: every BASELINE config on one GPU (median of 5 x 480 steps) with the CPU baseline of
# configs 1 and 2, the GPU suite and smoke()
#   bash tools/gpu/r05_final_b.sh <tag> -> gpurun_out/<tag>/
set -e
tag=${1:-r05fb}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $out/gpu_tests.log 2>&1
tail -2 $out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
B="python bench.py --steps 480 --warmup 48 --repeats 5"
timeout -k 10 300 $B --num-envs 64 --mesh plane --cpu-envs 64 --cpu-seconds 20 > $out/cfg1_64_plane.json 2> $out/cfg1.err
timeout -k 10 300 $B --num-envs 4096 --mesh plane --cpu-envs 4096 --cpu-seconds 20 > $out/cfg2_4096_plane.json 2> $out/cfg2.err
timeout -k 10 200 $B --num-envs 16384 --mesh trimesh --no-cpu-baseline > $out/n16384_trimesh.json 2> $out/n16384.err
timeout -k 10 200 $B --num-envs 32768 --mesh heightfield --push --no-cpu-baseline > $out/cfg5_32768_hf_push_fp32.json 2> $out/cfg5a.err
timeout -k 10 200 $B --num-envs 32768 --mesh heightfield --push --state-dtype fp16 --no-cpu-baseline > $out/cfg5_32768_hf_push_fp16.json 2> $out/cfg5b.err
echo done
