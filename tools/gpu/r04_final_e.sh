# round-4 final tree (second session): every BASELINE config on one GPU, median of 5 x 480 steps (the CPU baselines of
# configs 1 / 2 do not depend on the GPU kernel: profiles/r04fb_cfg*.json)
#   bash tools/gpu/r04_final_e.sh <tag> -> gpurun_out/<tag>/
set -e
tag=${1:-r04ff}
out=gpurun_out/$tag
mkdir -p $out
B="python bench.py --steps 480 --warmup 48 --repeats 5 --no-cpu-baseline"
timeout -k 10 200 $B --num-envs 64 --mesh plane > $out/cfg1_64_plane.json 2> $out/cfg1.err
timeout -k 10 200 $B --num-envs 4096 --mesh plane > $out/cfg2_4096_plane.json 2> $out/cfg2.err
timeout -k 10 200 $B --num-envs 16384 --mesh trimesh > $out/n16384_trimesh.json 2> $out/n16384.err
timeout -k 10 200 $B --num-envs 32768 --mesh heightfield --push > $out/cfg5_32768_hf_push_fp32.json 2> $out/cfg5a.err
timeout -k 10 200 $B --num-envs 32768 --mesh heightfield --push --state-dtype fp16 > $out/cfg5_32768_hf_push_fp16.json 2> $out/cfg5b.err
for f in $out/*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']/1e6,2), 'M', d['ms_per_step'], d['roofline'].get('kernel'))"; done
