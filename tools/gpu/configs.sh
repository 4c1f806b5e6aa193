# bench.py over the BASELINE configs on one GPU (uninstrumented, 300 steps).
#   bash tools/gpu/configs.sh <tag> -> gpurun_out/<tag>/cfg_*.json
set -e
tag=${1:-cfg}
out=gpurun_out/$tag
mkdir -p $out
B="python bench.py --steps 300 --warmup 50 --no-cpu-baseline --time-every 0"
timeout -k 10 120 $B --num-envs 64 --mesh plane > $out/cfg1_64_plane.json 2> $out/cfg1.err
timeout -k 10 120 $B --num-envs 4096 --mesh plane > $out/cfg2_4096_plane.json 2> $out/cfg2.err
timeout -k 10 120 $B --num-envs 8192 --mesh trimesh > $out/cfg3_8192_trimesh.json 2> $out/cfg3.err
timeout -k 10 120 $B --num-envs 16384 --mesh trimesh > $out/n16384_trimesh.json 2> $out/n16384.err
timeout -k 10 120 $B --num-envs 32768 --mesh heightfield --push > $out/cfg5_32768_hf_push_fp32.json 2> $out/cfg5a.err
timeout -k 10 120 $B --num-envs 32768 --mesh heightfield --push --state-dtype fp16 > $out/cfg5_32768_hf_push_fp16.json 2> $out/cfg5b.err
