# Other BASELINE configs (parity-test cases, reported in DESIGN.md) + PPO end-to-end, on the current build.
#   bash tools/gpu/configs.sh <tag>
set -e
tag=${1:-cfg}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 180 python bench.py --steps 200 --warmup 30 --no-cpu-baseline --num-envs 4096 --mesh plane > $out/cfg2_4096_plane.json 2> $out/cfg.err
timeout -k 10 240 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --num-envs 32768 --mesh heightfield > $out/cfg5_32768_hf.json 2>> $out/cfg.err
timeout -k 10 180 python bench.py --steps 200 --warmup 30 --no-cpu-baseline --num-envs 16384 --mesh trimesh > $out/n16384_trimesh.json 2>> $out/cfg.err
timeout -k 10 300 python tools/bench_ppo.py --num-envs 8192 --iters 3 > $out/ppo_8192.json 2> $out/ppo.err
