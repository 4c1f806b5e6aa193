# round-4 (second session) probe: the HEAD tree's bench line (k_dyn5, fused epilogue on four waves) and its per-wave
# phase profile.   bash tools/gpu/r04b_probe.sh <tag> -> gpurun_out/<tag>/
set -e
tag=${1:-r04g}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 300 python bench.py --steps 480 --warmup 48 --repeats 3 --no-cpu-baseline > $out/bench.json 2> $out/bench.err
timeout -k 10 300 python tools/prof_dynamics_phases.py --steps 100 > $out/phases5.txt 2> $out/phases5.err
cat $out/bench.json $out/phases5.txt
