# r02l: -O3 guard test, SQ instruction counters of the fused step kernel, phase profile.   bash tools/gpu/r02l.sh <tag>
set -e
tag=${1:-r02l}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_opt_levels.py -x -v --timeout 500 --timeout-method thread > $out/opt_guard.log 2>&1
bash tools/gpu/pmc_sq.sh $tag
timeout -k 10 300 python tools/prof_dynamics_phases.py > $out/phases.txt 2>&1
