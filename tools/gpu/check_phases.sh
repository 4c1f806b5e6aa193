# GPU check (tests + bench) followed by the fused-kernel phase profile
set -e
tag=${1:-check}
bash tools/gpu/check.sh $tag
timeout -k 10 300 python tools/prof_dynamics_phases.py > gpurun_out/$tag/phases.txt 2>&1
