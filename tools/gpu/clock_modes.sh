# The shader clock vs the step time of k_dyn6 builds across fresh processes (tools/clock_probe.py, T1_PROBE_CLOCK builds)
#   bash tools/gpu/clock_modes.sh <tag> <reps> <name>=<lib.so> ... -> gpurun_out/<tag>/clock.txt
set -e
tag=$1; reps=$2; shift 2
out=gpurun_out/$tag
mkdir -p $out
for rep in $(seq $reps); do
  for nv in "$@"; do
    n=${nv%%=*}; lib=$PWD/${nv#*=}
    T1ENV_LIB=$lib timeout -k 10 200 python tools/clock_probe.py | sed "s/^/$n $rep /" | tee -a $out/clock.txt
  done
done
