# rocprofv3 kernel statistics of the rollout's act() (tools/act_bench.py) at 8192 envs, 64-env heads (default) and the
# 32-env heads (T1POLICY_HEADS64=0).   bash tools/gpu/act_probe.sh <tag>
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/${1:-actprobe}; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out -o h64 -- python3 $GRAFT_REPO_ROOT/tools/act_bench.py --iters 200 > $out/h64.json 2> $out/h64.err
T1POLICY_HEADS64=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out -o h32 -- python3 $GRAFT_REPO_ROOT/tools/act_bench.py --iters 200 > $out/h32.json 2> $out/h32.err
