# phase profile (capsules on / off) and the PPO benches
set -e
t=${1:-r03q}
o=$GRAFT_REPO_ROOT/gpurun_out/$t
mkdir -p $o
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/prof_dynamics_phases.py > $o/phases_self_on.txt 2>&1
timeout -k 10 300 python tools/prof_dynamics_phases.py --no-self-collision > $o/phases_self_off.txt 2>&1
timeout -k 10 300 python tools/bench_ppo.py --bf16 --iters 6 > $o/ppo_bf16.json 2> $o/ppo_bf16.err
timeout -k 10 300 python tools/bench_ppo.py --iters 6 > $o/ppo_fp32.json 2> $o/ppo_fp32.err
