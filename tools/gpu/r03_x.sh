# tests (MFMA conv, contact, dynamics, fused), self-collision A/B, rollout profile, PPO update profiles
set -e
t=${1:-r03x}
o=$GRAFT_REPO_ROOT/gpurun_out/$t
mkdir -p $o
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -s tests/test_gpu_policy_conv.py tests/test_gpu_dynamics_contact.py tests/test_gpu_dynamics.py tests/test_gpu_fused.py > $o/tests.log 2>&1
bash tools/gpu/r03_ab_self.sh $t
timeout -k 10 300 python tools/prof_rollout.py > $o/rollout_profile.txt 2>&1
bash tools/gpu/r03_w.sh $t
