# contact / dynamics / fused / policy-conv tests, then the what-if A/B and the rollout profile
set -e
t=${1:-r03v}
o=$GRAFT_REPO_ROOT/gpurun_out/$t
mkdir -p $o
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -s tests/test_gpu_policy_conv.py tests/test_gpu_dynamics_contact.py tests/test_gpu_dynamics.py tests/test_gpu_fused.py > $o/tests.log 2>&1
timeout -k 10 300 python tools/prof_rollout.py > $o/rollout_profile.txt 2>&1
bash tools/gpu/r03_whatif.sh $t
