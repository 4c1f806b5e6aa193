# restructured k_dyn4 (forward pass before S1, kinematics via LDS) + faster capsules: correctness, A/B, phases
set -e
t=${1:-r03s}
o=$GRAFT_REPO_ROOT/gpurun_out/$t
mkdir -p $o
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_dynamics_contact.py tests/test_gpu_dynamics.py tests/test_gpu_dynamics_kane.py tests/test_gpu_fused.py tests/test_gpu_product_parity.py tests/test_gpu_substep_log_identity.py > $o/tests.log 2>&1
bash tools/gpu/r03_ab_self.sh $t
timeout -k 10 300 python tools/prof_dynamics_phases.py > $o/phases_self_on.txt 2>&1
