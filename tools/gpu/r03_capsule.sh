# capsule self-collision: contact / dynamics GPU checks, then the on/off A/B and the phase profile
set -e
o=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03k}
mkdir -p $o
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -s tests/test_gpu_dynamics_contact.py tests/test_gpu_dynamics.py tests/test_gpu_dynamics_kane.py > $o/tests.log 2>&1
bash tools/gpu/r03_ab_self.sh ${1:-r03k}
timeout -k 10 300 python tools/prof_dynamics_phases.py > $o/phases_self_on.txt 2>&1
