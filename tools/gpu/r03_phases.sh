# phase profile of k_dyn4 (T1_PHASE_PROF build) with and without self-collision
set -e
o=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03j}
mkdir -p $o
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python tools/prof_dynamics_phases.py > $o/phases_self_on.txt 2>&1
timeout -k 10 300 python tools/prof_dynamics_phases.py --no-self-collision > $o/phases_self_off.txt 2>&1
