# self-collision A/B (on/off, twice) and the phase profile with it on
set -e
t=${1:-r03r}
o=$GRAFT_REPO_ROOT/gpurun_out/$t
mkdir -p $o
cd $GRAFT_REPO_ROOT
bash tools/gpu/r03_ab_self.sh $t
timeout -k 10 300 python tools/prof_dynamics_phases.py > $o/phases_self_on.txt 2>&1
