# phase profiles of k_dynamics: fused vs split, and fused without the shift-side release fence (timing only)
set -e
o=gpurun_out/phases3.txt
: > $o
timeout -k 10 300 python tools/prof_dynamics_phases.py >> $o 2>&1
timeout -k 10 300 python tools/prof_dynamics_phases.py --split >> $o 2>&1
cp ti5_isaacgym_amd/_lib/libt1env_hip_prof_nofence.so ti5_isaacgym_amd/_lib/libt1env_hip_prof.so
echo "=== no shift fence (experiment) ===" >> $o
timeout -k 10 300 python tools/prof_dynamics_phases.py >> $o 2>&1
