# round-5: k_dyn6 phase profile and timing-only what-ifs (the distal half of W0's CRBA skipped; no fold-in)
#   bash tools/gpu/r05_wi.sh <tag>
set -e
tag=${1:-r05wi}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/prof_dynamics_phases.py --kernel 6 > $out/phases6.txt 2>&1
head -3 $out/phases6.txt
V=ti5_isaacgym_amd/_lib/var
bash tools/gpu/r05_ab.sh $tag 2 k6 $V/libd6_crbahalf.so $V/libd6_nofoldin.so
