# round-5: is the -O2 build's fast mode (r05ab2: 0.119 ms) a property of the box?  -O1 / -O2 interleaved, 3 reps
set -e
tag=${1:-r05o2b}
cd $GRAFT_REPO_ROOT
bash tools/gpu/r05_ab.sh $tag 3 ti5_isaacgym_amd/_lib/var/libd6_o1.so ti5_isaacgym_amd/_lib/var/libd6_o2.so
