# round-5: one copy of the contact law per call site (no merged copies indexing a scratch copy of the query), -O1 / -O2
set -e
tag=${1:-r05n}
cd $GRAFT_REPO_ROOT
V=ti5_isaacgym_amd/_lib/var
bash tools/gpu/r05_ab.sh $tag 3 $V/libd6_base.so $V/libd6_n1.so $V/libd6_n2.so
