# round-5: the fold-in split across W0 / W4 (T1_D6_FOLD_SPLIT) against the product build
set -e
tag=${1:-r05fs}
cd $GRAFT_REPO_ROOT
V=ti5_isaacgym_amd/_lib/var
bash tools/gpu/r05_ab.sh $tag 3 $V/libd6_base.so $V/libd6_fs.so
