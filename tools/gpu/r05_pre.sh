# round-5: W0's post-S2 LDS reads issued earlier (the shank's terms before joints 5-4; W4's base block before the
# elimination) against the product build
set -e
tag=${1:-r05pre}
cd $GRAFT_REPO_ROOT
V=ti5_isaacgym_amd/_lib/var
bash tools/gpu/r05_ab.sh $tag 3 $V/libd6_base.so $V/libd6_se.so $V/libd6_wb.so $V/libd6_both.so
