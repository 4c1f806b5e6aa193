# round-5: k_dyn6 build-level A/B (-O1 / -O2 / -O3, the W0 lane launder) and the GPU suite on the -O2 build
#   bash tools/gpu/r05_o2.sh <tag>
set -e
tag=${1:-r05o2}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
V=ti5_isaacgym_amd/_lib/var
bash tools/gpu/r05_ab.sh $tag 2 $V/libd6_o1nl.so $V/libd6_o2.so $V/libd6_o2nl.so $V/libd6_o3.so
T1ENV_LIB=$GRAFT_REPO_ROOT/$V/libd6_o2.so timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $out/tests_o2.log 2>&1
tail -3 $out/tests_o2.log
