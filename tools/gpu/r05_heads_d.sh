# round-5 A/B: the 8-wave heads kernel's fragment-ring depths (T1_HEADS_D1/D2/D3 variants relinked into _lib/var),
# act() timing alternated; then a rocprof kernel trace of the product's act()
set -e
tag=${1:-r05hd}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for rep in 1 2; do
  for v in base h12_6_2 h4_2_1 h6_3_2; do
    if [ $v = base ]; then L=""; else L=$GRAFT_REPO_ROOT/ti5_isaacgym_amd/_lib/var/lib$v.so; fi
    T1ENV_LIB=${L:-} timeout -k 10 120 python tools/act_bench.py --iters 300 > $out/act_${v}_$rep.json 2>> $out/err.log
    echo "rep $rep $v $(cat $out/act_${v}_$rep.json)"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o act -- python tools/act_bench.py --iters 100 > $out/act_prof.json 2> $out/prof.err
echo profiled
