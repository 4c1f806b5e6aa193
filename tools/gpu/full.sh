# Round-end style check: GPU tests, smoke, default bench (with CPU baseline), rocprof kernel stats + PMC passes.
#   bash tools/gpu/full.sh <tag> -> gpurun_out/<tag>/...
set -e
tag=${1:-full}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/tests.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
bash tools/gpu/profile.sh $tag
