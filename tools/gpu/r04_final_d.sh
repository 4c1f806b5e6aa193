# round-4 final tree (second session): every -m gpu test and smoke(), then measurement set A on the metric's config
# (bench line with the CPU baseline, median of 5 x 480, rocprof kernel stats, PMC HBM traffic, SQ counters).
#   bash tools/gpu/r04_final_d.sh <tag> -> gpurun_out/<tag>/
set -e
tag=${1:-r04fe}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd $GRAFT_REPO_ROOT
T1_PARITY_REPORT=$out/parity_report.json timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 \
    --timeout-method thread > $out/tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
tail -1 $out/smoke.log
bash tools/gpu/r04_final_a.sh $tag
