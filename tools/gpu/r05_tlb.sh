# round-5: the per-process bimodal step time (0.125 vs 0.130 ms at -O1, 0.117 vs 0.131 at -O2): TLB / cache counters of
# fast and slow processes.  Lists the available counters first.
set -e
tag=${1:-r05tlb}
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > $out/avail.txt 2>&1 || true
grep -i -E "UTCL|TLB|TRANSLATION" $out/avail.txt | head -40 > $out/tlb_counters.txt || true
cat $out/tlb_counters.txt | head -20
