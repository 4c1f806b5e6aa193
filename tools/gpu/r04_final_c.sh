# round-4 final check: every -m gpu test, smoke(), and the BASELINE configs with the kernel choice by env count
#   bash tools/gpu/r04_final_c.sh <tag> -> gpurun_out/<tag>/
set -e
tag=${1:-r04fc}
out=gpurun_out/$tag
mkdir -p $out
T1_PARITY_REPORT=$out/parity_report.json timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 \
    --timeout-method thread > $out/tests.log 2>&1 || echo "TESTS FAILED rc=$?" >> $out/tests.log
grep -q "Fatal\|core dumped\|Aborted\|Segmentation" $out/tests.log && exit 3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
B="python bench.py --steps 480 --warmup 48 --repeats 5 --no-cpu-baseline"
timeout -k 10 200 $B --num-envs 16384 --mesh trimesh > $out/n16384_trimesh.json 2> $out/n16384.err
timeout -k 10 200 $B --num-envs 32768 --mesh heightfield --push > $out/cfg5_32768_hf_push_fp32.json 2> $out/cfg5a.err
timeout -k 10 200 $B --num-envs 32768 --mesh heightfield --push --state-dtype fp16 > $out/cfg5_32768_hf_push_fp16.json 2> $out/cfg5b.err
tail -3 $out/tests.log
cat $out/smoke.log | tail -2
