"""Summarise gpurun_out/<tag>/bench*.json lines: value, ms/step, per-kernel event averages."""
import glob
import json
import sys

for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/bench*.json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable:", e)
        continue
    k = {n: v["avg_ms"] for n, v in d["roofline"]["kernels"].items()}
    print(f, d["value"], d["ms_per_step"], k, d["roofline"].get("step_span_ms_timed"))
