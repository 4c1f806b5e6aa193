"""SQ counter summary of the fused step kernel from the rocprofv3 databases tools/gpu/pmc_sq.sh writes.

    python tools/pmc_sq_summary.py gpurun_out/<tag>/sq1_results.db gpurun_out/<tag>/sq2_results.db \
        --envs 8192 -o profiles/<tag>_sq_counters.json

Per counter: the value summed over the kernel's per-SE instances of one dispatch, averaged over the dispatches
of k_dyn4.  Derived: VALU instructions per dynamics wave, the issue fraction (VALU quad-cycles over wave
quad-cycles), and the VALU-issue roofline bench.py reports beside the HBM one ("Roofline").
"""
import argparse
import json
import sqlite3
from collections import defaultdict

KERNEL = "k_dyn4"


def collect(db):
    c = sqlite3.connect(db)
    per = defaultdict(lambda: defaultdict(float))
    for disp, name, counter, value in c.execute(
            "select dispatch_id, kernel_name, counter_name, value from counters_collection"):
        if KERNEL in name:
            per[counter][disp] += value
    return {k: sum(v.values()) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dbs", nargs="+")
    p.add_argument("--envs", type=int, default=8192)
    p.add_argument("-o", "--out")
    a = p.parse_args()
    vals, n = {}, {}
    for db in a.dbs:
        v, k = collect(db)
        vals.update(v)
        n.update(k)
    dyn_waves = 4 * ((a.envs + 63) // 64)
    d = {}
    if "SQ_INSTS_VALU" in vals:
        d["valu_insts_per_dyn_wave"] = vals["SQ_INSTS_VALU"] / dyn_waves
    if "SQ_WAVE_CYCLES" in vals and "SQ_WAVES" in vals:
        d["quad_cycles_per_wave"] = vals["SQ_WAVE_CYCLES"] / vals["SQ_WAVES"]
    if "SQ_ACTIVE_INST_VALU" in vals and "SQ_WAVE_CYCLES" in vals:
        # VALU quad-cycles over wave quad-cycles: the share of every wave's lifetime spent issuing VALU
        d["valu_issue_frac"] = vals["SQ_ACTIVE_INST_VALU"] / vals["SQ_WAVE_CYCLES"]
    if "SQ_WAIT_ANY" in vals and "SQ_WAVE_CYCLES" in vals:
        d["wait_any_frac"] = vals["SQ_WAIT_ANY"] / vals["SQ_WAVE_CYCLES"]
    out = {"kernel": KERNEL, "envs": a.envs, "dispatches": n, "counters": vals, "derived": d,
           "sources": a.dbs}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
