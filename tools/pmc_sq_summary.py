"""SQ counter summary of the fused step kernel from the rocprofv3 databases tools/gpu/pmc_sq.sh writes.

    python tools/pmc_sq_summary.py gpurun_out/<tag>/sq1_results.db gpurun_out/<tag>/sq2_results.db \
        --envs 8192 -o profiles/<tag>_sq_counters.json

Per counter: the value summed over the kernel's per-SE instances of one dispatch, averaged over the dispatches
of --kernel (k_dyn6, the default step kernel up to 32 envs per CU; k_dyn5; k_dyn4).  Derived ("Roofline"):
  * k_dyn6 (two role waves per SIMD): valu_insts_per_simd = SQ_INSTS_VALU / (4 SIMDs x workgroups) and
    simd_issue_frac = 2 valu_insts_per_simd / kernel_cycles, against the SIMD's one wave64 VALU instruction per 2
    cycles (what bench.py's roofline.issue reports for k_dyn6);
  * valu_insts_per_dyn_wave: SQ_INSTS_VALU over the dynamics waves: k_dyn5 4 ceil(N / 32) (four role waves per 32
    envs, each also shifting history rows), k_dyn4 4 ceil(N / 64) (the shift waves issue a few hundred VALU each, so
    this slightly overstates a dynamics wave);
  * kernel_cycles = SQ_BUSY_CYCLES / 32 shader engines (SQ_BUSY_CYCLES is summed over the SEs) and the effective
    shader clock = kernel_cycles / the traced mean duration of the same dispatches;
  * dyn_wave_issue_frac = 4 valu_insts_per_dyn_wave / kernel_cycles: a dynamics wave's VALU issue over the launch,
    against one instruction per 4 cycles (a wave alone on its SIMD).  This is what bench.py's roofline.issue reports
    (it divides by the live launch duration x this clock);
  * valu_active_frac_all_waves = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: the same ratio averaged over EVERY wave of the
    launch, the history-shift waves (almost no VALU) included -- lower, and not the dynamics waves' issue fraction
    (round 2 reported this one as valu_issue_frac);
  * wait_any_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES (all waves).
"""
import argparse
import json
import sqlite3
from collections import defaultdict

KERNEL = "k_dyn5"
NUM_SE = 32   # MI355X shader engines (MI355X_MICROARCH.md)


def collect(db):
    c = sqlite3.connect(db)
    per = defaultdict(lambda: defaultdict(float))
    for disp, name, counter, value in c.execute(
            "select dispatch_id, kernel_name, counter_name, value from counters_collection"):
        if KERNEL in name:
            per[counter][disp] += value
    return {k: sum(v.values()) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def durations_ns(db):
    """traced durations of the kernel's dispatches (rocprofv3 --kernel-trace in the same pass)"""
    c = sqlite3.connect(db)
    ids = [kid for kid, name in c.execute("select id, display_name from rocpd_info_kernel_symbol") if KERNEL in name]
    out = []
    for kid in ids:
        out += [e - s for s, e in c.execute("select start, end from rocpd_kernel_dispatch where kernel_id = ?", (kid,))]
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dbs", nargs="+")
    p.add_argument("--envs", type=int, default=8192)
    p.add_argument("--kernel", default="k_dyn6", choices=["k_dyn6", "k_dyn5", "k_dyn4"])
    p.add_argument("-o", "--out")
    a = p.parse_args()
    global KERNEL
    KERNEL = a.kernel
    vals, n, durs = {}, {}, []
    for db in a.dbs:
        v, k = collect(db)
        vals.update(v)
        n.update(k)
        try:
            durs += durations_ns(db)
        except sqlite3.Error:
            pass
    dyn_waves = {"k_dyn6": 8 * ((a.envs + 31) // 32), "k_dyn5": 4 * ((a.envs + 31) // 32)}.get(
        a.kernel, 4 * ((a.envs + 63) // 64))
    d = {}
    if "SQ_INSTS_VALU" in vals:
        d["valu_insts_per_dyn_wave"] = vals["SQ_INSTS_VALU"] / dyn_waves
    if "SQ_WAVE_CYCLES" in vals and "SQ_WAVES" in vals:
        d["quad_cycles_per_wave"] = vals["SQ_WAVE_CYCLES"] / vals["SQ_WAVES"]
    if "SQ_BUSY_CYCLES" in vals:
        d["kernel_cycles"] = vals["SQ_BUSY_CYCLES"] / NUM_SE
        if durs:
            d["mean_duration_us"] = sum(durs) / len(durs) / 1e3
            d["shader_clock_ghz"] = d["kernel_cycles"] / (sum(durs) / len(durs))
        if "valu_insts_per_dyn_wave" in d:
            d["dyn_wave_issue_frac"] = 4.0 * d["valu_insts_per_dyn_wave"] / d["kernel_cycles"]
        if a.kernel == "k_dyn6" and "SQ_INSTS_VALU" in vals:
            d["valu_insts_per_simd"] = vals["SQ_INSTS_VALU"] / (4 * ((a.envs + 31) // 32))
            d["simd_issue_frac"] = 2.0 * d["valu_insts_per_simd"] / d["kernel_cycles"]
    if "SQ_ACTIVE_INST_VALU" in vals and "SQ_WAVE_CYCLES" in vals:
        # VALU quad-cycles over wave quad-cycles, averaged over every wave of the launch (shift waves included)
        d["valu_active_frac_all_waves"] = vals["SQ_ACTIVE_INST_VALU"] / vals["SQ_WAVE_CYCLES"]
    if "SQ_WAIT_ANY" in vals and "SQ_WAVE_CYCLES" in vals:
        d["wait_any_frac"] = vals["SQ_WAIT_ANY"] / vals["SQ_WAVE_CYCLES"]
    if "SQ_WAIT_INST_ANY" in vals and "SQ_WAVE_CYCLES" in vals:
        d["wait_inst_any_frac"] = vals["SQ_WAIT_INST_ANY"] / vals["SQ_WAVE_CYCLES"]
    if "SQC_ICACHE_MISSES" in vals and "SQC_ICACHE_HITS" in vals:
        d["icache_miss_rate"] = vals["SQC_ICACHE_MISSES"] / max(1.0, vals["SQC_ICACHE_HITS"] + vals["SQC_ICACHE_MISSES"])
    out = {"kernel": a.kernel, "envs": a.envs, "dispatches": n, "counters": vals, "derived": d,
           "sources": a.dbs}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
