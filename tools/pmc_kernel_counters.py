"""Dev tool: per-dispatch means of the PMC counters rocprofv3 --pmc collected for one kernel (name substring), with the
traced mean duration, from one or more rocprofv3 databases (one pass each).

    python tools/pmc_kernel_counters.py gpurun_out/<tag>/p1_results.db gpurun_out/<tag>/p2_results.db --kernel k_gemm
"""
import argparse
import json
import sqlite3
from collections import defaultdict


def main():
    p = argparse.ArgumentParser()
    p.add_argument("dbs", nargs="+")
    p.add_argument("--kernel", required=True)
    a = p.parse_args()
    out, dur = {}, []
    for db in a.dbs:
        c = sqlite3.connect(db)
        per = defaultdict(lambda: defaultdict(float))
        for disp, name, counter, value in c.execute(
                "select dispatch_id, kernel_name, counter_name, value from counters_collection"):
            if a.kernel in name:
                per[counter][disp] += value
        out.update({k: sum(v.values()) / len(v) for k, v in per.items()})
        ids = [kid for kid, name in c.execute("select id, display_name from rocpd_info_kernel_symbol") if a.kernel in name]
        for kid in ids:
            dur += [e - s for s, e in c.execute("select start, end from rocpd_kernel_dispatch where kernel_id = ?", (kid,))]
    res = {"kernel": a.kernel, "mean_us": round(sum(dur) / len(dur) / 1e3, 2) if dur else None,
           "counters": {k: round(v, 1) for k, v in sorted(out.items())}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
