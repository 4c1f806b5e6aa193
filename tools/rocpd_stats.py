"""Kernel statistics (rocprofv3 --stats layout) from a rocprofv3 rocpd SQLite database.

    python tools/rocpd_stats.py gpurun_out/prof/run_results.db [-o profiles/rNN_kernel_stats.csv] [--top 12]

Also reports each kernel's register/LDS/scratch footprint from the code-object metadata.
"""
import argparse
import csv
import sqlite3
import statistics
import sys


def stats(db):
    c = sqlite3.connect(db)
    names = {}
    for kid, disp, sgpr, vgpr, agpr, lds, scratch in c.execute(
            "select id, display_name, sgpr_count, arch_vgpr_count, accum_vgpr_count, group_segment_size, "
            "private_segment_size from rocpd_info_kernel_symbol"):
        names[kid] = (disp, sgpr, vgpr, agpr, lds, scratch)
    durs = {}
    for kid, s, e in c.execute("select kernel_id, start, end from rocpd_kernel_dispatch"):
        durs.setdefault(kid, []).append(e - s)
    total = sum(sum(v) for v in durs.values())
    rows = []
    for kid, d in durs.items():
        disp, sgpr, vgpr, agpr, lds, scratch = names.get(kid, (str(kid), 0, 0, 0, 0, 0))
        rows.append({"Name": disp, "Calls": len(d), "TotalDurationNs": sum(d), "AverageNs": sum(d) / len(d),
                     "Percentage": 100.0 * sum(d) / total, "MinNs": min(d), "MaxNs": max(d),
                     "StdDev": statistics.pstdev(d), "SGPR": sgpr, "VGPR": vgpr, "AGPR": agpr, "LDS": lds,
                     "Scratch": scratch})
    rows.sort(key=lambda r: -r["TotalDurationNs"])
    return rows


def main():
    p = argparse.ArgumentParser()
    p.add_argument("db")
    p.add_argument("-o", "--out")
    p.add_argument("--top", type=int, default=12)
    a = p.parse_args()
    rows = stats(a.db)
    if a.out:
        with open(a.out, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()), quoting=csv.QUOTE_NONNUMERIC)
            w.writeheader()
            w.writerows(rows)
    for r in rows[:a.top]:
        sys.stdout.write(f"{r['Percentage']:6.2f}%  calls {r['Calls']:5d}  avg {r['AverageNs'] / 1e3:9.2f} us  "
                         f"vgpr {r['VGPR']:3d} agpr {r['AGPR']:3d} lds {r['LDS']:6d} scratch {r['Scratch']:5d}  "
                         f"{r['Name'][:90]}\n")


if __name__ == "__main__":
    main()
