"""HBM traffic per env step from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE), for bench.py's `traffic`.

    rocprofv3 --kernel-trace --pmc FETCH_SIZE -d OUT -o fetch -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
    rocprofv3 --kernel-trace --pmc WRITE_SIZE -d OUT -o write -- python3 bench.py ...
    python tools/pmc_traffic.py OUT/fetch_results.db OUT/write_results.db --num-envs 8192 --mesh trimesh \
        -o profiles/traffic_r01.json

Counters are collected in separate passes (FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2).  Both are KB per
dispatch.  gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of a
wide coalesced read, so it is doubled; WRITE_SIZE is taken as is.  Per kernel the median over the step's
dispatches is used; the env step is one dispatch of each kernel in STEP_KERNELS.
"""
import argparse
import json
import sqlite3
import statistics

STEP_KERNELS = ["k_dyn6", "k_dyn5", "k_shift5", "k_shift4c", "k_dyn4", "k_dynamics", "k_post_a", "k_post_b", "k_shift", "k_stack", "k_finalize", "k_terrain_level_sum"]
FETCH_CORRECTION = 2.0


def per_kernel(db, counter):
    c = sqlite3.connect(db)
    q = """select s.display_name, p.value from rocpd_pmc_event p
           join rocpd_info_pmc i on p.pmc_id = i.id
           join rocpd_kernel_dispatch d on d.event_id = p.event_id
           join rocpd_info_kernel_symbol s on s.id = d.kernel_id
           where i.name = ?"""
    out = {}
    for name, val in c.execute(q, (counter,)):
        short = name.split("(")[0].split("<")[0].replace("void ", "").strip()
        out.setdefault(short, []).append(float(val))
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch_db")
    p.add_argument("write_db")
    p.add_argument("--num-envs", type=int, required=True)
    p.add_argument("--mesh", required=True)
    p.add_argument("-o", "--out")
    a = p.parse_args()
    fetch, write = per_kernel(a.fetch_db, "FETCH_SIZE"), per_kernel(a.write_db, "WRITE_SIZE")
    kernels, total = {}, 0.0
    for k in STEP_KERNELS:
        if k not in fetch or k not in write:
            continue
        f_kb, w_kb = statistics.median(fetch[k]), statistics.median(write[k])
        hbm = (FETCH_CORRECTION * f_kb + w_kb) * 1024.0
        kernels[k] = {"fetch_kb_raw": round(f_kb, 1), "write_kb": round(w_kb, 1), "hbm_bytes": round(hbm),
                      "dispatches": len(fetch[k])}
        total += hbm
    res = {"num_envs": a.num_envs, "mesh": a.mesh, "fetch_correction": FETCH_CORRECTION,
           "hbm_bytes_per_step": round(total), "hbm_bytes_per_env_step": round(total / a.num_envs, 1),
           "kernels": kernels}
    print(json.dumps(res, indent=1))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
