"""Dev probe: the shader clock k_dyn6 runs at (a -DT1_PROBE_CLOCK build: lane 0 of every workgroup's wave 0 reads the
shader-cycle counter (s_memtime) and the 100 MHz constant counter (s_memrealtime) at the start and end of the launch and
adds the deltas to two device counters), against the step time -- to tell a clock (power-management) mode from a code
mode when a build's step time differs across processes (VERDICT r5 #1b, the -O2 slow mode).

    T1ENV_LIB=ti5_isaacgym_amd/_lib/var/<probe build>.so python tools/clock_probe.py [--steps 300]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd import make_t1_env  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--num-envs", type=int, default=8192)
    p.add_argument("--dump", default=None, help="save the per-workgroup (life, S1 wait, S2 wait) us array (.npy)")
    a = p.parse_args()
    N = a.num_envs
    env = make_t1_env(num_envs=N, mesh_type="trimesh", seed=5, device="cuda:0")
    env.reset()
    acts = torch.randn(8, N, 12, device="cuda:0")
    for i in range(50):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    lib = ctypes.CDLL(os.environ["T1ENV_LIB"])
    out = np.zeros(4, np.uint64)
    lib.t1env_debug_clock6(out.ctypes.data_as(ctypes.c_void_p), 1)   # read and reset
    wg = (N + 31) // 32
    sums = np.zeros((wg, 3), np.uint64)
    lib.t1env_debug_wgsum6(sums.ctypes.data_as(ctypes.c_void_p), wg, 1)
    t0 = time.perf_counter()
    for i in range(a.steps):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / a.steps * 1e3
    lib.t1env_debug_clock6(out.ctypes.data_as(ctypes.c_void_p), 0)
    cycles, ticks, launches = int(out[0]), int(out[1]), int(out[2])
    mhz = cycles / (ticks / 100.0) if ticks else None   # s_memrealtime: 100 MHz
    # per workgroup over the timed steps: W0's lifetime and its S1 / S2 waits (us per launch at the measured clock),
    # and by terrain type (the reference's floor(i / (N / 20)), legged_robot.py:1490) of the workgroup's first env
    lib.t1env_debug_wgsum6(sums.ctypes.data_as(ctypes.c_void_p), wg, 0)
    per = sums.astype(np.float64) / a.steps / (mhz if mhz else 2400.0)   # us per launch
    ttype = (np.arange(wg) * 32) // max(1, N // 20)
    by_type = {int(k): [round(float(per[ttype == k, j].mean()), 2) for j in range(3)] for k in np.unique(ttype)}
    slow = np.argsort(-per[:, 0])[:8]
    if a.dump:
        np.save(a.dump, per)
    # the last launch's timeline (us from its first workgroup's start): start spread, W0 lifetimes, last-wave ends
    tl = np.zeros((wg, 4), np.uint64)
    lib.t1env_debug_wgtime6(tl.ctypes.data_as(ctypes.c_void_p), wg)
    t0 = int(tl[:, 0].min())
    st, w0e, end, lend = ((tl[:, k].astype(np.int64) - t0) / 100.0 for k in range(4))
    # the last launch's resets per workgroup (the reset buffer after the step) against its loop / epilogue times
    rs = env.reset_buf.detach().to(torch.int32).cpu().numpy()[: wg * 32].reshape(wg, 32).sum(1)
    loop_t, epi_t = lend - st, w0e - lend
    epi_by_resets = {"0": round(float(epi_t[rs == 0].mean()), 2) if (rs == 0).any() else None,
                     ">=1": round(float(epi_t[rs > 0].mean()), 2) if (rs > 0).any() else None,
                     "wgs_with_resets": int((rs > 0).sum())}
    q = lambda v: [round(float(x), 2) for x in np.quantile(v, [0, 0.5, 0.9, 1.0])]  # noqa: E731
    print(json.dumps({"ms_per_step": round(ms, 4), "launches_x_workgroups": launches,
                      "shader_mhz": round(mhz, 1) if mhz else None,
                      "w0_lifetime_us_mean": round(ticks / max(1, launches) / 100.0, 2),
                      "last_launch_us": {"start_q0_50_90_100": q(st), "w0_life_q": q(w0e - st),
                                         "wg_end_q": q(end), "after_w0_q": q(end - w0e),
                                         "loop_q": q(loop_t), "epilogue_q": q(epi_t),
                                         "epilogue_by_resets": epi_by_resets,
                                         "slowest_end_wgs": [[int(b), round(float(loop_t[b]), 2), round(float(epi_t[b]), 2),
                                                              int(rs[b])] for b in np.argsort(-end)[:6]]},
                      "per_wg_us_life_s1wait_s2wait_q": [q(per[:, j]) for j in range(3)],
                      "by_terrain_type_life_s1_s2": by_type,
                      "slowest_wgs": [[int(b), [round(float(x), 2) for x in per[b]]] for b in slow],
                      "lib": os.path.basename(os.environ["T1ENV_LIB"])}))


if __name__ == "__main__":
    main()
