"""Dev probe: split the fused step's time into its per-substep part and its fixed part (prologue, post-physics
epilogue, launch) by timing the same env at several decimations (substeps per env step).  Timing only: a
decimation other than 10 is not the task's physics.

    python tools/decimation_timing.py [--num-envs 8192] [--mesh trimesh] [--decimations 10 5 2 1]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def time_env(n, mesh, dec, steps, warmup):
    import torch
    from ti5_isaacgym_amd import make_t1_env

    def hook(cfg):  # the lag rings assume 10 substeps: lags 0 at every decimation, so the sizes compare like for like
        cfg.control.decimation = dec
        dr = cfg.domain_rand
        dr.lag_timesteps_range, dr.dof_lag_timesteps_range, dr.imu_lag_timesteps_range = [0, 0], [0, 0], [0, 0]
    env = make_t1_env(num_envs=n, mesh_type=mesh, seed=5, device="cuda:0", cfg_hook=hook)
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(0)
    acts = [torch.randn(n, 12, device="cuda:0", generator=g) for _ in range(8)]
    for i in range(warmup):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--num-envs", type=int, default=8192)
    p.add_argument("--mesh", default="trimesh")
    p.add_argument("--decimations", type=int, nargs="+", default=[10, 5, 2, 1])
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--warmup", type=int, default=50)
    a = p.parse_args()
    res = {d: time_env(a.num_envs, a.mesh, d, a.steps, a.warmup) for d in a.decimations}
    ds = sorted(res)
    # least-squares line ms = fixed + per_substep * decimation
    import numpy as np
    A = np.array([[1.0, d] for d in ds])
    fixed, per = np.linalg.lstsq(A, np.array([res[d] for d in ds]), rcond=None)[0]
    print(json.dumps({"num_envs": a.num_envs, "mesh": a.mesh, "ms_per_step": {str(d): round(res[d], 4) for d in ds},
                      "fit_fixed_ms": round(float(fixed), 4), "fit_per_substep_ms": round(float(per), 4),
                      "lib": os.environ.get("T1ENV_LIB", "product")}))


if __name__ == "__main__":
    main()
