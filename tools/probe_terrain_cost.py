"""Dev probe: k_dynamics time on trimesh terrain vs the same height-field code path on a flat height field.

Separates the cost of height-field queries from the cost of the different robot behaviour on rough terrain.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd import make_t1_env  # noqa: E402


def run(flat, steps=100, warmup=20, n=8192):
    env = make_t1_env(num_envs=n, mesh_type="trimesh", seed=5, device="cuda:0")
    if flat:
        env.height_samples.zero_()
        env._lib.t1env_set_terrain(env._handle, env.height_samples.data_ptr(), env.height_samples.shape[0], env.height_samples.shape[1],
                                   env.cfg.terrain.horizontal_scale, env.cfg.terrain.vertical_scale,
                                   env.cfg.terrain.border_size, 2)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(1234)
    pool = [torch.randn(n, 12, device="cuda:0", generator=g) for _ in range(8)]
    env.reset()
    for i in range(warmup):
        env.step(pool[i % 8])
    env.set_timing(True)
    for i in range(steps):
        env.step(pool[i % 8])
    t = env.get_timing()
    resets = float(env.reset_buf.float().mean())
    return t["k_dynamics"]["ms"] / t["k_dynamics"]["launches"], resets


for flat in (False, True):
    ms, r = run(flat)
    print(f"{'flat height field' if flat else 'trimesh curriculum'}: k_dynamics {ms:.4f} ms  reset fraction {r:.4f}")
