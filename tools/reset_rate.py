"""Dev probe: envs reset per step (and per 64-env wave) in the default bench workload."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd import make_t1_env
N = 8192
env = make_t1_env(num_envs=N, mesh_type="trimesh", seed=5, device="cuda:0")
g = torch.Generator(device="cuda:0").manual_seed(1234)
pool = [torch.randn(N, 12, device="cuda:0", generator=g) for _ in range(8)]
env.reset()
tot, waves_any, steps = 0.0, 0.0, 250
for i in range(steps):
    env.step(pool[i % 8])
    if i >= 50:
        r = env.reset_buf.view(-1, 64).bool()
        tot += r.sum().item()
        waves_any += r.any(1).float().mean().item()
print(f"resets per step {tot / (steps - 50):.1f} of {N}; waves with >= 1 reset {waves_any / (steps - 50):.3f}")
