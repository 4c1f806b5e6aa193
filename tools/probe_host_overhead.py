"""Dev probe: host-side cost of env.step() (Python + ctypes + HIP launches), no device sync in the loop."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd import make_t1_env  # noqa: E402

N = 8192
env = make_t1_env(num_envs=N, mesh_type="trimesh", seed=5, device="cuda:0")
pool = [torch.randn(N, 12, device="cuda:0") for _ in range(8)]
env.reset()
for i in range(30):
    env.step(pool[i % 8])
torch.cuda.synchronize()
host = []
t0 = time.perf_counter()
for i in range(200):
    a = time.perf_counter()
    env.step(pool[i % 8])
    host.append(time.perf_counter() - a)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
host.sort()
print(f"host per step: median {host[100] * 1e6:.1f} us, p90 {host[180] * 1e6:.1f} us; "
      f"submit loop {((t1 - t0) / 200) * 1e6:.1f} us/step; wall incl. drain {((t2 - t0) / 200) * 1e6:.1f} us/step")
# breakdown of the Python side
import cProfile  # noqa: E402
import pstats  # noqa: E402
pr = cProfile.Profile()
pr.enable()
for i in range(200):
    env.step(pool[i % 8])
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(12)
