"""Diagnostics: one synced env step of the GPU env vs the host fp64 replica (tests/test_gpu_dynamics.py)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle.cpu_env import CpuT1Env  # noqa: E402
from ti5_isaacgym_amd import make_t1_env  # noqa: E402

N = 64
env = make_t1_env(num_envs=N, mesh_type="plane", seed=5, device="cuda:0")
c64 = CpuT1Env(env._model, N, seed=5, mesh_type="plane", fp64=True)
env.reset()
c64.reset()
print("after reset |root diff|", np.abs(env.root_states.cpu().numpy() - c64.o.root).max(axis=0))
rng = np.random.default_rng(3)
for t in range(3):
    a = (0.5 * rng.standard_normal((N, 12))).astype(np.float32)
    if t == 2:
        a[:] = 0
    root, dof = c64.o.root.copy(), c64.o.dof.copy()
    env.root_states.copy_(torch.from_numpy(root))
    env.dof_state.copy_(torch.from_numpy(dof.reshape(N * 12, 2)))
    env.step(torch.from_numpy(a).to("cuda:0"))
    c64.step(a)
    g = env.root_states.cpu().numpy()
    gd = env.dof_state.view(N, 12, 2).cpu().numpy()
    print(f"step {t}")
    print("  root err per component", np.array2string(np.abs(g - c64.o.root).max(axis=0), precision=2))
    print("  q err per joint", np.array2string(np.abs(gd[..., 0] - c64.o.dof[..., 0]).max(axis=0), precision=2))
    print("  qd err per joint", np.array2string(np.abs(gd[..., 1] - c64.o.dof[..., 1]).max(axis=0), precision=2))
    print("  torque err per joint (last substep)",
          np.array2string(np.abs(env.torques.cpu().numpy() - c64.o.torques).max(axis=0), precision=2))
    print("  rigid pos err per body", np.array2string(
        np.abs(env.rigid_state.cpu().numpy()[..., :3] - c64.o.rigid[..., :3]).max(axis=(0, 2)), precision=2))
    print("  z gpu/cpu env0", g[0, 2], c64.o.root[0, 2], "vz", g[0, 9], c64.o.root[0, 9])
    print("  reset gpu/cpu", int(env.reset_buf.sum()), int(c64.o.reset_buf.sum()))
