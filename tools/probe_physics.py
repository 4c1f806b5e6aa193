"""Dev probe: step the real HIP physics and print a few trajectory statistics."""
import sys
import time

import torch

sys.path.insert(0, ".")
from ti5_isaacgym_amd import make_t1_env  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
mesh = sys.argv[3] if len(sys.argv) > 3 else "plane"
env = make_t1_env(num_envs=n, mesh_type=mesh)
env.reset()
torch.cuda.synchronize()
resets = 0
for t in range(steps):
    a = torch.zeros(n, 12, device="cuda:0") if t < steps // 2 else 0.3 * torch.randn(n, 12, device="cuda:0")
    obs, priv, rew, done, ex = env.step(a)
    resets += int(done.sum())
    if t % 20 == 0 or t == steps - 1:
        z = env.root_states[:, 2]
        fz = env.contact_forces[:, [6, 12], 2]
        print(f"t={t:4d} z mean {z.mean():.3f} min {z.min():.3f} max {z.max():.3f} | base contact resets so far {resets}"
              f" | foot Fz mean {fz.mean():.1f} | rew mean {rew.mean():.4f} | q err "
              f"{(env.dof_pos - env.default_dof_pos).abs().mean():.3f} | finite {bool(torch.isfinite(env.root_states).all())}",
              flush=True)
torch.cuda.synchronize()
t0 = time.time()
for _ in range(20):
    env.step(torch.zeros(n, 12, device="cuda:0"))
torch.cuda.synchronize()
dt = (time.time() - t0) / 20
print(f"{n} envs: {dt * 1e3:.2f} ms/step -> {n / dt:.0f} env-steps/s")
