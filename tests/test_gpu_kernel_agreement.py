"""The selectable step kernels agree with each other -- needs the MI355X.

The product runs k_dyn6 at every env count (t1_dyn_waves_default, since r05; until r04 the choice went by env count,
so the same global envs ran on different kernels in an 8-GPU run and on one GPU), and T1ENV_DYN_KERNEL=4|5 selects
the older kernels.  The kernels solve
the same linear system per substep (compute_delta / _split / _roles / _roles6 agree in fp64, tests/test_dynamics.py)
but sum it in different fp32 orders, so their trajectories are not bit-identical, and contact dynamics amplify
rounding chaotically over a trajectory.  The bound is therefore on the ONE-STEP gap, as in tests/test_gpu_dynamics.py:
before every env step all three kernels' envs and a host fp32 replica are set to the fp64 host replica's state, all
advance one env step (10 substeps) with the same actions, and every pair of kernels must agree within a small multiple
of the host fp32 build's own distance from fp64 (plus the same absolute floor) -- 40 steps through the drop, touchdown
and stance, on the plane and on the curriculum trimesh.
"""
import numpy as np
import pytest
import torch

from test_gpu_dynamics import FLOOR, N, STEPS, _cpu_env, _state, _terrain_hook

pytestmark = pytest.mark.gpu

KERNELS = ("4", "5", "6")
PAIR_FACTOR = 10.0   # |kA - kB| <= PAIR_FACTOR * |cpu32 - fp64| + FLOOR


@pytest.mark.parametrize("mesh", ["plane", "trimesh"])
def test_step_kernels_agree_one_step(mesh, monkeypatch):
    from ti5_isaacgym_amd import make_t1_env
    envs = {}
    for k in KERNELS:   # the kernel is read when an env is created
        monkeypatch.setenv("T1ENV_DYN_KERNEL", k)
        envs[k] = make_t1_env(num_envs=N, mesh_type=mesh, seed=5, device="cuda:0",
                              cfg_hook=_terrain_hook if mesh != "plane" else None)
    env0 = envs[KERNELS[0]]
    c64, c32 = _cpu_env(env0, True), _cpu_env(env0, False)
    for e in envs.values():
        e.reset()
    c64.reset()
    c32.reset()
    rng = np.random.default_rng(11)
    worst = {}
    for t in range(STEPS):
        a = (0.5 * rng.standard_normal((N, 12))).astype(np.float32)
        root, dof = c64.o.root.copy(), c64.o.dof.copy()
        for e in envs.values():
            e.root_states.copy_(torch.from_numpy(root))
            e.dof_state.copy_(torch.from_numpy(dof.reshape(N * 12, 2)))
            e.contact_vimp.copy_(torch.from_numpy(c64.vimp))
        c32.o.root[:] = root
        c32.o.dof[:] = dof
        c32.vimp[:] = c64.vimp
        at = torch.from_numpy(a).to("cuda:0")
        for e in envs.values():
            e.step(at)
        c64.step(a)
        c32.step(a)
        r64, r32 = _state(c64.o.root, c64.o.dof), _state(c32.o.root, c32.o.dof)
        g = {k: _state(e.root_states.cpu().numpy(), e.dof_state.view(N, 12, 2).cpu().numpy()) for k, e in envs.items()}
        # rows whose reset differs between any two of the runs are not physics (the post-reset state is a redraw)
        rs = [e.reset_buf.cpu().numpy().astype(bool) for e in envs.values()] + [c64.o.reset_buf.astype(bool)]
        same = np.all([r == rs[0] for r in rs], axis=0)
        for q in r64:
            e32 = float(np.abs(r32[q] - r64[q])[same].max())
            for i, ka in enumerate(KERNELS):
                for kb in KERNELS[i + 1:]:
                    gap = float(np.abs(g[ka][q] - g[kb][q])[same].max())
                    key = (ka, kb, q)
                    worst[key] = max(worst.get(key, 0.0), gap / (e32 + FLOOR[q]))
                    assert gap <= PAIR_FACTOR * e32 + FLOOR[q], \
                        f"[{mesh} step {t}] k_dyn{ka} vs k_dyn{kb} {q}: gap {gap:.3g}, |cpu32-fp64| {e32:.3g}"
    print(mesh, {f"{a}-{b} {q}": f"{v:.2f}" for (a, b, q), v in sorted(worst.items())})
