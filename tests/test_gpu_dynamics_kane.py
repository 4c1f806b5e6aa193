"""The GPU solver (k_dyn4, fp32) against an INDEPENDENT fp64 formulation of the equations of motion -- needs the MI355X.

tests/test_gpu_dynamics.py compares the kernel with the same header compiled for the host in fp64; here the
reference is oracle/dynamics_ref.py (Kane's projected Newton-Euler equations from finite-difference Jacobians of
plain forward kinematics: nothing shared with the product's CRBA / RNEA / LTDL code).  PhysX itself is absent, so
this pins the equations of motion, not PhysX parity.

Airborne robots (base 5 m up, joints inside their limits, speeds well below the velocity limits): no contact and no joint-limit term enters, so one substep of the semi-implicit integrator changes the
generalized speeds by exactly dt times the accelerations at the substep's start state.  The kernel's substep log
(t1env_set_substep_log) gives the state after substep 0 and the PD torques of substep 0; the test recovers the
kernel's velocity change from the logged root / dof rows (undoing the COM-velocity report and the base-origin
velocity update of integrate_base) and compares delta_u / dt with Kane's accelerations for the same state, torques
and per-env randomized masses, COM displacement, inertia scales and armatures.

The second case also sets a random base force in `applied_force` (the _add_ext_force force the next simulate applies,
t1_dh_stand_env.py:233-247; the kernel applies it on the step's first substep at the base COM), which enters Kane's
equations as Jv_base^T f.

Tolerance: |gpu - ref| <= 2e-4 (1 + |ref|_max) per env (the fp32 velocity change divided by dt = 1 ms; measured
worst 1.2e-5 on the MI355X, profiles/r02am_gpu_kane.log).
"""
import numpy as np
import pytest
import torch

from oracle.dynamics_ref import Robot, quat_to_R

pytestmark = pytest.mark.gpu

N = 64


def _skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


@pytest.mark.parametrize("ext_force", [False, True], ids=["no_force", "base_ext_force"])
def test_one_substep_matches_kane_equations(ext_force, dyn_solver):
    from ti5_isaacgym_amd import make_t1_env
    from ti5_isaacgym_amd.utils.urdf import load_model

    def hook(cfg):
        cfg.domain_rand.push_robots = False
        # Kane's equations here have no contact terms: self-collision off (asset.self_collisions is Isaac Gym's
        # filter, 1 = disabled), since random joint offsets of +-0.15 rad can press the feet into each other
        # (tests/test_gpu_dynamics_contact.py checks those contacts)
        cfg.asset.self_collisions = 1

    env = make_t1_env(num_envs=N, mesh_type="plane", seed=11, device="cuda:0", cfg_hook=hook)
    tab = load_model()
    env.set_substep_log(True)
    env.reset()
    rng = np.random.default_rng(7)
    lo = np.array([-0.5, -0.17, -0.78, 0.01, -1.9, -2.9] * 2)
    hi = np.array([0.5, 0.17, 0.78, 2.0, 1.9, 2.9] * 2)
    lim = np.asarray(tab["limits"])
    lo, hi = np.maximum(lo, lim[:, 0] + 0.05), np.minimum(hi, lim[:, 1] - 0.05)
    q0 = np.clip(np.array([0, 0, -0.3, 0.6, -0.3, 0] * 2) + rng.uniform(-0.15, 0.15, (N, 12)), lo, hi)
    qd0 = np.clip(rng.normal(0, 1.5, (N, 12)), -0.3 * lim[:, 3], 0.3 * lim[:, 3])
    quat = rng.normal(size=(N, 4))
    quat /= np.linalg.norm(quat, axis=1, keepdims=True)
    root = np.zeros((N, 13), np.float32)
    root[:, 0:2] = env.env_origins[:, 0:2].cpu().numpy()
    root[:, 2] = 5.0
    root[:, 3:7] = quat
    root[:, 7:10] = rng.normal(0, 0.5, (N, 3))   # COM velocity (the root-state convention)
    root[:, 10:13] = rng.normal(0, 0.8, (N, 3))
    env.root_states.copy_(torch.from_numpy(root))
    env.dof_state.copy_(torch.from_numpy(np.stack([q0, qd0], -1).reshape(N * 12, 2).astype(np.float32)))
    fb = np.zeros((N, 3))
    if ext_force:   # the t1 cfg's ranges: x U(-300, 600), y U(-400, 400), z U(-5, 5)
        fb = np.stack([rng.uniform(-300, 600, N), rng.uniform(-400, 400, N), rng.uniform(-5, 5, N)], 1)
    env.applied_force.copy_(torch.from_numpy(fb.astype(np.float32)))
    fb = fb.astype(np.float32).astype(np.float64)
    env.step(torch.from_numpy(rng.normal(0, 0.5, (N, 12)).astype(np.float32)).to("cuda:0"))
    lg = {k: v.cpu().numpy().astype(np.float64) for k, v in env.substep_log.items()}
    env.set_substep_log(False)

    dt = float(env.sim_params.dt)
    base_mass = env.body_mass.cpu().numpy().reshape(N).astype(np.float64)
    link_scale = env.link_mass_scale.cpu().numpy().astype(np.float64)
    com_disp = env.com_displacements.cpu().numpy().astype(np.float64)
    arm = env.joint_armatures.cpu().numpy().astype(np.float64)
    mass0 = np.asarray(tab["mass"], float)
    com_base = np.asarray(tab["com"], float)[0]
    r0 = root.astype(np.float64)
    q0, qd0 = q0.astype(np.float32).astype(np.float64), qd0.astype(np.float32).astype(np.float64)
    worst = 0.0
    for n in range(N):
        mass = mass0.copy()
        mass[0] = base_mass[n]
        mass[1:] = mass0[1:] * link_scale[n]
        isc = np.concatenate([[base_mass[n] / mass0[0]], link_scale[n]])
        R0, w0 = quat_to_R(r0[n, 3:7]), r0[n, 10:13]
        vo0 = r0[n, 7:10] - np.cross(w0, R0 @ (com_base + com_disp[n]))
        tau = lg["torque"][0, n]
        ref, _ = Robot(tab, mass, isc, com_disp[n], arm[n]).accel(r0[n, 0:3], r0[n, 3:7], w0, vo0, q0[n], qd0[n], tau,
                                                                  f_base=fb[n])
        ref_sp = ref.copy()
        ref_sp[3:6] = ref[3:6] - np.cross(w0, vo0)   # classical -> spatial acceleration of the base origin
        # the kernel's velocity change over substep 0 (integrate_base: vb = vO_new + dt w_new x vO_new, reported at
        # the COM)
        r1 = lg["root"][0, n]
        R1, w1 = quat_to_R(r1[3:7] / np.linalg.norm(r1[3:7])), r1[10:13]
        vb1 = r1[7:10] - np.cross(w1, R1 @ (com_base + com_disp[n]))
        vo1 = np.linalg.solve(np.eye(3) + dt * _skew(w1), vb1)
        du = np.concatenate([w1 - w0, vo1 - vo0, lg["dof"][0, n, :, 1] - qd0[n]]) / dt
        err = np.abs(du - ref_sp).max()
        scale = np.abs(ref_sp).max() + 1.0
        worst = max(worst, err / scale)
        assert err <= 2e-4 * scale, f"env {n}: |gpu - kane| {err:.3g} (scale {scale:.3g})\n{du}\n{ref_sp}"
    print(f"worst |gpu - kane| / (1 + |ref|max) over {N} envs: {worst:.2e}")
