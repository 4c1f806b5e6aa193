"""The GPU solver (k_dyn4, fp32) IN CONTACT against an independent dense formulation -- needs the MI355X.

tests/test_gpu_dynamics_kane.py checks one airborne substep against Kane's equations; tests/test_dynamics_contact.py
checks the host fp64 build of the same header in contact against oracle/dynamics_ref.py ContactRobot (point Jacobians
by finite differences of plain forward kinematics, the contact law restated per point, one dense implicit solve).
Here the product kernel itself is the thing checked: robots on the plane with their feet (some shanks) below the
surface, legs pressed into each other (self-collision across the legs and shank-foot within a leg), joints past their
limits, and impacts faster than the bounce threshold with restitution episodes under way (contact_vimp), one substep
of k_dyn4 from its substep log (the state after substep 0 and the PD torques of substep 0), with each env's own
randomized masses, COM, armature, friction and restitution.  The kernel's velocity change is recovered from the
logged root / dof rows as in the Kane test.

Tolerance: |du_gpu - du_ref| <= 1e-4 (1 + |du_ref|_max) per env (fp32 against fp64; the host fp64 build meets 1e-5).
"""
import numpy as np
import pytest
import torch

from oracle.dynamics_ref import ContactRobot, quat_to_R

pytestmark = pytest.mark.gpu

PER, KINDS = 16, ("stance", "self", "limits", "impact")


def _skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


def test_one_substep_in_contact_matches_independent_formulation(dyn_solver):
    from test_dynamics_contact import _place_on_ground, scenario
    from ti5_isaacgym_amd import make_t1_env
    from ti5_isaacgym_amd.envs.t1_env import SOLVER
    from ti5_isaacgym_amd.utils.urdf import load_model

    n = PER * len(KINDS)

    def hook(cfg):
        cfg.domain_rand.push_robots = False

    env = make_t1_env(num_envs=n, mesh_type="plane", seed=13, device="cuda:0", cfg_hook=hook)
    tab = load_model()
    env.set_substep_log(True)
    env.reset()
    rob0 = ContactRobot(tab, solver={})
    roots, dofs, vimps = [], [], []
    for i, kind in enumerate(KINDS):
        rng = np.random.default_rng(100 + i)
        root, dof = scenario(kind, PER, rng, tab)
        _place_on_ground(rob0, root, dof, rng, depth=(0.001, 0.004) if kind != "self" else (-0.05, -0.02))
        vimp = np.zeros((PER, 6))
        if kind == "impact":
            root[:, 9] = -rng.uniform(0.8, 1.5, PER)
            vimp = np.where(rng.uniform(size=(PER, 6)) < 0.6, rng.uniform(0.6, 2.0, (PER, 6)), 0.0)
        roots.append(root)
        dofs.append(dof)
        vimps.append(vimp)
    root = np.concatenate(roots)
    dof = np.concatenate(dofs)
    vimp = np.concatenate(vimps).astype(np.float32)
    root[:, 0:2] += env.env_origins[:, 0:2].cpu().numpy()
    env.root_states.copy_(torch.from_numpy(root.astype(np.float32)))
    env.dof_state.copy_(torch.from_numpy(dof.reshape(n * 12, 2).astype(np.float32)))
    env.contact_vimp.copy_(torch.from_numpy(vimp))
    env.applied_force.zero_()
    rng = np.random.default_rng(7)
    env.step(torch.from_numpy(rng.normal(0, 0.5, (n, 12)).astype(np.float32)).to("cuda:0"))
    lg = {k: v.cpu().numpy().astype(np.float64) for k, v in env.substep_log.items()}
    env.set_substep_log(False)

    dt = float(env.sim_params.dt)
    m = env._model
    solver = dict(SOLVER, bounce_threshold=float(m.bounce_threshold))
    lim = np.array([[m.q_lower[j], m.q_upper[j]] for j in range(12)], float)
    base_mass = env.body_mass.cpu().numpy().reshape(n).astype(np.float64)
    link_scale = env.link_mass_scale.cpu().numpy().astype(np.float64)
    com_disp = env.com_displacements.cpu().numpy().astype(np.float64)
    arm = env.joint_armatures.cpu().numpy().astype(np.float64)
    fr = env.env_frictions.cpu().numpy().reshape(n).astype(np.float64)
    rst = env.restitution_coeffs.cpu().numpy().reshape(n).astype(np.float64)
    mass0 = np.asarray(tab["mass"], float)
    com_base = np.asarray(tab["com"], float)[0]
    r0 = root.astype(np.float32).astype(np.float64)
    d0 = dof.astype(np.float32).astype(np.float64)
    worst, contacts = {}, {}
    for i in range(n):
        kind = KINDS[i // PER]
        mass = mass0.copy()
        mass[0] = base_mass[i]
        mass[1:] = mass0[1:] * link_scale[i]
        isc = np.concatenate([[base_mass[i] / mass0[0]], link_scale[i]])
        rob = ContactRobot(tab, mass, isc, com_disp[i], arm[i], solver=solver, limits=lim)
        R0, w0 = quat_to_R(r0[i, 3:7]), r0[i, 10:13]
        vo0 = r0[i, 7:10] - np.cross(w0, R0 @ (com_base + com_disp[i]))
        mu_g = 0.5 * (fr[i] + float(m.ground_friction))
        e_g = 0.5 * (rst[i] + float(m.ground_restitution))
        p0 = r0[i, 0:3] - np.array([env.env_origins[i, 0].item(), env.env_origins[i, 1].item(), 0.0])
        contacts[kind] = contacts.get(kind, 0) + len(rob.contacts(p0, R0, d0[i, :, 0], None, mu_g, e_g, fr[i], rst[i]))
        ref, _ = rob.step(p0, r0[i, 3:7], w0, vo0, d0[i, :, 0], d0[i, :, 1], lg["torque"][0, i], dt, mu_g, e_g, fr[i],
                          rst[i], vimp=vimp[i].astype(np.float64))
        r1 = lg["root"][0, i]
        R1, w1 = quat_to_R(r1[3:7] / np.linalg.norm(r1[3:7])), r1[10:13]
        vb1 = r1[7:10] - np.cross(w1, R1 @ (com_base + com_disp[i]))
        vo1 = np.linalg.solve(np.eye(3) + dt * _skew(w1), vb1)
        du = np.concatenate([w1 - w0, vo1 - vo0, lg["dof"][0, i, :, 1] - d0[i, :, 1]])
        scale = np.abs(ref).max() + 1.0
        err = np.abs(du - ref).max()
        worst[kind] = max(worst.get(kind, 0.0), err / scale)
        assert err <= 1e-4 * scale, f"{kind} env {i}: |gpu - ref| {err:.3g} (scale {scale:.3g})\n{du}\n{ref}"
    assert all(contacts[k] > 0 for k in KINDS), contacts
    print("worst |gpu - ref| / (1 + |ref|max):", {k: f"{v:.2e}" for k, v in worst.items()}, "contacts:", contacts)
