"""The solver's contact, self-collision, restitution and joint-limit terms against an INDEPENDENT dense formulation
(oracle/dynamics_ref.py ContactRobot: point Jacobians by finite differences of plain forward kinematics, the contact
law restated per point, one dense implicit solve) -- host build of the product header in fp64, no GPU.

tests/test_dynamics.py pins the contact-free equations of motion (Kane) and the split vs assembled compositions;
here one substep IN CONTACT is compared: robots on the plane with feet (and some shanks) below the surface, legs
pressed into each other (self-collision across the legs), joints past their limits, and impacts faster than the
bounce threshold (restitution), for both compositions the product has (assembled compute_delta, and the k_dyn4 split
compute_delta_split).  tests/test_gpu_dynamics_contact.py runs the same check on the MI355X kernel.

Tolerance: |du_solver - du_ref| <= 1e-5 (1 + |du_ref|_max) per env (the reference's Jacobians are central differences
with step 1e-6; fp64 otherwise).
"""
import ctypes as C

import numpy as np
import pytest

from oracle import build_cpu
from oracle.dynamics_ref import ContactRobot, quat_to_R

DT = 0.001


def _skew(w):
    return np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])


@pytest.fixture(scope="module")
def setup():
    return make_setup()


def make_setup():
    from ti5_isaacgym_amd import _lib
    from ti5_isaacgym_amd.envs.t1_env import SOLVER, set_self_collision
    from ti5_isaacgym_amd.utils.urdf import load_model
    tab = load_model()
    m = _lib.Model()
    for b in range(13):
        for k in range(3):
            m.joint_offset[b][k], m.joint_axis[b][k], m.com[b][k] = tab["joint_offset"][b][k], tab["joint_axis"][b][k], tab["com"][b][k]
        m.parent[b], m.mass[b] = tab["parent"][b], tab["mass"][b]
        for k in range(6):
            m.inertia[b][k] = tab["inertia"][b][k]
        m.contact_start[b], m.contact_count[b] = tab["contact_start"][b], tab["contact_count"][b]
    lim = np.asarray(tab["limits"])
    for j in range(12):
        m.q_lower[j], m.q_upper[j], m.vel_limit[j], m.torque_limit[j] = lim[j, 0], lim[j, 1], lim[j, 3], lim[j, 2] * 0.85
    m.n_contact = len(tab["contact_point"])
    for c, p in enumerate(tab["contact_point"]):
        for k in range(3):
            m.contact_point[c][k] = p[k]
    for k, v in SOLVER.items():
        setattr(m, k, v)
    m.ground_friction, m.ground_restitution = 0.6, 0.0
    set_self_collision(m, tab, enabled=True, bounce_threshold=0.5)
    return C.CDLL(build_cpu.build()), m, tab


def scenario(kind, n, rng, tab):
    """robot states (root Gym rows, dof rows) for one contact scenario"""
    q0 = np.array([0, 0, -0.3, 0.6, -0.3, 0] * 2)
    root = np.zeros((n, 13))
    dof = np.zeros((n, 12, 2))
    yaw = rng.uniform(-np.pi, np.pi, n)
    root[:, 5], root[:, 6] = np.sin(yaw / 2), np.cos(yaw / 2)
    root[:, 0:2] = rng.uniform(-1, 1, (n, 2))
    q = q0 + rng.uniform(-0.1, 0.1, (n, 12))
    qd = rng.normal(0, 0.5, (n, 12))
    vel = rng.normal(0, 0.2, (n, 6))
    if kind == "self":
        # hips rolled / yawed inward: the feet (and shanks) press into each other
        q[:, 1] = rng.uniform(-0.17, -0.08, n)
        q[:, 7] = rng.uniform(0.08, 0.17, n)
        q[:, 0] = rng.uniform(-0.3, 0.3, n)
        q[:, 6] = rng.uniform(-0.3, 0.3, n)
        # every third robot mirrors its legs: the feet (and shanks) run near parallel, the capsules' overlap-midpoint
        # rule (and the fixed pair order both legs evaluate it in)
        mir = np.arange(n) % 3 == 0
        q[mir, 6] = q[mir, 0]
        q[mir, 7] = -q[mir, 1]
        q[mir, 8:12] = q[mir, 2:6]
    if kind == "limits":
        lim = np.asarray(tab["limits"])
        j = rng.integers(0, 12, n)
        side = rng.integers(0, 2, n)
        q[np.arange(n), j] = np.where(side == 0, lim[j, 0] - rng.uniform(0.001, 0.02, n), lim[j, 1] + rng.uniform(0.001, 0.02, n))
        qd[np.arange(n), j] = np.where(side == 0, -1.0, 1.0) * rng.uniform(0.1, 1.0, n)
    dof[..., 0], dof[..., 1] = q, qd
    root[:, 7:13] = vel
    return root, dof


def _place_on_ground(robot, root, dof, rng, depth=(0.001, 0.004)):
    """lower each robot so that its lowest contact point is `depth` below the plane"""
    pts = np.asarray(robot.tab["contact_point"], float)
    for i in range(root.shape[0]):
        R = quat_to_R(root[i, 3:7])
        Rs, ps, _ = robot.fk(np.zeros(3), R, dof[i, :, 0])
        zmin = min((ps[b] + Rs[b] @ pts[c])[2] for b in range(13)
                   for c in range(robot.tab["contact_start"][b], robot.tab["contact_start"][b] + robot.tab["contact_count"][b]))
        root[i, 2] = -zmin - rng.uniform(*depth)


def host_du(setup, root, dof, tau, fr, rst, flags, dt=DT, vimp=None):
    """the product header's substep (fp64 host build) -> du per env (and the restitution episodes after it)"""
    dyn, m, tab = setup
    n = root.shape[0]
    fp = C.POINTER(C.c_float)
    r = np.ascontiguousarray(root, np.float32).copy()
    d = np.ascontiguousarray(dof.reshape(n, 24), np.float32).copy()
    r0, d0 = r.astype(np.float64), d.astype(np.float64).reshape(n, 12, 2)
    bm = np.full(n, m.mass[0], np.float32)
    ls = np.ones((n, 12), np.float32)
    cd = np.zeros((n, 3), np.float32)
    arm = np.full((n, 12), 0.1, np.float32)
    f32 = lambda a: np.ascontiguousarray(a, np.float32)  # noqa: E731
    t, fr, rst = f32(tau), f32(fr), f32(rst)
    hf = np.zeros((2, 2), np.int16)
    vi = np.ascontiguousarray(np.zeros((n, 6)) if vimp is None else vimp, np.float32).copy()
    rc = dyn.t1dyn_substeps(C.byref(m), n, flags, r.ctypes.data_as(fp), d.ctypes.data_as(fp), t.ctypes.data_as(fp),
                            bm.ctypes.data_as(fp), ls.ctypes.data_as(fp), cd.ctypes.data_as(fp), arm.ctypes.data_as(fp),
                            fr.ctypes.data_as(fp), rst.ctypes.data_as(fp), vi.ctypes.data_as(fp), None, C.c_float(dt), 1,
                            hf.ctypes.data_as(C.POINTER(C.c_int16)), 2, 2, C.c_float(0.1), C.c_float(0.005),
                            C.c_float(0.0), 0, None, None)
    assert rc == 0
    com0 = np.asarray(tab["com"], float)[0]
    out = []
    r1, d1 = r.astype(np.float64), d.astype(np.float64).reshape(n, 12, 2)
    for i in range(n):
        R0, w0 = quat_to_R(r0[i, 3:7]), r0[i, 10:13]
        vo0 = r0[i, 7:10] - np.cross(w0, R0 @ com0)
        R1, w1 = quat_to_R(r1[i, 3:7] / np.linalg.norm(r1[i, 3:7])), r1[i, 10:13]
        vb1 = r1[i, 7:10] - np.cross(w1, R1 @ com0)
        vo1 = np.linalg.solve(np.eye(3) + dt * _skew(w1), vb1)
        out.append(np.concatenate([w1 - w0, vo1 - vo0, d1[i, :, 1] - d0[i, :, 1]]))
    return np.array(out), r0, d0, vi


def ref_du(setup, r0, d0, tau, fr, rst, dt=DT, count=None, vimp=None, episodes=None):
    from ti5_isaacgym_amd.envs.t1_env import SOLVER
    dyn, m, tab = setup
    com0 = np.asarray(tab["com"], float)[0]
    solver = dict(SOLVER, bounce_threshold=m.bounce_threshold)
    lim = np.array([[m.q_lower[j], m.q_upper[j]] for j in range(12)], float)
    rob = ContactRobot(tab, armature=np.full(12, np.float32(0.1)), solver=solver, limits=lim)
    out = []
    for i in range(r0.shape[0]):
        R0, w0 = quat_to_R(r0[i, 3:7]), r0[i, 10:13]
        vo0 = r0[i, 7:10] - np.cross(w0, R0 @ com0)
        mu_g, e_g = 0.5 * (float(np.float32(fr[i])) + m.ground_friction), 0.5 * (float(np.float32(rst[i])) + 0.0)
        if count is not None:
            count.append(len(rob.contacts(r0[i, 0:3], R0, d0[i, :, 0], None, mu_g, e_g, float(np.float32(fr[i])),
                                          float(np.float32(rst[i])))))
        du, ep = rob.step(r0[i, 0:3], r0[i, 3:7], w0, vo0, d0[i, :, 0], d0[i, :, 1], np.asarray(tau[i], np.float64), dt,
                          mu_g, e_g, float(np.float32(fr[i])), float(np.float32(rst[i])),
                          vimp=None if vimp is None else np.asarray(vimp[i], np.float32).astype(np.float64))
        out.append(du)
        if episodes is not None:
            episodes.append(ep)
    return np.array(out)


@pytest.mark.parametrize("kind", ["stance", "self", "limits", "impact"])
@pytest.mark.parametrize("flags", [1, 3], ids=["assembled", "split"])
def test_contact_substep_matches_independent_formulation(setup, kind, flags):
    rng = np.random.default_rng({"stance": 0, "self": 1, "limits": 2, "impact": 3}[kind])
    n = 12
    dyn, m, tab = setup
    root, dof = scenario(kind, n, rng, tab)
    rob = ContactRobot(tab, solver={})
    _place_on_ground(rob, root, dof, rng, depth=(0.001, 0.004) if kind != "self" else (-0.05, -0.02))
    vimp = None
    if kind == "impact":   # falling onto the plane faster than the bounce threshold (0.5 m/s), episodes under way
        root[:, 9] = -rng.uniform(0.8, 1.5, n)
        vimp = np.where(rng.uniform(size=(n, 6)) < 0.6, rng.uniform(0.6, 2.0, (n, 6)), 0.0).astype(np.float32)
    tau = rng.normal(0, 20, (n, 12))
    fr = rng.uniform(0.2, 1.3, n)
    rst = rng.uniform(0.0, 0.4, n)
    du, r0, d0, ep_host = host_du(setup, root, dof, tau, fr, rst, flags, vimp=vimp)
    cnt, ep_ref = [], []
    ref = ref_du(setup, r0, d0, np.asarray(tau, np.float32), fr, rst, count=cnt, vimp=vimp, episodes=ep_ref)
    assert sum(cnt) > 0, "no contact in the scenario"
    # the restitution episodes after the substep: same slots open / closed, the same impact speeds
    np.testing.assert_allclose(ep_host, np.array(ep_ref), rtol=1e-5, atol=1e-6)
    for i in range(n):
        scale = np.abs(ref[i]).max() + 1.0
        err = np.abs(du[i] - ref[i]).max()
        assert err <= 1e-5 * scale, f"{kind} env {i} ({cnt[i]} contacts): |solver - ref| {err:.3g} (scale {scale:.3g})"


def test_self_collision_scenario_has_self_contacts(setup):
    """the "self" scenario really presses the legs into each other: airborne (no terrain contact), every env has
    self-contacts"""
    dyn, m, tab = setup
    rob = ContactRobot(tab, solver={})
    rng = np.random.default_rng(1)
    root, dof = scenario("self", 12, rng, tab)
    from oracle.dynamics_ref import _capsules
    caps, parallel = _capsules(tab), 0
    for i in range(12):
        c = rob.contacts(root[i, 0:3] + np.array([0, 0, 5.0]), quat_to_R(root[i, 3:7]), dof[i, :, 0], None,
                         0.5, 0.0, 0.5, 0.0)
        assert len(c) > 0 and all(x[4] is not None for x in c), i
        Rs, ps, _ = rob.fk(root[i, 0:3], quat_to_R(root[i, 3:7]), dof[i, :, 0])
        dl, dr = (Rs[b] @ (caps[b][1] - caps[b][0]) for b in (6, 12))
        touching = any({x[0], x[4][0]} == {6, 12} for x in c)
        parallel += touching and np.linalg.norm(np.cross(dl, dr)) ** 2 < 1e-3 * (dl @ dl) * (dr @ dr)
    assert parallel > 0, "no near-parallel foot contact in the scenario"


def test_restitution_makes_impacts_bounce(setup):
    """A robot holding its stance with a PD loop hits the plane at 1.5 m/s (above the 0.5 m/s bounce threshold): with
    restitution 0.4 (0.2 combined with the ground's 0) its feet are pushed out toward 0.3 m/s while separating, so the
    robot rebounds faster than with 0; below the threshold (0.3 m/s) the two are identical.  (The compliant law has a
    rebound of its own -- the spring's stored energy -- so the exit speed is at least ~e v_imp)"""
    dyn, m, tab = setup
    from test_dynamics import Sim
    q0 = np.array([0, 0, -0.3, 0.6, -0.3, 0] * 2, np.float32)
    rob = ContactRobot(tab, solver={})

    def rebound(e, v0):
        s = Sim(dyn, m, n=1)
        s.dof[0, 0::2] = q0
        s.rst[:] = e
        r = s.root.astype(np.float64)
        d = np.stack([q0, np.zeros(12)], -1)[None]
        _place_on_ground(rob, r, d, np.random.default_rng(0), depth=(-0.002, -0.001))   # 1-2 mm above the plane
        s.root[0, 2] = r[0, 2]
        s.root[0, 9] = -v0
        vz = []
        for _ in range(120):
            q, qd = s.dof[0, 0::2], s.dof[0, 1::2]
            s.step(800.0 * (q0 - q) - 40.0 * qd, nsub=1)
            vz.append(float(s.root[0, 9]))
        return max(vz)

    fast0, fast4 = rebound(0.0, 1.5), rebound(0.4, 1.5)
    slow0, slow4 = rebound(0.0, 0.3), rebound(0.4, 0.3)
    assert fast4 > fast0 + 0.02, (fast0, fast4)
    assert abs(slow4 - slow0) < 1e-6, (slow0, slow4)
