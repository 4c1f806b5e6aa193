"""Physics checks on the host (no GPU): the product dynamics header compiled with g++ in fp64
(oracle/_build/libt1dyn_cpu.so) against an independent formulation and physical invariants.

PhysX is unavailable, so physics parity with the reference is UNPINNED; these tests pin the equations of
motion themselves (see oracle/dynamics_ref.py)."""
import ctypes as C

import numpy as np
import pytest

from oracle import build_cpu
from oracle.dynamics_ref import Robot


@pytest.fixture(scope="module")
def dyn():
    lib = C.CDLL(build_cpu.build())
    return lib


@pytest.fixture(scope="module")
def model():
    from ti5_isaacgym_amd import _lib
    from ti5_isaacgym_amd.envs.t1_env import SOLVER
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
    m.ground_friction = 0.6
    from ti5_isaacgym_amd.envs.t1_env import set_self_collision
    set_self_collision(m, tab, enabled=True, bounce_threshold=0.5)
    return m, tab


def rand_state(rng):
    q = np.array([0, 0, -0.3, 0.6, -0.3, 0] * 2) + rng.uniform(-0.15, 0.15, 12)
    q = np.clip(q, [-0.5, -0.17, -0.78, 0.01, -1.9, -2.9] * 2, [0.5, 0.17, 0.78, 2.0, 1.9, 2.9] * 2)
    quat = rng.normal(size=4)
    quat /= np.linalg.norm(quat)
    return dict(p=np.array([0.3, -0.2, 5.0]), quat=quat, w=rng.normal(0, 1.0, 3), v=rng.normal(0, 1.0, 3), q=q,
                qd=rng.normal(0, 2.0, 12), tau=rng.normal(0, 20.0, 12))


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_accelerations_match_independent_formulation(dyn, model, seed):
    m, tab = model
    rng = np.random.default_rng(seed)
    s = rand_state(rng)
    mass = np.array(tab["mass"]) * rng.uniform(0.9, 1.1, 13)
    isc = mass / np.array(tab["mass"])
    com = rng.uniform(-0.05, 0.05, 3)
    arm = rng.uniform(0.01, 3.0, 12)
    st = np.concatenate([s["p"], s["quat"], s["w"], s["v"], s["q"], s["qd"]]).astype(np.float64)
    out = np.zeros(18)
    dp = lambda a: np.ascontiguousarray(a, np.float64).ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
    keep = [np.ascontiguousarray(x, np.float64) for x in (mass, isc, com, arm, st, s["tau"])]
    rc = dyn.t1dyn_accel(C.byref(m), *[k.ctypes.data_as(C.POINTER(C.c_double)) for k in keep], dp(out) if False else
                         out.ctypes.data_as(C.POINTER(C.c_double)))
    assert rc == 0
    ref, M = Robot(tab, mass, isc, com, arm).accel(s["p"], s["quat"], s["w"], s["v"], s["q"], s["qd"], s["tau"])
    scale = np.abs(ref).max() + 1.0
    np.testing.assert_allclose(out, ref, atol=2e-5 * scale, rtol=1e-5)


# ----------------------------------------------------------------------------------------------------
# invariants on the full substep (contact + integration), fp64 host build
# ----------------------------------------------------------------------------------------------------
class Sim:
    def __init__(self, dyn, m, n=1):
        self.dyn, self.m, self.n = dyn, m, n
        self.root = np.zeros((n, 13), np.float32)
        self.root[:, 6] = 1.0
        self.dof = np.zeros((n, 24), np.float32)
        self.bm = np.full(n, m.mass[0], np.float32)
        self.ls = np.ones((n, 12), np.float32)
        self.cd = np.zeros((n, 3), np.float32)
        self.arm = np.full((n, 12), 0.1, np.float32)
        self.fr = np.full(n, 0.8, np.float32)
        self.rst = np.zeros(n, np.float32)
        self.vimp = np.zeros((n, 6), np.float32)
        self.rigid = np.zeros((n, 13, 13), np.float32)
        self.contact = np.zeros((n, 13, 3), np.float32)
        self.hf = np.zeros((2, 2), np.int16)

    def step(self, tau, nsub=1, dt=0.001):
        fp = C.POINTER(C.c_float)
        tau = np.ascontiguousarray(tau, np.float32).reshape(self.n, 12)
        rc = self.dyn.t1dyn_substeps(C.byref(self.m), self.n, 1, self.root.ctypes.data_as(fp), self.dof.ctypes.data_as(fp),
                                     tau.ctypes.data_as(fp), self.bm.ctypes.data_as(fp), self.ls.ctypes.data_as(fp),
                                     self.cd.ctypes.data_as(fp), self.arm.ctypes.data_as(fp), self.fr.ctypes.data_as(fp),
                                     self.rst.ctypes.data_as(fp), self.vimp.ctypes.data_as(fp), None,
                                     C.c_float(dt), nsub, self.hf.ctypes.data_as(C.POINTER(C.c_int16)), 2, 2,
                                     C.c_float(0.1), C.c_float(0.005), C.c_float(0.0), 0,
                                     self.rigid.ctypes.data_as(fp), self.contact.ctypes.data_as(fp))
        assert rc == 0

    def momentum(self, masses):
        return (masses[None, :, None] * self.rigid[:, :, 7:10]).sum(1)


def test_free_fall_momentum(dyn, model):
    """Airborne, zero torques: linear momentum changes at exactly M g; joints keep their initial speeds' energy."""
    m, tab = model
    s = Sim(dyn, m)
    s.root[0, 2] = 50.0
    rng = np.random.default_rng(0)
    s.dof[0, 0::2] = [0, 0, -0.3, 0.6, -0.3, 0] * 2
    s.dof[0, 1::2] = rng.normal(0, 1.0, 12)
    s.root[0, 10:13] = rng.normal(0, 0.5, 3)
    masses = np.array(tab["mass"], np.float32)
    s.step(np.zeros(12), nsub=1)
    p0 = s.momentum(masses)[0].astype(np.float64)
    s.step(np.zeros(12), nsub=100)
    p1 = s.momentum(masses)[0].astype(np.float64)
    expect = p0 + np.array([0, 0, -9.81]) * masses.sum() * 0.1
    np.testing.assert_allclose(p1, expect, atol=2e-3 * masses.sum())


def test_energy_conserved_without_gravity(dyn, model):
    m, tab = model
    g0 = m.gravity
    m.gravity = 0.0
    try:
        s = Sim(dyn, m)
        s.root[0, 2] = 50.0
        rng = np.random.default_rng(1)
        s.dof[0, 0::2] = [0, 0, -0.3, 0.6, -0.3, 0] * 2
        s.dof[0, 1::2] = rng.normal(0, 1.0, 12)
        s.arm[:] = 0.0
        masses = np.array(tab["mass"])
        I_body = [np.array([[a, d, e], [d, b, f], [e, f, c]]) for a, b, c, d, e, f in tab["inertia"]]

        def energy():
            s.step(np.zeros(12), nsub=0)
            E = 0.0
            from oracle.dynamics_ref import quat_to_R
            for b in range(13):
                v = s.rigid[0, b, 7:10].astype(float)
                w = s.rigid[0, b, 10:13].astype(float)
                R = quat_to_R(s.rigid[0, b, 3:7].astype(float))
                E += 0.5 * masses[b] * v @ v + 0.5 * w @ (R @ I_body[b] @ R.T) @ w
            return E
        e0 = energy()
        s.step(np.zeros(12), nsub=200)
        e1 = energy()
        assert abs(e1 - e0) / e0 < 0.02, (e0, e1)
    finally:
        m.gravity = g0


def test_stance_supports_weight_and_limits(dyn, model):
    """Stiff PD stance on the plane: feet carry the weight (Newton), joints stay within limits (+ small
    compliant overshoot), nothing penetrates more than a few mm."""
    m, tab = model
    s = Sim(dyn, m, n=1)
    q0 = np.array([0, 0, -0.3, 0.6, -0.3, 0] * 2, np.float32)
    s.root[0, 2] = 0.945
    s.dof[0, 0::2] = q0
    kp, kd = 800.0, 40.0
    for _ in range(300):
        q, qd = s.dof[0, 0::2], s.dof[0, 1::2]
        s.step(kp * (q0 - q) - kd * qd, nsub=1)
    total_mass = np.array(tab["mass"]).sum()
    fz = s.contact[0, :, 2].sum()
    assert abs(fz - total_mass * 9.81) < 0.1 * total_mass * 9.81, fz
    assert s.contact[0, 0].sum() == 0.0
    lo = np.array([m.q_lower[j] for j in range(12)])
    hi = np.array([m.q_upper[j] for j in range(12)])
    assert np.all(s.dof[0, 0::2] > lo - 0.02) and np.all(s.dof[0, 0::2] < hi + 0.02)
    assert s.rigid[0, 6, 2] > 0.0 and s.rigid[0, 12, 2] > 0.0


def test_joint_limit_holds_against_torque(dyn, model):
    m, tab = model
    s = Sim(dyn, m)
    s.root[0, 2] = 50.0
    s.dof[0, 0::2] = [0, 0, -0.3, 0.6, -0.3, 0] * 2
    tau = np.zeros(12)
    tau[3] = -150.0   # drive the left knee below its 0 rad lower limit
    for _ in range(300):
        s.step(tau, nsub=1)
    assert s.dof[0, 6] > -0.02, s.dof[0, 6]


def _run_flags(dyn, m, flags, root, dof, tau, hf, mesh, nsub):
    """t1dyn_substeps on copies of (root, dof); returns (root, dof, rigid, contact)."""
    fp = C.POINTER(C.c_float)
    n = root.shape[0]
    root, dof = root.copy(), dof.copy()
    bm = np.full(n, m.mass[0], np.float32)
    rng = np.random.default_rng(7)
    ls = rng.uniform(0.9, 1.1, (n, 12)).astype(np.float32)
    cd = rng.uniform(-0.05, 0.05, (n, 3)).astype(np.float32)
    arm = rng.uniform(0.05, 0.5, (n, 12)).astype(np.float32)
    fr = rng.uniform(0.2, 1.3, n).astype(np.float32)
    rst = rng.uniform(0.0, 0.4, n).astype(np.float32)
    rigid = np.zeros((n, 13, 13), np.float32)
    contact = np.zeros((n, 13, 3), np.float32)
    tau = np.ascontiguousarray(tau, np.float32)
    hf = np.ascontiguousarray(hf)
    rc = dyn.t1dyn_substeps(C.byref(m), n, flags, root.ctypes.data_as(fp), dof.ctypes.data_as(fp),
                            tau.ctypes.data_as(fp), bm.ctypes.data_as(fp), ls.ctypes.data_as(fp), cd.ctypes.data_as(fp),
                            arm.ctypes.data_as(fp), fr.ctypes.data_as(fp), rst.ctypes.data_as(fp),
                            np.zeros((n, 6), np.float32).ctypes.data_as(fp), None, C.c_float(0.001), nsub,
                            hf.ctypes.data_as(C.POINTER(C.c_int16)), hf.shape[0], hf.shape[1], C.c_float(0.1),
                            C.c_float(0.005), C.c_float(1.0), mesh, rigid.ctypes.data_as(fp), contact.ctypes.data_as(fp))
    assert rc == 0
    return root, dof, rigid, contact


@pytest.mark.parametrize("mesh", [0, 2])
def test_split_composition_matches_assembled(dyn, model, mesh):
    """k_dyn4's split composition (contact-free passes + contact fold-in, compute_delta_split), k_dyn5's four-role
    composition (bias / torque rhs from the RNEA wave, compute_delta_roles) and k_dyn6's eight-role composition (each
    terrain contact body as two halves of its points, its restitution episode from the halves' fastest approach,
    compute_delta_roles6) are the same linear system as the assembled one (compute_delta): in fp64 they agree to
    rounding, with the feet and shanks in contact on a plane and on a rough height field."""
    m, _ = model
    n = 48
    rng = np.random.default_rng(3)
    root = np.zeros((n, 13), np.float32)
    root[:, 0:2] = rng.uniform(1.5, 2.5, (n, 2))
    root[:, 2] = rng.uniform(0.90, 0.96, n)
    yaw = rng.uniform(-np.pi, np.pi, n)
    root[:, 5], root[:, 6] = np.sin(yaw / 2), np.cos(yaw / 2)
    root[:, 7:13] = rng.normal(0, 0.3, (n, 6))
    dof = np.zeros((n, 24), np.float32)
    dof[:, 0::2] = np.array([0, 0, -0.3, 0.6, -0.3, 0] * 2) + rng.uniform(-0.3, 0.3, (n, 12))
    dof[:, 1::2] = rng.normal(0, 2.0, (n, 12))
    tau = rng.normal(0, 30.0, (n, 12)).astype(np.float32)
    hf = (rng.integers(-20, 20, (40, 40)) if mesh else np.zeros((2, 2))).astype(np.int16)
    a = _run_flags(dyn, m, 1, root, dof, tau, hf, mesh, 20)
    assert np.abs(a[3]).sum() > 0, "no contact exercised"
    # flags 3: k_dyn4's split composition; 5: k_dyn5's four-role composition (compute_delta_roles, t1_dyn5.h); 9:
    # k_dyn6's eight-role composition (compute_delta_roles6)
    for flags in (3, 5, 9):
        b = _run_flags(dyn, m, flags, root, dof, tau, hf, mesh, 20)
        for x, y, name in zip(a, b, ["root", "dof", "rigid", "contact"]):
            scale = np.abs(x).max() + 1.0
            np.testing.assert_allclose(y, x, rtol=1e-6, atol=1e-6 * scale, err_msg=f"flags {flags}: {name}")


def test_host_dynamics_under_sanitizers(model, tmp_path):
    """The dynamics header's host build (assembled and split compositions, fp32 and fp64, contact on a rough
    height field) runs clean under AddressSanitizer + UndefinedBehaviorSanitizer (sanitizers
    on host code)."""
    import os
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    m, _ = model
    blob = tmp_path / "model.bin"
    blob.write_bytes(bytes(m))
    exe = tmp_path / "asan_dyn"
    here = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fopenmp", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-o", str(exe),
                    os.path.join(here, "asan_main.cpp")], check=True)
    # verify_asan_link_order=0: the process environment may preload other libraries ahead of the ASan runtime
    env = dict(os.environ, OMP_NUM_THREADS="2", ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0")
    r = subprocess.run([str(exe), str(blob)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "ok", (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
