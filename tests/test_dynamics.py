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
