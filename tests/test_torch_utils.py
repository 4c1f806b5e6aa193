"""a7: the restated Isaac Gym torch_utils quaternion helpers vs an independent fp64 rotation-matrix formulation.

Isaac Gym Preview 4 (third party, absent here) supplies quat_rotate_inverse / quat_rotate / quat_apply / quat_mul /
normalize on the hot path (call sites legged_robot.py:201-205, 476-478, 598-600, 1006-1013; t1_dh_stand_env.py:
550-552; utils/math.py:4-12).  Two restatements exist: the test-only stand-in the golden fixtures were generated
with (tests/golden/harness/isaacgym/torch_utils.py) and the oracle's (oracle/t1_oracle.py, which the HIP kernels are
pinned to through the fixtures).  Neither is pinned by a reference test, so both are checked here against a
formulation that shares no code with them: the xyzw unit quaternion's 3x3 rotation matrix, built in fp64,
    R = I + 2w[u]x + 2[u]x^2,   u = (x, y, z),
with quat_rotate(q, v) = R v, quat_rotate_inverse(q, v) = R^T v, quat_mul(a, b) <-> R(a) R(b), and the XYZ euler
angles of get_euler_xyz_tensor (legged_robot.py:27-53) recovered from R (roll = atan2(R21, R22), pitch = asin(-R20),
yaw = atan2(R10, R00)).  Tolerance: fp32 restatements vs fp64 truth, 8e-6 absolute on rotated N(0,1) vectors
(a few fp32 ulps of |v| <= ~4), 5e-5 rad on the euler angles away from gimbal lock.
"""
import os
import sys

import numpy as np
import pytest
import torch

from oracle.t1_oracle import euler_xyz, quat_rotate_inverse as oracle_qri

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "harness"))
from isaacgym import torch_utils as tu  # noqa: E402  (the stand-in, not Isaac Gym)


def rotmat(q):
    """fp64 rotation matrices of xyzw quaternions (normalised here)."""
    q = q / np.linalg.norm(q, axis=-1, keepdims=True)
    x, y, z, w = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    u = np.stack([x, y, z], -1)
    K = np.zeros(q.shape[:-1] + (3, 3))
    K[..., 0, 1], K[..., 0, 2], K[..., 1, 2] = -z, y, -x
    K[..., 1, 0], K[..., 2, 0], K[..., 2, 1] = z, -y, x
    eye = np.broadcast_to(np.eye(3), K.shape)
    R = eye + 2 * w[..., None, None] * K + 2 * (K @ K)
    assert np.allclose(np.einsum("...ij,...i->...j", K, u), 0)   # K u = u x u = 0
    return R


def random_quats(n, rng):
    q = rng.standard_normal((n, 4))
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    # edge cases: identity, 180-degree turns, gimbal lock (pitch = +-90 deg), w < 0 twins
    s = np.sqrt(0.5)
    edge = np.array([[0, 0, 0, 1], [1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, s, 0, s], [0, -s, 0, s],
                     [0, 0, 0, -1], [0.5, 0.5, 0.5, 0.5], [-0.5, 0.5, -0.5, 0.5]], np.float64)
    return np.concatenate([edge, q, -q[:50]])


@pytest.fixture(scope="module")
def data():
    rng = np.random.default_rng(7)
    q = random_quats(4000, rng)
    v = rng.standard_normal((q.shape[0], 3))
    return q, v, rotmat(q)


def test_quat_rotate_and_inverse(data):
    q, v, R = data
    qf, vf = q.astype(np.float32), v.astype(np.float32)
    fwd = np.einsum("nij,nj->ni", R, v)
    inv = np.einsum("nji,nj->ni", R, v)
    tq, tv = torch.from_numpy(qf), torch.from_numpy(vf)
    np.testing.assert_allclose(tu.quat_rotate(tq, tv).numpy(), fwd, atol=8e-6)
    np.testing.assert_allclose(tu.quat_rotate_inverse(tq, tv).numpy(), inv, atol=8e-6)
    np.testing.assert_allclose(tu.quat_apply(tq, tv).numpy(), fwd, atol=8e-6)
    np.testing.assert_allclose(oracle_qri(qf, vf), inv, atol=8e-6)
    # projected gravity (legged_robot.py:478): the body-frame image of -z
    g = np.tile([0.0, 0.0, -1.0], (q.shape[0], 1))
    np.testing.assert_allclose(oracle_qri(qf, g.astype(np.float32)), np.einsum("nji,nj->ni", R, g), atol=2e-6)


def test_quat_mul_and_normalize(data):
    q, _, R = data
    a, b = q[:2000], q[2000:4000]
    ab = tu.quat_mul(torch.from_numpy(a.astype(np.float32)), torch.from_numpy(b.astype(np.float32))).numpy()
    np.testing.assert_allclose(rotmat(ab.astype(np.float64)), R[:2000] @ R[2000:4000], atol=1e-5)
    x = torch.from_numpy((3.0 * q).astype(np.float32))
    np.testing.assert_allclose(tu.normalize(x).numpy(), q, atol=1e-6)
    z = torch.zeros(2, 4)
    assert torch.isfinite(tu.normalize(z)).all()   # eps clamp (torch_utils.normalize)


def test_euler_xyz_vs_rotation_matrix(data):
    q, _, R = data
    e = euler_xyz(q.astype(np.float32)).astype(np.float64)
    roll = np.arctan2(R[:, 2, 1], R[:, 2, 2])
    pitch = np.arcsin(np.clip(-R[:, 2, 0], -1, 1))
    yaw = np.arctan2(R[:, 1, 0], R[:, 0, 0])
    ref = np.stack([roll, pitch, yaw], 1)
    # away from gimbal lock the three angles are unique; at |pitch| = 90 deg only pitch is defined
    ok = np.abs(np.cos(pitch)) > 1e-3
    d = np.angle(np.exp(1j * (e - ref)))     # compare on the circle ((-pi, pi] wrap of get_euler_xyz)
    assert np.abs(d[ok]).max() < 5e-5, np.abs(d[ok]).max()
    assert np.abs(d[~ok, 1]).max() < 2e-3
    assert (e > -np.pi - 1e-6).all() and (e <= np.pi + 1e-6).all()
    # the rotation the angles describe reproduces R (R = Rz(yaw) Ry(pitch) Rx(roll))
    cr, sr, cp, sp, cy, sy = np.cos(e[:, 0]), np.sin(e[:, 0]), np.cos(e[:, 1]), np.sin(e[:, 1]), np.cos(e[:, 2]), np.sin(e[:, 2])
    Rz = np.zeros_like(R); Ry = np.zeros_like(R); Rx = np.zeros_like(R)  # noqa: E702
    Rz[:, 0, 0], Rz[:, 0, 1], Rz[:, 1, 0], Rz[:, 1, 1], Rz[:, 2, 2] = cy, -sy, sy, cy, 1
    Ry[:, 0, 0], Ry[:, 0, 2], Ry[:, 2, 0], Ry[:, 2, 2], Ry[:, 1, 1] = cp, sp, -sp, cp, 1
    Rx[:, 1, 1], Rx[:, 1, 2], Rx[:, 2, 1], Rx[:, 2, 2], Rx[:, 0, 0] = cr, -sr, sr, cr, 1
    np.testing.assert_allclose((Rz @ Ry @ Rx)[ok], R[ok], atol=1e-4)
