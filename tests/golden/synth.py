"""Deterministic synthetic physics states for parity tests (TEST INFRASTRUCTURE).

PhysX cannot run anywhere in this pipeline, so obs/reward/reset parity is pinned on *injected* physics:
the reference (via FakeGym.simulate) and our HIP path (via the injected-physics step) both consume the
states produced here.  States are plain numpy functions of (seed, env, global substep) so the fixture
only needs to store the seed.  They are chosen to straddle every threshold in the reward/termination
code (contact > 5 N, base contact > 1 N, |F| > 500 N, feet height 0.02/0.08 m, |sin| < 0.1, ...).
"""
import numpy as np

from oracle import rng as R

NB, ND = 13, 12
Q0 = np.array([0, 0, -0.3, 0.6, -0.3, 0] * 2, dtype=np.float32)


def _u(seed, env, g, slot):
    return R.uniform(seed, env, g, 7_000_000 + slot).astype(np.float64)


def _n(seed, env, g, slot):
    # Box-Muller normal from two counter draws
    u1 = np.maximum(_u(seed, env, g, 2 * slot), 1e-7)
    u2 = _u(seed, env, g, 2 * slot + 1)
    return np.sqrt(-2 * np.log(u1)) * np.cos(2 * np.pi * u2)


def _quat_from_euler(r, p, y):
    cr, sr = np.cos(r / 2), np.sin(r / 2)
    cp, sp = np.cos(p / 2), np.sin(p / 2)
    cy, sy = np.cos(y / 2), np.sin(y / 2)
    w = cr * cp * cy + sr * sp * sy
    x = sr * cp * cy - cr * sp * sy
    yy = cr * sp * cy + sr * cp * sy
    z = cr * cp * sy - sr * sp * cy
    return np.stack([x, yy, z, w], axis=-1)


def state(seed, num_envs, g, origins=None, env_offset=0):
    """Physics state after global substep ``g`` (0-based count of simulate() calls).

    ``origins`` (N,3): env origins the robots wander around (envs with e % 4 == 1 drift 5 m away so the
    terrain curriculum sees both "walked far" and "walked too little").
    Returns root (N,13), dof (N,12,2) [pos, vel], rigid (N,13,13), contact (N,13,3), all float32.
    """
    e = np.arange(num_envs, dtype=np.int64) + env_offset
    t = g * 0.001
    ph = _u(seed, e, 0, 1) * 6.28
    root = np.zeros((num_envs, 13))
    root[:, 0] = 0.3 * np.sin(t + ph) + 0.02 * _n(seed, e, g, 10)
    root[:, 1] = 0.3 * np.cos(0.7 * t + ph) + 0.02 * _n(seed, e, g, 11)
    root[:, 2] = 0.98 + 0.05 * np.sin(3 * t + ph) + 0.01 * _n(seed, e, g, 12)
    roll = 0.08 * _n(seed, e, g, 13)
    pitch = 0.08 * _n(seed, e, g, 14)
    yaw = np.pi * (2 * _u(seed, e, g // 50, 15) - 1)
    # a few envs far from upright: exercises the euler wrap / asin clamp paths
    big = (e % 7) == 3
    roll = np.where(big, 2.8 * (2 * _u(seed, e, g, 16) - 1), roll)
    pitch = np.where(big, 1.5 * (2 * _u(seed, e, g, 17) - 1), pitch)
    root[:, 3:7] = _quat_from_euler(roll, pitch, yaw)
    root[:, 7:10] = 0.4 * np.stack([_n(seed, e, g, 20 + k) for k in range(3)], axis=1)
    root[:, 10:13] = 0.6 * np.stack([_n(seed, e, g, 23 + k) for k in range(3)], axis=1)

    if origins is not None:
        root[:, 0] += origins[:, 0] + np.where((e % 4) == 1, 5.0, 0.0)
        root[:, 1] += origins[:, 1]
        root[:, 2] += origins[:, 2]
    dof = np.zeros((num_envs, ND, 2))
    for j in range(ND):
        dof[:, j, 0] = Q0[j] + 0.15 * np.sin(5 * t + ph + j) + 0.03 * _n(seed, e, g, 30 + j)
        dof[:, j, 1] = 2.0 * _n(seed, e, g, 50 + j)
    # exact zero velocities for some joints: exercises sign(0) in the Coulomb term
    dof[:, 0, 1] = np.where((e % 5) == 0, 0.0, dof[:, 0, 1])

    rigid = np.zeros((num_envs, NB, 13))
    for b in range(NB):
        rigid[:, b, 0] = root[:, 0] + 0.1 * np.sin(b + ph) + 0.01 * _n(seed, e, g, 70 + b)
        rigid[:, b, 1] = root[:, 1] + (0.12 if 1 <= b <= 6 else -0.12 if b >= 7 else 0.0) \
            + 0.08 * _n(seed, e, g // 20, 90 + b)
        rigid[:, b, 2] = root[:, 2] - 0.08 * (b if b <= 6 else b - 6) + 0.01 * _n(seed, e, g, 110 + b)
        q = _quat_from_euler(0.1 * _n(seed, e, g, 130 + b), 0.4 * _n(seed, e, g, 150 + b),
                             0.2 * _n(seed, e, g, 170 + b))
        rigid[:, b, 3:7] = q
        rigid[:, b, 7:13] = 0.7 * np.stack([_n(seed, e, g, 190 + 6 * b + k) for k in range(6)], axis=1)
    # feet: heights straddling the clearance band [0.02, 0.08]
    for side, b in enumerate((6, 12)):
        rigid[:, b, 2] = 0.05 + 0.05 * np.sin(8 * t + ph + np.pi * side) + 0.01 * _n(seed, e, g, 300 + side)

    contact = np.zeros((num_envs, NB, 3))
    for side, b in enumerate((6, 12)):
        on = np.sin(8 * t + ph + np.pi * side) < 0.2
        fz = np.where(on, 350 + 250 * _u(seed, e, g, 310 + side), 8 * _u(seed, e, g, 312 + side))
        contact[:, b, 2] = fz
        contact[:, b, 0] = 40 * _n(seed, e, g, 314 + side) * on
        contact[:, b, 1] = 40 * _n(seed, e, g, 316 + side) * on
    # knees / others: small noise so norms straddle the 0.1 N collision threshold
    for b in (1, 2, 3, 4, 5, 7, 8, 9, 10, 11):
        contact[:, b] = 0.05 * np.stack([_n(seed, e, g, 320 + 3 * b + k) for k in range(3)], axis=1)
    # base: occasional hard contact -> termination; otherwise sub-threshold noise
    hit = _u(seed, e, g // 10, 400) < 0.04
    contact[:, 0, :] = np.where(hit[:, None], 5.0, 0.3) * np.stack(
        [_n(seed, e, g, 401 + k) for k in range(3)], axis=1)
    f32 = np.float32
    return root.astype(f32), dof.astype(f32), rigid.astype(f32), contact.astype(f32)
