"""Independent fp64 equations of motion for the collapsed T1 articulation (TEST INFRASTRUCTURE).

PhysX (the reference's physics) cannot run anywhere here, so the HIP dynamics is pinned against physics
itself: this module derives the floating-base equations of motion with a formulation that shares nothing
with the product's CRBA/RNEA/LTDL code -- Kane's projected Newton-Euler equations

    sum_b  Jv_b^T (m_b a_b - m_b g) + Jw_b^T (I_b alpha_b + w_b x I_b w_b) = [0, 0, tau]

with partial-velocity Jacobians Jv_b, Jw_b of every body's COM velocity / angular velocity w.r.t. the
generalized speeds u = [omega_base (world), v_base_origin (world), qd], obtained by central finite
differences of plain homogeneous-transform forward kinematics, and the velocity-product terms J_dot u by
differentiating J along the motion.  Armature adds to the joint diagonal (PhysX joint-space armature).
"""
import numpy as np


def _rot(axis, a):
    c, s = np.cos(a), np.sin(a)
    x, y, z = axis
    C = 1 - c
    return np.array([[c + x * x * C, x * y * C - z * s, x * z * C + y * s],
                     [y * x * C + z * s, c + y * y * C, y * z * C - x * s],
                     [z * x * C - y * s, z * y * C + x * s, c + z * z * C]])


def quat_to_R(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


class Robot:
    def __init__(self, tab, mass=None, inertia_scale=None, com_disp=(0, 0, 0), armature=None):
        self.parent = tab["parent"]
        self.off = np.array(tab["joint_offset"])
        self.axis = np.array(tab["joint_axis"], dtype=float)
        self.mass = np.array(tab["mass"] if mass is None else mass, dtype=float)
        self.com = np.array(tab["com"], dtype=float)
        self.com[0] += np.asarray(com_disp, float)
        sc = np.ones(13) if inertia_scale is None else np.asarray(inertia_scale, float)
        self.I = []
        for b, (xx, yy, zz, xy, xz, yz) in enumerate(tab["inertia"]):
            self.I.append(sc[b] * np.array([[xx, xy, xz], [xy, yy, yz], [xz, yz, zz]]))
        self.arm = np.zeros(12) if armature is None else np.asarray(armature, float)

    def fk(self, p, R, q):
        Rs, ps = [R], [p]
        for b in range(1, 13):
            pr = self.parent[b]
            ps.append(ps[pr] + Rs[pr] @ self.off[b])
            Rs.append(Rs[pr] @ _rot(self.axis[b], q[b - 1]))
        coms = [ps[b] + Rs[b] @ self.com[b] for b in range(13)]
        return Rs, ps, coms

    @staticmethod
    def _move(p, R, q, u, eps):
        """configuration after moving for time eps with generalized speeds u (first order in eps)."""
        w, v, qd = u[0:3], u[3:6], u[6:18]
        n = np.linalg.norm(w)
        Rw = _rot(w / n, n * eps) if n > 0 else np.eye(3)
        return p + eps * v, Rw @ R, q + eps * qd

    def jacobians(self, p, R, q, eps=1e-6):
        Jv = np.zeros((13, 3, 18))
        Jw = np.zeros((13, 3, 18))
        for k in range(18):
            e = np.zeros(18)
            e[k] = 1.0
            Rp, _, cp = self.fk(*self._move(p, R, q, e, eps))
            Rm, _, cm = self.fk(*self._move(p, R, q, e, -eps))
            for b in range(13):
                Jv[b, :, k] = (cp[b] - cm[b]) / (2 * eps)
                W = (Rp[b] - Rm[b]) @ Rp[b].T / (2 * eps)   # skew(w) to first order
                Jw[b, :, k] = [W[2, 1], W[0, 2], W[1, 0]]
        return Jv, Jw

    def accel(self, p, quat, w, v, q, qd, tau, g=9.81, eps=1e-5, f_base=None):
        """generalized accelerations; f_base: an external world-frame force on the base body at its COM (Isaac Gym
        apply_rigid_body_force_tensors without positions), entering as Jv_base^T f."""
        R = quat_to_R(quat)
        u = np.concatenate([w, v, qd])
        Jv, Jw = self.jacobians(p, R, q)
        Jvp, Jwp = self.jacobians(*self._move(p, R, q, u, eps))
        Jvm, Jwm = self.jacobians(*self._move(p, R, q, u, -eps))
        Rs, _, _ = self.fk(p, R, q)
        M = np.zeros((18, 18))
        h = np.zeros(18)
        grav = np.array([0, 0, -g])
        for b in range(13):
            Ib = Rs[b] @ self.I[b] @ Rs[b].T
            wb = Jw[b] @ u
            Jvd_u = (Jvp[b] - Jvm[b]) @ u / (2 * eps)
            Jwd_u = (Jwp[b] - Jwm[b]) @ u / (2 * eps)
            M += self.mass[b] * Jv[b].T @ Jv[b] + Jw[b].T @ Ib @ Jw[b]
            h += Jv[b].T @ (self.mass[b] * (Jvd_u - grav)) + Jw[b].T @ (Ib @ Jwd_u + np.cross(wb, Ib @ wb))
        M[6:, 6:] += np.diag(self.arm)
        f = np.concatenate([np.zeros(6), tau])
        if f_base is not None:
            f = f + Jv[0].T @ np.asarray(f_base, float)
        return np.linalg.solve(M, f - h), M
