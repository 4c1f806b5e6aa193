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


# ---------------------------------------------------------------------------------------------------------------
# One implicit substep WITH contact, written independently of the product's assembly (TEST INFRASTRUCTURE).
#
# The product (t1_dynamics.h) folds its contact and joint-limit terms into a tree-sparse LTDL; this restates the
# same discrete law densely from plain kinematics:
#   * point Jacobians J_x (velocity of a body-fixed point w.r.t. u = [omega, v_O, qd]) by central differences of
#     forward kinematics -- no spatial algebra shared with the product;
#   * terrain: the plane z = 0 (normal +z), contact candidates = the model's contact points below it;
#   * self-collision: the legs' capsules (utils/urdf.py self_capsules: left shank, left foot, right shank, right foot);
#     per overlapping pair one contact at the middle of the overlap along the segments' closest points (found here by
#     enumerating the 2-parameter problem's interior stationary point and its four edges; near-parallel segments,
#     sin^2 < 1e-3, by the overlap-midpoint rule the product documents); pairs {l, r} x {shank, foot} across the legs
#     and shank-foot within a leg; each body gets the force at that point, the other body the reaction;
#   * the law per contact: normal spring k pen, damper d while approaching (implicit: cn = dt k + d) and,
#     with a restitution target v_tgt, while separating slower than it (cn = d, f_n += d v_tgt), regularised Coulomb friction ct = mu fn_est / max(|v_t|, v_s) as an implicit tangential
#     damper: C = cn n n^T + ct (I - n n^T), f = (k pen - cn v_n + d v_tgt) n - ct v_t;
#   * restitution: each terrain-contact body (shanks, feet, the base box's two halves) keeps the approach speed v_imp
#     of its contact episode; v_tgt = e v_imp above the bounce threshold, else 0 (self-contacts: 0);
#   * soft joint limits k_l, d_l (implicit damper when moving further out);
#   * implicit Euler in the contact / limit velocities with each body's own terms implicit (a self-contact's other
#     body enters through its current velocity):
#       (M + dt sum J^T C J + dt diag(c_l)) du = dt (tau - h + sum J^T f + f_limit).
# ---------------------------------------------------------------------------------------------------------------
SELF_BODIES = (4, 6, 10, 12)


def _capsules(tab):
    """{body: (a, b, r)}: each self-collision box (tab["self_box"], link frame) as the capsule along its longest axis,
    radius the smaller cross-section half extent, ends inset by the radius (the model's definition)"""
    out = {}
    for body, box in zip(SELF_BODIES, tab["self_box"]):
        c, h = np.asarray(box[:3], float), np.asarray(box[3:], float)
        ax = int(np.argmax(h))
        r = float(np.min(np.delete(h, ax)))
        e = np.eye(3)[ax] * max(h[ax] - r, 1e-3)
        out[body] = (c - e, c + e, r)
    return out


def _closest_segments(p1, q1, p2, q2):
    """closest points of the segments p1-q1, p2-q2: min over the interior stationary point (if inside [0,1]^2) and the
    best point of each edge of the parameter square; near-parallel segments: the overlap-midpoint rule"""
    d1, d2 = q1 - p1, q2 - p2
    a, e, b = d1 @ d1, d2 @ d2, d1 @ d2
    clip = lambda x: min(max(x, 0.0), 1.0)  # noqa: E731
    if a * e - b * b < 1e-3 * a * e:
        s0, s1 = sorted(((p2 - p1) @ d1 / a, (q2 - p1) @ d1 / a))
        c1 = p1 + 0.5 * (clip(s0) + clip(s1)) * d1
        return c1, p2 + clip((c1 - p2) @ d2 / e) * d2
    cands = []
    st = np.linalg.solve(np.array([[a, -b], [-b, e]]), np.array([-(p1 - p2) @ d1, (p1 - p2) @ d2]))
    if 0 <= st[0] <= 1 and 0 <= st[1] <= 1:
        cands.append(tuple(st))
    for sv in (0.0, 1.0):
        cands.append((sv, clip((p1 + sv * d1 - p2) @ d2 / e)))
    for tv in (0.0, 1.0):
        cands.append((clip((p2 + tv * d2 - p1) @ d1 / a), tv))
    dist = [np.linalg.norm(p1 + sv * d1 - p2 - tv * d2) for sv, tv in cands]
    sv, tv = cands[int(np.argmin(dist))]
    return p1 + sv * d1, p2 + tv * d2


class ContactRobot(Robot):
    def __init__(self, tab, mass=None, inertia_scale=None, com_disp=(0, 0, 0), armature=None, solver=None,
                 limits=None):
        super().__init__(tab, mass, inertia_scale, com_disp, armature)
        self.tab = tab
        self.sv = dict(solver)
        lim = np.asarray(tab["limits"], float) if limits is None else np.asarray(limits, float)
        self.lo, self.hi = lim[:, 0], lim[:, 1]

    def _points(self, Rs, ps, b, local):
        return ps[b] + Rs[b] @ local

    def point_jacobian(self, p, R, q, b, local, eps=1e-6):
        """d x / d u of the body-fixed point `local` of body b (world position x)"""
        J = np.zeros((3, 18))
        for k in range(18):
            e = np.zeros(18)
            e[k] = 1.0
            Rp, pp, _ = self.fk(*self._move(p, R, q, e, eps))
            Rm, pm, _ = self.fk(*self._move(p, R, q, e, -eps))
            J[:, k] = (self._points(Rp, pp, b, local) - self._points(Rm, pm, b, local)) / (2 * eps)
        return J

    def contacts(self, p, R, q, u, mu_ground, e_ground, mu_self, e_self, self_collision=True):
        """[(body, local point, normal, pen, other body's point or None, mu, episode slot or None)] of the state;
        episode slots: 2 leg + (0 shank, 1 foot), 4 + leg for the base box half the point belongs to"""
        Rs, ps, _ = self.fk(p, R, q)
        out = []
        pts = np.asarray(self.tab["contact_point"], float)
        for b in range(13):
            s, n = self.tab["contact_start"][b], self.tab["contact_count"][b]
            for c in range(s, s + n):
                x = self._points(Rs, ps, b, pts[c])
                if x[2] < 0:
                    slot = 4 + (c - s) * 2 // n if b == 0 else 2 * ((b - 1) // 6) + (1 if (b - 1) % 6 == 5 else 0)
                    out.append((b, pts[c], np.array([0.0, 0.0, 1.0]), -x[2], None, mu_ground, slot))
        if self_collision:
            caps = _capsules(self.tab)
            pairs = [(4, 10), (4, 12), (6, 10), (6, 12), (4, 6), (10, 12)]
            for a, bb in pairs:
                (a0, a1, ra), (b0, b1, rb) = caps[a], caps[bb]
                ca, cb = _closest_segments(self._points(Rs, ps, a, a0), self._points(Rs, ps, a, a1),
                                           self._points(Rs, ps, bb, b0), self._points(Rs, ps, bb, b1))
                dist = np.linalg.norm(ca - cb)
                if dist >= ra + rb:
                    continue
                n = (ca - cb) / dist            # pushes a out of b
                pen = ra + rb - dist
                x = cb + (rb - 0.5 * pen) * n   # the middle of the overlap
                la, lb = Rs[a].T @ (x - ps[a]), Rs[bb].T @ (x - ps[bb])
                out.append((a, la, n, pen, (bb, lb), mu_self, None))
                out.append((bb, lb, -n, pen, (a, la), mu_self, None))
        return out

    def step(self, p, quat, w, v, q, qd, tau, dt, mu_ground, e_ground, mu_self, e_self, f_base=None,
             self_collision=True, g=9.81, vimp=None):
        """(du over one substep (u = [omega, v_O, qd]), the restitution episodes after it)"""
        sv = self.sv
        k, d, vs = sv["k_contact"], sv["d_contact"], sv["friction_vs"]
        R = quat_to_R(quat)
        u = np.concatenate([w, v, qd])
        acc, Mm = self.accel(p, quat, w, v, q, qd, np.zeros(12), g=g, f_base=f_base)
        # accel() gives the classical acceleration of the (moving) base origin; the substep's du is taken about the point
        # O fixed where the base origin is at the substep's start: the spatial acceleration a_O - w x v_O
        acc = acc.copy()
        acc[3:6] -= np.cross(w, v)
        f0 = Mm @ acc                        # the generalized force without tau: J_base^T f_base - h(q, u)
        A = Mm.copy()
        rhs = dt * (np.concatenate([np.zeros(6), tau]) + f0)
        vimp = np.zeros(6) if vimp is None else np.asarray(vimp, float)
        amax = np.full(6, -1.0)
        for b, local, n, pen, other, mu, slot in self.contacts(p, R, q, u, mu_ground, e_ground, mu_self, e_self,
                                                               self_collision):
            J = self.point_jacobian(p, R, q, b, local)
            vp = J @ u
            if other is not None:
                vp = vp - self.point_jacobian(p, R, q, other[0], other[1]) @ u
            vn = n @ vp
            vt = vp - vn * n
            vtg = 0.0
            if slot is not None:
                vtg = e_ground * vimp[slot] if vimp[slot] > sv["bounce_threshold"] else 0.0
                amax[slot] = max(amax[slot], max(-vn, 0.0))
            approach, below = vn < 0, 0 <= vn < vtg
            cn = dt * k + d if approach else (d if below else 0.0)
            fn_est = k * pen + (-d * vn if approach else (d * (vtg - vn) if below else 0.0))
            ct = mu * fn_est / max(np.linalg.norm(vt), vs)
            f = (k * pen - cn * vn + (d * vtg if below else 0.0)) * n - ct * vt
            C = cn * np.outer(n, n) + ct * (np.eye(3) - np.outer(n, n))
            A += dt * J.T @ C @ J
            rhs += dt * J.T @ f
        for j in range(12):
            kl, dl = sv["k_limit"], sv["d_limit"]
            if q[j] < self.lo[j]:
                cl = dt * kl + dl if qd[j] < 0 else 0.0
                A[6 + j, 6 + j] += dt * cl
                rhs[6 + j] += dt * (kl * (self.lo[j] - q[j]) - cl * qd[j])
            elif q[j] > self.hi[j]:
                cl = dt * kl + dl if qd[j] > 0 else 0.0
                A[6 + j, 6 + j] += dt * cl
                rhs[6 + j] += dt * (kl * (self.hi[j] - q[j]) - cl * qd[j])
        new = np.where(amax < 0, 0.0, np.where(vimp > 0, vimp, np.maximum(amax, 1e-6)))
        return np.linalg.solve(A, rhs), new   # du = change of [omega, v_O (spatial, about O), qd]; episodes
