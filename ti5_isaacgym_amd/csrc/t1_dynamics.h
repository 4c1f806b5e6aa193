// t1_dynamics.h -- floating-base articulated dynamics + compliant terrain contact for the Ti5 T1 biped.
//
// Replaces Isaac Gym Preview 4 / PhysX `gym.simulate` on the LeggedRobot.step() path
// (legged_robot.py:399-410).  PhysX is a closed binary that cannot run here, so
// physics parity is UNPINNED; DESIGN.md §physics documents the model and tests/test_dynamics*.py pin it
// against an independent fp64 formulation and physical invariants.
//
// Model (one env):
//   * generalized coords: base pose (p, quat) + 12 revolute joints; generalized velocity
//     u = [omega (3), v_o (3), qd (12)] with the base spatial velocity taken at the base origin, world axes.
//   * all spatial quantities in world-aligned axes about the point O = base origin at the start of the
//     substep (a fixed inertial frame for that substep, so plain spatial algebra applies and fp32 positions
//     stay O(1 m) whatever the terrain coordinates).
//   * bias forces by RNEA (gravity as a fictitious base acceleration), joint-space inertia by CRBA;
//     compliant contact (spring k, damper d, regularised Coulomb friction) and soft joint limits are
//     integrated implicitly: their J^T C J terms are per-body 6x6 matrices that the CRBA folds into the
//     composite inertias, so the augmented matrix keeps the kinematic-tree sparsity and one LTDL
//     factorisation per substep solves everything (no contact iterations).
//   * tree-sparse LTDL (Featherstone RBDA §6.5) over DOF order [base 0..5 | left leg | right leg]: each leg
//     is eliminated into the 6x6 base block, the base block is factored densely, legs back-substitute.
//   * semi-implicit Euler; joint speeds clamped to the URDF velocity limits like PhysX max joint velocity.
#pragma once
#include "t1_common.h"

namespace t1 {

constexpr int NB = 13, ND = 12, NLEG = 6;

// Model in the form the kernels consume (built from t1env_model at create time).
struct DynModel {
  float joint_offset[NB][3];
  int32_t axis_idx[NB];
  float axis_sign[NB];
  float mass[NB];
  float com[NB][3];
  float inertia[NB][6];  // xx yy zz xy xz yz about COM, body frame
  float q_lower[ND], q_upper[ND], vel_limit[ND], torque_limit[ND];
  float default_dof_pos[ND], p_gains[ND], d_gains[ND];
  int32_t contact_start[NB], contact_count[NB];
  float contact_point[48][3];
  float k_contact, d_contact, friction_vs, k_limit, d_limit, gravity;
  float ground_friction, ground_restitution;
  float base_init_state[13];
};

// Terrain: plane (type 0) or height field sampled like the trimesh the reference builds from it
// (type 1/2; two triangles per cell split along the (i,j)-(i+1,j+1) diagonal).
struct Terrain {
  const int16_t* h;  // (rows, cols), rows along x
  int32_t rows, cols, type;
  float hscale, vscale, border;
};

template <typename R> struct EnvParams {
  R mass[NB];
  R inertia_scale[NB];
  R com_disp[3];
  R armature[ND];
  R friction;
};

template <typename R> struct BodyState {  // per-body kinematics of one substep (world axes, about O)
  M3<R> Rot;
  V3<R> p;   // frame origin rel. O
};

template <typename R> struct Sym6 {
  // packed upper triangle of a symmetric 6x6: (0,0)(0,1)..(0,5)(1,1)..(5,5)
  R a[21];
};
T1_HD constexpr int sidx(int i, int j) {  // i <= j
  return i * 6 - (i * (i - 1)) / 2 + (j - i);
}
template <typename R> T1_HD R sget(const Sym6<R>& S, int i, int j) { return i <= j ? S.a[sidx(i, j)] : S.a[sidx(j, i)]; }
template <typename R> T1_HD void sym_zero(Sym6<R>& S) {
#pragma unroll
  for (int k = 0; k < 21; ++k) S.a[k] = R(0);
}
template <typename R> T1_HD void sym_add(Sym6<R>& S, const Sym6<R>& T) {
#pragma unroll
  for (int k = 0; k < 21; ++k) S.a[k] += T.a[k];
}
// S += c * w w^T
template <typename R> T1_HD void sym_rank1(Sym6<R>& S, R c, const R w[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    R ci = c * w[i];
#pragma unroll
    for (int j = i; j < 6; ++j) S.a[sidx(i, j)] += ci * w[j];
  }
}
template <typename R> T1_HD void sym_mul(const Sym6<R>& S, const R x[6], R y[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    R acc = R(0);
#pragma unroll
    for (int j = 0; j < 6; ++j) acc += sget(S, i, j) * x[j];
    y[i] = acc;
  }
}
// spatial inertia of a body about O in world axes from (m, com c rel O, Ic world) ; [[Io, [h]x],[[h]x^T, m]]
template <typename R> T1_HD void inertia_spatial(Sym6<R>& S, R m, V3<R> c, const R Ic[6] /*xx yy zz xy xz yz*/) {
  R cc = dot(c, c);
  // Io = Ic + m (|c|^2 I - c c^T)
  S.a[sidx(0, 0)] = Ic[0] + m * (cc - c.x * c.x);
  S.a[sidx(1, 1)] = Ic[1] + m * (cc - c.y * c.y);
  S.a[sidx(2, 2)] = Ic[2] + m * (cc - c.z * c.z);
  S.a[sidx(0, 1)] = Ic[3] - m * c.x * c.y;
  S.a[sidx(0, 2)] = Ic[4] - m * c.x * c.z;
  S.a[sidx(1, 2)] = Ic[5] - m * c.y * c.z;
  V3<R> h = m * c;
  // top-right [h]x = [[0,-hz,hy],[hz,0,-hx],[-hy,hx,0]]
  S.a[sidx(0, 3)] = R(0);  S.a[sidx(0, 4)] = -h.z; S.a[sidx(0, 5)] = h.y;
  S.a[sidx(1, 3)] = h.z;   S.a[sidx(1, 4)] = R(0); S.a[sidx(1, 5)] = -h.x;
  S.a[sidx(2, 3)] = -h.y;  S.a[sidx(2, 4)] = h.x;  S.a[sidx(2, 5)] = R(0);
  S.a[sidx(3, 3)] = m; S.a[sidx(4, 4)] = m; S.a[sidx(5, 5)] = m;
  S.a[sidx(3, 4)] = R(0); S.a[sidx(3, 5)] = R(0); S.a[sidx(4, 5)] = R(0);
}
// motion x motion: [w;v] x [w2;v2] = [w x w2 ; w x v2 + v x w2]
template <typename R> T1_HD void crm(const R a[6], const R b[6], R out[6]) {
  V3<R> w{a[0], a[1], a[2]}, v{a[3], a[4], a[5]}, w2{b[0], b[1], b[2]}, v2{b[3], b[4], b[5]};
  V3<R> o1 = cross(w, w2), o2 = cross(w, v2) + cross(v, w2);
  out[0] = o1.x; out[1] = o1.y; out[2] = o1.z; out[3] = o2.x; out[4] = o2.y; out[5] = o2.z;
}
// motion x* force: [w;v] x* [n;f] = [w x n + v x f ; w x f]
template <typename R> T1_HD void crf(const R a[6], const R b[6], R out[6]) {
  V3<R> w{a[0], a[1], a[2]}, v{a[3], a[4], a[5]}, n{b[0], b[1], b[2]}, f{b[3], b[4], b[5]};
  V3<R> o1 = cross(w, n) + cross(v, f), o2 = cross(w, f);
  out[0] = o1.x; out[1] = o1.y; out[2] = o1.z; out[3] = o2.x; out[4] = o2.y; out[5] = o2.z;
}
template <typename R> T1_HD R dot6(const R a[6], const R b[6]) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}

// ---------------------------------------------------------------------------------------------------
// terrain query: height + unit normal at world (x, y)
// ---------------------------------------------------------------------------------------------------
template <typename R> T1_HD R terrain_height(const Terrain& T, R x, R y, V3<R>& n) {
  if (T.type == 0) { n = v3<R>(0, 0, 1); return R(0); }
  R fx = (x + R(T.border)) / R(T.hscale), fy = (y + R(T.border)) / R(T.hscale);
  R ix = floor(fx), iy = floor(fy);
  int i = (int)ix, j = (int)iy;
  R u = fx - ix, v = fy - iy;
  if (i < 0) { i = 0; u = 0; }
  if (j < 0) { j = 0; v = 0; }
  if (i > T.rows - 2) { i = T.rows - 2; u = 1; }
  if (j > T.cols - 2) { j = T.cols - 2; v = 1; }
  const int16_t* r0 = T.h + (size_t)i * T.cols + j;
  R vs = R(T.vscale);
  R h00 = vs * r0[0], h01 = vs * r0[1], h10 = vs * r0[T.cols], h11 = vs * r0[T.cols + 1];
  R dhdu, dhdv, h;
  if (u >= v) {  // triangle (i,j)-(i+1,j)-(i+1,j+1)
    dhdu = h10 - h00; dhdv = h11 - h10; h = h00 + u * dhdu + v * dhdv;
  } else {       // triangle (i,j)-(i+1,j+1)-(i,j+1)
    dhdv = h01 - h00; dhdu = h11 - h01; h = h00 + v * dhdv + u * dhdu;
  }
  R gx = dhdu / R(T.hscale), gy = dhdv / R(T.hscale);
  R inv = R(1) / sqrt(R(1) + gx * gx + gy * gy);
  n = v3<R>(-gx * inv, -gy * inv, inv);
  return h;
}

// ---------------------------------------------------------------------------------------------------
// kinematics of one leg (bodies b0+1 .. b0+6), world axes about O
// ---------------------------------------------------------------------------------------------------
template <typename R>
T1_HD void leg_fk(const DynModel& M, int leg, const M3<R>& Rbase, const R q[ND], BodyState<R> B[NLEG]) {
  M3<R> Rp = Rbase;
  V3<R> pp = v3<R>(0, 0, 0);
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    const int b = 1 + 6 * leg + k;
    V3<R> off = v3<R>(M.joint_offset[b][0], M.joint_offset[b][1], M.joint_offset[b][2]);
    V3<R> p = pp + mul(Rp, off);
    R ang = R(M.axis_sign[b]) * q[6 * leg + k];
    R s = sin(ang), c = cos(ang);
    M3<R> Rb = mul_axis_rot(Rp, M.axis_idx[b], c, s);
    B[k].Rot = Rb;
    B[k].p = p;
    Rp = Rb;
    pp = p;
  }
}

template <typename R> T1_HD void motion_subspace(const DynModel& M, int b, const BodyState<R>& B, R S[6]) {
  V3<R> a = R(M.axis_sign[b]) * col(B.Rot, M.axis_idx[b]);
  V3<R> l = cross(B.p, a);
  S[0] = a.x; S[1] = a.y; S[2] = a.z; S[3] = l.x; S[4] = l.y; S[5] = l.z;
}

// world inertia about COM (xx yy zz xy xz yz) of body b
template <typename R>
T1_HD void world_inertia(const DynModel& M, int b, const M3<R>& Rb, R scale, R out[6]) {
  const float* I = M.inertia[b];
  // Ib (sym) -> R Ib R^T
  R Ib[9] = {R(I[0]), R(I[3]), R(I[4]), R(I[3]), R(I[1]), R(I[5]), R(I[4]), R(I[5]), R(I[2])};
  R T[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c)
      T[3 * r + c] = Rb.m[3 * r + 0] * Ib[0 + c] + Rb.m[3 * r + 1] * Ib[3 + c] + Rb.m[3 * r + 2] * Ib[6 + c];
  R W[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = r; c < 3; ++c)
      W[3 * r + c] = T[3 * r + 0] * Rb.m[3 * c + 0] + T[3 * r + 1] * Rb.m[3 * c + 1] + T[3 * r + 2] * Rb.m[3 * c + 2];
  out[0] = scale * W[0]; out[1] = scale * W[4]; out[2] = scale * W[8];
  out[3] = scale * W[1]; out[4] = scale * W[2]; out[5] = scale * W[5];
}

// ---------------------------------------------------------------------------------------------------
// contact of one body against the terrain: accumulates dt * J^T C J (6x6, about O) and the impulse wrench.
// Per point: normal spring k*pen (+ implicit damping when approaching), regularised Coulomb friction as an
// implicit tangential damper whose coefficient keeps |F_t| <= mu F_n (Stribeck speed friction_vs).
// ---------------------------------------------------------------------------------------------------
template <typename R>
T1_HD void body_contact(const DynModel& M, const Terrain& T, int b, const M3<R>& Rb, V3<R> pb, V3<R> base_abs,
                        const R Vb[6], R mu, R dt, Sym6<R>& K, R w[6], bool& any) {
  const int c0 = M.contact_start[b], nc = M.contact_count[b];
  const R k = R(M.k_contact), d = R(M.d_contact);
  for (int c = c0; c < c0 + nc; ++c) {
    V3<R> r = v3<R>(M.contact_point[c][0], M.contact_point[c][1], M.contact_point[c][2]);
    V3<R> x = pb + mul(Rb, r);  // rel O
    V3<R> X = x + base_abs;
    V3<R> n;
    R h = terrain_height(T, X.x, X.y, n);
    R pen = (h - X.z) * n.z;
    if (pen > R(0)) {
      any = true;
      V3<R> om{Vb[0], Vb[1], Vb[2]}, vo{Vb[3], Vb[4], Vb[5]};
      V3<R> vp = vo + cross(om, x);
      R vn = dot(n, vp);
      V3<R> vt = vp - vn * n;
      R vtn = sqrt(dot(vt, vt));
      R cn = vn < R(0) ? dt * k + d : R(0);
      R fn_est = k * pen + (vn < R(0) ? -d * vn : R(0));
      R ct = mu * fn_est / (vtn > R(M.friction_vs) ? vtn : R(M.friction_vs));
      // force at the current velocity (explicit part) f = k pen n - C vp, C = cn nn^T + ct (I - nn^T)
      V3<R> f = (k * pen - cn * vn) * n - ct * vt;
      V3<R> tq = cross(x, f);
      w[0] += dt * tq.x; w[1] += dt * tq.y; w[2] += dt * tq.z;
      w[3] += dt * f.x;  w[4] += dt * f.y;  w[5] += dt * f.z;
      // C = ct I + (cn - ct) n n^T ; J^T C J = ct * sum_e w_e w_e^T + (cn - ct) w_n w_n^T, e over world axes
      V3<R> xn = cross(x, n);
      R wn[6] = {xn.x, xn.y, xn.z, n.x, n.y, n.z};
      sym_rank1(K, dt * (cn - ct), wn);
      R ex[6] = {R(0), x.z, -x.y, R(1), R(0), R(0)};   // [x cross e_x ; e_x]
      R ey[6] = {-x.z, R(0), x.x, R(0), R(1), R(0)};
      R ez[6] = {x.y, -x.x, R(0), R(0), R(0), R(1)};
      sym_rank1(K, dt * ct, ex);
      sym_rank1(K, dt * ct, ey);
      sym_rank1(K, dt * ct, ez);
    }
  }
}

// contact force (world) a body receives at velocity Vb (used for the net-contact-force report)
template <typename R>
T1_HD V3<R> body_contact_force(const DynModel& M, const Terrain& T, int b, const M3<R>& Rb, V3<R> pb,
                               V3<R> base_abs, const R Vb[6], R mu, R dt) {
  const int c0 = M.contact_start[b], nc = M.contact_count[b];
  const R k = R(M.k_contact), d = R(M.d_contact);
  V3<R> F = v3<R>(0, 0, 0);
  for (int c = c0; c < c0 + nc; ++c) {
    V3<R> r = v3<R>(M.contact_point[c][0], M.contact_point[c][1], M.contact_point[c][2]);
    V3<R> x = pb + mul(Rb, r);
    V3<R> X = x + base_abs;
    V3<R> n;
    R h = terrain_height(T, X.x, X.y, n);
    R pen = (h - X.z) * n.z;
    if (pen > R(0)) {
      V3<R> om{Vb[0], Vb[1], Vb[2]}, vo{Vb[3], Vb[4], Vb[5]};
      V3<R> vp = vo + cross(om, x);
      R vn = dot(n, vp);
      V3<R> vt = vp - vn * n;
      R vtn = sqrt(dot(vt, vt));
      R fn = k * pen - (vn < R(0) ? d * vn : R(0));
      fn = fn > R(0) ? fn : R(0);
      R ct = mu * fn / (vtn > R(M.friction_vs) ? vtn : R(M.friction_vs));
      F = F + fn * n - ct * vt;
    }
  }
  return F;
}

// ---------------------------------------------------------------------------------------------------
// Per-env state kept in registers across the decimation loop
// ---------------------------------------------------------------------------------------------------
template <typename R> struct EnvState {
  R pos[3];   // base origin, world (absolute)
  R quat[4];  // xyzw
  R w[3];     // base angular velocity, world
  R vo[3];    // base origin velocity, world
  R q[ND], qd[ND];
};

// Leg block of the augmented system after assembly / elimination.
template <typename R> struct LegBlock {
  R L[21];      // leg-leg (sym, packed, index (i<=j) over leg dofs 0..5 from root to leaf)
  R Bl[6][6];   // base-leg coupling: Bl[r][j] = A(base r, leg j)
  R rhs[6];
};

// ---------------------------------------------------------------------------------------------------
// assemble one leg: forward kinematics/velocity/bias, per-body inertia (+contact), backward composite
// pass producing A(leg,leg), A(base,leg), rhs(leg) and the leg's contribution to the base composite.
// ---------------------------------------------------------------------------------------------------
template <typename R>
T1_HD void assemble_leg(const DynModel& M, const Terrain& T, const EnvParams<R>& P, const EnvState<R>& s, int leg,
                        const M3<R>& Rbase, V3<R> base_abs, const R V0[6], const R A0[6], const R tau[ND], R dt,
                        LegBlock<R>& out, Sym6<R>& Ac_up, R gc_up[6], bool& any_contact) {
  BodyState<R> B[NLEG];
  leg_fk(M, leg, Rbase, s.q, B);
  R S[NLEG][6], g[NLEG][6];
  Sym6<R> Abody[NLEG];
  R V[6], A[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) { V[i] = V0[i]; A[i] = A0[i]; }
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    const int b = 1 + 6 * leg + k, j = 6 * leg + k;
    motion_subspace(M, b, B[k], S[k]);
    R vj[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) vj[i] = S[k][i] * s.qd[j];
#pragma unroll
    for (int i = 0; i < 6; ++i) V[i] += vj[i];
    R cr[6];
    crm(V, vj, cr);  // V_i x (S qd)
#pragma unroll
    for (int i = 0; i < 6; ++i) A[i] += cr[i];
    // inertia about O
    R Icw[6];
    world_inertia(M, b, B[k].Rot, P.inertia_scale[b], Icw);
    V3<R> c = B[k].p + mul(B[k].Rot, v3<R>(M.com[b][0], M.com[b][1], M.com[b][2]));
    inertia_spatial(Abody[k], P.mass[b], c, Icw);
    // RNEA body force f = I a + V x* (I V)
    R IA[6], IV[6], vf[6];
    sym_mul(Abody[k], A, IA);
    sym_mul(Abody[k], V, IV);
    crf(V, IV, vf);
#pragma unroll
    for (int i = 0; i < 6; ++i) g[k][i] = dt * (IA[i] + vf[i]);
    if (M.contact_count[b] > 0) {
      R w[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
      Sym6<R> K;
      sym_zero(K);
      bool any = false;
      body_contact(M, T, b, B[k].Rot, B[k].p, base_abs, V, P.friction, dt, K, w, any);
      if (any) {
        any_contact = true;
        sym_add(Abody[k], K);
#pragma unroll
        for (int i = 0; i < 6; ++i) g[k][i] -= w[i];
      }
    }
  }
  // backward: composites from the leaf up
  Sym6<R> Ac;
  sym_zero(Ac);
  R gc[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
#pragma unroll
  for (int k = NLEG - 1; k >= 0; --k) {
    const int j = 6 * leg + k;
    sym_add(Ac, Abody[k]);
#pragma unroll
    for (int i = 0; i < 6; ++i) gc[i] += g[k][i];
    R F[6];
    sym_mul(Ac, S[k], F);
    // diagonal (+ armature + soft joint limit)
    R Ajj = dot6(S[k], F) + P.armature[j];
    R rj = dt * tau[j] - dot6(S[k], gc);
    R lo = R(M.q_lower[j]), hi = R(M.q_upper[j]);
    R qj = s.q[j], qdj = s.qd[j];
    if (qj < lo) {
      R cl = qdj < R(0) ? dt * R(M.k_limit) + R(M.d_limit) : R(0);
      Ajj += dt * cl;
      rj += dt * (R(M.k_limit) * (lo - qj) - cl * qdj);
    } else if (qj > hi) {
      R cl = qdj > R(0) ? dt * R(M.k_limit) + R(M.d_limit) : R(0);
      Ajj += dt * cl;
      rj += dt * (R(M.k_limit) * (hi - qj) - cl * qdj);
    }
    out.L[sidx(k, k)] = Ajj;
    out.rhs[k] = rj;
#pragma unroll
    for (int i = 0; i < k; ++i) out.L[sidx(i, k)] = dot6(S[i], F);
#pragma unroll
    for (int r = 0; r < 6; ++r) out.Bl[r][k] = F[r];
  }
  sym_add(Ac_up, Ac);
#pragma unroll
  for (int i = 0; i < 6; ++i) gc_up[i] += gc[i];
}

// Eliminate a leg's 6 DOF (leaf first) into the base block: Featherstone LTDL restricted to the path
// [base 0..5, leg 0..5].  On return out.L/Bl hold the unit factor L (off-diagonal) and D (diagonal), Abb and
// rhs_b hold the Schur-complement updates, and out.rhs holds the forward-substituted leg rhs.
template <typename R> T1_HD void eliminate_leg(LegBlock<R>& lb, Sym6<R>& Abb, R rhs_b[6]) {
#pragma unroll
  for (int k = NLEG - 1; k >= 0; --k) {
    const R Dk = lb.L[sidx(k, k)];
    const R inv = R(1) / Dk;
    // ancestors of leg dof k: leg dofs i < k, then base dofs 5..0
    R a_leg[NLEG], a_base[6];
#pragma unroll
    for (int i = 0; i < k; ++i) a_leg[i] = lb.L[sidx(i, k)] * inv;
#pragma unroll
    for (int r = 0; r < 6; ++r) a_base[r] = lb.Bl[r][k] * inv;
    // H_ij -= a_i * H_kj for ancestor pairs (i, j) -- every pair on the path
#pragma unroll
    for (int i = 0; i < k; ++i) {
#pragma unroll
      for (int jj = 0; jj <= i; ++jj) lb.L[sidx(jj, i)] -= a_leg[i] * lb.L[sidx(jj, k)];
#pragma unroll
      for (int r = 0; r < 6; ++r) lb.Bl[r][i] -= a_leg[i] * lb.Bl[r][k];
    }
#pragma unroll
    for (int r = 0; r < 6; ++r)
#pragma unroll
      for (int c = r; c < 6; ++c) Abb.a[sidx(r, c)] -= a_base[r] * lb.Bl[c][k];
    // forward substitution of the rhs (L^-T pass): b_i -= L_ki b_k
    const R bk = lb.rhs[k];
#pragma unroll
    for (int i = 0; i < k; ++i) lb.rhs[i] -= a_leg[i] * bk;
#pragma unroll
    for (int r = 0; r < 6; ++r) rhs_b[r] -= a_base[r] * bk;
    // store the factor
#pragma unroll
    for (int i = 0; i < k; ++i) lb.L[sidx(i, k)] = a_leg[i];
#pragma unroll
    for (int r = 0; r < 6; ++r) lb.Bl[r][k] = a_base[r];
  }
}

// dense LDL^T of the 6x6 base block with the same (leaf-first) convention and solve in place.
template <typename R> T1_HD void solve_base(Sym6<R>& A, R b[6]) {
#pragma unroll
  for (int k = 5; k >= 0; --k) {
    const R inv = R(1) / A.a[sidx(k, k)];
    R a[6];
#pragma unroll
    for (int i = 0; i < k; ++i) a[i] = A.a[sidx(i, k)] * inv;
#pragma unroll
    for (int i = 0; i < k; ++i)
#pragma unroll
      for (int jj = 0; jj <= i; ++jj) A.a[sidx(jj, i)] -= a[i] * A.a[sidx(jj, k)];
#pragma unroll
    for (int i = 0; i < k; ++i) { b[i] -= a[i] * b[k]; A.a[sidx(i, k)] = a[i]; }
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) b[k] /= A.a[sidx(k, k)];
#pragma unroll
  for (int k = 0; k < 6; ++k)
#pragma unroll
    for (int i = 0; i < k; ++i) b[k] -= A.a[sidx(i, k)] * b[i];
}

// back substitution for a leg once the base solution x_b is known: x_k = rhs_k / D_k - sum_anc L_ki x_i
template <typename R> T1_HD void backsub_leg(const LegBlock<R>& lb, const R xb[6], R x[NLEG]) {
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    R v = lb.rhs[k] / lb.L[sidx(k, k)];
#pragma unroll
    for (int r = 0; r < 6; ++r) v -= lb.Bl[r][k] * xb[r];
#pragma unroll
    for (int i = 0; i < k; ++i) v -= lb.L[sidx(i, k)] * x[i];
    x[k] = v;
  }
}

// ---------------------------------------------------------------------------------------------------
// Assemble and solve one substep: delta = change of u = [omega, v_O (spatial, about the fixed point O),
// qd] over dt, including implicit contact / joint-limit terms.  tau: joint torques; ext_f: world force at
// the base COM (apply_rigid_body_force_tensors ENV_SPACE semantics).
// ---------------------------------------------------------------------------------------------------
template <typename R>
T1_HD void compute_delta(const DynModel& M, const Terrain& T, const EnvParams<R>& P, const EnvState<R>& s,
                         const R tau[ND], V3<R> ext_f, R dt, R delta[6 + ND]) {
  M3<R> R0 = quat_to_mat(s.quat[0], s.quat[1], s.quat[2], s.quat[3]);
  V3<R> base_abs = v3<R>(s.pos[0], s.pos[1], s.pos[2]);
  R V0[6] = {s.w[0], s.w[1], s.w[2], s.vo[0], s.vo[1], s.vo[2]};
  R A0[6] = {R(0), R(0), R(0), R(0), R(0), R(M.gravity)};  // fictitious base acceleration -g
  Sym6<R> Ac;
  R Icw[6];
  world_inertia(M, 0, R0, P.inertia_scale[0], Icw);
  V3<R> c0 = mul(R0, v3<R>(R(M.com[0][0]) + P.com_disp[0], R(M.com[0][1]) + P.com_disp[1],
                           R(M.com[0][2]) + P.com_disp[2]));
  inertia_spatial(Ac, P.mass[0], c0, Icw);
  R gc[6];
  {
    R IA[6], IV[6], vf[6];
    sym_mul(Ac, A0, IA);
    sym_mul(Ac, V0, IV);
    crf(V0, IV, vf);
    V3<R> tq = cross(c0, ext_f);
    R fe[6] = {tq.x, tq.y, tq.z, ext_f.x, ext_f.y, ext_f.z};
#pragma unroll
    for (int i = 0; i < 6; ++i) gc[i] = dt * (IA[i] + vf[i] - fe[i]);
  }
  bool any = false;
  if (M.contact_count[0] > 0) {
    R w[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
    Sym6<R> K;
    sym_zero(K);
    bool a = false;
    body_contact(M, T, 0, R0, v3<R>(0, 0, 0), base_abs, V0, P.friction, dt, K, w, a);
    if (a) {
      sym_add(Ac, K);
#pragma unroll
      for (int i = 0; i < 6; ++i) gc[i] -= w[i];
    }
  }
  LegBlock<R> lb[2];
#pragma unroll
  for (int leg = 0; leg < 2; ++leg) assemble_leg(M, T, P, s, leg, R0, base_abs, V0, A0, tau, dt, lb[leg], Ac, gc, any);
  R rb[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) rb[i] = -gc[i];
#pragma unroll
  for (int leg = 0; leg < 2; ++leg) eliminate_leg(lb[leg], Ac, rb);
  solve_base(Ac, rb);
#pragma unroll
  for (int i = 0; i < 6; ++i) delta[i] = rb[i];
#pragma unroll
  for (int leg = 0; leg < 2; ++leg) backsub_leg(lb[leg], rb, delta + 6 + 6 * leg);
}

// Semi-implicit Euler with the solved velocity change (+ the omega x v term that turns the spatial base
// acceleration into the classical acceleration of the base origin); joint speeds clamped like PhysX.
template <typename R>
T1_HD void integrate(const DynModel& M, EnvState<R>& s, const R delta[6 + ND], R dt) {
  V3<R> w_new = v3<R>(s.w[0] + delta[0], s.w[1] + delta[1], s.w[2] + delta[2]);
  V3<R> vO_new = v3<R>(s.vo[0] + delta[3], s.vo[1] + delta[4], s.vo[2] + delta[5]);
  V3<R> vb_new = vO_new + dt * cross(w_new, vO_new);
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    R v = s.qd[j] + delta[6 + j];
    R vl = R(M.vel_limit[j]);
    v = v > vl ? vl : (v < -vl ? -vl : v);
    s.qd[j] = v;
    s.q[j] += dt * v;
  }
  s.w[0] = w_new.x; s.w[1] = w_new.y; s.w[2] = w_new.z;
  s.vo[0] = vb_new.x; s.vo[1] = vb_new.y; s.vo[2] = vb_new.z;
  s.pos[0] += dt * vb_new.x; s.pos[1] += dt * vb_new.y; s.pos[2] += dt * vb_new.z;
  // quaternion: q += 0.5 dt [w, 0] (x) q  (world-frame angular velocity), renormalised
  R qx = s.quat[0], qy = s.quat[1], qz = s.quat[2], qw = s.quat[3];
  R hx = R(0.5) * dt * w_new.x, hy = R(0.5) * dt * w_new.y, hz = R(0.5) * dt * w_new.z;
  R nx = qx + (hx * qw + hy * qz - hz * qy);
  R ny = qy + (hy * qw + hz * qx - hx * qz);
  R nz = qz + (hz * qw + hx * qy - hy * qx);
  R nw = qw - (hx * qx + hy * qy + hz * qz);
  R inv = R(1) / sqrt(nx * nx + ny * ny + nz * nz + nw * nw);
  s.quat[0] = nx * inv; s.quat[1] = ny * inv; s.quat[2] = nz * inv; s.quat[3] = nw * inv;
}

template <typename R>
T1_HD void substep(const DynModel& M, const Terrain& T, const EnvParams<R>& P, EnvState<R>& s, const R tau[ND],
                   V3<R> ext_f, R dt) {
  R delta[6 + ND];
  compute_delta(M, T, P, s, tau, ext_f, dt, delta);
  integrate(M, s, delta, dt);
}

// ---------------------------------------------------------------------------------------------------
// Gym-shaped outputs after the last substep: root (13), rigid (13 x 13), net contact force (13 x 3).
// Linear velocities are COM velocities (PhysX reports link COM velocity); positions are link frame origins.
// ---------------------------------------------------------------------------------------------------
template <typename R, typename Writer>
T1_HD void report(const DynModel& M, const Terrain& T, const EnvParams<R>& P, const EnvState<R>& s, R dt, Writer& W) {
  M3<R> R0 = quat_to_mat(s.quat[0], s.quat[1], s.quat[2], s.quat[3]);
  V3<R> base_abs = v3<R>(s.pos[0], s.pos[1], s.pos[2]);
  R V0[6] = {s.w[0], s.w[1], s.w[2], s.vo[0], s.vo[1], s.vo[2]};
  V3<R> c0 = mul(R0, v3<R>(R(M.com[0][0]) + P.com_disp[0], R(M.com[0][1]) + P.com_disp[1],
                           R(M.com[0][2]) + P.com_disp[2]));
  V3<R> vcom = v3<R>(s.vo[0], s.vo[1], s.vo[2]) + cross(v3<R>(s.w[0], s.w[1], s.w[2]), c0);
  R body[13];
  body[0] = s.pos[0]; body[1] = s.pos[1]; body[2] = s.pos[2];
  body[3] = s.quat[0]; body[4] = s.quat[1]; body[5] = s.quat[2]; body[6] = s.quat[3];
  body[7] = vcom.x; body[8] = vcom.y; body[9] = vcom.z;
  body[10] = s.w[0]; body[11] = s.w[1]; body[12] = s.w[2];
  W.root(body);
  W.rigid(0, body);
  V3<R> F0 = body_contact_force(M, T, 0, R0, v3<R>(0, 0, 0), base_abs, V0, P.friction, dt);
  W.contact(0, F0);
#pragma unroll
  for (int leg = 0; leg < 2; ++leg) {
    BodyState<R> B[NLEG];
    leg_fk(M, leg, R0, s.q, B);
    R V[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) V[i] = V0[i];
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      const int b = 1 + 6 * leg + k;
      R S[6];
      motion_subspace(M, b, B[k], S);
#pragma unroll
      for (int i = 0; i < 6; ++i) V[i] += S[i] * s.qd[6 * leg + k];
      V3<R> c = B[k].p + mul(B[k].Rot, v3<R>(M.com[b][0], M.com[b][1], M.com[b][2]));
      V3<R> om{V[0], V[1], V[2]};
      V3<R> vc = v3<R>(V[3], V[4], V[5]) + cross(om, c);
      R qb[4];
      mat_to_quat(B[k].Rot, qb);
      R out[13] = {B[k].p.x + base_abs.x, B[k].p.y + base_abs.y, B[k].p.z + base_abs.z, qb[0], qb[1], qb[2], qb[3],
                   vc.x, vc.y, vc.z, om.x, om.y, om.z};
      W.rigid(b, out);
      V3<R> F = M.contact_count[b] > 0 ? body_contact_force(M, T, b, B[k].Rot, B[k].p, base_abs, V, P.friction, dt)
                                       : v3<R>(0, 0, 0);
      W.contact(b, F);
    }
  }
}

}  // namespace t1
