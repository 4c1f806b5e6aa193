// t1_dyn5.h -- the substep of t1_dynamics.h split into the four roles of k_dyn5 (t1env_dyn5.hip).
//
// k_dyn5 runs 32 envs per workgroup with BOTH legs of an env in one wave (lanes 0-31 the left legs, 32-63 the
// right legs), so each of the four waves of a workgroup is a different role of the same substep and the step's
// dynamics spread over twice the lanes per env of k_dyn4 (8 instead of 4) -- at 8192 envs 256 workgroups, every
// CU of the MI355X, instead of 128:
//   W0 core    forward chain (poses only), contact-free CRBA backward pass without the bias (leg_backward_crba);
//              after S2: fold-in of every other role's terms (leg_apply_terms), elimination, the base system of
//              the two halves (permlane32 exchange, no LDS round trip, no third barrier), back-substitution,
//              integration
//   W1 bias    forward pass with the RNEA bias, PD torques, the bias/torque part of every joint rhs and of the
//              leg composite (leg_bias_rhs), the base block and the base-box contacts of both halves summed
//   W2 terrain shank and foot terrain contacts (restitution episodes)
//   W3 self    the capsule self-contact terms (the other leg's capsules by permlane32 from the other half)
// All of it is the same linear system as compute_delta (the assembled CRBA with contacts folded into the
// composites) up to fp32 summation order: the bias enters each joint rhs as rg_k = dt tau_k - S_k . sum_{j>=k} g_j
// and the leg composite's bias as G = sum_j g_j, exactly the terms leg_backward_nc accumulates, moved to the wave
// that computes g.  compute_delta_roles composes the roles on one host thread; tests/test_dynamics.py checks it
// against compute_delta in fp64 (flag bit 2 of t1dyn_substeps).
#pragma once
#include "t1_dynamics.h"

namespace t1 {

// W0: joint sin/cos and the leaf pose by leg_forward_nc's pose operations (the same values, in the same order)
template <typename R> struct LegFK {
  R sn[NLEG], cs[NLEG];
  M3<R> Rk;  // leaf pose
  V3<R> pk;
};
template <typename R>
T1_HD void leg_fk_chain(const DynModel& M, const M3<R>& R0, const R q[NLEG], int leg, LegFK<R>& st) {
  M3<R> Rk = R0;
  V3<R> pk = v3<R>(0, 0, 0);
  auto fwd = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int AX = T1_LEG_AXIS[k];
    const int b = 1 + 6 * leg + k;
    pk = pk + mul(Rk, v3<R>(M.joint_offset[b][0], M.joint_offset[b][1], M.joint_offset[b][2]));
    fsincos(R(M.axis_sign[b]) * q[k], &st.sn[k], &st.cs[k]);
    Rk = joint_rot<AX>(M, b, Rk, st.cs[k], st.sn[k]);
  };
  fwd(kconst<0>{});
  fwd(kconst<1>{});
  fwd(kconst<2>{});
  fwd(kconst<3>{});
  fwd(kconst<4>{});
  fwd(kconst<5>{});
  st.Rk = Rk;
  st.pk = pk;
}

// W0: leg_backward_nc without the RNEA bias and the torques (W1's leg_bias_rhs supplies them): the contact-free
// composite of the leg (Ac_up), D0, H0, Bl = F0 and the joint-limit part of each rhs; S[k] for the fold-in.
template <typename R>
T1_HD void leg_backward_crba(const DynModel& M, const LegParams<R>& P, const R q[NLEG], const R qd[NLEG], int leg, R dt,
                             const LegFK<R>& st, R (&S)[NLEG][6], LegBlock<R>& out, Sym6<R>& Ac_up) {
  M3<R> Rk = st.Rk;
  V3<R> pk = st.pk;
  Composite<R> Ac;
  composite_zero(Ac);
  auto step = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const int b = 1 + 6 * leg + k, j = 6 * leg + k;
    if constexpr (k < NLEG - 1) {  // step up from child k+1
      constexpr int AXC = T1_LEG_AXIS[k + 1];
      const int bc = b + 1;
      Rk = joint_rot<AXC>(M, bc, Rk, st.cs[k + 1], -st.sn[k + 1]);
      pk = pk - mul(Rk, v3<R>(M.joint_offset[bc][0], M.joint_offset[bc][1], M.joint_offset[bc][2]));
    }
    R* Sk = S[k];
    joint_subspace<T1_LEG_AXIS[k]>(M, b, Rk, pk, Sk);
    {
      R Icw[6];
      world_inertia(M, b, Rk, P.inertia_scale[k], Icw);
      const V3<R> c = pk + mul(Rk, v3<R>(M.com[b][0], M.com[b][1], M.com[b][2]));
      composite_add(Ac, P.mass[k], c, Icw);
    }
    R Fk[6];
    composite_mul(Ac, Sk, Fk);
    R Ajj = dot6(Sk, Fk) + P.armature[k];
    R rj = R(0);
    const R lo = R(M.q_lower[j]), hi = R(M.q_upper[j]);
    const R qj = q[k], qdj = qd[k];
    if (qj < lo) {
      const R cl = qdj < R(0) ? dt * R(M.k_limit) + R(M.d_limit) : R(0);
      Ajj += dt * cl;
      rj = dt * (R(M.k_limit) * (lo - qj) - cl * qdj);
    } else if (qj > hi) {
      const R cl = qdj > R(0) ? dt * R(M.k_limit) + R(M.d_limit) : R(0);
      Ajj += dt * cl;
      rj = dt * (R(M.k_limit) * (hi - qj) - cl * qdj);
    }
    out.L[sidx(k, k)] = Ajj;
    out.rhs[k] = rj;
#pragma unroll
    for (int jj = k + 1; jj < NLEG; ++jj) {
      R Fj[6] = {out.Bl[0][jj], out.Bl[1][jj], out.Bl[2][jj], out.Bl[3][jj], out.Bl[4][jj], out.Bl[5][jj]};
      out.L[sidx(k, jj)] = dot6(Sk, Fj);
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) out.Bl[r][k] = Fk[r];
  };
#ifndef T1_WHATIF_CRBA_HALF  // timing-only what-if build (never the product): the distal half of the pass skipped
  step(kconst<5>{});
  step(kconst<4>{});
  step(kconst<3>{});
#else  // joints 3-5 decoupled with a unit inertia (a bounded, wrong system: timing only)
#pragma unroll
  for (int k = 3; k < NLEG; ++k) {
#pragma unroll
    for (int jj = 0; jj < NLEG; ++jj) out.L[sidx(jj < k ? jj : k, jj < k ? k : jj)] = jj == k ? R(1) : R(0);
#pragma unroll
    for (int r = 0; r < 6; ++r) out.Bl[r][k] = R(0);
    out.rhs[k] = R(0);
#pragma unroll
    for (int i = 0; i < 6; ++i) S[k][i] = R(0);
  }
#endif
  step(kconst<2>{});
  step(kconst<1>{});
  step(kconst<0>{});
  composite_to_sym(Ac, Ac_up);
}

// W1: leg_forward_nc's pass (poses, velocities, velocity-product accelerations, RNEA bias g_k at each COM), then
// the bias / torque part of the joint rhs, rg_k = dt tau_k - S_k . sum_{j>=k} g_j, and the leg's total bias G.
template <typename R>
T1_HD void leg_bias_rhs(const DynModel& M, const LegParams<R>& P, const BaseFrame<R>& F, const R q[NLEG],
                        const R qd[NLEG], const R tau[NLEG], int leg, R dt, R rg[NLEG], R G[6]) {
  M3<R> Rk = F.R0;
  V3<R> pk = v3<R>(0, 0, 0);
  R V[6], A[6], S[NLEG][6], g[NLEG][6];
#pragma unroll
  for (int i = 0; i < 6; ++i) { V[i] = F.V0[i]; A[i] = R(0); }
  A[5] = R(M.gravity);
  auto fwd = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int AX = T1_LEG_AXIS[k];
    const int b = 1 + 6 * leg + k;
    pk = pk + mul(Rk, v3<R>(M.joint_offset[b][0], M.joint_offset[b][1], M.joint_offset[b][2]));
    R sn, cs;
    fsincos(R(M.axis_sign[b]) * q[k], &sn, &cs);
    Rk = joint_rot<AX>(M, b, Rk, cs, sn);
    R* Sk = S[k];
    joint_subspace<AX>(M, b, Rk, pk, Sk);
    R vj[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) vj[i] = Sk[i] * qd[k];
#pragma unroll
    for (int i = 0; i < 6; ++i) V[i] += vj[i];
    R cr[6];
    crm(V, vj, cr);  // V_k x (S qd)
#pragma unroll
    for (int i = 0; i < 6; ++i) A[i] += cr[i];
    R Icw[6];
    world_inertia(M, b, Rk, P.inertia_scale[k], Icw);
    const V3<R> c = pk + mul(Rk, v3<R>(M.com[b][0], M.com[b][1], M.com[b][2]));
    rnea_bias_com(P.mass[k], c, Icw, V, A, dt, g[k]);
  };
  fwd(kconst<0>{});
  fwd(kconst<1>{});
  fwd(kconst<2>{});
  fwd(kconst<3>{});
  fwd(kconst<4>{});
  fwd(kconst<5>{});
  R gc[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
#pragma unroll
  for (int k = NLEG - 1; k >= 0; --k) {
#pragma unroll
    for (int i = 0; i < 6; ++i) gc[i] += g[k][i];
    rg[k] = dt * tau[k] - dot6(S[k], gc);
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) G[i] = gc[i];
}

// W0 after S2: leg_apply_contacts with the bias / torque terms of W1 instead of the torques: the contact terms of
// bodies K0 < K1 (C0/c0, C1/c1), rg into every joint rhs, G and the contact wrenches into the leg's bias gc_up
template <int K0, int K1, typename R>
T1_HD void leg_apply_terms(const Sym6<R>& C0, const R c0[6], const Sym6<R>& C1, const R c1[6], const R rg[NLEG],
                           const R G[6], const R (&S)[NLEG][6], LegBlock<R>& out, Sym6<R>& Ac_up, R gc_up[6]) {
  static_assert(0 <= K0 && K0 < K1 && K1 < NLEG, "contact bodies K0 < K1 of the leg");
  Sym6<R> Cs = C0;
  sym_add(Cs, C1);
  R cs[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) cs[i] = c0[i] + c1[i];
  R u[NLEG][6];  // Cs_k S_k
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    if (k <= K0) sym_mul(Cs, S[k], u[k]);
    else if (k <= K1) sym_mul(C1, S[k], u[k]);
    else
#pragma unroll
      for (int i = 0; i < 6; ++i) u[k][i] = R(0);
  }
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    const R sc = k <= K0 ? dot6(S[k], cs) : (k <= K1 ? dot6(S[k], c1) : R(0));
    out.L[sidx(k, k)] += dot6(S[k], u[k]);
    out.rhs[k] += rg[k] - sc;
#pragma unroll
    for (int jj = k + 1; jj < NLEG; ++jj) out.L[sidx(k, jj)] += dot6(S[k], u[jj]);
  }
#pragma unroll
  for (int k = 0; k < NLEG; ++k)
#pragma unroll
    for (int r = 0; r < 6; ++r) out.Bl[r][k] += u[k][r];
  sym_add(Ac_up, Cs);
#pragma unroll
  for (int i = 0; i < 6; ++i) gc_up[i] += G[i] + cs[i];
}

// the four roles composed on one thread in k_dyn5's order (host builds; tests/test_dynamics.py)
template <typename R>
T1_HD void compute_delta_roles(const DynModel& M, const Terrain& T, const EnvParams<R>& P, EnvState<R>& s,
                               const R tau[ND], V3<R> ext_f, R dt, R delta[6 + ND]) {
  constexpr int KS = 3, KF = 5;
  static_assert(T1_LEG_CONTACT_MASK == ((1 << KS) | (1 << KF)), "roles assume shank + foot contacts");
  BaseFrame<R> F;
  base_frame(s, F);
  const R mu = P.base.friction, e = ground_restitution(M, P.base.restitution);
  // W1: the base block and the base-box contact halves, summed (left half first)
  Sym6<R> Bs;
  R rbs[6];
  base_block(M, P.base, F, ext_f, dt, Bs, rbs);
#pragma unroll
  for (int i = 0; i < 6; ++i) rbs[i] = -rbs[i];
  const int32_t bound_b = terrain_bound_raw_any(T, F.abs.x, F.abs.y);
  for (int leg = 0; leg < 2; ++leg) {
    int cb, ce;
    base_contact_range(M, leg, cb, ce);
    Sym6<R> Cb;
    R gw[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
    sym_zero(Cb);
    body_contact_fixed<T1_POINTS_PER_BODY / 2>(M, T, F.abs.z - R(M.contact_radius[0]), bound_b, cb, F.R0,
                                               v3<R>(0, 0, 0), F.abs, F.V0, mu, e, s.vimp[vimp_base(leg)], dt, Cb, gw);
    sym_add(Bs, Cb);
#pragma unroll
    for (int i = 0; i < 6; ++i) rbs[i] -= gw[i];
  }
  // W3: self-contact terms of both legs (from the substep's state)
  SelfTerms<R> ST;
  self_terms_env(M, F, s.q, s.qd, P.base, dt, ST);
  LegBlock<R> lb[2];
  Sym6<R> Ab[2];
  R rb[2][6];
  for (int leg = 0; leg < 2; ++leg) {
    const R* q = s.q + 6 * leg;
    const R* qd = s.qd + 6 * leg;
    // W0 before S2
    LegFK<R> fk;
    leg_fk_chain(M, F.R0, q, leg, fk);
    R S[NLEG][6];
    sym_zero(Ab[leg]);
    leg_backward_crba(M, P.leg[leg], q, qd, leg, dt, fk, S, lb[leg], Ab[leg]);
    // W1
    R rg[NLEG], G[6];
    leg_bias_rhs(M, P.leg[leg], F, q, qd, tau + 6 * leg, leg, dt, rg, G);
    // W2: terrain terms of the shank and the foot from their kinematics
    BodyKin<R> K[2];
    leg_body_kinematics(M, F, q, qd, leg, K);
    Sym6<R> Ct[2];
    R ct[2][6];
    for (int i = 0; i < 2; ++i) {
      const int b = 1 + 6 * leg + (i ? KF : KS);
      sym_zero(Ct[i]);
      for (int j = 0; j < 6; ++j) ct[i][j] = R(0);
      const int32_t bound = terrain_bound_raw_any(T, K[i].p.x + F.abs.x, K[i].p.y + F.abs.y);
      body_contact_fixed<T1_POINTS_PER_BODY>(M, T, K[i].p.z + F.abs.z - R(M.contact_radius[b]), bound,
                                             M.contact_start[b], K[i].Rb, K[i].p, F.abs, K[i].V, mu, e,
                                             s.vimp[i ? vimp_foot(leg) : vimp_shank(leg)], dt, Ct[i], ct[i]);
      // W0: terrain + self terms of the body
      sym_add(Ct[i], ST.C[leg][i]);
      for (int j = 0; j < 6; ++j) ct[i][j] += ST.c[leg][i][j];
    }
    // W0 after S2
    R g6[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
    leg_apply_terms<KS, KF>(Ct[0], ct[0], Ct[1], ct[1], rg, G, S, lb[leg], Ab[leg], g6);
#pragma unroll
    for (int i = 0; i < 6; ++i) rb[leg][i] = -g6[i];
    eliminate_leg(lb[leg], Ab[leg], rb[leg]);
  }
  // W0: base system = (base + base-box halves) + left leg + right leg
  Sym6<R> Ac = Bs;
  R r[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) r[i] = rbs[i];
  for (int leg = 0; leg < 2; ++leg) {
    sym_add(Ac, Ab[leg]);
#pragma unroll
    for (int i = 0; i < 6; ++i) r[i] += rb[leg][i];
  }
  solve_base(Ac, r);
  for (int i = 0; i < 6; ++i) delta[i] = r[i];
  for (int leg = 0; leg < 2; ++leg) backsub_leg(lb[leg], r, delta + 6 + 6 * leg);
}

// one half (NP points from c_begin) of a contact body against the terrain: contact_query + contact_apply, the fastest
// approach of its points in amax (k_dyn6's contact_half, t1env_dyn6.hip, on one host thread)
template <int NP, typename R>
T1_HD void contact_points_half(const DynModel& M, const Terrain& T, int c_begin, const M3<R>& Rb, V3<R> pb,
                               V3<R> base_abs, const R Vb[6], R mu, R vtg, R dt, Sym6<R>& A, R g[6], R& amax) {
  ContactQuery<NP, R> Q;
  if (T.type == 0) {
    contact_query<false, NP>(M, T, c_begin, Rb, pb, base_abs, Q);
    contact_apply<false, NP>(M, Q, Vb, mu, vtg, dt, A, g, amax);
  } else {
    contact_query<true, NP>(M, T, c_begin, Rb, pb, base_abs, Q);
    contact_apply<true, NP>(M, Q, Vb, mu, vtg, dt, A, g, amax);
  }
}

// k_dyn6's eight roles (t1env_dyn6.hip) composed on one thread: k_dyn5's composition with each terrain contact body
// evaluated as two halves of its points (W2 / W6: the shank, W3 / W7: the foot) whose terms are summed, then the
// self-contact terms added ((half 0 + half 1) + self), and the body's restitution episode taken from the larger of the
// halves' fastest approach (the core wave, W0).  The base-box halves and the leg passes are k_dyn5's.
template <typename R>
T1_HD void compute_delta_roles6(const DynModel& M, const Terrain& T, const EnvParams<R>& P, EnvState<R>& s,
                                const R tau[ND], V3<R> ext_f, R dt, R delta[6 + ND]) {
  constexpr int KS = 3, KF = 5, NH = T1_POINTS_PER_BODY / 2;
  static_assert(T1_LEG_CONTACT_MASK == ((1 << KS) | (1 << KF)), "roles assume shank + foot contacts");
  BaseFrame<R> F;
  base_frame(s, F);
  const R mu = P.base.friction, e = ground_restitution(M, P.base.restitution);
  // W0: the base block and the base-box contact halves, summed (left half first)
  Sym6<R> Bs;
  R rbs[6];
  base_block(M, P.base, F, ext_f, dt, Bs, rbs);
#pragma unroll
  for (int i = 0; i < 6; ++i) rbs[i] = -rbs[i];
  const int32_t bound_b = terrain_bound_raw_any(T, F.abs.x, F.abs.y);
  for (int leg = 0; leg < 2; ++leg) {
    int cb, ce;
    base_contact_range(M, leg, cb, ce);
    Sym6<R> Cb;
    R gw[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
    sym_zero(Cb);
    body_contact_fixed<T1_POINTS_PER_BODY / 2>(M, T, F.abs.z - R(M.contact_radius[0]), bound_b, cb, F.R0,
                                               v3<R>(0, 0, 0), F.abs, F.V0, mu, e, s.vimp[vimp_base(leg)], dt, Cb, gw);
    sym_add(Bs, Cb);
#pragma unroll
    for (int i = 0; i < 6; ++i) rbs[i] -= gw[i];
  }
  // W5: self-contact terms of both legs (from the substep's state)
  SelfTerms<R> ST;
  self_terms_env(M, F, s.q, s.qd, P.base, dt, ST);
  LegBlock<R> lb[2];
  Sym6<R> Ab[2];
  R rb[2][6];
  R vnew[2][2];  // the shank / foot episodes after this substep (W0 updates them after S2)
  for (int leg = 0; leg < 2; ++leg) {
    const R* q = s.q + 6 * leg;
    const R* qd = s.qd + 6 * leg;
    // W4
    LegFK<R> fk;
    leg_fk_chain(M, F.R0, q, leg, fk);
    R S[NLEG][6];
    sym_zero(Ab[leg]);
    leg_backward_crba(M, P.leg[leg], q, qd, leg, dt, fk, S, lb[leg], Ab[leg]);
    // W1
    R rg[NLEG], G[6];
    leg_bias_rhs(M, P.leg[leg], F, q, qd, tau + 6 * leg, leg, dt, rg, G);
    // W2 / W6 (shank), W3 / W7 (foot): the terrain terms of each half of the body's points
    BodyKin<R> K[2];
    leg_body_kinematics(M, F, q, qd, leg, K);
    Sym6<R> Ct[2];
    R ct[2][6];
    for (int i = 0; i < 2; ++i) {
      const int b = 1 + 6 * leg + (i ? KF : KS);
      const int vi = i ? vimp_foot(leg) : vimp_shank(leg);
      const R vtg = restitution_target(M, e, s.vimp[vi]);
      // the shank is skipped when out of the terrain's reach by its height bound (both halves: no contact)
      const bool skip = i == 0 && K[i].p.z + F.abs.z - R(M.contact_radius[b]) >
                                      bound_height<R>(T, terrain_bound_raw_any(T, K[i].p.x + F.abs.x, K[i].p.y + F.abs.y));
      Sym6<R> Ch[2];
      R ch[2][6], am[2] = {R(-1), R(-1)};
      for (int h = 0; h < 2; ++h) {
        sym_zero(Ch[h]);
        for (int j = 0; j < 6; ++j) ch[h][j] = R(0);
        if (!skip)
          contact_points_half<NH>(M, T, M.contact_start[b] + h * NH, K[i].Rb, K[i].p, F.abs, K[i].V, mu, vtg, dt,
                                  Ch[h], ch[h], am[h]);
      }
      vnew[leg][i] = restitution_episode(s.vimp[vi], am[0] > am[1] ? am[0] : am[1]);
      // W0: (half 0 + half 1) + self
      for (int j = 0; j < 21; ++j) Ct[i].a[j] = (Ch[0].a[j] + Ch[1].a[j]) + ST.C[leg][i].a[j];
      for (int j = 0; j < 6; ++j) ct[i][j] = (ch[0][j] + ch[1][j]) + ST.c[leg][i][j];
    }
    // W0 after S2
    R g6[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
    leg_apply_terms<KS, KF>(Ct[0], ct[0], Ct[1], ct[1], rg, G, S, lb[leg], Ab[leg], g6);
#pragma unroll
    for (int i = 0; i < 6; ++i) rb[leg][i] = -g6[i];
    eliminate_leg(lb[leg], Ab[leg], rb[leg]);
  }
  for (int leg = 0; leg < 2; ++leg) {
    s.vimp[vimp_shank(leg)] = vnew[leg][0];
    s.vimp[vimp_foot(leg)] = vnew[leg][1];
  }
  // W0: base system = (base + base-box halves) + left leg + right leg
  Sym6<R> Ac = Bs;
  R r[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) r[i] = rbs[i];
  for (int leg = 0; leg < 2; ++leg) {
    sym_add(Ac, Ab[leg]);
#pragma unroll
    for (int i = 0; i < 6; ++i) r[i] += rb[leg][i];
  }
  solve_base(Ac, r);
  for (int i = 0; i < 6; ++i) delta[i] = r[i];
  for (int leg = 0; leg < 2; ++leg) backsub_leg(lb[leg], r, delta + 6 + 6 * leg);
}

template <typename R>
T1_HD void substep_roles6(const DynModel& M, const Terrain& T, const EnvParams<R>& P, EnvState<R>& s, const R tau[ND],
                          V3<R> ext_f, R dt) {
  R delta[6 + ND];
  compute_delta_roles6(M, T, P, s, tau, ext_f, dt, delta);
  integrate_base(s, delta, dt);
  for (int leg = 0; leg < 2; ++leg) integrate_leg(M, leg, s.q + 6 * leg, s.qd + 6 * leg, delta + 6 + 6 * leg, dt);
}

template <typename R>
T1_HD void substep_roles(const DynModel& M, const Terrain& T, const EnvParams<R>& P, EnvState<R>& s, const R tau[ND],
                         V3<R> ext_f, R dt) {
  R delta[6 + ND];
  compute_delta_roles(M, T, P, s, tau, ext_f, dt, delta);
  integrate_base(s, delta, dt);
  for (int leg = 0; leg < 2; ++leg) integrate_leg(M, leg, s.q + 6 * leg, s.qd + 6 * leg, delta + 6 + 6 * leg, dt);
}

}  // namespace t1
