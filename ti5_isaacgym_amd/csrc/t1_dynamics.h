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
//     The leg work is written per leg (leg_assemble / eliminate_leg / backsub_leg) and the base block is the
//     sum  base + contribution(left) + contribution(right)  in that order, so the GPU can run the two legs of
//     an env on two waves that exchange a 27-float contribution, and the host build runs them in a loop --
//     same arithmetic either way.
//   * semi-implicit Euler; joint speeds clamped to the URDF velocity limits like PhysX max joint velocity.
#pragma once
#include <type_traits>

#include "t1_common.h"

// phase profiling hook (t1env_dynamics.hip built with -DT1_PHASE_PROF); compiled out otherwise
#ifndef T1_PROF_MARK
#define T1_PROF_MARK(i) ((void)0)
#endif

namespace t1 {

constexpr int NB = 13, ND = 12, NLEG = 6;

// Contact layout known at compile time: CM = bit mask of the leg bodies (k = 0..5) that carry NPC contact
// points each (the T1: shank k=3 and foot k=5, 8 points each; base box 8 points = 4 per leg).  CM < 0: read
// the layout from the model at run time (host build, other robots).  The GPU kernel requires the T1 layout
// (t1_model_conv.h checks it) so every contact loop is fully unrolled with its loads batched.
constexpr int T1_LEG_CONTACT_MASK = (1 << 3) | (1 << 5);
constexpr int T1_POINTS_PER_BODY = 8;
// joint axis of leg joint k (0 = x, 1 = y, 2 = z): hip yaw z, hip roll x, hip pitch y, knee y, ankle pitch y,
// ankle roll x -- compiled in with the fixed layout (checked at create) so rotations use static indices
constexpr int T1_LEG_AXIS[NLEG] = {2, 0, 1, 1, 1, 0};


// A self-collision capsule in its link frame: segment a-b and radius r (t1env_model.self_capsule).
struct SelfCapsule {
  float a[3], b[3], r;
};

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
  float contact_radius[NB];  // max distance of a body's contact points from its frame origin
  float k_contact, d_contact, friction_vs, k_limit, d_limit, gravity;
  float ground_friction, ground_restitution;
  float base_init_state[13];
  SelfCapsule self_cap[2][2];  // [leg][0 shank, 1 foot]
  int32_t self_collisions;
  float bounce_threshold;  // restitution acts on contacts approaching faster than this [m/s]
};

// Terrain: plane (type 0) or height field sampled like the trimesh the reference builds from it
// (type 1/2; two triangles per cell split along the (i,j)-(i+1,j+1) diagonal).
struct Terrain {
  const int16_t* h;  // (rows, cols), rows along x
  int32_t rows, cols, type;
  float hscale, vscale, border;
  float inv_hscale;  // 1 / hscale
  // coarse bound: hmax[ci][cj] = highest sample within K cells of coarse cell (ci, cj) (K * cell >= every
  // contact radius), raw units; lets a contact body far above the ground skip its point queries exactly.
  const int16_t* hmax;  // (hm_rows, hm_cols) or null (no bound: always query)
  int32_t hm_rows, hm_cols;
  float hm_inv_cell;    // 1 / coarse cell size [1/m]
};
inline Terrain make_terrain(const int16_t* h, int32_t rows, int32_t cols, int32_t type, float hscale, float vscale,
                            float border) {
  return Terrain{h, rows, cols, type, hscale, vscale, border, 1.0f / hscale, nullptr, 0, 0, 0.0f};
}

template <typename R> struct BaseParams {
  R mass, inertia_scale, com_disp[3];
  R friction;       // combined shape/ground friction coefficient
  R restitution;    // the env's shape restitution (DR, restitution_range); ground contacts combine it with the ground's
  R self_friction;  // the env's shape friction (a self-contact is between two shapes of the same env)
};
// PhysX's default combine mode (average) for a robot shape against the ground: friction (load_base_params) and
// restitution alike (third-party semantics, unpinned)
template <typename R> T1_HD R ground_restitution(const DynModel& M, R e_env) { return R(0.5) * (e_env + R(M.ground_restitution)); }
template <typename R> struct LegParams {
  R mass[NLEG], inertia_scale[NLEG], armature[NLEG];
};
template <typename R> struct EnvParams {
  BaseParams<R> base;
  LegParams<R> leg[2];
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
// terrain query at world (x, y): height h and slope (gx, gy) = dh/dx, dh/dy; the unit normal
// (-gx, -gy, 1) / |.| is formed only for points in contact (terrain_normal).  HF=false: the plane z=0.
// ---------------------------------------------------------------------------------------------------
template <bool HF, typename R> T1_HD R terrain_height(const Terrain& T, R x, R y, R& gx, R& gy) {
  if constexpr (!HF) {
    gx = gy = R(0);
    return R(0);
  } else {
    const R ih = R(T.inv_hscale);
    R fx = (x + R(T.border)) * ih, fy = (y + R(T.border)) * ih;
    R ix = floor(fx), iy = floor(fy);
    int i = (int)ix, j = (int)iy;
    R u = fx - ix, v = fy - iy;
    if (i < 0) { i = 0; u = 0; }
    if (j < 0) { j = 0; v = 0; }
    if (i > T.rows - 2) { i = T.rows - 2; u = 1; }
    if (j > T.cols - 2) { j = T.cols - 2; v = 1; }
    const int16_t* r0 = T.h + (i * T.cols + j);
    R vs = R(T.vscale);
    R h00 = vs * r0[0], h01 = vs * r0[1], h10 = vs * r0[T.cols], h11 = vs * r0[T.cols + 1];
    // triangle (i,j)-(i+1,j)-(i+1,j+1) if u >= v else (i,j)-(i+1,j+1)-(i,j+1)
    const bool lo = u >= v;
    R dhdu = lo ? h10 - h00 : h11 - h01;
    R dhdv = lo ? h11 - h10 : h01 - h00;
    gx = dhdu * ih;
    gy = dhdv * ih;
    return h00 + u * dhdu + v * dhdv;
  }
}
template <bool HF, typename R> T1_HD V3<R> terrain_normal(R gx, R gy) {
  if constexpr (!HF) {
    return v3<R>(0, 0, 1);
  } else {
    R inv = rcp(fsqrt(R(1) + gx * gx + gy * gy));
    return v3<R>(-gx * inv, -gy * inv, inv);
  }
}
template <bool HF, typename R> T1_HD R terrain_height(const Terrain& T, R x, R y, V3<R>& n) {
  R gx, gy;
  R h = terrain_height<HF>(T, x, y, gx, gy);
  n = terrain_normal<HF>(gx, gy);
  return h;
}

// Highest terrain a body whose frame origin is at world (x, y) can touch with points within its contact radius
// (hmax covers every contact radius): a body with origin height - radius above it cannot be in contact.
// Exact -- the trimesh interpolation never exceeds its vertices.  Split from the test so the load can be
// issued early and consumed later.  No bound (always query): +inf.
// The raw bound sample (height-field units) is returned so the load's consumer -- and its wait -- stays where
// the bound is tested (bound_height).
template <bool HF, typename R> T1_HD int32_t terrain_bound_raw(const Terrain& T, R x, R y) {
  if constexpr (!HF) {
    return 0;
  } else {
    if (!T.hmax) return 0x7fffffff;
    int ci = (int)floor((x + R(T.border)) * R(T.hm_inv_cell));
    int cj = (int)floor((y + R(T.border)) * R(T.hm_inv_cell));
    ci = ci < 0 ? 0 : (ci > T.hm_rows - 1 ? T.hm_rows - 1 : ci);
    cj = cj < 0 ? 0 : (cj > T.hm_cols - 1 ? T.hm_cols - 1 : cj);
    return T.hmax[ci * T.hm_cols + cj];
  }
}
template <typename R> T1_HD R bound_height(const Terrain& T, int32_t raw) {
  return raw == 0x7fffffff ? R(INFINITY) : R(T.vscale) * R(raw);
}
template <bool HF, typename R> T1_HD R terrain_bound(const Terrain& T, R x, R y) {
  return bound_height<R>(T, terrain_bound_raw<HF>(T, x, y));
}
template <typename R> T1_HD int32_t terrain_bound_raw_any(const Terrain& T, R x, R y) {
  return T.type == 0 ? terrain_bound_raw<false>(T, x, y) : terrain_bound_raw<true>(T, x, y);
}


// ---------------------------------------------------------------------------------------------------
// kinematics of one leg (bodies 1+6*leg .. 6+6*leg), world axes about O
// ---------------------------------------------------------------------------------------------------
template <typename R>
T1_HD void leg_fk(const DynModel& M, int leg, const M3<R>& Rbase, const R q[NLEG], BodyState<R> B[NLEG]) {
  M3<R> Rp = Rbase;
  V3<R> pp = v3<R>(0, 0, 0);
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    const int b = 1 + 6 * leg + k;
    V3<R> off = v3<R>(M.joint_offset[b][0], M.joint_offset[b][1], M.joint_offset[b][2]);
    V3<R> p = pp + mul(Rp, off);
    R s, c;
    fsincos(R(M.axis_sign[b]) * q[k], &s, &c);
    M3<R> Rb = mul_axis_rot(Rp, M.axis_idx[b], c, s);
    B[k].Rot = Rb;
    B[k].p = p;
    Rp = Rb;
    pp = p;
  }
}

template <typename R> T1_HD void motion_subspace(const DynModel& M, int b, const BodyState<R>& B, R S[6]) {
  // a = Rot * (sign e_axis); the 0/+-1 weights are exact, and no register array is indexed at run time
  const int ax = M.axis_idx[b];
  const R sg = R(M.axis_sign[b]);
  V3<R> a = mul(B.Rot, v3<R>(ax == 0 ? sg : R(0), ax == 1 ? sg : R(0), ax == 2 ? sg : R(0)));
  V3<R> l = cross(B.p, a);
  S[0] = a.x; S[1] = a.y; S[2] = a.z; S[3] = l.x; S[4] = l.y; S[5] = l.z;
}

// world inertia about COM (xx yy zz xy xz yz) of body b
// timing-only what-if builds (never the product): the body-frame inertia used as if the body were unrotated
template <typename R> T1_HD void world_inertia_unrotated(const DynModel& M, int b, R scale, R out[6]) {
#pragma unroll
  for (int i = 0; i < 6; ++i) out[i] = scale * R(M.inertia[b][i]);
}
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
// contact of one body's points [c_begin, c_end) against the terrain: accumulates dt * J^T C J (6x6, about
// O) into A and subtracts the impulse wrench from g.  Per point: normal spring k*pen (+ implicit damping
// when approaching), regularised Coulomb friction as an implicit tangential damper whose coefficient keeps
// |F_t| <= mu F_n (Stribeck speed friction_vs).
// ---------------------------------------------------------------------------------------------------
// Sum over a body's contact points of c * sum_e w_e w_e^T with w_e = [x cross e ; e] over the world axes e:
// that is the spatial inertia of point masses c at x, [[ |x|^2 I - x x^T, [x]x ], [[x]x^T, I]] * c, so the
// friction stiffness accumulates as 10 moments per body instead of three 6x6 rank-1 updates per point.
template <typename R> struct PointMoments {
  R m, hx, hy, hz, sxx, syy, szz, sxy, sxz, syz;
};
template <typename R> T1_HD void moments_zero(PointMoments<R>& P) {
  P.m = P.hx = P.hy = P.hz = P.sxx = P.syy = P.szz = P.sxy = P.sxz = P.syz = R(0);
}
template <typename R> T1_HD void moments_add(PointMoments<R>& P, R c, V3<R> x) {
  const R cx = c * x.x, cy = c * x.y, cz = c * x.z;
  P.m += c; P.hx += cx; P.hy += cy; P.hz += cz;
  P.sxx += cx * x.x; P.syy += cy * x.y; P.szz += cz * x.z;
  P.sxy += cx * x.y; P.sxz += cx * x.z; P.syz += cy * x.z;
}
template <typename R> T1_HD void moments_flush(const PointMoments<R>& P, Sym6<R>& A) {
  A.a[sidx(0, 0)] += P.syy + P.szz; A.a[sidx(1, 1)] += P.sxx + P.szz; A.a[sidx(2, 2)] += P.sxx + P.syy;
  A.a[sidx(0, 1)] -= P.sxy; A.a[sidx(0, 2)] -= P.sxz; A.a[sidx(1, 2)] -= P.syz;
  A.a[sidx(0, 4)] -= P.hz; A.a[sidx(0, 5)] += P.hy;
  A.a[sidx(1, 3)] += P.hz; A.a[sidx(1, 5)] -= P.hx;
  A.a[sidx(2, 3)] -= P.hy; A.a[sidx(2, 4)] += P.hx;
  A.a[sidx(3, 3)] += P.m; A.a[sidx(4, 4)] += P.m; A.a[sidx(5, 5)] += P.m;
}

// Restitution (PhysX's bounce: sim.physx.bounce_threshold_velocity and the shapes' restitution e).  A contact body
// keeps the approach speed v_imp its contact episode began with (the fastest approaching point of the episode's
// first substep; 0 while the body touches nothing, t1env_buffers.contact_vimp).  When v_imp exceeds the threshold,
// the points' normal damper, which otherwise acts only while they approach, also acts while they separate slower than
// v_tgt = e v_imp, pushing them out toward that speed -- PhysX's restitution target (exit) velocity, as a set point of
// the damper in the separation phase:  approaching (v_n < 0): cn = dt k + d, f_n = k pen - cn v_n (unchanged);
// separating below the target (0 <= v_n < v_tgt): cn = d, f_n = k pen - d (v_n - v_tgt); otherwise no damper.  The
// compliant law's own rebound (the spring's stored energy) comes on top: the exit speed is at least ~e v_imp.
// v_tgt = 0 is the plain compliant law.
template <typename R> T1_HD R restitution_target(const DynModel& M, R e, R vimp) {
#ifdef T1_WHATIF_NO_RESTITUTION  // timing-only what-if build: no restitution set point
  return R(0);
#endif
  return vimp > R(M.bounce_threshold) ? e * vimp : R(0);
}
// the episode after this substep: amax = the fastest approach among the body's points in contact (< 0: none)
template <typename R> T1_HD R restitution_episode(R vimp, R amax) {
  return amax < R(0) ? R(0) : (vimp > R(0) ? vimp : (amax > R(1e-6) ? amax : R(1e-6)));
}

// One contact point of a body: x (about O), unit normal n pushing the body out, depth pen, the body's spatial velocity
// Vb, friction mu, restitution target speed vtg; vs = the velocity of the surface it touches at x (zero for the
// terrain, the other body's point velocity for a self-contact, whose own-side terms are implicit and the other side's
// motion explicit).  amax (optional): raised to this point's approach speed max(-v_n, 0).
template <typename R>
T1_HD void contact_point(const DynModel& M, V3<R> x, V3<R> n, R pen, const R Vb[6], R mu, R vtg, R dt, Sym6<R>& A,
                         R g[6], PointMoments<R>& fric, V3<R> vs = V3<R>{R(0), R(0), R(0)}, R* amax = nullptr) {
  const R k = R(M.k_contact), d = R(M.d_contact);
  V3<R> om{Vb[0], Vb[1], Vb[2]}, vo{Vb[3], Vb[4], Vb[5]};
  V3<R> vp = vo + cross(om, x) - vs;
  R vn = dot(n, vp);
  V3<R> vt = vp - vn * n;
  R vtn = fsqrt(dot(vt, vt));
  const bool ap = vn < R(0), rs = !ap && vn < vtg;  // approaching; separating below the restitution target
  R cn = ap ? dt * k + d : (rs ? d : R(0));
  R fn_est = k * pen + (ap ? -d * vn : (rs ? d * (vtg - vn) : R(0)));
  R ct = mu * fn_est * rcp(vtn > R(M.friction_vs) ? vtn : R(M.friction_vs));
  if (amax) *amax = *amax > -vn ? *amax : (-vn > R(0) ? -vn : R(0));
  // force at the current velocity (explicit part) f = (k pen - cn vn + d vtg) n - ct vt, C = cn nn^T + ct (I - nn^T)
  V3<R> f = (k * pen - cn * vn + (rs ? d * vtg : R(0))) * n - ct * vt;
  V3<R> tq = cross(x, f);
  g[0] -= dt * tq.x; g[1] -= dt * tq.y; g[2] -= dt * tq.z;
  g[3] -= dt * f.x;  g[4] -= dt * f.y;  g[5] -= dt * f.z;
  // C = ct I + (cn - ct) n n^T ; J^T C J = ct * sum_e w_e w_e^T + (cn - ct) w_n w_n^T, e over world axes
  V3<R> xn = cross(x, n);
  R wn[6] = {xn.x, xn.y, xn.z, n.x, n.y, n.z};
  sym_rank1(A, dt * (cn - ct), wn);
  moments_add(fric, dt * ct, x);
}

#if defined(__HIP_DEVICE_COMPILE__)
// Device, fp32: contact_point for two points of a body at once, every arithmetic step on float2 (v_pk_fma/mul/add_f32:
// the pair shares the body velocity, so nothing needs shuffling) into pair accumulators folded once per body.  A
// point not in contact (c0/c1 false) contributes exactly zero.  The same algebra as contact_point; only the
// summation order of the per-body sums differs.
typedef float t1f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ t1f2 t1f2_of(float a, float b) { return t1f2{a, b}; }
struct PairAcc {
  t1f2 A[21];  // dt J^T C J, packed upper triangle (sidx), summed over the pair halves at the end
  t1f2 g[6];   // dt * [torque; force] of the points
  t1f2 m, hx, hy, hz, sxx, syy, szz, sxy, sxz, syz;  // friction point-mass moments (PointMoments)
};
__device__ __forceinline__ void pair_acc_zero(PairAcc& P) {
#pragma unroll
  for (int k = 0; k < 21; ++k) P.A[k] = t1f2{0.0f, 0.0f};
#pragma unroll
  for (int k = 0; k < 6; ++k) P.g[k] = t1f2{0.0f, 0.0f};
  P.m = P.hx = P.hy = P.hz = P.sxx = P.syy = P.szz = P.sxy = P.sxz = P.syz = t1f2{0.0f, 0.0f};
}
__device__ __forceinline__ void contact_pair(const DynModel& M, const V3<float>& x0, const V3<float>& x1, const V3<float>& n0,
                                             const V3<float>& n1, float pen0, float pen1, bool c0, bool c1,
                                             const float Vb[6], float mu, float vtg, float dt, PairAcc& P,
                                             float& amax) {
  const float k = M.k_contact, d = M.d_contact;
  const t1f2 xx = t1f2_of(x0.x, x1.x), xy = t1f2_of(x0.y, x1.y), xz = t1f2_of(x0.z, x1.z);
  const t1f2 nx = t1f2_of(n0.x, n1.x), ny = t1f2_of(n0.y, n1.y), nz = t1f2_of(n0.z, n1.z);
  const t1f2 pen = t1f2_of(c0 ? pen0 : 0.0f, c1 ? pen1 : 0.0f);
  // vp = v_O + omega x x
  const t1f2 vpx = Vb[3] + (Vb[1] * xz - Vb[2] * xy);
  const t1f2 vpy = Vb[4] + (Vb[2] * xx - Vb[0] * xz);
  const t1f2 vpz = Vb[5] + (Vb[0] * xy - Vb[1] * xx);
  const t1f2 vn = nx * vpx + ny * vpy + nz * vpz;
  const t1f2 vtx = vpx - vn * nx, vty = vpy - vn * ny, vtz = vpz - vn * nz;
  const t1f2 vt2 = vtx * vtx + vty * vty + vtz * vtz;
  const float vs = M.friction_vs;
  const float vtn0 = fsqrt(vt2.x), vtn1 = fsqrt(vt2.y);
  // approaching; separating below the restitution target (contact_point)
  const bool ap0 = vn.x < 0.0f, ap1 = vn.y < 0.0f, rs0 = !ap0 && vn.x < vtg, rs1 = !ap1 && vn.y < vtg;
  const t1f2 cn = t1f2_of(c0 ? (ap0 ? dt * k + d : (rs0 ? d : 0.0f)) : 0.0f, c1 ? (ap1 ? dt * k + d : (rs1 ? d : 0.0f)) : 0.0f);
  const t1f2 fn_est = k * pen + t1f2_of(ap0 ? -d * vn.x : (rs0 ? d * (vtg - vn.x) : 0.0f),
                                        ap1 ? -d * vn.y : (rs1 ? d * (vtg - vn.y) : 0.0f));
  const t1f2 ct = mu * fn_est * t1f2_of(c0 ? rcp(vtn0 > vs ? vtn0 : vs) : 0.0f, c1 ? rcp(vtn1 > vs ? vtn1 : vs) : 0.0f);
  if (c0) amax = fmaxf(amax, fmaxf(-vn.x, 0.0f));
  if (c1) amax = fmaxf(amax, fmaxf(-vn.y, 0.0f));
  // force at the current velocity f = (k pen - cn vn + d vtg) n - ct vt, and its moment about O
  const float dv = d * vtg;
  const t1f2 fs = k * pen - cn * vn + t1f2_of(c0 && rs0 ? dv : 0.0f, c1 && rs1 ? dv : 0.0f);
  const t1f2 fx = fs * nx - ct * vtx, fy = fs * ny - ct * vty, fz = fs * nz - ct * vtz;
  P.g[0] += dt * (xy * fz - xz * fy);
  P.g[1] += dt * (xz * fx - xx * fz);
  P.g[2] += dt * (xx * fy - xy * fx);
  P.g[3] += dt * fx;
  P.g[4] += dt * fy;
  P.g[5] += dt * fz;
  // (cn - ct) w_n w_n^T with w_n = [x cross n; n]
  const t1f2 w[6] = {xy * nz - xz * ny, xz * nx - xx * nz, xx * ny - xy * nx, nx, ny, nz};
  const t1f2 cc = dt * (cn - ct);
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const t1f2 ci = cc * w[i];
#pragma unroll
    for (int j = i; j < 6; ++j) P.A[sidx(i, j)] += ci * w[j];
  }
  // friction stiffness ct (I - n n^T) folded as point-mass moments of weight dt ct
  const t1f2 cm = dt * ct, cx = cm * xx, cy = cm * xy, cz = cm * xz;
  P.m += cm; P.hx += cx; P.hy += cy; P.hz += cz;
  P.sxx += cx * xx; P.syy += cy * xy; P.szz += cz * xz;
  P.sxy += cx * xy; P.sxz += cx * xz; P.syz += cy * xz;
}
// fold the pair accumulators into A (Sym6) and g (subtracted, like contact_point)
__device__ __forceinline__ void pair_acc_flush(const PairAcc& P, Sym6<float>& A, float g[6]) {
#pragma unroll
  for (int k = 0; k < 21; ++k) A.a[k] += P.A[k].x + P.A[k].y;
#pragma unroll
  for (int k = 0; k < 6; ++k) g[k] -= P.g[k].x + P.g[k].y;
  PointMoments<float> F;
  F.m = P.m.x + P.m.y; F.hx = P.hx.x + P.hx.y; F.hy = P.hy.x + P.hy.y; F.hz = P.hz.x + P.hz.y;
  F.sxx = P.sxx.x + P.sxx.y; F.syy = P.syy.x + P.syy.y; F.szz = P.szz.x + P.szz.y;
  F.sxy = P.sxy.x + P.sxy.y; F.sxz = P.sxz.x + P.sxz.y; F.syz = P.syz.x + P.syz.y;
  moments_flush(F, A);
}
#endif

// NP points known at compile time: phase 1 transforms every point and queries the terrain with no branch
// in between, so all coordinate (scalar) and height-field (vector) loads issue together and the body pays
// one memory latency instead of one per point; phase 2 runs the contact math for the points in contact
// (on the device in fp32: two points per packed instruction, contact_pair).
#ifndef T1_CONTACT_BATCH
#define T1_CONTACT_BATCH 8
#endif
template <bool HF, int NP, typename R>
T1_HD void body_contact_np(const DynModel& M, const Terrain& T, int c_begin, const M3<R>& Rb, V3<R> pb,
                           V3<R> base_abs, const R Vb[6], R mu, R vtg, R dt, Sym6<R>& A, R g[6], R& amax) {
  constexpr int CH = NP < T1_CONTACT_BATCH ? NP : T1_CONTACT_BATCH;  // points in flight (bounds live registers)
  static_assert(NP % CH == 0, "contact points per body must be a multiple of the batch");
  PointMoments<R> fric;
  moments_zero(fric);
#if defined(__HIP_DEVICE_COMPILE__) && !defined(T1_SCALAR_CONTACT)
  PairAcc pacc;
  if constexpr (std::is_same<R, float>::value && CH % 2 == 0) pair_acc_zero(pacc);
#endif
#pragma unroll
  for (int c0 = 0; c0 < NP; c0 += CH) {
    V3<R> xs[CH];
    R dz[CH], gxs[CH], gys[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int c = c_begin + c0 + i;
      xs[i] = pb + mul(Rb, v3<R>(M.contact_point[c][0], M.contact_point[c][1], M.contact_point[c][2]));
      V3<R> X = xs[i] + base_abs;
      dz[i] = terrain_height<HF>(T, X.x, X.y, gxs[i], gys[i]) - X.z;
    }
    T1_PROF_MARK(16);
#ifdef T1_PHASE_PROF
    __builtin_amdgcn_s_waitcnt(0);  // profiling build: separate the height loads' latency from the math
    T1_PROF_MARK(17);
#endif
#if defined(__HIP_DEVICE_COMPILE__) && !defined(T1_SCALAR_CONTACT)
    if constexpr (std::is_same<R, float>::value && CH % 2 == 0) {
#pragma unroll
      for (int i = 0; i < CH; i += 2) {
        // the pair's inputs as values before the branch: the unrolled pairs' identical bodies may be merged into one
        // block, which then takes phis of these values instead of indexing the arrays (a scratch copy at -O2)
        const V3<R> x0 = xs[i], x1 = xs[i + 1];
        const R dz0 = dz[i], dz1 = dz[i + 1], gx0 = gxs[i], gy0 = gys[i], gx1 = gxs[i + 1], gy1 = gys[i + 1];
        const bool c0 = dz0 > R(0), c1 = dz1 > R(0);  // below the surface (the normal's z is positive)
        if (c0 || c1) {
          const V3<R> n0 = terrain_normal<HF>(gx0, gy0), n1 = terrain_normal<HF>(gx1, gy1);
          contact_pair(M, x0, x1, n0, n1, dz0 * n0.z, dz1 * n1.z, c0, c1, Vb, mu, vtg, dt, pacc, amax);
        }
      }
    } else
#endif
    {
#pragma unroll
      for (int i = 0; i < CH; ++i)
        if (dz[i] > R(0)) {  // below the surface (the normal's z is positive)
          const V3<R> n = terrain_normal<HF>(gxs[i], gys[i]);
          contact_point(M, xs[i], n, dz[i] * n.z, Vb, mu, vtg, dt, A, g, fric, V3<R>{R(0), R(0), R(0)}, &amax);
        }
    }
    T1_PROF_MARK(18);
  }
#if defined(__HIP_DEVICE_COMPILE__) && !defined(T1_SCALAR_CONTACT)
  if constexpr (std::is_same<R, float>::value && CH % 2 == 0) pair_acc_flush(pacc, A, g);
#endif
  moments_flush(fric, A);
}

#if defined(__HIP_DEVICE_COMPILE__) && !defined(T1_SCALAR_CONTACT)
// one pair of queried points into the pair accumulators (contact_apply), every input by value
template <bool HF>
__device__ __forceinline__ void contact_pair_q(const DynModel& M, V3<float> x0, V3<float> x1, float dz0, float dz1,
                                               float gx0, float gy0, float gx1, float gy1, const float Vb[6], float mu,
                                               float vtg, float dt, PairAcc& pacc, float& amax) {
  const bool c0 = dz0 > 0.0f, c1 = dz1 > 0.0f;  // below the surface (the normal's z is positive)
  if (c0 || c1) {
    const V3<float> n0 = terrain_normal<HF>(gx0, gy0), n1 = terrain_normal<HF>(gx1, gy1);
    contact_pair(M, x0, x1, n0, n1, dz0 * n0.z, dz1 * n1.z, c0, c1, Vb, mu, vtg, dt, pacc, amax);
  }
}
#endif

// body_contact_np in two halves, for a caller with independent work to run while the height loads are in flight:
// contact_query (phase 1: transforms and terrain queries, one batch of NP <= T1_CONTACT_BATCH points) and
// contact_apply (phase 2: the contact math), the same operations in the same order.
template <int NP, typename R> struct ContactQuery {
  V3<R> xs[NP];
  R dz[NP], gx[NP], gy[NP];
};
template <bool HF, int NP, typename R>
T1_HD void contact_query(const DynModel& M, const Terrain& T, int c_begin, const M3<R>& Rb, V3<R> pb, V3<R> base_abs,
                         ContactQuery<NP, R>& Q) {
  static_assert(NP <= T1_CONTACT_BATCH, "one batch");
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int c = c_begin + i;
    Q.xs[i] = pb + mul(Rb, v3<R>(M.contact_point[c][0], M.contact_point[c][1], M.contact_point[c][2]));
    V3<R> X = Q.xs[i] + base_abs;
    Q.dz[i] = terrain_height<HF>(T, X.x, X.y, Q.gx[i], Q.gy[i]) - X.z;
  }
}
template <bool HF, int NP, typename R>
T1_HD void contact_apply(const DynModel& M, const ContactQuery<NP, R>& Q, const R Vb[6], R mu, R vtg, R dt, Sym6<R>& A,
                         R g[6], R& amax) {
  PointMoments<R> fric;
  moments_zero(fric);
#if defined(__HIP_DEVICE_COMPILE__) && !defined(T1_SCALAR_CONTACT)
  if constexpr (std::is_same<R, float>::value && NP % 2 == 0) {
    PairAcc pacc;
    pair_acc_zero(pacc);
    // the pairs unrolled by hand, their inputs passed by value (at -O2 the pragma'd loop, and a lambda capturing Q,
    // kept a scratch copy of Q indexed per pair)
    static_assert(NP == 4 || NP == 8, "two or four pairs");
    contact_pair_q<HF>(M, Q.xs[0], Q.xs[1], Q.dz[0], Q.dz[1], Q.gx[0], Q.gy[0], Q.gx[1], Q.gy[1], Vb, mu, vtg, dt, pacc,
                       amax);
    contact_pair_q<HF>(M, Q.xs[2], Q.xs[3], Q.dz[2], Q.dz[3], Q.gx[2], Q.gy[2], Q.gx[3], Q.gy[3], Vb, mu, vtg, dt, pacc,
                       amax);
    if constexpr (NP == 8) {
      contact_pair_q<HF>(M, Q.xs[4], Q.xs[5], Q.dz[4], Q.dz[5], Q.gx[4], Q.gy[4], Q.gx[5], Q.gy[5], Vb, mu, vtg, dt,
                         pacc, amax);
      contact_pair_q<HF>(M, Q.xs[6], Q.xs[7], Q.dz[6], Q.dz[7], Q.gx[6], Q.gy[6], Q.gx[7], Q.gy[7], Vb, mu, vtg, dt,
                         pacc, amax);
    }
    pair_acc_flush(pacc, A, g);
  } else
#endif
  {
#pragma unroll
    for (int i = 0; i < NP; ++i)
      if (Q.dz[i] > R(0)) {
        const V3<R> n = terrain_normal<HF>(Q.gx[i], Q.gy[i]);
        contact_point(M, Q.xs[i], n, Q.dz[i] * n.z, Vb, mu, vtg, dt, A, g, fric, V3<R>{R(0), R(0), R(0)}, &amax);
      }
  }
  moments_flush(fric, A);
}

template <bool HF, typename R>
T1_HD void body_contact_t(const DynModel& M, const Terrain& T, int c_begin, int c_end, const M3<R>& Rb, V3<R> pb,
                          V3<R> base_abs, const R Vb[6], R mu, R vtg, R dt, Sym6<R>& A, R g[6], R& amax) {
  // the T1 model: 8 points per contact body (base box split 4 + 4 between the legs)
  if (c_end - c_begin == 8) return body_contact_np<HF, 8>(M, T, c_begin, Rb, pb, base_abs, Vb, mu, vtg, dt, A, g, amax);
  if (c_end - c_begin == 4) return body_contact_np<HF, 4>(M, T, c_begin, Rb, pb, base_abs, Vb, mu, vtg, dt, A, g, amax);
  PointMoments<R> fric;
  moments_zero(fric);
  for (int c = c_begin; c < c_end; ++c) {
    V3<R> x = pb + mul(Rb, v3<R>(M.contact_point[c][0], M.contact_point[c][1], M.contact_point[c][2]));
    V3<R> X = x + base_abs;
    V3<R> n;
    R h = terrain_height<HF>(T, X.x, X.y, n);
    R pen = (h - X.z) * n.z;
    if (pen > R(0)) contact_point(M, x, n, pen, Vb, mu, vtg, dt, A, g, fric, V3<R>{R(0), R(0), R(0)}, &amax);
  }
  moments_flush(fric, A);
}
// a body's terrain contact (generic layout, host builds) with its restitution episode vimp (updated)
template <typename R>
T1_HD void body_contact(const DynModel& M, const Terrain& T, int c_begin, int c_end, const M3<R>& Rb, V3<R> pb,
                        V3<R> base_abs, const R Vb[6], R mu, R e, R& vimp, R dt, Sym6<R>& A, R g[6]) {
  const R vtg = restitution_target(M, e, vimp);
  R amax = R(-1);
  if (T.type == 0) body_contact_t<false>(M, T, c_begin, c_end, Rb, pb, base_abs, Vb, mu, vtg, dt, A, g, amax);
  else body_contact_t<true>(M, T, c_begin, c_end, Rb, pb, base_abs, Vb, mu, vtg, dt, A, g, amax);
  vimp = restitution_episode(vimp, amax);
}

// contact force (world) a body receives at velocity Vb (used for the net-contact-force report)
template <typename R>
T1_HD V3<R> point_contact_force(const DynModel& M, V3<R> x, V3<R> n, R pen, const R Vb[6], R mu, R vtg,
                                V3<R> vs = V3<R>{R(0), R(0), R(0)}) {
  const R k = R(M.k_contact), d = R(M.d_contact);
  V3<R> om{Vb[0], Vb[1], Vb[2]}, vo{Vb[3], Vb[4], Vb[5]};
  V3<R> vp = vo + cross(om, x) - vs;
  R vn = dot(n, vp);
  V3<R> vt = vp - vn * n;
  R vtn = fsqrt(dot(vt, vt));
  R fn = k * pen - (vn < vtg ? d * (vn - vtg) : R(0));  // approaching, or separating below the restitution target
  fn = fn > R(0) ? fn : R(0);
  R ct = mu * fn * rcp(vtn > R(M.friction_vs) ? vtn : R(M.friction_vs));
  return fn * n - ct * vt;
}
template <bool HF, typename R>
T1_HD V3<R> body_contact_force_t(const DynModel& M, const Terrain& T, int b, const M3<R>& Rb, V3<R> pb,
                                 V3<R> base_abs, const R Vb[6], R mu, R vtg) {
  const int c0 = M.contact_start[b], nc = M.contact_count[b];
  V3<R> F = v3<R>(0, 0, 0);
  const V3<R> W = pb + base_abs;
  if (W.z - R(M.contact_radius[b]) > terrain_bound<HF>(T, W.x, W.y)) return F;
  if (nc == T1_POINTS_PER_BODY) {  // batched: all queries of the body in flight together
    constexpr int NP = T1_POINTS_PER_BODY;
    V3<R> xs[NP];
    R dz[NP], gxs[NP], gys[NP];
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const int c = c0 + i;
      xs[i] = pb + mul(Rb, v3<R>(M.contact_point[c][0], M.contact_point[c][1], M.contact_point[c][2]));
      V3<R> X = xs[i] + base_abs;
      dz[i] = terrain_height<HF>(T, X.x, X.y, gxs[i], gys[i]) - X.z;
    }
#pragma unroll
    for (int i = 0; i < NP; ++i)
      if (dz[i] > R(0)) {
        const V3<R> n = terrain_normal<HF>(gxs[i], gys[i]);
        F = F + point_contact_force(M, xs[i], n, dz[i] * n.z, Vb, mu, vtg);
      }
    return F;
  }
  for (int c = c0; c < c0 + nc; ++c) {
    V3<R> r = v3<R>(M.contact_point[c][0], M.contact_point[c][1], M.contact_point[c][2]);
    V3<R> x = pb + mul(Rb, r);
    V3<R> X = x + base_abs;
    V3<R> n;
    R h = terrain_height<HF>(T, X.x, X.y, n);
    R pen = (h - X.z) * n.z;
    if (pen > R(0)) F = F + point_contact_force(M, x, n, pen, Vb, mu, vtg);
  }
  return F;
}
template <typename R>
T1_HD V3<R> body_contact_force(const DynModel& M, const Terrain& T, int b, const M3<R>& Rb, V3<R> pb,
                               V3<R> base_abs, const R Vb[6], R mu, R vtg) {
  return T.type == 0 ? body_contact_force_t<false>(M, T, b, Rb, pb, base_abs, Vb, mu, vtg)
                     : body_contact_force_t<true>(M, T, b, Rb, pb, base_abs, Vb, mu, vtg);
}

// ---------------------------------------------------------------------------------------------------
// Self-collision between the legs' collision bodies (asset.self_collisions = 0 enables it in the reference,
// t1_dh_stand_config.py:51; PhysX collides every non-adjacent pair of shapes of the articulation).  The bodies that
// carry shapes are the base box, the shanks and the feet; the base box cannot be reached by a shank or a foot within
// the joint limits, which leaves the pairs {left, right} x {shank, foot} across the legs and the
// shank-foot pair within a leg (not adjacent: the ankle-pitch link lies between them).  Volumes: each shank box and
// each foot hull's bounding box as a capsule along its long axis (SelfCapsule, utils/urdf.py), the representation
// legged-robot self-collision usually takes: one closest-point query per pair.  A pair whose capsules overlap is one
// contact at the middle of the overlap, under the same compliant law as the terrain (contact_point, with the other
// body's point velocity as the surface velocity): each body's own terms are implicit (folded into its composite like
// a terrain contact), the other body's motion enters explicitly, and each leg's helper evaluates the pair for its own
// body (the reaction on the other body is the other helper's evaluation of the same pair).
// ---------------------------------------------------------------------------------------------------
template <typename R> T1_HD R clamp01(R x) { return x < R(0) ? R(0) : (x > R(1) ? R(1) : x); }
// Closest points c1, c2 of the segments p1-q1 and p2-q2 (non-degenerate), by selects (no divergent branch).  Crossing
// segments: the unconstrained minimum, then clamped (the convex 2-parameter problem's solution).  Segments within
// ~1.8 deg of parallel (sin^2 < 1e-3; the crossing point is ill-conditioned there, and both legs' shanks are parallel
// whenever the legs mirror each other): the middle of the overlap of segment 2's projection onto segment 1.
template <typename R>
T1_HD void closest_segments(V3<R> p1, V3<R> q1, V3<R> p2, V3<R> q2, V3<R>& c1, V3<R>& c2) {
  const V3<R> d1 = q1 - p1, d2 = q2 - p2, r = p1 - p2;
  const R a = dot(d1, d1), e = dot(d2, d2), f = dot(d2, r), c = dot(d1, r), b = dot(d1, d2);
  const R den = a * e - b * b, ia = rcp(a), ie = rcp(e);
  const bool parallel = den < R(1e-3) * a * e;
  // crossing
  R sx = clamp01((b * f - c * e) * rcp(parallel ? R(1) : den));
  const R tx = (b * sx + f) * ie;
  sx = tx < R(0) ? clamp01(-c * ia) : (tx > R(1) ? clamp01((b - c) * ia) : sx);
  // parallel: segment 2's ends project to s = -c / a and (b - c) / a
  const R s0 = -c * ia, s1 = (b - c) * ia;
  const R sp = R(0.5) * (clamp01(s0 < s1 ? s0 : s1) + clamp01(s0 < s1 ? s1 : s0));
  const R sv = parallel ? sp : sx;
  c1 = p1 + sv * d1;
  c2 = p2 + clamp01(dot(c1 - p2, d2) * ie) * d2;
}
// a capsule in world axes about O: segment p-q, radius r
template <typename R> struct CapPose {
  V3<R> p, q;
  R r;
};
template <typename R> T1_HD CapPose<R> cap_pose(const SelfCapsule& c, const M3<R>& Rb, V3<R> pb) {
  return CapPose<R>{pb + mul(Rb, v3<R>(R(c.a[0]), R(c.a[1]), R(c.a[2]))),
                    pb + mul(Rb, v3<R>(R(c.b[0]), R(c.b[1]), R(c.b[2]))), R(c.r)};
}

template <typename R> T1_HD V3<R> point_velocity(const R V[6], V3<R> x) {
  return v3<R>(V[3], V[4], V[5]) + cross(v3<R>(V[0], V[1], V[2]), x);
}
// The contact of capsule O (own body) with capsule X, if they overlap: x the middle of the overlap, n the unit normal
// pushing O out, pen the overlap depth.  Returns false when apart.  o_first: O is the pair's first body (the left leg's
// across the legs, the shank within a leg); the segments go to closest_segments in that fixed order, so both bodies'
// evaluations of a pair use the same closest points (the near-parallel rule is not symmetric in its arguments).
template <typename R>
T1_HD bool capsule_contact(const CapPose<R>& O, const CapPose<R>& X, bool o_first, V3<R>& x, V3<R>& n, R& pen) {
  V3<R> c1, c2;
  closest_segments(o_first ? O.p : X.p, o_first ? O.q : X.q, o_first ? X.p : O.p, o_first ? X.q : O.q, c1, c2);
  const V3<R> co = o_first ? c1 : c2, cx = o_first ? c2 : c1;
  const V3<R> d = co - cx;
  const R d2 = dot(d, d), rs = O.r + X.r;
  if (!(d2 < rs * rs)) return false;
  const R dist = fsqrt(d2);
  // axes crossing (dist ~ 0): push apart along the line between the segment midpoints (fallback +z)
  const V3<R> m = R(0.5) * (O.p + O.q) - R(0.5) * (X.p + X.q);
  const R mm = dot(m, m);
  n = dist > R(1e-6) ? rcp(dist) * d : (mm > R(1e-12) ? rcp(fsqrt(mm)) * m : v3<R>(R(0), R(0), R(1)));
  pen = rs - dist;
  x = cx + (X.r - R(0.5) * pen) * n;
  return true;
}
// the self-contact terms one body (capsule O, velocity Vo) receives from another (capsule X, velocity Vx)
template <typename R>
T1_HD void self_pair_terms(const DynModel& M, const CapPose<R>& O, const R Vo[6], const CapPose<R>& X, const R Vx[6],
                           bool o_first, R mu, R dt, Sym6<R>& A, R g[6], PointMoments<R>& fric) {
  V3<R> x, n;
  R pen;
  if (capsule_contact(O, X, o_first, x, n, pen)) contact_point(M, x, n, pen, Vo, mu, R(0), dt, A, g, fric, point_velocity(Vx, x));
}
// the self-contact force on body O (the report): that contact's explicit force
template <typename R>
T1_HD V3<R> self_pair_force(const DynModel& M, const CapPose<R>& O, const R Vo[6], const CapPose<R>& X, const R Vx[6],
                            bool o_first, R mu) {
  V3<R> x, n;
  R pen;
  if (!capsule_contact(O, X, o_first, x, n, pen)) return v3<R>(R(0), R(0), R(0));
  return point_contact_force(M, x, n, pen, Vo, mu, R(0), point_velocity(Vx, x));
}
// Pose (rotation, origin about O) and spatial velocity of one contact body, as the kinematics publish them
template <typename R> struct BodyKin {
  M3<R> Rb;
  V3<R> p;
  R V[6];
};
// One body's view for the self-contact terms: its capsule in world axes about O and its spatial velocity.
template <typename R> struct SelfBody {
  CapPose<R> cap;
  R V[6];
};
template <typename R> T1_HD SelfBody<R> self_body(const DynModel& M, int leg, int s, const BodyKin<R>& K) {
  SelfBody<R> B;
  B.cap = cap_pose(M.self_cap[leg][s], K.Rb, K.p);
#pragma unroll
  for (int i = 0; i < 6; ++i) B.V[i] = K.V[i];
  return B;
}
// Self-contact terms of the shank (s = 0) and foot (s = 1) of leg `own` (bodies O) against the other leg's (X):
// accumulated (contact_point's convention) into C[s] / c[s].  mu: the robot's own shapes' friction (the env's; PhysX's
// average of two equal values).  Self-contacts keep no restitution episode (v_tgt = 0): a leg striking the other leg
// faster than the bounce threshold is not given a bounce.
template <typename R>
T1_HD void self_terms_bodies(const DynModel& M, int own, const SelfBody<R> (&O)[2], const SelfBody<R> (&X)[2], R mu, R dt,
                             Sym6<R> (&C)[2], R (&c)[2][6]) {
  // the shank-foot pair within the leg: one query for both bodies (shank first)
  V3<R> xi, ni;
  R peni;
  const bool intra = capsule_contact(O[0].cap, O[1].cap, true, xi, ni, peni);
  // one instantiation per body (a plain loop this large is not unrolled, and its register arrays would go to scratch)
  auto body = [&](auto sc) {
    constexpr int s = decltype(sc)::value;
    PointMoments<R> fric;
    moments_zero(fric);
    self_pair_terms(M, O[s].cap, O[s].V, X[0].cap, X[0].V, own == 0, mu, dt, C[s], c[s], fric);
    self_pair_terms(M, O[s].cap, O[s].V, X[1].cap, X[1].V, own == 0, mu, dt, C[s], c[s], fric);
    if (intra)
      contact_point(M, xi, s == 0 ? ni : R(-1) * ni, peni, O[s].V, mu, R(0), dt, C[s], c[s], fric,
                    point_velocity(O[1 - s].V, xi));
    moments_flush(fric, C[s]);
  };
  body(std::integral_constant<int, 0>{});
  body(std::integral_constant<int, 1>{});
}
// the same from the contact-body kinematics of the two legs (Ko: leg `own`, Kx: the other)
template <typename R>
T1_HD void self_terms_leg(const DynModel& M, int own, const BodyKin<R> (&Ko)[2], const BodyKin<R> (&Kx)[2], R mu, R dt,
                          Sym6<R> (&C)[2], R (&c)[2][6]) {
  SelfBody<R> O[2], X[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    O[s] = self_body(M, own, s, Ko[s]);
    X[s] = self_body(M, 1 - own, s, Kx[s]);
  }
  self_terms_bodies(M, own, O, X, mu, dt, C, c);
}
// the net self-contact forces on the shank / foot of leg `own` (report)
template <typename R>
T1_HD void self_forces_bodies(const DynModel& M, int own, const SelfBody<R> (&O)[2], const SelfBody<R> (&X)[2], R mu,
                              V3<R> (&F)[2]) {
  auto body = [&](auto sc) {
    constexpr int s = decltype(sc)::value;
    F[s] = self_pair_force(M, O[s].cap, O[s].V, X[0].cap, X[0].V, own == 0, mu) +
           self_pair_force(M, O[s].cap, O[s].V, X[1].cap, X[1].V, own == 0, mu) +
           self_pair_force(M, O[s].cap, O[s].V, O[1 - s].cap, O[1 - s].V, s == 0, mu);
  };
  body(std::integral_constant<int, 0>{});
  body(std::integral_constant<int, 1>{});
}
template <typename R>
T1_HD void self_forces_leg(const DynModel& M, int own, const BodyKin<R> (&Ko)[2], const BodyKin<R> (&Kx)[2], R mu,
                           V3<R> (&F)[2]) {
  SelfBody<R> O[2], X[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    O[s] = self_body(M, own, s, Ko[s]);
    X[s] = self_body(M, 1 - own, s, Kx[s]);
  }
  self_forces_bodies(M, own, O, X, mu, F);
}

// ---------------------------------------------------------------------------------------------------
// Per-env state kept in registers across the decimation loop
// ---------------------------------------------------------------------------------------------------
template <typename R> struct BaseState {
  R pos[3];   // base origin, world (absolute)
  R quat[4];  // xyzw
  R w[3];     // base angular velocity, world
  R vo[3];    // base origin velocity, world
};
template <typename R> struct EnvState : BaseState<R> {
  R q[ND], qd[ND];
  R vimp[6];  // restitution episodes of the contact bodies (vimp_shank / vimp_foot / vimp_base)
};

// base quantities of one substep shared by both legs
template <typename R> struct BaseFrame {
  M3<R> R0;
  V3<R> abs;  // O in world coordinates
  R V0[6];    // base spatial velocity about O
};
template <typename R> T1_HD void base_frame(const BaseState<R>& s, BaseFrame<R>& F) {
  F.R0 = quat_to_mat(s.quat[0], s.quat[1], s.quat[2], s.quat[3]);
  F.abs = v3<R>(s.pos[0], s.pos[1], s.pos[2]);
  F.V0[0] = s.w[0]; F.V0[1] = s.w[1]; F.V0[2] = s.w[2];
  F.V0[3] = s.vo[0]; F.V0[4] = s.vo[1]; F.V0[5] = s.vo[2];
}
template <typename R> T1_HD V3<R> base_com(const DynModel& M, const BaseParams<R>& P, const M3<R>& R0) {
  return mul(R0, v3<R>(R(M.com[0][0]) + P.com_disp[0], R(M.com[0][1]) + P.com_disp[1], R(M.com[0][2]) + P.com_disp[2]));
}

// Leg block of the augmented system after assembly / elimination.
template <typename R> struct LegBlock {
  R L[21];      // leg-leg (sym, packed, index (i<=j) over leg dofs 0..5 from root to leaf)
  R Bl[6][6];   // base-leg coupling: Bl[r][j] = A(base r, leg j)
  R rhs[6];
};

// ---------------------------------------------------------------------------------------------------
// base block: the base body's spatial inertia about O, its RNEA bias (gravity as the fictitious base
// acceleration -g) and the external force at the base COM (apply_rigid_body_force_tensors ENV_SPACE).
// ---------------------------------------------------------------------------------------------------
template <typename R>
T1_HD void base_block(const DynModel& M, const BaseParams<R>& P, const BaseFrame<R>& F, V3<R> ext_f, R dt,
                      Sym6<R>& Ac, R gc[6]) {
  const R A0[6] = {R(0), R(0), R(0), R(0), R(0), R(M.gravity)};
  R Icw[6];
  world_inertia(M, 0, F.R0, P.inertia_scale, Icw);
  V3<R> c0 = base_com(M, P, F.R0);
  inertia_spatial(Ac, P.mass, c0, Icw);
  R IA[6], IV[6], vf[6];
  sym_mul(Ac, A0, IA);
  sym_mul(Ac, F.V0, IV);
  crf(F.V0, IV, vf);
  V3<R> tq = cross(c0, ext_f);
  R fe[6] = {tq.x, tq.y, tq.z, ext_f.x, ext_f.y, ext_f.z};
#pragma unroll
  for (int i = 0; i < 6; ++i) gc[i] = dt * (IA[i] + vf[i] - fe[i]);
}

// base-body contact points handled together with leg `leg` (the base's points are split between the legs so
// that the two-wave GPU kernel does each point once)
T1_HD void base_contact_range(const DynModel& M, int leg, int& c_begin, int& c_end) {
  const int c0 = M.contact_start[0], nc = M.contact_count[0];
  c_begin = c0 + (nc * leg) / 2;
  c_end = c0 + (nc * (leg + 1)) / 2;
}

// spatial inertia about O (world axes) of leg body b at pose (Rk, pk)
template <typename R>
T1_HD void body_inertia(const DynModel& M, int b, R mass, R iscale, const M3<R>& Rk, V3<R> pk, Sym6<R>& I) {
  R Icw[6];
  world_inertia(M, b, Rk, iscale, Icw);
  V3<R> c = pk + mul(Rk, v3<R>(M.com[b][0], M.com[b][1], M.com[b][2]));
  inertia_spatial(I, mass, c, Icw);
}

// ---------------------------------------------------------------------------------------------------
// assemble one leg.  Forward pass (root to leaf): poses, velocities, velocity-product accelerations and the
// RNEA bias g_k = dt (I_k a_k + v_k x* I_k v_k).  Backward pass (leaf to root): each body's pose and velocity
// are rebuilt from its child (R_k = R_{k+1} Rot_{k+1}^T, p_k = p_{k+1} - R_k off_{k+1},
// v_k = v_{k+1} - S_{k+1} qd_{k+1}), its inertia and contact stiffness join the composite, and column k of
// the leg block is formed; the off-diagonal H(k, j>k) = S_k . (Ic_j S_j) reuses the stored coupling
// columns.  Only g_k, the joint sin/cos and the leaf pose/velocity cross between the passes (66 floats),
// which is what keeps a leg inside the register file.  Ac_up / gc_up accumulate the leg composite.
// ---------------------------------------------------------------------------------------------------
// joint rotation / motion subspace with the axis known at compile time (AX >= 0) or read from the model
template <int AX, typename R> T1_HD M3<R> joint_rot(const DynModel& M, int b, const M3<R>& A, R c, R s) {
  if constexpr (AX >= 0) return mul_axis_rot_t<AX>(A, c, s);
  else return mul_axis_rot(A, M.axis_idx[b], c, s);
}
template <int AX, typename R> T1_HD void joint_subspace(const DynModel& M, int b, const M3<R>& Rb, V3<R> p, R S[6]) {
  if constexpr (AX >= 0) {
    const R sg = R(M.axis_sign[b]);
    const V3<R> a = v3<R>(sg * Rb.m[AX], sg * Rb.m[3 + AX], sg * Rb.m[6 + AX]);
    const V3<R> l = cross(p, a);
    S[0] = a.x; S[1] = a.y; S[2] = a.z; S[3] = l.x; S[4] = l.y; S[5] = l.z;
  } else {
    BodyState<R> Bk{Rb, p};
    motion_subspace(M, b, Bk, S);
  }
}

// true if p holds on any lane of the wave (wave-uniform); the host runs one env at a time
T1_HD bool t1_wave_any(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ballot(p) != 0;
#else
  return p;
#endif
}
// contact of a body with NP points; `lowest` = its origin height minus its contact radius, `bound` = the
// terrain_bound at its origin (fetched earlier): skipped when the body cannot reach the terrain
// terrain: e = the combined restitution, vimp = the body's restitution episode (updated).
template <int NP, typename R>
T1_HD void body_contact_fixed(const DynModel& M, const Terrain& T, R lowest, int32_t bound_raw, int c_begin,
                              const M3<R>& Rb, V3<R> pb, V3<R> base_abs, const R Vb[6], R mu, R e, R& vimp, R dt,
                              Sym6<R>& A, R g[6]) {
  if (lowest > bound_height<R>(T, bound_raw)) {
    vimp = R(0);  // cannot touch the terrain: no contact episode
    return;
  }
  const R vtg = restitution_target(M, e, vimp);
  R amax = R(-1);
  // a restitution set point is rare (an episode opened above the bounce threshold): a wave with none anywhere runs the
  // law with v_tgt = 0 folded in (the same values: the separation branch is empty at v_tgt = 0), -7% of the step
  if (t1_wave_any(vtg > R(0))) {
    if (T.type == 0) body_contact_np<false, NP>(M, T, c_begin, Rb, pb, base_abs, Vb, mu, vtg, dt, A, g, amax);
    else body_contact_np<true, NP>(M, T, c_begin, Rb, pb, base_abs, Vb, mu, vtg, dt, A, g, amax);
  } else {
    if (T.type == 0) body_contact_np<false, NP>(M, T, c_begin, Rb, pb, base_abs, Vb, mu, R(0), dt, A, g, amax);
    else body_contact_np<true, NP>(M, T, c_begin, Rb, pb, base_abs, Vb, mu, R(0), dt, A, g, amax);
  }
  vimp = restitution_episode(vimp, amax);
}
// body_contact_fixed with the terrain queries already issued (contact_query, possibly before the bound was known:
// a speculative query costs the loads of a body that turns out to be out of reach, and saves the round trip the
// bound test put between the bound's load and the heights' loads); the same operations in the same order
template <bool HF, int NP, typename R>
T1_HD void body_contact_fixed_q(const DynModel& M, const ContactQuery<NP, R>& Q, R lowest, int32_t bound_raw,
                                const Terrain& T, const R Vb[6], R mu, R e, R& vimp, R dt, Sym6<R>& A, R g[6]) {
  if (lowest > bound_height<R>(T, bound_raw)) {
    vimp = R(0);  // cannot touch the terrain: no contact episode
    return;
  }
  const R vtg = restitution_target(M, e, vimp);
  R amax = R(-1);
#ifdef T1_CONTACT_ONE_COPY  // one copy of the contact law (k_dyn6's unit: see t1env_dyn6.hip)
  contact_apply<HF, NP>(M, Q, Vb, mu, vtg, dt, A, g, amax);
#else
  if (t1_wave_any(vtg > R(0))) contact_apply<HF, NP>(M, Q, Vb, mu, vtg, dt, A, g, amax);
  else contact_apply<HF, NP>(M, Q, Vb, mu, R(0), dt, A, g, amax);
#endif
  vimp = restitution_episode(vimp, amax);
}
// body_contact_fixed for a body that is always evaluated (no height bound), with `between()` run after its terrain
// queries are issued and before their heights are used (the helper's self-contact terms hide the load latency)
template <int NP, typename R, typename Between>
T1_HD void body_contact_query_apply(const DynModel& M, const Terrain& T, int c_begin, const M3<R>& Rb, V3<R> pb,
                                    V3<R> base_abs, const R Vb[6], R mu, R e, R& vimp, R dt, Sym6<R>& A, R g[6],
                                    Between&& between) {
  ContactQuery<NP, R> Q;
  if (T.type == 0) contact_query<false, NP>(M, T, c_begin, Rb, pb, base_abs, Q);
  else contact_query<true, NP>(M, T, c_begin, Rb, pb, base_abs, Q);
  between();
  const R vtg = restitution_target(M, e, vimp);
  R amax = R(-1);
  if (t1_wave_any(vtg > R(0))) {
    if (T.type == 0) contact_apply<false, NP>(M, Q, Vb, mu, vtg, dt, A, g, amax);
    else contact_apply<true, NP>(M, Q, Vb, mu, vtg, dt, A, g, amax);
  } else {
    if (T.type == 0) contact_apply<false, NP>(M, Q, Vb, mu, R(0), dt, A, g, amax);
    else contact_apply<true, NP>(M, Q, Vb, mu, R(0), dt, A, g, amax);
  }
  vimp = restitution_episode(vimp, amax);
}
// slots of an env's restitution episodes (t1env_buffers.contact_vimp, EnvState::vimp): the shank and the foot of each
// leg, and the base box's two halves (one per leg: base_contact_range)
T1_HD constexpr int vimp_shank(int leg) { return 2 * leg; }
T1_HD constexpr int vimp_foot(int leg) { return 2 * leg + 1; }
T1_HD constexpr int vimp_base(int leg) { return 4 + leg; }
constexpr int NVIMP = 6;

template <int K> using kconst = std::integral_constant<int, K>;

// selfC / selfc: the self-contact terms of the leg's shank [0] and foot [1] (self_terms_leg), or null
// vimp_leg: the restitution episodes of the leg's shank [0] and foot [1] (updated)
template <int CM, typename R>
T1_HD void leg_assemble(const DynModel& M, const Terrain& T, const LegParams<R>& P, R mu, R e, R (&vimp_leg)[2],
                        const BaseFrame<R>& F, const R q[NLEG], const R qd[NLEG], const R tau[NLEG], int leg, R dt,
                        LegBlock<R>& out, Sym6<R>& Ac_up, R gc_up[6], const Sym6<R>* selfC = nullptr,
                        const R (*selfc)[6] = nullptr) {
  R sn[NLEG], cs[NLEG], g[NLEG][6];
  M3<R> Rk = F.R0;
  V3<R> pk = v3<R>(0, 0, 0);
  R V[6], A[6], Sk[6];
  R lowest[NLEG];  // contact bodies (fixed layout): origin height - radius, and the terrain bound sample
  int32_t bound[NLEG];  // fetched in the forward pass, tested in the backward pass
#pragma unroll
  for (int i = 0; i < 6; ++i) { V[i] = F.V0[i]; A[i] = R(0); }
  A[5] = R(M.gravity);
  auto fwd = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int AX = CM >= 0 ? T1_LEG_AXIS[k] : -1;
    const int b = 1 + 6 * leg + k;
    pk = pk + mul(Rk, v3<R>(M.joint_offset[b][0], M.joint_offset[b][1], M.joint_offset[b][2]));
    fsincos(R(M.axis_sign[b]) * q[k], &sn[k], &cs[k]);
    Rk = joint_rot<AX>(M, b, Rk, cs[k], sn[k]);
    if constexpr (CM >= 0 && ((CM >> k) & 1)) {
      lowest[k] = pk.z + F.abs.z - R(M.contact_radius[b]);
      bound[k] = terrain_bound_raw_any(T, pk.x + F.abs.x, pk.y + F.abs.y);
    }
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
    Sym6<R> I;
    body_inertia(M, b, P.mass[k], P.inertia_scale[k], Rk, pk, I);
    R IA[6], IV[6], vf[6];
    sym_mul(I, A, IA);
    sym_mul(I, V, IV);
    crf(V, IV, vf);
#pragma unroll
    for (int i = 0; i < 6; ++i) g[k][i] = dt * (IA[i] + vf[i]);
  };
  fwd(kconst<0>{});
  fwd(kconst<1>{});
  fwd(kconst<2>{});
  fwd(kconst<3>{});
  fwd(kconst<4>{});
  fwd(kconst<5>{});
  T1_PROF_MARK(1);
  Sym6<R> Ac;
  sym_zero(Ac);
  R gc[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
  // one instantiation per body (leaf first): every array index below is a compile-time constant
  auto step = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const int b = 1 + 6 * leg + k, j = 6 * leg + k;
    if constexpr (k < NLEG - 1) {  // step up from child k+1 (Sk still holds S_{k+1})
      constexpr int AXC = CM >= 0 ? T1_LEG_AXIS[k + 1] : -1;
      const int bc = b + 1;
#pragma unroll
      for (int i = 0; i < 6; ++i) V[i] -= Sk[i] * qd[k + 1];
      Rk = joint_rot<AXC>(M, bc, Rk, cs[k + 1], -sn[k + 1]);
      pk = pk - mul(Rk, v3<R>(M.joint_offset[bc][0], M.joint_offset[bc][1], M.joint_offset[bc][2]));
    }
    joint_subspace<(CM >= 0 ? T1_LEG_AXIS[k] : -1)>(M, b, Rk, pk, Sk);
    {
      Sym6<R> I;
      body_inertia(M, b, P.mass[k], P.inertia_scale[k], Rk, pk, I);
      sym_add(Ac, I);
    }
    if constexpr (CM >= 0) {
      if constexpr ((CM >> k) & 1) {
        T1_PROF_MARK(2);
        body_contact_fixed<T1_POINTS_PER_BODY>(M, T, lowest[k], bound[k], M.contact_start[b], Rk, pk, F.abs, V, mu,
                                               e, vimp_leg[k == NLEG - 1 ? 1 : 0], dt, Ac, gc);
        if (selfC) {
          constexpr int sfs = k == NLEG - 1 ? 1 : 0;  // shank (k = 3) -> 0, foot (k = 5) -> 1
          sym_add(Ac, selfC[sfs]);
#pragma unroll
          for (int i = 0; i < 6; ++i) gc[i] += selfc[sfs][i];
        }
        T1_PROF_MARK(3);
      }
    } else {
      const int c0 = M.contact_start[b], nc = M.contact_count[b];
      if (nc > 0) {  // the T1's contact bodies of a leg are the shank and the foot; others keep no episode
        R dummy = R(0);
        R& vi = k == 3 ? vimp_leg[0] : (k == NLEG - 1 ? vimp_leg[1] : dummy);
        body_contact(M, T, c0, c0 + nc, Rk, pk, F.abs, V, mu, e, vi, dt, Ac, gc);
      }
      if (selfC && (k == 3 || k == NLEG - 1)) {  // the T1's self-collision bodies: shank, foot
        const int sfs = k == NLEG - 1 ? 1 : 0;
        sym_add(Ac, selfC[sfs]);
        for (int i = 0; i < 6; ++i) gc[i] += selfc[sfs][i];
      }
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) gc[i] += g[k][i];
    R Fk[6];
    sym_mul(Ac, Sk, Fk);
    // diagonal (+ armature + soft joint limit)
    R Ajj = dot6(Sk, Fk) + P.armature[k];
    R rj = dt * tau[k] - dot6(Sk, gc);
    R lo = R(M.q_lower[j]), hi = R(M.q_upper[j]);
    R qj = q[k], qdj = qd[k];
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
    for (int jj = k + 1; jj < NLEG; ++jj) {
      R Fj[6] = {out.Bl[0][jj], out.Bl[1][jj], out.Bl[2][jj], out.Bl[3][jj], out.Bl[4][jj], out.Bl[5][jj]};
      out.L[sidx(k, jj)] = dot6(Sk, Fj);
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) out.Bl[r][k] = Fk[r];
  };
  static_assert(NLEG == 6, "backward pass is written out for 6-DOF legs");
  step(kconst<5>{});
  step(kconst<4>{});
  step(kconst<3>{});
  step(kconst<2>{});
  step(kconst<1>{});
  step(kconst<0>{});
  sym_add(Ac_up, Ac);
#pragma unroll
  for (int i = 0; i < 6; ++i) gc_up[i] += gc[i];
}

// Eliminate a leg's 6 DOF (leaf first) into the base block: Featherstone LTDL restricted to the path
// [base 0..5, leg 0..5].  On return out.L/Bl hold the unit factor L (off-diagonal), L's diagonal holds
// 1/D, Abb and rhs_b hold the Schur-complement updates, and out.rhs the forward-substituted leg rhs.
// The Schur updates do not depend on Abb's value, so a leg can be eliminated into its own contribution.
template <typename R> T1_HD void eliminate_leg(LegBlock<R>& lb, Sym6<R>& Abb, R rhs_b[6]) {
#pragma unroll
  for (int k = NLEG - 1; k >= 0; --k) {
    const R inv = rcp(lb.L[sidx(k, k)]);
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
    lb.L[sidx(k, k)] = inv;
#pragma unroll
    for (int i = 0; i < k; ++i) lb.L[sidx(i, k)] = a_leg[i];
#pragma unroll
    for (int r = 0; r < 6; ++r) lb.Bl[r][k] = a_base[r];
  }
}

// dense LDL^T of the 6x6 base block with the same (leaf-first) convention and solve in place.
template <typename R> T1_HD void solve_base(Sym6<R>& A, R b[6]) {
  R invd[6];
#pragma unroll
  for (int k = 5; k >= 0; --k) {
    const R inv = rcp(A.a[sidx(k, k)]);
    invd[k] = inv;
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
  for (int k = 0; k < 6; ++k) b[k] *= invd[k];
#pragma unroll
  for (int k = 0; k < 6; ++k)
#pragma unroll
    for (int i = 0; i < k; ++i) b[k] -= A.a[sidx(i, k)] * b[i];
}

// back substitution for a leg once the base solution x_b is known: x_k = rhs_k / D_k - sum_anc L_ki x_i
template <typename R> T1_HD void backsub_leg(const LegBlock<R>& lb, const R xb[6], R x[NLEG]) {
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    R v = lb.rhs[k] * lb.L[sidx(k, k)];
#pragma unroll
    for (int r = 0; r < 6; ++r) v -= lb.Bl[r][k] * xb[r];
#pragma unroll
    for (int i = 0; i < k; ++i) v -= lb.L[sidx(i, k)] * x[i];
    x[k] = v;
  }
}

// One leg's contribution to the base block: base-contact share + leg composite - Schur complement.
// Returns the factored leg block (for backsub_leg) and (Ab, rb) to be summed into the base system.
template <int CM = -1, typename R>
T1_HD void leg_contribution(const DynModel& M, const Terrain& T, const BaseParams<R>& PB, const LegParams<R>& PL,
                            const BaseFrame<R>& F, const R q[NLEG], const R qd[NLEG], const R tau[NLEG], int leg,
                            R dt, LegBlock<R>& lb, Sym6<R>& Ab, R rb[6], R (&vimp)[NVIMP],
                            const Sym6<R>* selfC = nullptr, const R (*selfc)[6] = nullptr) {
  sym_zero(Ab);
  R g[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
  const R e = ground_restitution(M, PB.restitution);
  const int32_t base_bound = CM >= 0 ? terrain_bound_raw_any(T, F.abs.x, F.abs.y) : 0;  // tested after the leg pass
  R vl[2] = {vimp[vimp_shank(leg)], vimp[vimp_foot(leg)]};
  leg_assemble<CM>(M, T, PL, PB.friction, e, vl, F, q, qd, tau, leg, dt, lb, Ab, g, selfC, selfc);
  vimp[vimp_shank(leg)] = vl[0];
  vimp[vimp_foot(leg)] = vl[1];
  T1_PROF_MARK(2);
#pragma unroll
  for (int i = 0; i < 6; ++i) rb[i] = -g[i];
  eliminate_leg(lb, Ab, rb);
  T1_PROF_MARK(4);
  int cb, ce;
  base_contact_range(M, leg, cb, ce);
  R gw[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
  if constexpr (CM >= 0) {
    body_contact_fixed<T1_POINTS_PER_BODY / 2>(M, T, F.abs.z - R(M.contact_radius[0]), base_bound, cb, F.R0,
                                               v3<R>(0, 0, 0), F.abs, F.V0, PB.friction, e, vimp[vimp_base(leg)], dt,
                                               Ab, gw);
  } else {
    if (ce > cb)
      body_contact(M, T, cb, ce, F.R0, v3<R>(0, 0, 0), F.abs, F.V0, PB.friction, e, vimp[vimp_base(leg)], dt, Ab, gw);
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) rb[i] -= gw[i];
  T1_PROF_MARK(5);
}

// RNEA bias of one body, g = dt (I A + V x* I V) about O, evaluated at the body's COM instead of through the 6x6
// spatial inertia: with c the COM (rel. O), Icw its world inertia about the COM, V = [w; v_O], A = [alpha; a_O]
// (spatial), the classical COM acceleration is a_c = a_O + alpha x c + w x (v_O + w x c), so
//   g = dt [ Icw alpha + w x (Icw w) + c x (m a_c) ;  m a_c ]
// (Newton-Euler about the COM moved to O) -- the same vector in about 70 % of the arithmetic.
template <typename R>
T1_HD void rnea_bias_com(R m, V3<R> c, const R Icw[6] /*xx yy zz xy xz yz*/, const R V[6], const R A[6], R dt,
                         R g[6]) {
  const V3<R> w{V[0], V[1], V[2]}, al{A[0], A[1], A[2]};
  const V3<R> vc = v3<R>(V[3], V[4], V[5]) + cross(w, c);
  const V3<R> ac = v3<R>(A[3], A[4], A[5]) + cross(al, c) + cross(w, vc);
  const V3<R> f = m * ac;
  const V3<R> Lw{Icw[0] * w.x + Icw[3] * w.y + Icw[4] * w.z, Icw[3] * w.x + Icw[1] * w.y + Icw[5] * w.z,
                 Icw[4] * w.x + Icw[5] * w.y + Icw[2] * w.z};
  const V3<R> La{Icw[0] * al.x + Icw[3] * al.y + Icw[4] * al.z, Icw[3] * al.x + Icw[1] * al.y + Icw[5] * al.z,
                 Icw[4] * al.x + Icw[5] * al.y + Icw[2] * al.z};
  const V3<R> n = La + cross(w, Lw) + cross(c, f);
  g[0] = dt * n.x; g[1] = dt * n.y; g[2] = dt * n.z;
  g[3] = dt * f.x; g[4] = dt * f.y; g[5] = dt * f.z;
}

// Composite rigid-body inertia about O in its 10-parameter form: mass, first moment h = sum m c, and the
// rotational inertia about O, J = sum Icw + m (|c|^2 I - c c^T) (xx yy zz xy xz yz).  Sums of rigid bodies stay
// in this form, and its product with a motion vector needs 30 operations instead of a Sym6's 36.
template <typename R> struct Composite {
  R m, h[3], J[6];
};
template <typename R> T1_HD void composite_zero(Composite<R>& K) {
  K.m = R(0);
  K.h[0] = K.h[1] = K.h[2] = R(0);
#pragma unroll
  for (int i = 0; i < 6; ++i) K.J[i] = R(0);
}
template <typename R> T1_HD void composite_add(Composite<R>& K, R m, V3<R> c, const R Icw[6]) {
  const R cc = dot(c, c);
  const R mx = m * c.x, my = m * c.y, mz = m * c.z;
  K.m += m;
  K.h[0] += mx; K.h[1] += my; K.h[2] += mz;
  K.J[0] += Icw[0] + (m * cc - mx * c.x);
  K.J[1] += Icw[1] + (m * cc - my * c.y);
  K.J[2] += Icw[2] + (m * cc - mz * c.z);
  K.J[3] += Icw[3] - mx * c.y;
  K.J[4] += Icw[4] - mx * c.z;
  K.J[5] += Icw[5] - my * c.z;
}
// F = K S for a motion vector S = [a; l]:  [J a + h x l ; m l - h x a]
template <typename R> T1_HD void composite_mul(const Composite<R>& K, const R S[6], R F[6]) {
  const V3<R> a{S[0], S[1], S[2]}, l{S[3], S[4], S[5]}, h{K.h[0], K.h[1], K.h[2]};
  const V3<R> hl = cross(h, l), ha = cross(h, a);
  F[0] = K.J[0] * a.x + K.J[3] * a.y + K.J[4] * a.z + hl.x;
  F[1] = K.J[3] * a.x + K.J[1] * a.y + K.J[5] * a.z + hl.y;
  F[2] = K.J[4] * a.x + K.J[5] * a.y + K.J[2] * a.z + hl.z;
  F[3] = K.m * l.x - ha.x;
  F[4] = K.m * l.y - ha.y;
  F[5] = K.m * l.z - ha.z;
}
// S += K as a packed symmetric 6x6 ([[J, [h]x], [[h]x^T, m I]], the layout of inertia_spatial)
template <typename R> T1_HD void composite_to_sym(const Composite<R>& K, Sym6<R>& S) {
  S.a[sidx(0, 0)] += K.J[0]; S.a[sidx(1, 1)] += K.J[1]; S.a[sidx(2, 2)] += K.J[2];
  S.a[sidx(0, 1)] += K.J[3]; S.a[sidx(0, 2)] += K.J[4]; S.a[sidx(1, 2)] += K.J[5];
  S.a[sidx(0, 4)] -= K.h[2]; S.a[sidx(0, 5)] += K.h[1];
  S.a[sidx(1, 3)] += K.h[2]; S.a[sidx(1, 5)] -= K.h[0];
  S.a[sidx(2, 3)] -= K.h[1]; S.a[sidx(2, 4)] += K.h[0];
  S.a[sidx(3, 3)] += K.m; S.a[sidx(4, 4)] += K.m; S.a[sidx(5, 5)] += K.m;
}

// ---------------------------------------------------------------------------------------------------
// Leg assembly split for the 4-wave kernel (t1env_dynamics.hip k_dyn4): the leg wave runs the articulated-
// body passes without contact (leg_forward_nc, leg_backward_nc) while a helper wave computes the contact terms
// of the leg's contact bodies from the poses the forward pass publishes; leg_apply_contacts then folds them
// in.  Exact algebra, in world axes about O: the composite of body k is Ic_k = Ic0_k + Cs_k with
// Cs_k = sum over contact bodies c >= k of C_c (C_c = dt J^T C J of body c's points, c_c its impulse wrench,
// cs_k likewise), so every quantity of the backward pass is its contact-free value plus a linear term:
//   F_k = F0_k + Cs_k S_k,   D_k = D0_k + S_k.Cs_k S_k,   H(k,j) = H0(k,j) + S_k.Cs_j S_j  (j > k),
//   r_k = r0_k + dt tau_k - S_k.cs_k,   leg composite += sum_c C_c, bias += sum_c c_c.
// Same system as leg_assemble up to fp32 summation order (tests/test_gpu_dynamics.py bounds both).
// ---------------------------------------------------------------------------------------------------
template <typename R> struct LegPass {
  R sn[NLEG], cs[NLEG], g[NLEG][6];  // joint sin/cos, RNEA bias per body
  M3<R> Rk;                           // leaf pose after the forward pass
  V3<R> pk;
  R S[NLEG][6];                       // motion subspaces, filled by the backward pass
};

// forward pass (root to leaf) without contact: poses, velocities and the RNEA bias of every body;
// pub(kconst<k>, R_k, p_k, V_k) is called for every contact body k of the CM mask.  (Evaluating the bias in the
// backward pass instead, rebuilding each body's velocity and acceleration from its child's, publishes the poses
// earlier but measured 14 % slower: the backward pass is the register-pressure peak.)
template <int CM, typename R, typename Pub>
T1_HD void leg_forward_nc(const DynModel& M, const LegParams<R>& P, const BaseFrame<R>& F, const R q[NLEG],
                          const R qd[NLEG], int leg, R dt, LegPass<R>& st, Pub&& pub) {
  M3<R> Rk = F.R0;
  V3<R> pk = v3<R>(0, 0, 0);
  R V[6], A[6], Sk[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) { V[i] = F.V0[i]; A[i] = R(0); }
  A[5] = R(M.gravity);
  auto fwd = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int AX = T1_LEG_AXIS[k];
    const int b = 1 + 6 * leg + k;
    pk = pk + mul(Rk, v3<R>(M.joint_offset[b][0], M.joint_offset[b][1], M.joint_offset[b][2]));
    fsincos(R(M.axis_sign[b]) * q[k], &st.sn[k], &st.cs[k]);
    Rk = joint_rot<AX>(M, b, Rk, st.cs[k], st.sn[k]);
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
    if constexpr ((CM >> k) & 1) pub(kc, Rk, pk, V);
    R Icw[6];
#ifdef T1_WHATIF_FWD_NOROT
    world_inertia_unrotated(M, b, P.inertia_scale[k], Icw);
#else
    world_inertia(M, b, Rk, P.inertia_scale[k], Icw);
#endif
    const V3<R> c = pk + mul(Rk, v3<R>(M.com[b][0], M.com[b][1], M.com[b][2]));
    rnea_bias_com(P.mass[k], c, Icw, V, A, dt, st.g[k]);
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

// The contact bodies' poses and spatial velocities from the joint state, by the operations leg_forward_nc uses for
// them (no RNEA bias, no inertia): lets the contact helper wave of k_dyn4 start from the substep's state instead of
// waiting for the leg wave's forward pass.  pub(kconst<k>, R_k, p_k, V_k) for every contact body k of CM.
template <int CM, typename R, typename Pub>
T1_HD void leg_contact_kinematics(const DynModel& M, const BaseFrame<R>& F, const R q[NLEG], const R qd[NLEG], int leg,
                                  Pub&& pub) {
  M3<R> Rk = F.R0;
  V3<R> pk = v3<R>(0, 0, 0);
  R V[6], Sk[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) V[i] = F.V0[i];
  auto fwd = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int AX = T1_LEG_AXIS[k];
    const int b = 1 + 6 * leg + k;
    pk = pk + mul(Rk, v3<R>(M.joint_offset[b][0], M.joint_offset[b][1], M.joint_offset[b][2]));
    R sn, cs;
    fsincos(R(M.axis_sign[b]) * q[k], &sn, &cs);
    Rk = joint_rot<AX>(M, b, Rk, cs, sn);
    joint_subspace<AX>(M, b, Rk, pk, Sk);
#pragma unroll
    for (int i = 0; i < 6; ++i) V[i] += Sk[i] * qd[k];
    if constexpr ((CM >> k) & 1) pub(kc, Rk, pk, V);
  };
  fwd(kconst<0>{});
  fwd(kconst<1>{});
  fwd(kconst<2>{});
  fwd(kconst<3>{});
  fwd(kconst<4>{});
  fwd(kconst<5>{});
}

// one leg's contact-body kinematics (shank [0], foot [1]) from its joint state
template <typename R>
T1_HD void leg_body_kinematics(const DynModel& M, const BaseFrame<R>& F, const R q[NLEG], const R qd[NLEG], int leg,
                               BodyKin<R> (&K)[2]) {
  leg_contact_kinematics<T1_LEG_CONTACT_MASK>(M, F, q, qd, leg, [&](auto kc, const M3<R>& Rk, V3<R> pk, const R* V) {
    constexpr int i = decltype(kc)::value == NLEG - 1 ? 1 : 0;
    K[i].Rb = Rk;
    K[i].p = pk;
#pragma unroll
    for (int j = 0; j < 6; ++j) K[i].V[j] = V[j];
  });
}
// both legs' contact-body kinematics (shank [0], foot [1]) from the env's joint state
template <typename R>
T1_HD void contact_body_kinematics(const DynModel& M, const BaseFrame<R>& F, const R q[ND], const R qd[ND],
                                   BodyKin<R> (&K)[2][2]) {
  for (int leg = 0; leg < 2; ++leg)
    leg_contact_kinematics<T1_LEG_CONTACT_MASK>(M, F, q + 6 * leg, qd + 6 * leg, leg,
                                                [&](auto kc, const M3<R>& Rk, V3<R> pk, const R* V) {
                                                  constexpr int i = decltype(kc)::value == NLEG - 1 ? 1 : 0;
                                                  K[leg][i].Rb = Rk;
                                                  K[leg][i].p = pk;
                                                  for (int j = 0; j < 6; ++j) K[leg][i].V[j] = V[j];
                                                });
}
// self-contact terms of all four contact bodies [leg][shank, foot] (zero when self-collision is off)
template <typename R> struct SelfTerms {
  Sym6<R> C[2][2];
  R c[2][2][6];
};
template <typename R>
T1_HD void self_terms_env(const DynModel& M, const BaseFrame<R>& F, const R q[ND], const R qd[ND],
                          const BaseParams<R>& PB, R dt, SelfTerms<R>& S) {
  for (int l = 0; l < 2; ++l)
    for (int i = 0; i < 2; ++i) {
      sym_zero(S.C[l][i]);
      for (int j = 0; j < 6; ++j) S.c[l][i][j] = R(0);
    }
  if (!M.self_collisions) return;
  BodyKin<R> K[2][2];
  contact_body_kinematics(M, F, q, qd, K);
  for (int leg = 0; leg < 2; ++leg)
    self_terms_leg(M, leg, K[leg], K[1 - leg], PB.self_friction, dt, S.C[leg], S.c[leg]);
}

// backward pass (leaf to root) without contact and without the joint torque: D0, H0, F0 = Bl, r0 and the
// contact-free leg composite; stores each S_k for leg_apply_contacts
template <typename R>
T1_HD void leg_backward_nc(const DynModel& M, const LegParams<R>& P, const R q[NLEG], const R qd[NLEG], int leg,
                           R dt, LegPass<R>& st, LegBlock<R>& out, Sym6<R>& Ac_up, R gc_up[6]) {
  M3<R> Rk = st.Rk;
  V3<R> pk = st.pk;
  Composite<R> Ac;
  composite_zero(Ac);
  R gc[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
  auto step = [&](auto kc) {
    constexpr int k = decltype(kc)::value;
    const int b = 1 + 6 * leg + k, j = 6 * leg + k;
    if constexpr (k < NLEG - 1) {  // step up from child k+1
      constexpr int AXC = T1_LEG_AXIS[k + 1];
      const int bc = b + 1;
      Rk = joint_rot<AXC>(M, bc, Rk, st.cs[k + 1], -st.sn[k + 1]);
      pk = pk - mul(Rk, v3<R>(M.joint_offset[bc][0], M.joint_offset[bc][1], M.joint_offset[bc][2]));
    }
    R* Sk = st.S[k];
    joint_subspace<T1_LEG_AXIS[k]>(M, b, Rk, pk, Sk);
    {
      R Icw[6];
#ifdef T1_WHATIF_BWD_NOROT
      world_inertia_unrotated(M, b, P.inertia_scale[k], Icw);
#else
      world_inertia(M, b, Rk, P.inertia_scale[k], Icw);
#endif
      const V3<R> c = pk + mul(Rk, v3<R>(M.com[b][0], M.com[b][1], M.com[b][2]));
      composite_add(Ac, P.mass[k], c, Icw);
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) gc[i] += st.g[k][i];
    R Fk[6];
    composite_mul(Ac, Sk, Fk);
    R Ajj = dot6(Sk, Fk) + P.armature[k];
    R rj = -dot6(Sk, gc);
    const R lo = R(M.q_lower[j]), hi = R(M.q_upper[j]);
    const R qj = q[k], qdj = qd[k];
    if (qj < lo) {
      const R cl = qdj < R(0) ? dt * R(M.k_limit) + R(M.d_limit) : R(0);
      Ajj += dt * cl;
      rj += dt * (R(M.k_limit) * (lo - qj) - cl * qdj);
    } else if (qj > hi) {
      const R cl = qdj > R(0) ? dt * R(M.k_limit) + R(M.d_limit) : R(0);
      Ajj += dt * cl;
      rj += dt * (R(M.k_limit) * (hi - qj) - cl * qdj);
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
  step(kconst<5>{});
  step(kconst<4>{});
  step(kconst<3>{});
  step(kconst<2>{});
  step(kconst<1>{});
  step(kconst<0>{});
  composite_to_sym(Ac, Ac_up);
#pragma unroll
  for (int i = 0; i < 6; ++i) gc_up[i] += gc[i];
}

// fold the contact terms of contact bodies K0 < K1 (C0/c0, C1/c1) and the joint torques into the contact-free
// backward-pass result (see above)
template <int K0, int K1, typename R>
T1_HD void leg_apply_contacts(const Sym6<R>& C0, const R c0[6], const Sym6<R>& C1, const R c1[6],
                              const R tau[NLEG], R dt, const LegPass<R>& st, LegBlock<R>& out, Sym6<R>& Ac_up,
                              R gc_up[6]) {
  static_assert(0 <= K0 && K0 < K1 && K1 < NLEG, "contact bodies K0 < K1 of the leg");
  Sym6<R> Cs = C0;
  sym_add(Cs, C1);
  R cs[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) cs[i] = c0[i] + c1[i];
  R u[NLEG][6];  // Cs_k S_k
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    if (k <= K0) sym_mul(Cs, st.S[k], u[k]);
    else if (k <= K1) sym_mul(C1, st.S[k], u[k]);
    else
#pragma unroll
      for (int i = 0; i < 6; ++i) u[k][i] = R(0);
  }
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    const R sc = k <= K0 ? dot6(st.S[k], cs) : (k <= K1 ? dot6(st.S[k], c1) : R(0));
    out.L[sidx(k, k)] += dot6(st.S[k], u[k]);
    out.rhs[k] += dt * tau[k] - sc;
#pragma unroll
    for (int jj = k + 1; jj < NLEG; ++jj) out.L[sidx(k, jj)] += dot6(st.S[k], u[jj]);
  }
#pragma unroll
  for (int k = 0; k < NLEG; ++k)
#pragma unroll
    for (int r = 0; r < 6; ++r) out.Bl[r][k] += u[k][r];
  sym_add(Ac_up, Cs);
#pragma unroll
  for (int i = 0; i < 6; ++i) gc_up[i] += cs[i];
}

// Semi-implicit Euler of the base with the solved velocity change (+ the omega x v term that turns the
// spatial base acceleration into the classical acceleration of the base origin).
template <typename R> T1_HD void integrate_base(BaseState<R>& s, const R delta[6], R dt) {
  V3<R> w_new = v3<R>(s.w[0] + delta[0], s.w[1] + delta[1], s.w[2] + delta[2]);
  V3<R> vO_new = v3<R>(s.vo[0] + delta[3], s.vo[1] + delta[4], s.vo[2] + delta[5]);
  V3<R> vb_new = vO_new + dt * cross(w_new, vO_new);
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
  R inv = rcp(fsqrt(nx * nx + ny * ny + nz * nz + nw * nw));
  s.quat[0] = nx * inv; s.quat[1] = ny * inv; s.quat[2] = nz * inv; s.quat[3] = nw * inv;
}
// joint speeds clamped to the URDF velocity limit like PhysX max joint velocity
template <typename R>
T1_HD void integrate_leg(const DynModel& M, int leg, R q[NLEG], R qd[NLEG], const R delta[NLEG], R dt) {
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    R v = qd[k] + delta[k];
    R vl = R(M.vel_limit[6 * leg + k]);
    v = v > vl ? vl : (v < -vl ? -vl : v);
    qd[k] = v;
    q[k] += dt * v;
  }
}

// ---------------------------------------------------------------------------------------------------
// Whole-env substep on one thread (host build / fp64 checks): delta = change of u = [omega, v_O (spatial,
// about the fixed point O), qd] over dt, including implicit contact / joint-limit terms.
// ---------------------------------------------------------------------------------------------------
template <typename R>
T1_HD void compute_delta(const DynModel& M, const Terrain& T, const EnvParams<R>& P, EnvState<R>& s,
                         const R tau[ND], V3<R> ext_f, R dt, R delta[6 + ND]) {
  BaseFrame<R> F;
  base_frame(s, F);
  Sym6<R> Ac;
  R gc[6];
  base_block(M, P.base, F, ext_f, dt, Ac, gc);
  R rb[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) rb[i] = -gc[i];
  LegBlock<R> lb[2];
  SelfTerms<R> S;
  self_terms_env(M, F, s.q, s.qd, P.base, dt, S);
  for (int leg = 0; leg < 2; ++leg) {
    Sym6<R> Ab;
    R r[6];
    leg_contribution(M, T, P.base, P.leg[leg], F, s.q + 6 * leg, s.qd + 6 * leg, tau + 6 * leg, leg, dt, lb[leg], Ab, r,
                     s.vimp, M.self_collisions ? S.C[leg] : nullptr, S.c[leg]);
    sym_add(Ac, Ab);
    for (int i = 0; i < 6; ++i) rb[i] += r[i];
  }
  solve_base(Ac, rb);
  for (int i = 0; i < 6; ++i) delta[i] = rb[i];
  for (int leg = 0; leg < 2; ++leg) backsub_leg(lb[leg], rb, delta + 6 + 6 * leg);
}

// The same substep composed the way k_dyn4 runs it (t1env_dynamics.hip): per leg the contact-free passes
// (leg_forward_nc / leg_backward_nc), the shank / foot contact terms from the forward pass's poses, the fold-in
// (leg_apply_contacts), the elimination, and the base-box contact share of the leg; summed base block, solve,
// back-substitution.  Host builds run it to check the split algebra against compute_delta (tests/test_dynamics.py).
template <typename R>
T1_HD void compute_delta_split(const DynModel& M, const Terrain& T, const EnvParams<R>& P, EnvState<R>& s,
                               const R tau[ND], V3<R> ext_f, R dt, R delta[6 + ND]) {
  constexpr int KS = 3, KF = 5;
  static_assert(T1_LEG_CONTACT_MASK == ((1 << KS) | (1 << KF)), "split composition assumes shank + foot contacts");
  BaseFrame<R> F;
  base_frame(s, F);
  Sym6<R> Ac;
  R gc[6];
  base_block(M, P.base, F, ext_f, dt, Ac, gc);
  R rb[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) rb[i] = -gc[i];
  LegBlock<R> lb[2];
  const R mu = P.base.friction, e = ground_restitution(M, P.base.restitution);
  SelfTerms<R> S;
  self_terms_env(M, F, s.q, s.qd, P.base, dt, S);
  for (int leg = 0; leg < 2; ++leg) {
    const R* q = s.q + 6 * leg;
    const R* qd = s.qd + 6 * leg;
    LegPass<R> st;
    M3<R> Rc[2];
    V3<R> pc[2];
    R Vc[2][6];
    leg_forward_nc<T1_LEG_CONTACT_MASK>(M, P.leg[leg], F, q, qd, leg, dt, st,
                                        [&](auto kc, const M3<R>& Rk, V3<R> pk, const R* V) {
                                          constexpr int i = decltype(kc)::value == KF ? 1 : 0;
                                          Rc[i] = Rk;
                                          pc[i] = pk;
                                          for (int j = 0; j < 6; ++j) Vc[i][j] = V[j];
                                        });
    Sym6<R> Ab;
    R g6[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
    sym_zero(Ab);
    leg_backward_nc(M, P.leg[leg], q, qd, leg, dt, st, lb[leg], Ab, g6);
    Sym6<R> Cc[2];
    R cc[2][6];
    for (int i = 0; i < 2; ++i) {
      const int b = 1 + 6 * leg + (i ? KF : KS);
      Cc[i] = S.C[leg][i];  // the self-contact terms (zero without self-collision), then the terrain's
      for (int j = 0; j < 6; ++j) cc[i][j] = S.c[leg][i][j];
      const int32_t bound = terrain_bound_raw_any(T, pc[i].x + F.abs.x, pc[i].y + F.abs.y);
      body_contact_fixed<T1_POINTS_PER_BODY>(M, T, pc[i].z + F.abs.z - R(M.contact_radius[b]), bound,
                                             M.contact_start[b], Rc[i], pc[i], F.abs, Vc[i], mu, e,
                                             s.vimp[i ? vimp_foot(leg) : vimp_shank(leg)], dt, Cc[i], cc[i]);
    }
    leg_apply_contacts<KS, KF>(Cc[0], cc[0], Cc[1], cc[1], tau + 6 * leg, dt, st, lb[leg], Ab, g6);
    R r[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) r[i] = -g6[i];
    eliminate_leg(lb[leg], Ab, r);
    // base-box contact share of this leg
    int cb, ce;
    base_contact_range(M, leg, cb, ce);
    Sym6<R> Cb;
    R gw[6] = {R(0), R(0), R(0), R(0), R(0), R(0)};
    sym_zero(Cb);
    const int32_t bound = terrain_bound_raw_any(T, F.abs.x, F.abs.y);
    body_contact_fixed<T1_POINTS_PER_BODY / 2>(M, T, F.abs.z - R(M.contact_radius[0]), bound, cb, F.R0,
                                               v3<R>(0, 0, 0), F.abs, F.V0, mu, e, s.vimp[vimp_base(leg)], dt, Cb, gw);
    sym_add(Ac, Ab);
    sym_add(Ac, Cb);
#pragma unroll
    for (int i = 0; i < 6; ++i) rb[i] += r[i] - gw[i];
  }
  solve_base(Ac, rb);
  for (int i = 0; i < 6; ++i) delta[i] = rb[i];
  for (int leg = 0; leg < 2; ++leg) backsub_leg(lb[leg], rb, delta + 6 + 6 * leg);
}

template <typename R>
T1_HD void substep(const DynModel& M, const Terrain& T, const EnvParams<R>& P, EnvState<R>& s, const R tau[ND],
                   V3<R> ext_f, R dt, bool split = false) {
  R delta[6 + ND];
  if (split) compute_delta_split(M, T, P, s, tau, ext_f, dt, delta);
  else compute_delta(M, T, P, s, tau, ext_f, dt, delta);
  integrate_base(s, delta, dt);
  for (int leg = 0; leg < 2; ++leg) integrate_leg(M, leg, s.q + 6 * leg, s.qd + 6 * leg, delta + 6 + 6 * leg, dt);
}

// ---------------------------------------------------------------------------------------------------
// Gym-shaped outputs after the last substep: root (13), rigid (13 x 13), net contact force (13 x 3).
// Linear velocities are COM velocities (PhysX reports link COM velocity); positions are link frame origins.
// ---------------------------------------------------------------------------------------------------
template <typename R, typename Writer>
T1_HD void report_base(const DynModel& M, const Terrain& T, const BaseParams<R>& P, const BaseState<R>& s,
                       const BaseFrame<R>& F, Writer& W, const R vimp_b[2]) {
  V3<R> c0 = base_com(M, P, F.R0);
  V3<R> vcom = v3<R>(s.vo[0], s.vo[1], s.vo[2]) + cross(v3<R>(s.w[0], s.w[1], s.w[2]), c0);
  R body[13];
  body[0] = s.pos[0]; body[1] = s.pos[1]; body[2] = s.pos[2];
  body[3] = s.quat[0]; body[4] = s.quat[1]; body[5] = s.quat[2]; body[6] = s.quat[3];
  body[7] = vcom.x; body[8] = vcom.y; body[9] = vcom.z;
  body[10] = s.w[0]; body[11] = s.w[1]; body[12] = s.w[2];
  W.root(body);
  W.rigid(0, body);
  // the base box's halves keep separate episodes; the report uses the stronger set point of the two
  const R e = ground_restitution(M, P.restitution);
  const R vt0 = restitution_target(M, e, vimp_b[0]), vt1 = restitution_target(M, e, vimp_b[1]);
  W.contact(0, body_contact_force(M, T, 0, F.R0, v3<R>(0, 0, 0), F.abs, F.V0, P.friction, vt0 > vt1 ? vt0 : vt1));
}
// fself: the self-contact forces on the leg's shank [0] and foot [1] (self_forces_leg), added to their net force
template <typename R, typename Writer>
T1_HD void report_leg(const DynModel& M, const Terrain& T, R mu, R e, const R vimp_leg[2], const BaseFrame<R>& F,
                      const R q[NLEG], const R qd[NLEG], int leg, Writer& W, const V3<R>* fself = nullptr) {
  BodyState<R> B[NLEG];
  leg_fk(M, leg, F.R0, q, B);
  R V[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) V[i] = F.V0[i];
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    const int b = 1 + 6 * leg + k;
    R S[6];
    motion_subspace(M, b, B[k], S);
#pragma unroll
    for (int i = 0; i < 6; ++i) V[i] += S[i] * qd[k];
    V3<R> c = B[k].p + mul(B[k].Rot, v3<R>(M.com[b][0], M.com[b][1], M.com[b][2]));
    V3<R> om{V[0], V[1], V[2]};
    V3<R> vc = v3<R>(V[3], V[4], V[5]) + cross(om, c);
    R qb[4];
    mat_to_quat(B[k].Rot, qb);
    R out[13] = {B[k].p.x + F.abs.x, B[k].p.y + F.abs.y, B[k].p.z + F.abs.z, qb[0], qb[1], qb[2], qb[3],
                 vc.x, vc.y, vc.z, om.x, om.y, om.z};
    W.rigid(b, out);
    const R vtg = restitution_target(M, e, k == 3 ? vimp_leg[0] : (k == NLEG - 1 ? vimp_leg[1] : R(0)));
    V3<R> fc = M.contact_count[b] > 0 ? body_contact_force(M, T, b, B[k].Rot, B[k].p, F.abs, V, mu, vtg) : v3<R>(0, 0, 0);
    if (fself && (k == 3 || k == NLEG - 1)) fc = fc + fself[k == NLEG - 1 ? 1 : 0];
    W.contact(b, fc);
  }
}
template <typename R, typename Writer>
T1_HD void report(const DynModel& M, const Terrain& T, const EnvParams<R>& P, const EnvState<R>& s, Writer& W) {
  BaseFrame<R> F;
  base_frame(s, F);
  const R vb[2] = {s.vimp[vimp_base(0)], s.vimp[vimp_base(1)]};
  report_base(M, T, P.base, s, F, W, vb);
  V3<R> fs[2][2];
  for (int l = 0; l < 2; ++l) fs[l][0] = fs[l][1] = v3<R>(R(0), R(0), R(0));
  if (M.self_collisions) {
    BodyKin<R> K[2][2];
    contact_body_kinematics(M, F, s.q, s.qd, K);
    for (int leg = 0; leg < 2; ++leg)
      self_forces_leg(M, leg, K[leg], K[1 - leg], P.base.self_friction, fs[leg]);
  }
  const R e = ground_restitution(M, P.base.restitution);
  for (int leg = 0; leg < 2; ++leg) {
    const R vl[2] = {s.vimp[vimp_shank(leg)], s.vimp[vimp_foot(leg)]};
    report_leg(M, T, P.base.friction, e, vl, F, s.q + 6 * leg, s.qd + 6 * leg, leg, W, fs[leg]);
  }
}

}  // namespace t1
