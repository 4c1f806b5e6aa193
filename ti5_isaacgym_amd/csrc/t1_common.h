// t1_common.h -- host/device helpers shared by the HIP kernels (and by the CPU build of the dynamics).
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define T1_HD __host__ __device__ __forceinline__
#else
#define T1_HD inline
#endif

namespace t1 {

// ---------------------------------------------------------------------------------------------------
// Counter RNG: identical definition to oracle/rng.py (the two are compared by tests/test_rng.py).
// Every reference draw site maps to (seed, global env id, step counter, slot) -> uniform; see
// oracle/rng.py for the slot table and the reference file:line of each site.
// ---------------------------------------------------------------------------------------------------
T1_HD uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
T1_HD uint32_t hash4(uint32_t seed, uint32_t env, uint32_t ctr, uint32_t slot) {
  uint32_t h = mix32(seed ^ 0x9E3779B9u);
  h = mix32(h ^ env);
  h = mix32(h + ctr * 0x9E3779B1u);
  h = mix32(h ^ (slot * 0x85EBCA77u));
  return h;
}
T1_HD float uniform01(uint32_t seed, uint32_t env, uint32_t ctr, uint32_t slot) {
  return (float)(hash4(seed, env, ctr, slot) >> 8) * (1.0f / 16777216.0f);
}
// torch_rand_float(lo, hi) = (hi - lo) * rand + lo, two fp32 roundings, no fma (isaacgym torch_utils)
T1_HD float rand_float(float lo, float hi, uint32_t seed, uint32_t env, uint32_t ctr, uint32_t slot) {
  float u = uniform01(seed, env, ctr, slot);
#if defined(__HIP_DEVICE_COMPILE__)
  // __fmul_rn / __fadd_rn alone are contracted into one v_fmac by the compiler (r03: ext-force draws U(-300, 600)
  // off by up to 5e-5 from the two-rounding value); the empty asm makes the rounded product opaque to that fusion
  float p = __fmul_rn(hi - lo, u);
  asm volatile("" : "+v"(p));
  return __fadd_rn(p, lo);
#else
  volatile float p = (hi - lo) * u;
  return p + lo;
#endif
}
T1_HD int32_t rand_int(int32_t lo, int32_t hi, uint32_t seed, uint32_t env, uint32_t ctr, uint32_t slot) {
  uint64_t h = hash4(seed, env, ctr, slot) >> 8;
  return lo + (int32_t)((h * (uint64_t)(hi - lo)) >> 24);
}
// The first three mixes of hash4 depend only on (seed, env, ctr): a draw site that makes many draws for one env
// and step takes the key once and pays one mix per draw (same values as hash4 by construction).
struct RngKey { uint32_t h; };
T1_HD RngKey rng_key(uint32_t seed, uint32_t env, uint32_t ctr) {
  uint32_t h = mix32(seed ^ 0x9E3779B9u);
  h = mix32(h ^ env);
  return RngKey{mix32(h + ctr * 0x9E3779B1u)};
}
T1_HD uint32_t hash_k(RngKey k, uint32_t slot) { return mix32(k.h ^ (slot * 0x85EBCA77u)); }
T1_HD float uniform01(RngKey k, uint32_t slot) { return (float)(hash_k(k, slot) >> 8) * (1.0f / 16777216.0f); }
T1_HD float rand_float(float lo, float hi, RngKey k, uint32_t slot) {
  float u = uniform01(k, slot);
#if defined(__HIP_DEVICE_COMPILE__)
  // __fmul_rn / __fadd_rn alone are contracted into one v_fmac by the compiler (r03: ext-force draws U(-300, 600)
  // off by up to 5e-5 from the two-rounding value); the empty asm makes the rounded product opaque to that fusion
  float p = __fmul_rn(hi - lo, u);
  asm volatile("" : "+v"(p));
  return __fadd_rn(p, lo);
#else
  volatile float p = (hi - lo) * u;
  return p + lo;
#endif
}
T1_HD int32_t rand_int(int32_t lo, int32_t hi, RngKey k, uint32_t slot) {
  uint64_t h = hash_k(k, slot) >> 8;
  return lo + (int32_t)((h * (uint64_t)(hi - lo)) >> 24);
}

// reset_idx(env_ids) between steps keys its draws on (counter | T1_BETWEEN_STEP_SALT) (oracle/rng.py
// BETWEEN_STEP_SALT): the in-step resets of the step that produced `counter` used the plain counter
constexpr uint32_t T1_BETWEEN_STEP_SALT = 0x80000000u;

// slot table (mirror of oracle/rng.py)
enum : uint32_t {
  SLOT_TORQUE_MULT = 1000, SLOT_CMD_X = 2000, SLOT_CMD_Y = 2001, SLOT_CMD_YAW = 2002, SLOT_CMD_HEADING = 2003,
  SLOT_EXT_FORCE = 3000, SLOT_EXT_TORQUE = 3003, SLOT_PUSH_VEL = 3100, SLOT_PUSH_ANG = 3102,
  SLOT_OBS_NOISE = 4000, SLOT_RESET_DOF = 5000, SLOT_RESET_ROOT_XY = 5100, SLOT_DR_TORQUE = 5200,
  SLOT_DR_OFFSET = 5300, SLOT_DR_KP = 5400, SLOT_DR_KD = 5500, SLOT_DR_COULOMB = 5600, SLOT_DR_VISCOUS = 5700,
  SLOT_DR_ARMATURE = 5800, SLOT_LAG_ACTION = 5900, SLOT_LAG_DOF = 5901, SLOT_LAG_IMU = 5902,
  SLOT_GAIT_START = 5903, SLOT_GAIT_TIME = 5910, SLOT_TERRAIN_LEVEL_RAND = 5920,
  SLOT_PAYLOAD = 6000, SLOT_LINK_MASS = 6001, SLOT_COM = 6020, SLOT_FRICTION_BUCKET = 6030,
  SLOT_FRICTION_VALUE = 6031, SLOT_RESTITUTION_VALUE = 6032, SLOT_TERRAIN_LEVEL_INIT = 6040, SLOT_START_XY = 6050,
};

// ---------------------------------------------------------------------------------------------------
// small vector algebra (templated so the CPU build can run in double)
// ---------------------------------------------------------------------------------------------------
template <typename R> struct V3 { R x, y, z; };
template <typename R> T1_HD V3<R> v3(R x, R y, R z) { return V3<R>{x, y, z}; }
template <typename R> T1_HD V3<R> operator+(V3<R> a, V3<R> b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
template <typename R> T1_HD V3<R> operator-(V3<R> a, V3<R> b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
template <typename R> T1_HD V3<R> operator*(R s, V3<R> a) { return {s * a.x, s * a.y, s * a.z}; }
template <typename R> T1_HD R dot(V3<R> a, V3<R> b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
template <typename R> T1_HD V3<R> cross(V3<R> a, V3<R> b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// fast reciprocal / square root: hardware v_rcp_f32 / v_sqrt_f32 (1 ulp) on the device, exact on the host
T1_HD float rcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_rcpf(x);
#else
  return 1.0f / x;
#endif
}
T1_HD double rcp(double x) { return 1.0 / x; }
T1_HD float fsqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_sqrtf(x);
#else
  return sqrtf(x);
#endif
}
T1_HD double fsqrt(double x) { return sqrt(x); }
// sin/cos of a joint angle.  Device: branch-free Cody-Waite reduction by pi/2 (three-part constant, exact for
// |a| < ~1e3, far beyond any joint angle) and minimax polynomials on [-pi/4, pi/4] (about 1 ulp), ~25
// instructions against the library's ~45 fast path plus its large-argument branch.  Host: the C library.
T1_HD void fsincos(float a, float* s, float* c) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float k = __builtin_rintf(a * 0.636619772367581343f);
  float r = __builtin_fmaf(k, -1.5707962513e+00f, a);
  r = __builtin_fmaf(k, -7.5497894159e-08f, r);
  r = __builtin_fmaf(k, -5.3903029534e-15f, r);
  const float r2 = r * r;
  const float ps = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, r2, 8.3321608736e-3f), r2,
                                                 -1.6666654611e-1f), r2 * r, r);
  const float pc = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, r2, -1.388731625493765e-3f), r2,
                                                 4.166664568298827e-2f), r2 * r2, __builtin_fmaf(-0.5f, r2, 1.0f));
  const int q = (int)k;
  const float sv = (q & 1) ? pc : ps, cv = (q & 1) ? ps : pc;
  *s = (q & 2) ? -sv : sv;
  *c = ((q + 1) & 2) ? -cv : cv;
#else
  sincosf(a, s, c);
#endif
}
T1_HD void fsincos(double a, double* s, double* c) { sincos(a, s, c); }

// row-major 3x3
template <typename R> struct M3 { R m[9]; };
template <typename R> T1_HD V3<R> mul(const M3<R>& A, V3<R> v) {
  return {A.m[0] * v.x + A.m[1] * v.y + A.m[2] * v.z, A.m[3] * v.x + A.m[4] * v.y + A.m[5] * v.z,
          A.m[6] * v.x + A.m[7] * v.y + A.m[8] * v.z};
}
template <typename R> T1_HD V3<R> col(const M3<R>& A, int c) { return {A.m[c], A.m[3 + c], A.m[6 + c]}; }
template <typename R> T1_HD M3<R> quat_to_mat(R x, R y, R z, R w) {
  M3<R> A;
  A.m[0] = 1 - 2 * (y * y + z * z); A.m[1] = 2 * (x * y - z * w);     A.m[2] = 2 * (x * z + y * w);
  A.m[3] = 2 * (x * y + z * w);     A.m[4] = 1 - 2 * (x * x + z * z); A.m[5] = 2 * (y * z - x * w);
  A.m[6] = 2 * (x * z - y * w);     A.m[7] = 2 * (y * z + x * w);     A.m[8] = 1 - 2 * (x * x + y * y);
  return A;
}
// A * Rot(axis, angle) for a unit coordinate axis (0=x,1=y,2=z): rotates two columns of A.  The axis is a
// template parameter so every register index is static (a runtime column index would go to scratch).
template <int AX, typename R> T1_HD M3<R> mul_axis_rot_t(const M3<R>& A, R c, R s) {
  constexpr int i = (AX + 1) % 3, j = (AX + 2) % 3;  // e_i -> c e_i + s e_j ; e_j -> -s e_i + c e_j
  M3<R> B = A;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    R ai = A.m[3 * r + i], aj = A.m[3 * r + j];
    B.m[3 * r + i] = c * ai + s * aj;
    B.m[3 * r + j] = -s * ai + c * aj;
  }
  return B;
}
template <typename R> T1_HD M3<R> mul_axis_rot(const M3<R>& A, int axis, R c, R s) {
  // branch-free: with 0/1 weights ex, ey, ez for the axis, columns (i, j) = cyclic successors of the axis:
  // for x: (y, z); y: (z, x); z: (x, y).  Column blends are exact (weights are 0 or 1).
  const R ex = axis == 0 ? R(1) : R(0), ey = axis == 1 ? R(1) : R(0), ez = axis == 2 ? R(1) : R(0);
  M3<R> B;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const R a0 = A.m[3 * r], a1 = A.m[3 * r + 1], a2 = A.m[3 * r + 2];
    const R ai = ex * a1 + ey * a2 + ez * a0;  // column i
    const R aj = ex * a2 + ey * a0 + ez * a1;  // column j
    const R ni = c * ai + s * aj, nj = -s * ai + c * aj;
    // write back: axis column unchanged, i -> ni, j -> nj
    B.m[3 * r] = ex * a0 + ey * nj + ez * ni;
    B.m[3 * r + 1] = ex * ni + ey * a1 + ez * nj;
    B.m[3 * r + 2] = ex * nj + ey * ni + ez * a2;
  }
  return B;
}
// column of A selected without a runtime register index
template <typename R> T1_HD V3<R> col_sel(const M3<R>& A, int c) {
  return c == 0 ? V3<R>{A.m[0], A.m[3], A.m[6]} : (c == 1 ? V3<R>{A.m[1], A.m[4], A.m[7]} : V3<R>{A.m[2], A.m[5], A.m[8]});
}
// rotation matrix -> quaternion (x,y,z,w), Shepperd
template <typename R> T1_HD void mat_to_quat(const M3<R>& A, R q[4]) {
  R t = A.m[0] + A.m[4] + A.m[8];
  if (t > 0) {
    R s = fsqrt(t + 1) * 2, is = rcp(s);
    q[3] = R(0.25) * s; q[0] = (A.m[7] - A.m[5]) * is; q[1] = (A.m[2] - A.m[6]) * is; q[2] = (A.m[3] - A.m[1]) * is;
  } else if (A.m[0] > A.m[4] && A.m[0] > A.m[8]) {
    R s = fsqrt(1 + A.m[0] - A.m[4] - A.m[8]) * 2, is = rcp(s);
    q[3] = (A.m[7] - A.m[5]) * is; q[0] = R(0.25) * s; q[1] = (A.m[1] + A.m[3]) * is; q[2] = (A.m[2] + A.m[6]) * is;
  } else if (A.m[4] > A.m[8]) {
    R s = fsqrt(1 + A.m[4] - A.m[0] - A.m[8]) * 2, is = rcp(s);
    q[3] = (A.m[2] - A.m[6]) * is; q[0] = (A.m[1] + A.m[3]) * is; q[1] = R(0.25) * s; q[2] = (A.m[5] + A.m[7]) * is;
  } else {
    R s = fsqrt(1 + A.m[8] - A.m[0] - A.m[4]) * 2, is = rcp(s);
    q[3] = (A.m[3] - A.m[1]) * is; q[0] = (A.m[2] + A.m[6]) * is; q[1] = (A.m[5] + A.m[7]) * is; q[2] = R(0.25) * s;
  }
  if (q[3] < 0) { q[0] = -q[0]; q[1] = -q[1]; q[2] = -q[2]; q[3] = -q[3]; }
}

}  // namespace t1
