// t1env_roles.h -- LDS row helpers shared by the role-split step kernels k_dyn5 (t1env_dyn5.hip, four waves) and
// k_dyn6 (t1env_dyn6.hip, eight waves).  Both put the two legs of an env in the two halves of one wave (lane l: env
// l & 31, leg l >> 5) and pass values between the roles of a substep through LDS rows [row][lane] of float4.
#pragma once
#include <hip/hip_runtime.h>

#include "t1_dynamics.h"
#include "t1env_fused.h"  // XCH, K_SHANK / K_FOOT

namespace t1 {

// float4 rows [row][lane]: one ds_write_b128 / ds_read_b128 per 4 values of a lane, conflict-free
template <int K> struct Rows4 { float4 r[(K + 3) / 4][64]; };
template <int K>
__device__ __forceinline__ void put4(Rows4<K>& D, int lane, const float (&v)[K]) {
#pragma unroll
  for (int r = 0; r < (K + 3) / 4; ++r)
    D.r[r][lane] = make_float4(v[4 * r], 4 * r + 1 < K ? v[4 * r + 1] : 0.0f, 4 * r + 2 < K ? v[4 * r + 2] : 0.0f,
                               4 * r + 3 < K ? v[4 * r + 3] : 0.0f);
}
template <int K>
__device__ __forceinline__ void get4(const Rows4<K>& D, int lane, float (&v)[K]) {
#pragma unroll
  for (int r = 0; r < (K + 3) / 4; ++r) {
    const float4 x = D.r[r][lane];
    v[4 * r] = x.x;
    if (4 * r + 1 < K) v[4 * r + 1] = x.y;
    if (4 * r + 2 < K) v[4 * r + 2] = x.z;
    if (4 * r + 3 < K) v[4 * r + 3] = x.w;
  }
}

// the value of the left-half lane and of the right-half lane of this lane's env, in every lane (v_permlane32_swap:
// lanes 32-63 of the first operand trade with lanes 0-31 of the second, both copies of v)
__device__ __forceinline__ void halves(float v, float& left, float& right) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  left = __uint_as_float(r[0]);
  right = __uint_as_float(r[1]);
}

// The substep state the core wave publishes (each half: the env's base state and its leg's joints)
enum : int { Q_POS = 0, Q_QUAT = 3, Q_W = 7, Q_VO = 10, Q_Q = 13, Q_QD = 19, Q_N = 25 };
constexpr int CAP5_N = 2 * NLEG + 8;  // the core wave's sensor-lag capture: q, qd of the leg; the raw IMU sample (leg 0)

__device__ __forceinline__ void state_pack(const BaseState<float>& sb, const float q[NLEG], const float qd[NLEG],
                                           float (&v)[Q_N]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) { v[Q_POS + i] = sb.pos[i]; v[Q_W + i] = sb.w[i]; v[Q_VO + i] = sb.vo[i]; }
#pragma unroll
  for (int i = 0; i < 4; ++i) v[Q_QUAT + i] = sb.quat[i];
#pragma unroll
  for (int k = 0; k < NLEG; ++k) { v[Q_Q + k] = q[k]; v[Q_QD + k] = qd[k]; }
}
__device__ __forceinline__ void state_unpack(const float (&v)[Q_N], BaseState<float>& sb, float q[NLEG], float qd[NLEG]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) { sb.pos[i] = v[Q_POS + i]; sb.w[i] = v[Q_W + i]; sb.vo[i] = v[Q_VO + i]; }
#pragma unroll
  for (int i = 0; i < 4; ++i) sb.quat[i] = v[Q_QUAT + i];
#pragma unroll
  for (int k = 0; k < NLEG; ++k) { q[k] = v[Q_Q + k]; qd[k] = v[Q_QD + k]; }
}
__device__ __forceinline__ void read_state_rows(const Rows4<Q_N>& st, int lane, BaseState<float>& sb, float q[NLEG],
                                                float qd[NLEG]) {
  float v[Q_N];
  get4(st, lane, v);
  state_unpack(v, sb, q, qd);
}
__device__ __forceinline__ void sym_pack(const Sym6<float>& A, const float g[6], float (&v)[XCH]) {
#pragma unroll
  for (int i = 0; i < 21; ++i) v[i] = A.a[i];
#pragma unroll
  for (int i = 0; i < 6; ++i) v[21 + i] = g[i];
}
__device__ __forceinline__ void sym_unpack(const float (&v)[XCH], Sym6<float>& A, float g[6]) {
#pragma unroll
  for (int i = 0; i < 21; ++i) A.a[i] = v[i];
#pragma unroll
  for (int i = 0; i < 6; ++i) g[i] = v[21 + i];
}

}  // namespace t1
