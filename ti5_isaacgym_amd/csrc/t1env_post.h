// t1env_post.h -- device functions of the post-physics pass (one env per lane).
//
// Mirrors, per env, T1DHStandEnv.post_physics_step (legged_robot.py:458-506) and what it calls in
// t1_dh_stand_env.py.  Every float expression keeps the reference's evaluation order (torch evaluates
// op by op in fp32), so results agree with the reference to the last few ulps; draw sites use the
// counter RNG (t1_common.h, slot table = oracle/rng.py).
#pragma once
#include "t1_common.h"

namespace t1 {

constexpr float PI_F = 3.14159265358979f;      // float32(np.pi)
constexpr float TWO_PI_F = 6.28318530717959f;   // float32(2 * np.pi)

__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub(float a, float b) { return __fsub_rn(a, b); }

// isaacgym torch_utils.quat_rotate_inverse (legged_robot.py:201-205 call sites), fp32 op order
__device__ __forceinline__ void quat_rotate_inverse(const float q[4], const float v[3], float out[3]) {
  const float qx = q[0], qy = q[1], qz = q[2], qw = q[3];
  const float s = fsub(fmul(2.0f, fmul(qw, qw)), 1.0f);
  const float a0 = fmul(v[0], s), a1 = fmul(v[1], s), a2 = fmul(v[2], s);
  // torch.cross(q_vec, v) * q_w * 2
  const float c0 = fsub(fmul(qy, v[2]), fmul(qz, v[1]));
  const float c1 = fsub(fmul(qz, v[0]), fmul(qx, v[2]));
  const float c2 = fsub(fmul(qx, v[1]), fmul(qy, v[0]));
  const float b0 = fmul(fmul(c0, qw), 2.0f), b1 = fmul(fmul(c1, qw), 2.0f), b2 = fmul(fmul(c2, qw), 2.0f);
  // q_vec * bmm(q_vec, v) * 2
  const float d = fadd(fadd(fmul(qx, v[0]), fmul(qy, v[1])), fmul(qz, v[2]));
  const float e0 = fmul(fmul(qx, d), 2.0f), e1 = fmul(fmul(qy, d), 2.0f), e2 = fmul(fmul(qz, d), 2.0f);
  out[0] = fadd(fsub(a0, b0), e0);
  out[1] = fadd(fsub(a1, b1), e1);
  out[2] = fadd(fsub(a2, b2), e2);
}

__device__ __forceinline__ float wrap_2pi_then_pi(float x) {
  // (x % 2pi) then x[x > pi] -= 2pi  (legged_robot.py:46, 52)
  float r = x < 0.0f ? fadd(x, TWO_PI_F) : x;
  if (r >= TWO_PI_F) r = fsub(r, TWO_PI_F);
  if (r > PI_F) r = fsub(r, TWO_PI_F);
  return r;
}

// get_euler_xyz_tensor (legged_robot.py:27-53)
__device__ __forceinline__ void euler_xyz(const float q[4], float e[3]) {
  const float qx = q[0], qy = q[1], qz = q[2], qw = q[3];
  const float sinr = fmul(2.0f, fadd(fmul(qw, qx), fmul(qy, qz)));
  const float cosr = fadd(fsub(fsub(fmul(qw, qw), fmul(qx, qx)), fmul(qy, qy)), fmul(qz, qz));
  const float roll = atan2f(sinr, cosr);
  const float sinp = fmul(2.0f, fsub(fmul(qw, qy), fmul(qz, qx)));
  float pitch;
  if (fabsf(sinp) >= 1.0f) pitch = sinp > 0.0f ? 1.57079637f : (sinp < 0.0f ? -1.57079637f : 0.0f);
  else pitch = asinf(sinp);
  const float siny = fmul(2.0f, fadd(fmul(qw, qz), fmul(qx, qy)));
  const float cosy = fsub(fsub(fadd(fmul(qw, qw), fmul(qx, qx)), fmul(qy, qy)), fmul(qz, qz));
  const float yaw = atan2f(siny, cosy);
  e[0] = wrap_2pi_then_pi(roll);
  e[1] = wrap_2pi_then_pi(pitch);
  e[2] = wrap_2pi_then_pi(yaw);
}

__device__ __forceinline__ float norm3(float a, float b, float c) { return sqrtf(fadd(fadd(fmul(a, a), fmul(b, b)), fmul(c, c))); }
__device__ __forceinline__ float norm2(float a, float b) { return sqrtf(fadd(fmul(a, a), fmul(b, b))); }
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
__device__ __forceinline__ float signf(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }

}  // namespace t1
