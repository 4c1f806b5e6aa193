// t1env_device.h -- device helpers shared by the physics kernels of both translation units
// (t1env.hip: injected-physics kernel; t1env_dynamics.hip: k_dynamics).  Included after t1_dynamics.h.
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/t1env.h"
#include "t1_dynamics.h"

namespace t1 {

struct DevWriter {
  float* rootp;
  float* rigidp;
  float* contactp;
  __device__ void root(const float* v) {
#pragma unroll
    for (int i = 0; i < 13; ++i) rootp[i] = v[i];
  }
  __device__ void rigid(int b, const float* v) {
#pragma unroll
    for (int i = 0; i < 13; ++i) rigidp[b * 13 + i] = v[i];
  }
  __device__ void contact(int b, V3<float> f) {
    contactp[b * 3 + 0] = f.x;
    contactp[b * 3 + 1] = f.y;
    contactp[b * 3 + 2] = f.z;
  }
};

// per-env base parameters; PhysX combines shape and ground friction by averaging (third-party semantics,
// unpinned)
__device__ __forceinline__ void load_base_params(const DynModel& M, const t1env_buffers& B, int n,
                                                 BaseParams<float>& P) {
  P.mass = B.body_mass[n];
  P.inertia_scale = P.mass / M.mass[0];
#pragma unroll
  for (int i = 0; i < 3; ++i) P.com_disp[i] = B.com_disp[n * 3 + i];
  P.friction = 0.5f * (B.friction[n] + M.ground_friction);
}
__device__ __forceinline__ void load_leg_params(const DynModel& M, const t1env_buffers& B, int n, int j0,
                                                LegParams<float>& P) {
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    const float s = B.link_mass_scale[n * 12 + j0 + k];
    P.mass[k] = M.mass[1 + j0 + k] * s;
    P.inertia_scale[k] = s;
    P.armature[k] = B.armature[n * 12 + j0 + k];
  }
}
// root state (COM velocity) -> internal base state (base-origin velocity)
__device__ __forceinline__ void load_base_state(const DynModel& M, const BaseParams<float>& P, const float* root,
                                                BaseState<float>& s) {
#pragma unroll
  for (int i = 0; i < 3; ++i) s.pos[i] = root[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) s.quat[i] = root[3 + i];
  V3<float> c0 = base_com(M, P, quat_to_mat(s.quat[0], s.quat[1], s.quat[2], s.quat[3]));
  V3<float> w = v3<float>(root[10], root[11], root[12]);
  V3<float> vo = v3<float>(root[7], root[8], root[9]) - cross(w, c0);
  s.w[0] = w.x; s.w[1] = w.y; s.w[2] = w.z;
  s.vo[0] = vo.x; s.vo[1] = vo.y; s.vo[2] = vo.z;
}

}  // namespace t1

// the PD torque and the IMU sample must round like the reference's torch ops: no FMA contraction from here on
#pragma clang fp contract(off)
#include "t1env_post.h"

namespace t1 {

// PD torque of one substep (legged_robot.py:1019-1074): lagged action, randomized gains, viscous +
// Coulomb friction, torque multiplier redrawn every substep, clip to 0.85 * effort.
// Joints j0 .. j0+NJ-1 (NJ = 12: whole env; NJ = 6: one leg of the two-wave kernel).
template <int NJ>
__device__ __forceinline__ void pd_torques(const DynModel& M, const t1env_config& C, const t1env_buffers& B, int n,
                                           uint32_t genv, uint32_t ctr, int sub, int lag, int j0, const float q[NJ],
                                           const float qd[NJ], float tau[NJ]) {
  const int d = lag > sub ? (lag - sub + 9) / 10 : 0;
  const float* la = B.act_hist + ((size_t)n * 4 + ((ctr - (uint32_t)d) & 3u)) * 12;
#pragma unroll
  for (int jj = 0; jj < NJ; ++jj) {
    const int j = j0 + jj;
    const float kp = B.kp[n * 12 + j], kd = B.kd[n * 12 + j];
    float t = kp * (((la[j] + M.default_dof_pos[j]) - q[jj]) + B.motor_offsets[n * 12 + j]);
    t = t - kd * qd[jj];
    t = t - B.viscous[n * 12 + j] * qd[jj];
    t = t - B.coulomb[n * 12 + j] * signf(qd[jj]);
    const float tm = rand_float(C.torque_mult_range[0], C.torque_mult_range[1], C.seed, genv, ctr,
                                SLOT_TORQUE_MULT + sub * 12 + j);
    t = t * tm;
    const float lim = M.torque_limit[j];
    tau[jj] = fminf(fmaxf(t, -lim), lim);
  }
}

__device__ __forceinline__ void capture_imu(const float quat[4], const float w_world[3], float* dst) {
  float av[3], e[3];
  quat_rotate_inverse(quat, w_world, av);
  euler_xyz(quat, e);
  dst[0] = av[0]; dst[1] = av[1]; dst[2] = av[2];
  dst[3] = e[0]; dst[4] = e[1]; dst[5] = e[2];
}

}  // namespace t1
