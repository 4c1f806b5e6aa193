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
  P.self_friction = B.friction[n];
  P.restitution = B.restitution[n];
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

// IMU lag ring entry: the raw base quaternion and world angular velocity of the captured substep (8 floats).
// The derived sample (base-frame angular velocity, euler angles: t1_dh_stand_env.py:398-404) is formed once
// per step where the observation reads it (imu_sample), not in the substep loop: lanes capture at
// different substeps, so in the loop the wave would evaluate it on most substeps.
// The per-env PD constants of one leg (randomized gains, motor offsets, viscous / Coulomb friction) and the
// 4-step action ring, staged in LDS once per env step ([value][joint][env]: conflict-free rows), so the
// substep loop reads LDS instead of re-gathering ~36 scattered rows from global memory every substep.
template <int LANES> struct PdStage {
  float kp[NLEG][LANES], kd[NLEG][LANES], off[NLEG][LANES], visc[NLEG][LANES], coul[NLEG][LANES];
  float act[4][NLEG][LANES];
};
template <int LANES>
__device__ __forceinline__ void pd_stage(const t1env_buffers& B, int n, int j0, int lane, PdStage<LANES>& P) {
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    const int j = j0 + k;
    P.kp[k][lane] = B.kp[n * 12 + j];
    P.kd[k][lane] = B.kd[n * 12 + j];
    P.off[k][lane] = B.motor_offsets[n * 12 + j];
    P.visc[k][lane] = B.viscous[n * 12 + j];
    P.coul[k][lane] = B.coulomb[n * 12 + j];
  }
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int k = 0; k < NLEG; ++k) P.act[s][k][lane] = B.act_hist[((size_t)n * 4 + s) * 12 + j0 + k];
}
// pd_torques<NLEG> with the constants from a PdStage (same arithmetic, same order)
// K = rng_key(C.seed, genv, ctr), taken once per env step by the caller (one mix per torque multiplier draw)
template <int LANES>
__device__ __forceinline__ void pd_torques_staged(const DynModel& M, const t1env_config& C, const PdStage<LANES>& P,
                                                  int lane, RngKey K, uint32_t ctr, int sub, int lag, int j0,
                                                  const float q[NLEG], const float qd[NLEG], float tau[NLEG]) {
  const int d = lag > sub ? (lag - sub + 9) / 10 : 0;
  const int slot = (int)((ctr - (uint32_t)d) & 3u);
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    const int j = j0 + k;
    const float kp = P.kp[k][lane], kd = P.kd[k][lane];
    float t = kp * (((P.act[slot][k][lane] + M.default_dof_pos[j]) - q[k]) + P.off[k][lane]);
    t = t - kd * qd[k];
    t = t - P.visc[k][lane] * qd[k];
    t = t - P.coul[k][lane] * signf(qd[k]);
    const float tm = rand_float(C.torque_mult_range[0], C.torque_mult_range[1], K, SLOT_TORQUE_MULT + sub * 12 + j);
    t = t * tm;
    const float lim = M.torque_limit[j];
    tau[k] = fminf(fmaxf(t, -lim), lim);
  }
}

__device__ __forceinline__ void capture_imu(const float quat[4], const float w_world[3], float* dst) {
  dst[0] = quat[0]; dst[1] = quat[1]; dst[2] = quat[2]; dst[3] = quat[3];
  dst[4] = w_world[0]; dst[5] = w_world[1]; dst[6] = w_world[2]; dst[7] = 0.0f;
}
__device__ __forceinline__ void imu_sample(const float raw[8], float out[6]) {
  const float quat[4] = {raw[0], raw[1], raw[2], raw[3]}, w[3] = {raw[4], raw[5], raw[6]};
  float av[3], e[3];
  quat_rotate_inverse(quat, w, av);
  euler_xyz(quat, e);
  out[0] = av[0]; out[1] = av[1]; out[2] = av[2];
  out[3] = e[0]; out[4] = e[1]; out[5] = e[2];
}


// =====================================================================================================
// history shift: out[n, :F*(H-1)] = in[n, F:] -- a flat shift by F floats of every row of the 66-frame obs
// and 3-frame critic history; the newest frame (columns >= F*(H-1)) is left to k_post_b, which also zeroes
// the older frames of reset envs.  One lane per 4 output floats, the shifted source assembled from two
// aligned 16-B loads.  SHIFT_UNROLL chunks per lane are loaded before any is stored (all loads are
// unconditional, clamped in bounds), so a lane keeps 8 x 16 B in flight: the shift reaches HBM rate with a
// few hundred workgroups, which is what k_dynamics' tail workgroups can field (each of its waves holds 240
// VGPRs).  It reads only the previous step's buffer, so it overlaps the dynamics inside one launch.
// =====================================================================================================
struct ShiftArgs {
  const float* obs_in;
  float* obs_out;
  const float* priv_in;
  float* priv_out;
  int64_t total_obs, total_priv;  // elements
  int32_t half;                   // 1: the histories hold fp16 (t1env_config.obs_half; the pointers are fp16 data)
};
constexpr int SHIFT_UNROLL = 4;

// Stores of the shift.  SC1 = the agent-coherent flavour (global_store ... sc1): the line leaves the XCD's L2
// and the store is visible to every XCD once it completes, so a later handoff needs only s_waitcnt, not an L2
// write-back (MI355X_MICROARCH.md, inter-workgroup visibility).  The fused step uses it for the rows whose
// reset zeroing may run on another XCD.
typedef float f32x4 __attribute__((ext_vector_type(4)));
template <bool SC1> __device__ __forceinline__ void store4(float* p, float4 v) {
  if constexpr (SC1) {
    const f32x4 x = {v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(x) : "memory");
  } else {
    *reinterpret_cast<float4*>(p) = v;
  }
}
template <bool SC1> __device__ __forceinline__ void store1(float* p, float v) {
  if constexpr (SC1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}

template <int F, int H, bool SC1>
__device__ __forceinline__ void shift_store(float* __restrict__ out, int64_t total, int64_t i, const float4 a,
                                            const float4 b, int rem) {
  constexpr int ROW = F * H;
  const float src[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  const int64_t row0 = i / ROW;
  const int col0 = (int)(i - row0 * ROW);
  // the 4 outputs are all older-frame columns of one row unless the chunk touches a row's newest frame
  if (col0 + 3 < ROW - F && i + 3 < total) {
    store4<SC1>(out + i, make_float4(src[rem], src[rem + 1], src[rem + 2], src[rem + 3]));
    return;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int64_t e = i + k;
    if (e >= total) break;
    const int64_t row = e / ROW;
    if ((int)(e - row * ROW) < ROW - F) store1<SC1>(out + e, src[rem + k]);
  }
}

// chunks [lo4, hi4) of one history buffer, lane t0 of `stride` lanes
template <int F, int H, bool SC1 = false, int U = SHIFT_UNROLL>
__device__ __forceinline__ void shift_range(const float* __restrict__ in, float* __restrict__ out, int64_t total,
                                            int64_t lo4, int64_t hi4, int64_t t0, int64_t stride) {
  for (int64_t base = lo4 + t0; base < hi4; base += U * stride) {
    float4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t sa = ((base + u * stride) * 4 + F) & ~(int64_t)3;
      const int64_t sc = sa + 8 <= total ? sa : (total - 8) & ~(int64_t)3;  // tail: aligned in-bounds dummy
      a[u] = *reinterpret_cast<const float4*>(in + sc);
      b[u] = *reinterpret_cast<const float4*>(in + sc + 4);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i4 = base + u * stride;
      if (i4 >= hi4) break;
      const int64_t i = i4 * 4, s = i + F, sa = s & ~(int64_t)3;
      float4 x = a[u], y = b[u];
      if (sa + 8 > total) {  // the last chunks of the buffer: element loads, zero past the end
        float t[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) t[k] = sa + k < total ? in[sa + k] : 0.0f;
        x = make_float4(t[0], t[1], t[2], t[3]);
        y = make_float4(t[4], t[5], t[6], t[7]);
      }
      shift_store<F, H, SC1>(out, total, i, x, y, (int)(s - sa));
    }
  }
}

// The in-launch shift's form of shift_range over whole rows [r0, r1): indices relative to the first row fit 32 bits,
// so the per-chunk row / column split is a 32-bit division by the constant row width instead of a 64-bit one (the
// fused step's shift workgroups run one wave per SIMD, where that integer work, not HBM, set their rate).
template <int F, int H, bool SC1, int U>
__device__ __forceinline__ void shift_rows_f32(const float* __restrict__ in, float* __restrict__ out, int64_t total,
                                               int64_t r0, int64_t r1, int t0, int stride) {
  constexpr uint32_t ROW = F * H;
  const float* __restrict__ in0 = in + r0 * ROW;
  float* __restrict__ out0 = out + r0 * ROW;
  const uint32_t lim = (uint32_t)(total - r0 * (int64_t)ROW);  // elements from in0 to the buffer end
  const uint32_t span = (uint32_t)((r1 - r0) * ROW);
  const uint32_t nel = span < lim ? span : lim;
  const uint32_t n4 = (nel + 3) / 4;
  for (uint32_t base = t0; base < n4; base += U * stride) {
    float4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t sa = ((base + u * stride) * 4 + F) & ~3u;
      const uint32_t sc = sa + 8 <= lim ? sa : (lim - 8) & ~3u;  // tail: aligned in-bounds dummy
      a[u] = *reinterpret_cast<const float4*>(in0 + sc);
      b[u] = *reinterpret_cast<const float4*>(in0 + sc + 4);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c = base + u * stride;
      if (c >= n4) break;
      const uint32_t i = c * 4, sidx = i + F, sa = sidx & ~3u;
      float4 x = a[u], y = b[u];
      if (sa + 8 > lim) {  // the last chunks of the buffer: element loads, zero past the end
        float t[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) t[k] = sa + k < lim ? in0[sa + k] : 0.0f;
        x = make_float4(t[0], t[1], t[2], t[3]);
        y = make_float4(t[4], t[5], t[6], t[7]);
      }
      const float src[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
      // sidx - sa = (4 c + F) mod 4: a compile-time offset (a run-time one indexes src through scratch at -O1)
      constexpr int rem = (int)(F & 3u);
      const uint32_t col0 = i - (i / ROW) * ROW;
      if (col0 + 3 < ROW - F && i + 3 < lim) {  // 4 older-frame columns of one row
        store4<SC1>(out0 + i, make_float4(src[rem], src[rem + 1], src[rem + 2], src[rem + 3]));
        continue;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t e = i + k;
        if (e >= lim) break;
        if (e - (e / ROW) * ROW < ROW - F) store1<SC1>(out0 + e, src[rem + k]);
      }
    }
  }
}

// ---- fp16 histories (BASELINE config 5's fp16 state, t1env_config.obs_half): the same flat shift by F elements
// over 16-B chunks of 8 halves.  The source offset inside the two aligned loads, F % 8, is a compile-time
// constant (every chunk starts on a multiple of 8), so the output chunk is four funnel shifts of 32-bit words
// (v_alignbyte) for odd F, or plain word moves for even F.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <bool SC1> __device__ __forceinline__ void store16B(uint16_t* p, u32x4 v) {
  if constexpr (SC1) asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
  else *reinterpret_cast<u32x4*>(p) = v;
}
template <bool SC1> __device__ __forceinline__ void store2B(uint16_t* p, uint16_t v) {
  if constexpr (SC1) {
    const uint32_t w = v;
    asm volatile("global_store_short %0, %1, off sc1" : : "v"(p), "v"(w) : "memory");
  } else {
    *p = v;
  }
}
template <int F, int H, bool SC1 = false, int U = SHIFT_UNROLL>
__device__ __forceinline__ void shift_range_h(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                              int64_t total, int64_t lo8, int64_t hi8, int64_t t0, int64_t stride) {
  constexpr int ROW = F * H, REM = F % 8, M = REM / 2;
  for (int64_t base = lo8 + t0; base < hi8; base += U * stride) {
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t sa = ((base + u * stride) * 8 + F) & ~(int64_t)7;
      const int64_t sc = sa + 16 <= total ? sa : (total - 16) & ~(int64_t)7;  // tail: aligned in-bounds dummy
      a[u] = *reinterpret_cast<const u32x4*>(in + sc);
      b[u] = *reinterpret_cast<const u32x4*>(in + sc + 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t c8 = base + u * stride;
      if (c8 >= hi8) break;
      const int64_t i = c8 * 8, sa = (i + F) & ~(int64_t)7;
      uint32_t w[8] = {a[u].x, a[u].y, a[u].z, a[u].w, b[u].x, b[u].y, b[u].z, b[u].w};
      if (sa + 16 > total) {  // the last chunks of the buffer: element loads, zero past the end
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t lo = sa + 2 * k < total ? in[sa + 2 * k] : 0u;
          const uint32_t hi = sa + 2 * k + 1 < total ? in[sa + 2 * k + 1] : 0u;
          w[k] = lo | (hi << 16);
        }
      }
      u32x4 o;
      if constexpr (REM % 2 == 0) {
        o = u32x4{w[M], w[M + 1], w[M + 2], w[M + 3]};
      } else {  // halves REM .. REM + 7 = the upper half of word M, ..., the lower half of word M + 4
        o = u32x4{__builtin_amdgcn_alignbyte(w[M + 1], w[M], 2), __builtin_amdgcn_alignbyte(w[M + 2], w[M + 1], 2),
                  __builtin_amdgcn_alignbyte(w[M + 3], w[M + 2], 2), __builtin_amdgcn_alignbyte(w[M + 4], w[M + 3], 2)};
      }
      const int64_t row0 = i / ROW;
      const int col0 = (int)(i - row0 * ROW);
      if (col0 + 7 < ROW - F && i + 7 < total) {
        store16B<SC1>(out + i, o);
        continue;
      }
      const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int64_t e = i + k;
        if (e >= total) break;
        const int64_t row = e / ROW;
        if ((int)(e - row * ROW) < ROW - F) store2B<SC1>(out + e, (uint16_t)(ow[k / 2] >> (16 * (k & 1))));
      }
    }
  }
}

// shift_range_h's in-launch form over whole rows [r0, r1) with 32-bit local indices (see shift_rows_f32)
template <int F, int H, bool SC1, int U>
__device__ __forceinline__ void shift_rows_f16(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                               int64_t total, int64_t r0, int64_t r1, int t0, int stride) {
  constexpr uint32_t ROW = F * H, REM = F % 8, M = REM / 2;
  const uint16_t* __restrict__ in0 = in + r0 * ROW;
  uint16_t* __restrict__ out0 = out + r0 * ROW;
  const uint32_t lim = (uint32_t)(total - r0 * (int64_t)ROW);
  const uint32_t span = (uint32_t)((r1 - r0) * ROW);
  const uint32_t nel = span < lim ? span : lim;
  const uint32_t n8 = (nel + 7) / 8;
  for (uint32_t base = t0; base < n8; base += U * stride) {
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t sa = ((base + u * stride) * 8 + F) & ~7u;
      const uint32_t sc = sa + 16 <= lim ? sa : (lim - 16) & ~7u;
      a[u] = *reinterpret_cast<const u32x4*>(in0 + sc);
      b[u] = *reinterpret_cast<const u32x4*>(in0 + sc + 8);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t c8 = base + u * stride;
      if (c8 >= n8) break;
      const uint32_t i = c8 * 8, sa = (i + F) & ~7u;
      uint32_t w[8] = {a[u].x, a[u].y, a[u].z, a[u].w, b[u].x, b[u].y, b[u].z, b[u].w};
      if (sa + 16 > lim) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t lo = sa + 2 * k < lim ? in0[sa + 2 * k] : 0u;
          const uint32_t hi = sa + 2 * k + 1 < lim ? in0[sa + 2 * k + 1] : 0u;
          w[k] = lo | (hi << 16);
        }
      }
      u32x4 o;
      if constexpr (REM % 2 == 0) {
        o = u32x4{w[M], w[M + 1], w[M + 2], w[M + 3]};
      } else {
        o = u32x4{__builtin_amdgcn_alignbyte(w[M + 1], w[M], 2), __builtin_amdgcn_alignbyte(w[M + 2], w[M + 1], 2),
                  __builtin_amdgcn_alignbyte(w[M + 3], w[M + 2], 2), __builtin_amdgcn_alignbyte(w[M + 4], w[M + 3], 2)};
      }
      const uint32_t col0 = i - (i / ROW) * ROW;
      if (col0 + 7 < ROW - F && i + 7 < lim) {
        store16B<SC1>(out0 + i, o);
        continue;
      }
      const uint32_t ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t e = i + k;
        if (e >= lim) break;
        if (e - (e / ROW) * ROW < ROW - F) store2B<SC1>(out0 + e, (uint16_t)(ow[k / 2] >> (16 * (k & 1))));
      }
    }
  }
}

// lane `t0` of `stride` lanes: the obs history, then the critic history
__device__ __forceinline__ void shift_history(const ShiftArgs& S, int64_t t0, int64_t stride) {
  if (S.half) {
    shift_range_h<T1_NOBS, T1_HIST>(reinterpret_cast<const uint16_t*>(S.obs_in), reinterpret_cast<uint16_t*>(S.obs_out),
                                    S.total_obs, 0, (S.total_obs + 7) / 8, t0, stride);
    shift_range_h<T1_NPRIV, T1_CHIST>(reinterpret_cast<const uint16_t*>(S.priv_in),
                                      reinterpret_cast<uint16_t*>(S.priv_out), S.total_priv, 0, (S.total_priv + 7) / 8,
                                      t0, stride);
    return;
  }
  shift_range<T1_NOBS, T1_HIST>(S.obs_in, S.obs_out, S.total_obs, 0, (S.total_obs + 3) / 4, t0, stride);
  shift_range<T1_NPRIV, T1_CHIST>(S.priv_in, S.priv_out, S.total_priv, 0, (S.total_priv + 3) / 4, t0, stride);
}

// the rows [r0, r1) of both histories (r0 a multiple of 8, so both row ranges start on a 16-B chunk of either
// element size), with agent-coherent (sc1) stores
template <int U = SHIFT_UNROLL>
__device__ __forceinline__ void shift_rows_range_sc1(const ShiftArgs& S, int64_t r0, int64_t r1, int64_t t0,
                                                 int64_t stride) {
  if (S.half) {
    shift_rows_f16<T1_NOBS, T1_HIST, true, U>(reinterpret_cast<const uint16_t*>(S.obs_in),
                                              reinterpret_cast<uint16_t*>(S.obs_out), S.total_obs, r0, r1, (int)t0,
                                              (int)stride);
    shift_rows_f16<T1_NPRIV, T1_CHIST, true, U>(reinterpret_cast<const uint16_t*>(S.priv_in),
                                                reinterpret_cast<uint16_t*>(S.priv_out), S.total_priv, r0, r1, (int)t0,
                                                (int)stride);
    return;
  }
  shift_rows_f32<T1_NOBS, T1_HIST, true, U>(S.obs_in, S.obs_out, S.total_obs, r0, r1, (int)t0, (int)stride);
  shift_rows_f32<T1_NPRIV, T1_CHIST, true, U>(S.priv_in, S.priv_out, S.total_priv, r0, r1, (int)t0, (int)stride);
}

// zero `count` elements of row `row` (row width `width`) of a history buffer, fp32 or fp16
__device__ __forceinline__ void zero_hist(float* buf, bool half, int64_t row, int width, int count, int t0, int stride) {
  if (half) {
    uint16_t* o = reinterpret_cast<uint16_t*>(buf) + row * width;
    for (int c = t0; c < count; c += stride) o[c] = 0;
  } else {
    float* o = buf + row * width;
    for (int c = t0; c < count; c += stride) o[c] = 0.0f;
  }
}

// reset_idx clears the obs / critic history deques of a reset env (t1_dh_stand_env.py:548-558): the 65 (2)
// older frames of `row` in the freshly shifted output, lane t0 of `stride` lanes
__device__ __forceinline__ void zero_history_row(const ShiftArgs& S, int64_t row, int t0, int stride) {
  zero_hist(S.obs_out, S.half, row, T1_NOBS * T1_HIST, T1_NOBS * (T1_HIST - 1), t0, stride);
  zero_hist(S.priv_out, S.half, row, T1_NPRIV * T1_CHIST, T1_NPRIV * (T1_CHIST - 1), t0, stride);
}

}  // namespace t1
