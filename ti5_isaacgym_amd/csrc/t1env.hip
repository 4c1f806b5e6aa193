// t1env.hip -- MI355X (gfx950) C ABI for the T1 humanoid LeggedRobot.step() hot path, plus the small kernels
// around the step (creation-time DR, reset_all, the split post-physics kernels, the stand-alone history shift).
//
// Per env step (t1env_step), normally ONE launch on the caller's stream and no host sync: k_dyn4 in
// t1env_dynamics.hip runs the 10 substeps, the post-physics epilogue and, in extra workgroups on the CUs the
// dynamics leave idle, the 65/2-frame history shift.  Split sequence (command-curriculum steps, golden parity):
//   k_dyn4<FUSED=false> (+ shift workgroups) -> k_post_a -> k_post_b
//   k_post_a   : base kinematics, command/ext-force callback, termination, 24 rewards (alphabetical),
//                episode sums, per-step extras reduction (legged_robot.py:458-489, 509-517, 654-680)
//   k_post_b   : masked reset_idx, compute_observations -> newest obs/priv frame, last_* bookkeeping, reset-row
//                zeroing, extras finalisation (legged_robot.py:490-502, t1_dh_stand_env.py:368-559)
// At large N (no idle CUs) the shift runs as its own launch (k_shift) ahead of the dynamics.
// See include/t1env.h for the ABI and DESIGN.md for layouts and rooflines.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

#include "../../include/t1env.h"
#include "t1_dynamics.h"
#include "t1_model_conv.h"
#include "t1env_device.h"
#include "t1env_internal.h"
#include "t1env_postphys.h"
#include "t1env_fused.h"

using namespace t1;

namespace {

thread_local char g_err[512] = "";
int fail(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}
#define HIP_TRY(expr)                                                                    \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    if (e_ != hipSuccess) {                                                              \
      snprintf(g_err, sizeof(g_err), "%s: %s", #expr, hipGetErrorString(e_));           \
      return (int)e_;                                                                    \
    }                                                                                    \
  } while (0)

constexpr int BLOCK = 64;  // one wave per workgroup: 8192 envs -> 128 workgroups spread over the CUs

}  // namespace

constexpr int NKERN = 6;  // 0 physics (+ shift), 1 post_a, 2 post_b, 3 shift alone, 4 unused, 5 whole step
constexpr int SHIFT_BLOCKS = 1024;       // grid of the stand-alone k_shift (256 threads)
constexpr int MAX_TIMED = 1 << 14;

struct t1env {
  t1env_config cfg;
  int timing;
  int n_timed;
  int timed_kernel[MAX_TIMED];
  hipEvent_t ev_start[MAX_TIMED], ev_stop[MAX_TIMED];
  int n_events;  // events created so far (reused across enable cycles)
  t1env_buffers buf;
  DynModel* d_model;
  t1env_config* d_cfg;
  Terrain terrain;
  DynLaunch dyn;          // dynamics kernel shape (T1ENV_DYN_WAVES / T1ENV_SHIFT_BLOCKS override; tuning)
  int shift_pending;      // phase A enqueued this step's history shift (phase B alone must run it)
  int fused;              // t1env_step runs the single fused launch (t1env_set_fused; default on)
  uint32_t epoch;         // fused launches so far (tags the shift-unit handoff words)
  uint32_t* d_unit_state; // per shift unit handoff word (fused step)
  int step_timer;         // timing slot of the current step span (phase A start .. phase B end)
  unsigned* d_done;       // k_post_b block-completion counter (its last block finalises the extras)
  float* d_ep_part;       // k_dyn4's per-workgroup partial extras sums (FusedArgs::ep_part)
  int16_t* d_hmax;        // coarse terrain height bound (Terrain::hmax), built by t1env_set_terrain
  float max_contact_radius;
  SubLog log;             // t1env_set_substep_log (tests): fused steps write it
  int log_on;
  hipStream_t side;       // k_dyn5's concurrent history shift (k_shift5), forked from / joined to the step's stream
  hipEvent_t ev_fork, ev_join;
};

// k_physics_injected: the same decimation loop with the physics states supplied by the caller (golden
// parity harness: the reference ran on identical injected states), so PD / lag / sensor capture are checked
// bit-for-bit without a simulator in the loop.
__global__ __launch_bounds__(BLOCK) void k_physics_injected(const DynModel* __restrict__ Mp,
                                                            const t1env_config* __restrict__ Cp, t1env_buffers B,
                                                            const float* __restrict__ actions, t1env_step_args A,
                                                            t1env_injected inj) {
  const int n = blockIdx.x * BLOCK + threadIdx.x;
  const t1env_config& C = *Cp;
  if (n >= C.num_envs) return;
  const DynModel& M = *Mp;
  const uint32_t genv = (uint32_t)(C.env_offset + n);
  const uint32_t ctr = A.counter;
  float* slot = B.act_hist + ((size_t)n * 4 + (ctr & 3u)) * 12;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    float a = fminf(fmaxf(actions[n * 12 + j], -C.clip_actions), C.clip_actions);
    B.actions[n * 12 + j] = a;
    slot[j] = a * C.action_scale;
  }
  const int lag = B.lag_timestep[n];
  const int s_dof = 9 - B.dof_lag_timestep[n] % 10, s_imu = 9 - B.imu_lag_timestep[n] % 10;
  float* dof_dst = B.dof_hist + ((size_t)n * 4 + (ctr & 3u)) * 24;
  float* imu_dst = B.imu_hist + ((size_t)n * 2 + (ctr & 1u)) * 8;
  const int N = C.num_envs;
  float tau[12];
  for (int sub = 0; sub < C.decimation; ++sub) {
    float q[12], qd[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) { q[j] = B.dof_state[n * 24 + 2 * j]; qd[j] = B.dof_state[n * 24 + 2 * j + 1]; }
    pd_torques<12>(M, C, B, n, genv, ctr, sub, lag, 0, q, qd, tau);
    if (inj.torque_log) {
#pragma unroll
      for (int j = 0; j < 12; ++j) inj.torque_log[((size_t)sub * N + n) * 12 + j] = tau[j];
    }
    const float* r = inj.root + ((size_t)sub * N + n) * 13;
    const float* d = inj.dof + ((size_t)sub * N + n) * 24;
#pragma unroll
    for (int i = 0; i < 13; ++i) B.root_states[n * 13 + i] = r[i];
#pragma unroll
    for (int i = 0; i < 24; ++i) B.dof_state[n * 24 + i] = d[i];
    if (sub == s_dof) {
#pragma unroll
      for (int j = 0; j < 12; ++j) { dof_dst[j] = d[2 * j]; dof_dst[12 + j] = d[2 * j + 1]; }
    }
    if (sub == s_imu) {
      float quat[4] = {r[3], r[4], r[5], r[6]}, w[3] = {r[10], r[11], r[12]};
      capture_imu(quat, w, imu_dst);
    }
  }
  for (int i = 0; i < 169; ++i) B.rigid_state[(size_t)n * 169 + i] = inj.rigid[(size_t)n * 169 + i];
  for (int i = 0; i < 39; ++i) B.contact_forces[(size_t)n * 39 + i] = inj.contact[(size_t)n * 39 + i];
#pragma unroll
  for (int j = 0; j < 12; ++j) B.torques[n * 12 + j] = tau[j];
}

// =====================================================================================================
// post-physics phase A: callback, termination, rewards (legged_robot.py:469-489) -- t1env_postphys.h
// =====================================================================================================
__global__ __launch_bounds__(BLOCK) void k_post_a(const DynModel* __restrict__ Mp, const t1env_config* __restrict__ Cp,
                                                  t1env_buffers B, t1env_step_args A) {
  (void)post_a_env(*Mp, *Cp, B, A, blockIdx.x * BLOCK + threadIdx.x);
}

__global__ __launch_bounds__(BLOCK) void k_post_b(const DynModel* __restrict__ Mp, const t1env_config* __restrict__ Cp,
                                                  t1env_buffers B, t1env_step_args A, unsigned* __restrict__ done) {
  const int n = blockIdx.x * BLOCK + threadIdx.x;
  const t1env_config& C = *Cp;
  const bool live = n < C.num_envs;
  const bool do_reset = live && B.reset_buf[n] != 0;
  const bool any_reset = B.ep_accum[24] > 0.0f;
  if (live) post_b_env(*Mp, C, B, A, n, do_reset, any_reset);
  // extras["episode"]["terrain_level"] = mean level over all envs after this step's resets (legged_robot.py:1158)
  if (C.custom_origins && any_reset) wave_atomic_add(B.ep_accum + 25, live ? (float)B.terrain_levels[n] : 0.0f);
  // reset_idx zeroes the obs / critic history of the reset envs (t1:548-558): k_shift wrote the 65 (2) older
  // frames of every row, so the wave zeroes those of its reset envs here, one row at a time, coalesced
  uint64_t m = __ballot(do_reset);
  while (m) {
    const int l = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    const size_t row = (size_t)blockIdx.x * BLOCK + l;
    zero_hist(B.obs_buf[A.obs_slot], C.obs_half, row, T1_NOBS * T1_HIST, T1_NOBS * (T1_HIST - 1), threadIdx.x, BLOCK);
    zero_hist(B.priv_buf[A.obs_slot], C.obs_half, row, T1_NPRIV * T1_CHIST, T1_NPRIV * (T1_CHIST - 1), threadIdx.x,
              BLOCK);
  }
  // the last block to finish finalises the step's extras (no separate launch)
  __threadfence();
  unsigned prev = 0;
  if (threadIdx.x == 0) prev = atomicAdd(done, 1u);
  prev = __shfl(prev, 0, 64);
  if (prev == gridDim.x - 1) {
    __threadfence();
    finalize_extras(B, C, (int)((A.counter + 1u) % T1ENV_EXTRAS_RING));
    if (threadIdx.x == 0) *done = 0u;
  }
}

// history shift for the paths that do not run k_dynamics (injected physics, phase B alone): the same
// shift_history as k_dynamics' tail workgroups, as its own launch on the caller's stream
__global__ __launch_bounds__(256) void k_shift(ShiftArgs S) {
  shift_history(S, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

// chunks per lane in flight in the concurrent shift launch (k_shift5): 93 VGPRs at 4 (8 spills), so one of its waves fits beside
// a k_dyn5 wave on every SIMD
#ifndef T1_D5_SHIFT_UNROLL
#define T1_D5_SHIFT_UNROLL 4
#endif
// ---------------------------------------------------------------------------------------------------
// k_shift5 (compiled here at -O3; the dynamics unit's -O1 spilled its 64-bit addresses): the history shift as a launch of its own, on a second stream beside k_dyn5 (DynLaunch::d5_shift = 1).
// One 256-thread workgroup per CU with no LDS but its handoff words and <= 96 VGPRs per wave, so it fits next to
// the k_dyn5 workgroup on every CU (k_dyn5 holds ~405 of a SIMD's 512 registers and 98 KB of LDS without the
// in-workgroup shift's staging ring) whichever launch the dispatcher places first: the shift's loads and stores
// issue in the dynamics waves' latency gaps instead of on their instruction stream and their vmcnt.  Each
// workgroup shifts a contiguous run of SHIFT_UNIT-row units; FUSED: then hands each unit off (unit_handoff, the
// k_dyn4 protocol, t1env_fused.h) -- whichever of the shift and k_dyn5's epilogue finishes a unit last zeroes its
// reset rows.  Not FUSED (the split step): k_post_b zeroes them after the caller's join.
// ---------------------------------------------------------------------------------------------------
template <bool FUSED, int U>
__device__ __forceinline__ void shift_conc_body(ShiftArgs S, FusedArgs FA, int N) {
  __shared__ uint32_t words[256];
  const int units = (N + SHIFT_UNIT - 1) / SHIFT_UNIT;
  const int nsw = gridDim.x, j = blockIdx.x;
  const int per = (units + nsw - 1) / nsw;
  const int u0 = j * per < units ? j * per : units, u1 = u0 + per < units ? u0 + per : units;
  const int mine = u1 - u0;
  if (mine > 0) {
    const int64_t r0 = (int64_t)u0 * SHIFT_UNIT, r1 = (int64_t)u1 * SHIFT_UNIT < N ? (int64_t)u1 * SHIFT_UNIT : N;
    shift_rows_range_sc1<U>(S, r0, r1, threadIdx.x, 256);
  }
  if constexpr (FUSED) {
    // every lane's sc1 stores complete (visible at agent scope) before any handoff
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int k0 = 0; k0 < mine; k0 += 256) {
      const int k = k0 + (int)threadIdx.x;
      if (k < mine) words[threadIdx.x] = unit_handoff(FA.unit_state + u0 + k, FA.epoch, HANDOFF_SHIFT);
      __syncthreads();
      const int cnt = mine - k0 < 256 ? mine - k0 : 256;
      for (int i = 0; i < cnt; ++i)
        if (handoff_complete(words[i])) zero_unit_resets(S, u0 + k0 + i, words[i], threadIdx.x, 256);
      __syncthreads();
    }
  }
}

template <bool FUSED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 8)))
void k_shift5(ShiftArgs S, FusedArgs FA, int N) {
  shift_conc_body<FUSED, T1_D5_SHIFT_UNROLL>(S, FA, N);
}

// k_shift4c: the same concurrent shift beside k_dyn4 (config 5: 32768 envs, fp16 histories).  A k_dyn4
// wave holds 433 of a SIMD's 512 registers per lane, so a shift wave must stay within 72 (amdgpu_waves_per_eu(7, 8)) to
// share the SIMD; its 148 KB of LDS leaves room for the shift's 1 KB of handoff words.
#ifndef T1_D4_SHIFT_UNROLL
#define T1_D4_SHIFT_UNROLL 3
#endif
template <bool FUSED>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7, 8)))
void k_shift4c(ShiftArgs S, FusedArgs FA, int N) {
  shift_conc_body<FUSED, T1_D4_SHIFT_UNROLL>(S, FA, N);
}

int t1_launch_shift5(const ShiftArgs& S, const FusedArgs* fused, int num_envs, int cus, hipStream_t s, bool beside4) {
  const int units = (num_envs + SHIFT_UNIT - 1) / SHIFT_UNIT;
  const int grid = units < cus ? units : cus;
  if (beside4) {
    if (fused) hipLaunchKernelGGL(k_shift4c<true>, dim3(grid), dim3(256), 0, s, S, *fused, num_envs);
    else hipLaunchKernelGGL(k_shift4c<false>, dim3(grid), dim3(256), 0, s, S, FusedArgs{}, num_envs);
  } else {
    if (fused) hipLaunchKernelGGL(k_shift5<true>, dim3(grid), dim3(256), 0, s, S, *fused, num_envs);
    else hipLaunchKernelGGL(k_shift5<false>, dim3(grid), dim3(256), 0, s, S, FusedArgs{}, num_envs);
  }
  return (int)hipGetLastError();
}

// extras finalisation for t1env_reset_all (one wave)
__global__ void k_finalize(t1env_buffers B, const t1env_config* __restrict__ Cp, int slot) {
  finalize_extras(B, *Cp, slot);
}

// terrain-level sum for extras["episode"]["terrain_level"] (only meaningful on reset steps)
__global__ __launch_bounds__(256) void k_terrain_level_sum(t1env_buffers B, const t1env_config* __restrict__ Cp) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const t1env_config& C = *Cp;
  const float v = (n < C.num_envs && C.custom_origins && B.ep_accum[24] > 0.0f) ? (float)B.terrain_levels[n] : 0.0f;
  wave_atomic_add(B.ep_accum + 25, v);
}

// -----------------------------------------------------------------------------------------------------
// Height scan (terrain.measure_heights; inactive in DHT1StandCfg).  k_measure_heights restates _get_heights
// (legged_robot.py:1551-1587) with quat_apply_yaw (utils/math.py:8-12) for every (env, point): the base-frame
// point rotated by the base yaw, offset by the base position and the border, truncated to a sample (`.long()`),
// clipped to [0, rows-2] x [0, cols-2], min of the sample and its +x / +y neighbours, times vertical_scale.  The
// sample index is discontinuous in the coordinates, so the chain is computed with the reference's fp32
// roundings (no FMA contraction, true division).  One thread per (env, point); reads root_states, which
// t1env_step_physics_and_rewards left at the post-physics, pre-reset pose the reference's callback samples.
// k_critic_heights assembles the critic history with heights (t1_dh_stand_env.py:466-468, 548-558): one
// thread per (env, column) of (N, 3, 73 + npts).
// -----------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_measure_heights(const float* __restrict__ root, const float* __restrict__ pts,
                                                         int npts, int N, Terrain T, float* __restrict__ measured) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * npts) return;
  const int n = (int)(i / npts), p = (int)(i - (int64_t)n * npts);
  if (T.type == 0) {  // plane (legged_robot.py:1564-1565)
    measured[i] = 0.0f;
    return;
  }
  const float* r = root + (size_t)n * 13;
  // normalize((0, 0, qz, qw)) with the norm clamped at 1e-9 (torch_utils.normalize)
  float qz = r[5], qw = r[6];
  const float nrm = fmaxf(__fsqrt_rn(__fadd_rn(__fmul_rn(qz, qz), __fmul_rn(qw, qw))), 1e-9f);
  qz = __fdiv_rn(qz, nrm);
  qw = __fdiv_rn(qw, nrm);
  // quat_apply(q, v), v = (px, py, 0): t = 2 (q_xyz x v); v + w t + q_xyz x t
  const float px = pts[2 * p], py = pts[2 * p + 1];
  const float tx = __fmul_rn(-__fmul_rn(qz, py), 2.0f), ty = __fmul_rn(__fmul_rn(qz, px), 2.0f);
  float x = __fadd_rn(__fadd_rn(px, __fmul_rn(qw, tx)), -__fmul_rn(qz, ty));
  float y = __fadd_rn(__fadd_rn(py, __fmul_rn(qw, ty)), __fmul_rn(qz, tx));
  x = __fadd_rn(__fadd_rn(x, r[0]), T.border);
  y = __fadd_rn(__fadd_rn(y, r[1]), T.border);
  int ix = (int)truncf(__fdiv_rn(x, T.hscale)), iy = (int)truncf(__fdiv_rn(y, T.hscale));
  ix = min(max(ix, 0), T.rows - 2);
  iy = min(max(iy, 0), T.cols - 2);
  const int16_t* h = T.h + (size_t)ix * T.cols + iy;
  const int hm = min(min((int)h[0], (int)h[T.cols]), (int)h[1]);
  measured[i] = __fmul_rn((float)hm, T.vscale);
}

__global__ __launch_bounds__(256) void k_critic_heights(const float* __restrict__ priv, const float* __restrict__ root,
                                                        const uint8_t* __restrict__ reset,
                                                        const float* __restrict__ measured,
                                                        const float* __restrict__ prev, float* __restrict__ out,
                                                        int npts, int N, float scale, float clip_obs) {
  const int W = T1_NPRIV + npts, RW = T1_CHIST * W;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)N * RW) return;
  const int n = (int)(i / RW), c = (int)(i - (int64_t)n * RW);
  const int f = c / W, k = c - f * W;
  float v;
  if (k < T1_NPRIV) {
    v = priv[(size_t)n * (T1_NPRIV * T1_CHIST) + f * T1_NPRIV + k];
  } else if (f < T1_CHIST - 1) {  // older frames: shifted by one, cleared for envs reset this step
    v = reset[n] ? 0.0f : prev[(size_t)n * RW + (f + 1) * W + k];
  } else {
    const float d = __fadd_rn(__fadd_rn(root[(size_t)n * 13 + 2], -0.5f), -measured[(size_t)n * npts + (k - T1_NPRIV)]);
    v = fminf(fmaxf(__fmul_rn(fminf(fmaxf(d, -1.0f), 1.0f), scale), -clip_obs), clip_obs);
  }
  out[i] = v;
}

// creation-time state (see t1env_init in include/t1env.h)
__global__ __launch_bounds__(BLOCK) void k_init(const DynModel* __restrict__ Mp, const t1env_config* __restrict__ Cp,
                                                t1env_buffers B) {
  const int n = blockIdx.x * BLOCK + threadIdx.x;
  const t1env_config& C = *Cp;
  if (n >= C.num_envs) return;
  const DynModel& M = *Mp;
  const uint32_t genv = (uint32_t)(C.env_offset + n), seed = C.seed, ctr = 0;
  const float payload = C.dr_base_mass
      ? rand_float(C.added_mass_range[0], C.added_mass_range[1], seed, genv, ctr, SLOT_PAYLOAD) : 0.0f;
  B.body_mass[n] = M.mass[0] + payload;
  for (int b = 0; b < 12; ++b)
    B.link_mass_scale[n * 12 + b] = C.dr_link_mass
        ? rand_float(C.link_mass_range[0], C.link_mass_range[1], seed, genv, ctr, SLOT_LINK_MASS + b) : 1.0f;
  for (int k = 0; k < 3; ++k)
    B.com_disp[n * 3 + k] = C.dr_com ? rand_float(C.com_range[k][0], C.com_range[k][1], seed, genv, ctr, SLOT_COM + k) : 0.0f;
  if (C.dr_friction) {  // 256 buckets; env -> bucket id, bucket -> (friction, restitution)
    const uint32_t bucket = (uint32_t)rand_int(0, 256, seed, genv, ctr, SLOT_FRICTION_BUCKET);
    B.friction[n] = rand_float(C.friction_range[0], C.friction_range[1], seed, bucket, 0, SLOT_FRICTION_VALUE);
    B.restitution[n] = rand_float(C.restitution_range[0], C.restitution_range[1], seed, bucket, 0, SLOT_RESTITUTION_VALUE);
  } else {
    B.friction[n] = 0.0f;
    B.restitution[n] = 0.0f;
  }
  if (C.custom_origins) {
    const int lv = rand_int(0, C.max_init_terrain_level + 1, seed, genv, ctr, SLOT_TERRAIN_LEVEL_INIT);
    const int ty = (int)floorf((float)genv / ((float)C.num_envs_total / (float)C.num_terrain_cols));
    B.terrain_levels[n] = lv;
    B.terrain_types[n] = ty;
    const float* to = B.terrain_origins + ((size_t)lv * C.num_terrain_cols + ty) * 3;
    for (int k = 0; k < 3; ++k) B.env_origins[n * 3 + k] = to[k];
  }
  B.gait_start[n] = (float)rand_int(0, 2, seed, genv, ctr, SLOT_GAIT_START) * 0.5f;
  B.lag_timestep[n] = rand_int(C.lag_range[0], C.lag_range[1] + 1, seed, genv, ctr, SLOT_LAG_ACTION);
  B.dof_lag_timestep[n] = rand_int(C.dof_lag_range[0], C.dof_lag_range[1] + 1, seed, genv, ctr, SLOT_LAG_DOF);
  B.imu_lag_timestep[n] = rand_int(C.imu_lag_range[0], C.imu_lag_range[1] + 1, seed, genv, ctr, SLOT_LAG_IMU);
  // start pose: origin + U(-1,1) xy jitter (legged_robot.py:1380-1383); DOF at the default pose
  float* r = B.root_states + n * 13;
  for (int i = 0; i < 13; ++i) r[i] = M.base_init_state[i];
  for (int k = 0; k < 3; ++k) r[k] += B.env_origins[n * 3 + k];
  r[0] += rand_float(-1.0f, 1.0f, seed, genv, ctr, SLOT_START_XY + 0);
  r[1] += rand_float(-1.0f, 1.0f, seed, genv, ctr, SLOT_START_XY + 1);
  for (int j = 0; j < 12; ++j) { B.dof_state[n * 24 + 2 * j] = M.default_dof_pos[j]; B.dof_state[n * 24 + 2 * j + 1] = 0.0f; }
  for (int i = 0; i < 169; ++i) B.rigid_state[(size_t)n * 169 + i] = (i % 13 == 6) ? 1.0f : 0.0f;
  for (int i = 0; i < 39; ++i) B.contact_forces[(size_t)n * 39 + i] = 0.0f;
  for (int j = 0; j < 12; ++j) {  // gains are still zero when randomize_dof_props first runs
    B.kp[n * 12 + j] = 0.0f; B.kd[n * 12 + j] = 0.0f; B.motor_offsets[n * 12 + j] = 0.0f;
    B.coulomb[n * 12 + j] = 0.0f; B.viscous[n * 12 + j] = 0.0f; B.armature[n * 12 + j] = 0.0f;
  }
}

// reset_idx(arange(N)) -- LeggedRobot.reset() (legged_robot.py:450-455)
// reset_idx of every env (mask == nullptr: t1env_reset_all) or of the masked envs (t1env_reset_idx)
__global__ __launch_bounds__(BLOCK) void k_reset_all(const DynModel* __restrict__ Mp, const t1env_config* __restrict__ Cp,
                                                     t1env_buffers B, t1env_step_args A,
                                                     const uint8_t* __restrict__ mask) {
  const int n0 = blockIdx.x * BLOCK + threadIdx.x;
  const t1env_config& C = *Cp;
  const bool live = n0 < C.num_envs && (mask == nullptr || mask[n0] != 0);
  const int n = live ? n0 : C.num_envs - 1;
  float contrib[T1_NREW];
  for (int k = 0; k < T1_NREW; ++k) contrib[k] = live ? B.episode_sums[(size_t)k * C.num_envs + n] : 0.0f;
  for (int k = 0; k < T1_NREW; ++k) wave_atomic_add(B.ep_accum + k, contrib[k]);
  wave_atomic_add(B.ep_accum + 24, live ? 1.0f : 0.0f);
  if (!live) return;
  const uint32_t genv = (uint32_t)(C.env_offset + n);
  // t1env_reset_idx (mask), and t1env_reset_all after the first step (env.reset() on a stepped env): the between-step
  // key domain, so an env reset in the step that produced A.counter draws fresh values here (t1_common.h
  // T1_BETWEEN_STEP_SALT; oracle T1Oracle.reset)
  const uint32_t key_ctr = (mask || A.counter > 0) ? (A.counter | T1_BETWEEN_STEP_SALT) : A.counter;
  reset_env(*Mp, C, B, A, n, genv, key_ctr, true);
  resample_commands(C, B, A, n, genv, key_ctr);
}

// reset_idx's obs / critic history clearing (t1_dh_stand_env.py:553-558) for the masked envs: every frame of
// their rows in the buffer the next step shifts from; one workgroup per env
__global__ __launch_bounds__(256) void k_zero_masked_rows(float* __restrict__ obs, float* __restrict__ priv,
                                                          const uint8_t* __restrict__ mask, int N, int half) {
  const int n = blockIdx.x;
  if (n >= N || mask[n] == 0) return;
  zero_hist(obs, half, n, T1_NOBS * T1_HIST, T1_NOBS * T1_HIST, threadIdx.x, blockDim.x);
  zero_hist(priv, half, n, T1_NPRIV * T1_CHIST, T1_NPRIV * T1_CHIST, threadIdx.x, blockDim.x);
}

// coarse height bound: out[ci][cj] = max height sample of rows [(ci-K)c, (ci+K+1)c] x cols [(cj-K)c, (cj+K+1)c]
// (clamped), c = HMAX_CELL -- every triangle a point within K cells of coarse cell (ci, cj) can fall on.
constexpr int HMAX_CELL = 3;
__global__ void k_hmax(const int16_t* __restrict__ h, int rows, int cols, int16_t* __restrict__ out, int hr, int hc,
                       int K) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= hr * hc) return;
  const int ci = t / hc, cj = t % hc;
  const int r0 = max(0, (ci - K) * HMAX_CELL), r1 = min(rows - 1, (ci + K + 1) * HMAX_CELL);
  const int c0 = max(0, (cj - K) * HMAX_CELL), c1 = min(cols - 1, (cj + K + 1) * HMAX_CELL);
  int m = -32768;
  for (int r = r0; r <= r1; ++r)
    for (int c = c0; c <= c1; ++c) m = max(m, (int)h[(size_t)r * cols + c]);
  out[t] = (int16_t)m;
}

// =====================================================================================================
// C ABI
// =====================================================================================================
static int grid(int n, int b) { return (n + b - 1) / b; }

// timing bracket around one launch: returns the slot (or -1 when timing is off / full)
static int t_begin(t1env* e, int kid, hipStream_t s) {
  if (!e->timing || e->n_timed >= MAX_TIMED) return -1;
  const int i = e->n_timed++;
  if (i >= e->n_events) {
    if (hipEventCreate(&e->ev_start[i]) != hipSuccess || hipEventCreate(&e->ev_stop[i]) != hipSuccess) return -1;
    e->n_events = i + 1;
  }
  e->timed_kernel[i] = kid;
  (void)hipEventRecord(e->ev_start[i], s);
  return i;
}
static void t_end(t1env* e, int i, hipStream_t s) {
  if (i >= 0) (void)hipEventRecord(e->ev_stop[i], s);
}

extern "C" {

const char* t1env_last_error(void) { return g_err; }
#ifndef T1_SOURCE_STAMP  // ti5_isaacgym_amd/build.py source_stamp(): the hash of the sources this library is built from
#define T1_SOURCE_STAMP "unstamped"
#endif
const char* t1env_version(void) { return "t1env-hip 0.1 (gfx950) src:" T1_SOURCE_STAMP; }

// one EP_PART_ROW-float row per k_dyn4 dynamics workgroup
// one row per dynamics workgroup: k_dyn5 has 32 envs per workgroup (k_dyn4 64)
static size_t ep_part_bytes(int num_envs) { return sizeof(float) * EP_PART_ROW * (size_t)((num_envs + 31) / 32); }

int t1env_create(const t1env_model* model, const t1env_config* cfg, const t1env_buffers* bufs, t1env** out) {
  if (!model || !cfg || !bufs || !out) return fail(T1ENV_E_ARG, "t1env_create: null argument");
  if (cfg->num_envs <= 0) return fail(T1ENV_E_SHAPE, "t1env_create: num_envs must be > 0");
  if (cfg->decimation <= 0 || cfg->decimation > 64) return fail(T1ENV_E_ARG, "t1env_create: bad decimation");
  if (model->n_contact > T1_MAXC) return fail(T1ENV_E_SHAPE, "t1env_create: too many contact points");
  for (int i = 0; i < 3; ++i) {
    if (cfg->lag_range[1] > 30 || cfg->dof_lag_range[1] > 30 || cfg->imu_lag_range[1] > 10 || cfg->lag_range[0] < 0 ||
        cfg->dof_lag_range[0] < 0 || cfg->imu_lag_range[0] < 0)
      return fail(T1ENV_E_ARG, "t1env_create: lag ranges must lie in [0,30] (dof/action) and [0,10] (imu)");
  }
  if (cfg->obs_half != 0 && cfg->obs_half != 1) return fail(T1ENV_E_ARG, "t1env_create: obs_half must be 0 or 1");
  if (cfg->decimation != 10 && (cfg->lag_range[1] > 0 || cfg->dof_lag_range[1] > 0 || cfg->imu_lag_range[1] > 0))
    return fail(T1ENV_E_ARG, "t1env_create: sensor/actuator lag rings assume decimation == 10");
  DynModel dm;
  if (const char* err = make_dyn_model(model, &dm)) return fail(T1ENV_E_ARG, err);
  if (const char* err = check_fixed_contact_layout(dm)) return fail(T1ENV_E_ARG, err);
  t1env* e = (t1env*)calloc(1, sizeof(t1env));
  if (!e) return fail(T1ENV_E_STATE, "t1env_create: out of host memory");
  e->cfg = *cfg;
  e->buf = *bufs;
  e->terrain = make_terrain(nullptr, 0, 0, 0, 0.1f, 0.005f, 0.0f);
  hipError_t err;
  if ((err = hipMalloc(&e->d_model, sizeof(DynModel))) != hipSuccess ||
      (err = hipMalloc(&e->d_cfg, sizeof(t1env_config))) != hipSuccess ||
      (err = hipMalloc(&e->d_done, sizeof(unsigned))) != hipSuccess ||
      (err = hipMalloc(&e->d_unit_state, sizeof(uint32_t) * (size_t)(cfg->num_envs / 8 + 1))) != hipSuccess ||
      (err = hipMalloc(&e->d_ep_part, ep_part_bytes(cfg->num_envs))) != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "t1env_create: hipMalloc: %s", hipGetErrorString(err));
    free(e);
    return (int)err;
  }
  HIP_TRY(hipMemcpy(e->d_model, &dm, sizeof(DynModel), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_cfg, cfg, sizeof(t1env_config), hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(e->buf.ep_accum, 0, 32 * sizeof(float)));
  HIP_TRY(hipMemset(e->d_done, 0, sizeof(unsigned)));
  HIP_TRY(hipMemset(e->d_unit_state, 0, sizeof(uint32_t) * (size_t)(cfg->num_envs / 8 + 1)));
  HIP_TRY(hipMemset(e->d_ep_part, 0, ep_part_bytes(cfg->num_envs)));
  e->fused = 1;
  {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess) cus = 256;
    e->dyn.cus = cus;
    e->dyn.waves = t1_dyn_waves_default(cfg->num_envs, cus, cfg->obs_half != 0);
    if (const char* dk = getenv("T1ENV_DYN_KERNEL"))  // A/B: 4 = k_dyn4, 5 = k_dyn5, 6 = k_dyn6
      if (atoi(dk) >= 4 && atoi(dk) <= 6) e->dyn.waves = atoi(dk);
    e->dyn.shift_blocks = 0;
    if (const char* sb = getenv("T1ENV_SHIFT_BLOCKS"))  // > 0: shift workgroups in the launch; -1: stand-alone shift
      if (atoi(sb) > 0 || atoi(sb) == -1) e->dyn.shift_blocks = atoi(sb);
    e->dyn.shift_delay = T1_SHIFT_DELAY_DEFAULT;
    e->dyn.d5_shift = 0;
    if (const char* ds = getenv("T1ENV_D5_SHIFT"))  // A/B: 1 = the shift as a concurrent launch (k_shift5)
      if (atoi(ds) == 0 || atoi(ds) == 1) e->dyn.d5_shift = atoi(ds);
    e->dyn.d4_shift = 1;
    if (const char* ds = getenv("T1ENV_D4_SHIFT"))  // A/B: 0 = k_dyn4's stand-alone shift ahead of it, in stream order
      if (atoi(ds) == 0 || atoi(ds) == 1) e->dyn.d4_shift = atoi(ds);
    if (const char* sd = getenv("T1ENV_SHIFT_DELAY"))  // tuning: delayed start of the in-launch shift (100 MHz ticks)
      if (atoi(sd) >= 0) e->dyn.shift_delay = atoi(sd);
  }
  for (int b = 0; b < NB; ++b) e->max_contact_radius = fmaxf(e->max_contact_radius, dm.contact_radius[b]);
  HIP_TRY(hipStreamCreateWithFlags(&e->side, hipStreamNonBlocking));
  HIP_TRY(hipEventCreateWithFlags(&e->ev_fork, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&e->ev_join, hipEventDisableTiming));
  *out = e;
  return 0;
}

int t1env_destroy(t1env* e) {
  if (!e) return 0;
  (void)hipFree(e->d_model);
  (void)hipFree(e->d_cfg);
  (void)hipFree(e->d_done);
  (void)hipFree(e->d_unit_state);
  (void)hipFree(e->d_ep_part);
  if (e->d_hmax) (void)hipFree(e->d_hmax);
  if (e->side) (void)hipStreamDestroy(e->side);
  if (e->ev_fork) (void)hipEventDestroy(e->ev_fork);
  if (e->ev_join) (void)hipEventDestroy(e->ev_join);
  for (int i = 0; i < e->n_events; ++i) {
    (void)hipEventDestroy(e->ev_start[i]);
    (void)hipEventDestroy(e->ev_stop[i]);
  }
  free(e);
  return 0;
}

int t1env_init(t1env* e, void* stream) {
  if (!e) return fail(T1ENV_E_ARG, "t1env_init: null env");
  const int N = e->cfg.num_envs;
  hipLaunchKernelGGL(k_init, dim3(grid(N, BLOCK)), dim3(BLOCK), 0, (hipStream_t)stream, e->d_model, e->d_cfg, e->buf);
  HIP_TRY(hipGetLastError());
  return 0;
}

int t1env_set_terrain(t1env* e, const int16_t* h, int32_t rows, int32_t cols, float hs, float vs, float border,
                      int32_t mesh_type) {
  if (!e) return fail(T1ENV_E_ARG, "t1env_set_terrain: null env");
  if (mesh_type != 0 && (!h || rows < 2 || cols < 2)) return fail(T1ENV_E_SHAPE, "t1env_set_terrain: bad height field");
  e->terrain = make_terrain(h, rows, cols, mesh_type, hs, vs, border);
  if (e->d_hmax) {
    (void)hipFree(e->d_hmax);
    e->d_hmax = nullptr;
  }
  if (mesh_type != 0) {
    // coarse cells of HMAX_CELL samples; window K cells each side with K * cell >= every contact radius
    const int hr = (rows + HMAX_CELL - 1) / HMAX_CELL, hc = (cols + HMAX_CELL - 1) / HMAX_CELL;
    const int K = (int)ceilf(e->max_contact_radius / (HMAX_CELL * hs));
    HIP_TRY(hipMalloc(&e->d_hmax, sizeof(int16_t) * (size_t)hr * hc));
    hipLaunchKernelGGL(k_hmax, dim3(grid(hr * hc, 256)), dim3(256), 0, 0, h, rows, cols, e->d_hmax, hr, hc, K);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(0));
    e->terrain.hmax = e->d_hmax;
    e->terrain.hm_rows = hr;
    e->terrain.hm_cols = hc;
    e->terrain.hm_inv_cell = 1.0f / (HMAX_CELL * hs);
  }
  return 0;
}

static ShiftArgs shift_args(const t1env* e, const t1env_step_args* a) {
  const int64_t N = e->cfg.num_envs;
  const int in = a->obs_slot ^ 1, out = a->obs_slot;
  return ShiftArgs{e->buf.obs_buf[in], e->buf.obs_buf[out], e->buf.priv_buf[in], e->buf.priv_buf[out],
                   N * T1_NOBS * T1_HIST, N * T1_NPRIV * T1_CHIST, e->cfg.obs_half ? 1 : 0};
}

// the history shift as its own launch, in stream order (paths without k_dynamics)
static int launch_shift(t1env* e, const t1env_step_args* a, hipStream_t s) {
  const int t = t_begin(e, 3, s);
  hipLaunchKernelGGL(k_shift, dim3(SHIFT_BLOCKS), dim3(256), 0, s, shift_args(e, a));
  t_end(e, t, s);
  HIP_TRY(hipGetLastError());
  return 0;
}

// The concurrent shift: k_dyn5 with DynLaunch::d5_shift, or k_dyn4 where its shift would otherwise run as its own
// launch ahead of it (t1_shift_prelaunch: config 5) with DynLaunch::d4_shift.  The side stream starts after everything
// enqueued on s so far (fork), runs the shift beside the dynamics launch, and s waits for it before anything after the
// step (join).  The fused epilogue and the shift hand each 8-row unit off (the k_dyn4 protocol, t1env_fused.h).
static bool concurrent_shift4(const t1env* e) {
  return e->dyn.waves == 4 && e->dyn.d4_shift == 1 && t1_shift_prelaunch(e->cfg.num_envs, e->dyn);
}
static bool concurrent_shift(const t1env* e) {
  return (e->dyn.waves == 5 && e->dyn.d5_shift == 1) || concurrent_shift4(e);
}
static int shift_fork(t1env* e, hipStream_t s) {
  HIP_TRY(hipEventRecord(e->ev_fork, s));
  HIP_TRY(hipStreamWaitEvent(e->side, e->ev_fork, 0));
  return 0;
}
static int shift_join(t1env* e, const t1env_step_args* a, const FusedArgs* fa, hipStream_t s) {
  const int t = t_begin(e, 3, e->side);  // the shift's own span, on its stream (bench.py: k_shift)
  HIP_TRY((hipError_t)t1_launch_shift5(shift_args(e, a), fa, e->cfg.num_envs, e->dyn.cus, e->side,
                                       e->dyn.waves == 4));
  t_end(e, t, e->side);
  HIP_TRY(hipEventRecord(e->ev_join, e->side));
  HIP_TRY(hipStreamWaitEvent(s, e->ev_join, 0));
  return 0;
}

static int launch_physics(t1env* e, const float* actions, const t1env_step_args* a, const t1env_injected* inj,
                          hipStream_t s) {
  if (a->obs_slot != 0 && a->obs_slot != 1) return fail(T1ENV_E_ARG, "obs_slot must be 0 or 1");
  if (e->log_on && !inj) return fail(T1ENV_E_STATE, "substep log set: only the fused step logs (t1env_set_substep_log)");
  const int N = e->cfg.num_envs;
  e->step_timer = t_begin(e, 5, s);
  // large N: the shift as its own launch, ahead of the dynamics or beside them (k_post_b zeroes the reset rows after
  // the join)
  const bool conc = !inj && concurrent_shift(e);
  const bool pre = !inj && t1_shift_prelaunch(N, e->dyn);
  if (pre && !conc)
    if (int rc = launch_shift(e, a, s)) return rc;
  if (conc)
    if (int rc = shift_fork(e, s)) return rc;
  int t = t_begin(e, 0, s);
  if (inj)
    hipLaunchKernelGGL(k_physics_injected, dim3(grid(N, BLOCK)), dim3(BLOCK), 0, s, e->d_model, e->d_cfg, e->buf,
                       actions, *a, *inj);
  else
    HIP_TRY((hipError_t)t1_launch_dynamics(e->d_model, e->d_cfg, e->buf, e->terrain, actions, *a, N,
                                           shift_args(e, a), e->dyn, nullptr, s, pre));
  t_end(e, t, s);
  HIP_TRY(hipGetLastError());
  if (conc)
    if (int rc = shift_join(e, a, nullptr, s)) return rc;
  if (inj) {
    if (int rc = launch_shift(e, a, s)) return rc;
  }
  e->shift_pending = 1;
  t = t_begin(e, 1, s);
  hipLaunchKernelGGL(k_post_a, dim3(grid(N, BLOCK)), dim3(BLOCK), 0, s, e->d_model, e->d_cfg, e->buf, *a);
  t_end(e, t, s);
  HIP_TRY(hipGetLastError());
  return 0;
}

int t1env_step_physics_and_rewards(t1env* e, const float* actions, const t1env_step_args* a, void* stream) {
  if (!e || !actions || !a) return fail(T1ENV_E_ARG, "t1env_step_physics_and_rewards: null argument");
  return launch_physics(e, actions, a, nullptr, (hipStream_t)stream);
}

int t1env_step_injected(t1env* e, const float* actions, const t1env_step_args* a, const t1env_injected* inj,
                        void* stream) {
  if (!e || !actions || !a || !inj || !inj->root || !inj->dof || !inj->rigid || !inj->contact)
    return fail(T1ENV_E_ARG, "t1env_step_injected: null argument");
  return launch_physics(e, actions, a, inj, (hipStream_t)stream);
}

int t1env_step_reset_and_observe(t1env* e, const t1env_step_args* a, void* stream) {
  if (!e || !a) return fail(T1ENV_E_ARG, "t1env_step_reset_and_observe: null argument");
  if (a->obs_slot != 0 && a->obs_slot != 1) return fail(T1ENV_E_ARG, "obs_slot must be 0 or 1");
  hipStream_t s = (hipStream_t)stream;
  const int N = e->cfg.num_envs;
  if (!e->shift_pending) {  // phase B without phase A on this env: shift now, in order
    e->step_timer = -1;
    if (int rc = launch_shift(e, a, s)) return rc;
  }
  e->shift_pending = 0;
  int t = t_begin(e, 2, s);
  hipLaunchKernelGGL(k_post_b, dim3(grid(N, BLOCK)), dim3(BLOCK), 0, s, e->d_model, e->d_cfg, e->buf, *a,
                     e->d_done);
  t_end(e, t, s);
  HIP_TRY(hipGetLastError());
  t_end(e, e->step_timer, s);
  e->step_timer = -1;
  return 0;
}

// the whole step as one launch (t1env_dynamics.hip, FUSED)
static int launch_fused(t1env* e, const float* actions, const t1env_step_args* a, hipStream_t s) {
  if (a->obs_slot != 0 && a->obs_slot != 1) return fail(T1ENV_E_ARG, "obs_slot must be 0 or 1");
  e->step_timer = t_begin(e, 5, s);
  // large N: no idle CUs for shift workgroups -- the shift runs as its own launch, beside the dynamics (concurrent:
  // the epilogue hands its reset rows off) or first (the epilogue then zeroes them without the handoff)
  const bool conc = concurrent_shift(e);
  const bool pre = t1_shift_prelaunch(e->cfg.num_envs, e->dyn);
  if (pre && !conc)
    if (int rc = launch_shift(e, a, s)) return rc;
  if (conc)
    if (int rc = shift_fork(e, s)) return rc;
  const int t = t_begin(e, 0, s);
  const FusedArgs FA{e->d_done, e->d_unit_state, ++e->epoch, (pre && !conc) ? 1 : 0, e->d_ep_part};
  HIP_TRY((hipError_t)t1_launch_dynamics(e->d_model, e->d_cfg, e->buf, e->terrain, actions, *a, e->cfg.num_envs,
                                         shift_args(e, a), e->dyn, &FA, s, pre, e->log_on ? &e->log : nullptr));
  t_end(e, t, s);
  if (conc)
    if (int rc = shift_join(e, a, &FA, s)) return rc;
  t_end(e, e->step_timer, s);
  e->step_timer = -1;
  e->shift_pending = 0;
  return 0;
}

int t1env_set_fused(t1env* e, int32_t enable) {
  if (!e) return fail(T1ENV_E_ARG, "t1env_set_fused: null env");
  e->fused = enable ? 1 : 0;
  return 0;
}

int t1env_set_substep_log(t1env* e, const t1env_substep_log* log) {
  if (!e) return fail(T1ENV_E_ARG, "t1env_set_substep_log: null env");
  if (!log) {
    e->log_on = 0;
    e->log = SubLog{};
    return 0;
  }
  if (!log->root || !log->dof || !log->torque) return fail(T1ENV_E_ARG, "t1env_set_substep_log: null buffer");
  e->log = SubLog{log->root, log->dof, log->torque};
  e->log_on = 1;
  return 0;
}

int t1env_measure_heights(t1env* e, const float* points, int32_t npts, float* measured, void* stream) {
  if (!e || !points || !measured || npts <= 0) return fail(T1ENV_E_ARG, "t1env_measure_heights: bad argument");
  const int N = e->cfg.num_envs;
  if (e->terrain.type != 0 && !e->terrain.h) return fail(T1ENV_E_STATE, "t1env_measure_heights: no terrain set");
  const int64_t total = (int64_t)N * npts;
  hipLaunchKernelGGL(k_measure_heights, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     e->buf.root_states, points, npts, N, e->terrain, measured);
  HIP_TRY(hipGetLastError());
  return 0;
}

int t1env_critic_heights(t1env* e, int32_t obs_slot, int32_t npts, float scale, const float* measured,
                         const float* prev, float* out, void* stream) {
  if (!e || !measured || !prev || !out || npts <= 0 || (obs_slot & ~1))
    return fail(T1ENV_E_ARG, "t1env_critic_heights: bad argument");
  if (e->cfg.obs_half) return fail(T1ENV_E_STATE, "t1env_critic_heights: fp16 histories (obs_half) are not supported");
  const int N = e->cfg.num_envs;
  const int64_t total = (int64_t)N * T1_CHIST * (T1_NPRIV + npts);
  hipLaunchKernelGGL(k_critic_heights, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     e->buf.priv_buf[obs_slot], e->buf.root_states, e->buf.reset_buf, measured, prev, out, npts, N,
                     scale, e->cfg.clip_obs);
  HIP_TRY(hipGetLastError());
  return 0;
}

int t1env_step(t1env* e, const float* actions, const t1env_step_args* a, void* stream) {
  if (!e || !actions || !a) return fail(T1ENV_E_ARG, "t1env_step: null argument");
  if (e->fused) return launch_fused(e, actions, a, (hipStream_t)stream);
  int rc = t1env_step_physics_and_rewards(e, actions, a, stream);
  if (rc) return rc;
  return t1env_step_reset_and_observe(e, a, stream);
}

int t1env_set_timing(t1env* e, int32_t enable) {
  if (!e) return fail(T1ENV_E_ARG, "t1env_set_timing: null env");
  e->timing = (enable & 1) ? 1 : 0;
  if (!(enable & 2)) e->n_timed = 0;  // bit 1: keep the events recorded so far (sampled timing)
  return 0;
}

int t1env_get_timing(t1env* e, double* ms, int32_t* launches) {
  if (!e || !ms || !launches) return fail(T1ENV_E_ARG, "t1env_get_timing: null argument");
  for (int k = 0; k < NKERN; ++k) { ms[k] = 0.0; launches[k] = 0; }
  if (e->n_timed > 0) HIP_TRY(hipEventSynchronize(e->ev_stop[e->n_timed - 1]));
  for (int i = 0; i < e->n_timed; ++i) {
    float t = 0.0f;
    HIP_TRY(hipEventElapsedTime(&t, e->ev_start[i], e->ev_stop[i]));
    ms[e->timed_kernel[i]] += t;
    launches[e->timed_kernel[i]] += 1;
  }
  return 0;
}

int t1env_reset_all(t1env* e, const t1env_step_args* a, void* stream) {
  if (!e || !a) return fail(T1ENV_E_ARG, "t1env_reset_all: null argument");
  hipStream_t s = (hipStream_t)stream;
  const int N = e->cfg.num_envs;
  hipLaunchKernelGGL(k_reset_all, dim3(grid(N, BLOCK)), dim3(BLOCK), 0, s, e->d_model, e->d_cfg, e->buf, *a,
                     (const uint8_t*)nullptr);
  HIP_TRY(hipGetLastError());
  if (e->cfg.custom_origins) {
    hipLaunchKernelGGL(k_terrain_level_sum, dim3(grid(N, 256)), dim3(256), 0, s, e->buf, e->d_cfg);
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s, e->buf, e->d_cfg, (int)(a->counter % T1ENV_EXTRAS_RING));
  HIP_TRY(hipGetLastError());
  // every history row restarts from zeros: clear both ping-pong buffers (the next step shifts from either)
  for (int k = 0; k < 2; ++k) {
    const size_t es = e->cfg.obs_half ? 2 : 4;
    HIP_TRY(hipMemsetAsync(e->buf.obs_buf[k], 0, es * (size_t)N * T1_NOBS * T1_HIST, s));
    HIP_TRY(hipMemsetAsync(e->buf.priv_buf[k], 0, es * (size_t)N * T1_NPRIV * T1_CHIST, s));
  }
  return 0;
}

int t1env_reset_idx(t1env* e, const uint8_t* mask, const t1env_step_args* a, void* stream) {
  if (!e || !mask || !a) return fail(T1ENV_E_ARG, "t1env_reset_idx: null argument");
  if (a->obs_slot & ~1) return fail(T1ENV_E_ARG, "t1env_reset_idx: obs_slot must be 0 or 1");
  hipStream_t s = (hipStream_t)stream;
  const int N = e->cfg.num_envs;
  hipLaunchKernelGGL(k_reset_all, dim3(grid(N, BLOCK)), dim3(BLOCK), 0, s, e->d_model, e->d_cfg, e->buf, *a, mask);
  HIP_TRY(hipGetLastError());
  if (e->cfg.custom_origins) {
    hipLaunchKernelGGL(k_terrain_level_sum, dim3(grid(N, 256)), dim3(256), 0, s, e->buf, e->d_cfg);
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s, e->buf, e->d_cfg, (int)(a->counter % T1ENV_EXTRAS_RING));
  HIP_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_zero_masked_rows, dim3(N), dim3(256), 0, s, e->buf.obs_buf[a->obs_slot],
                     e->buf.priv_buf[a->obs_slot], mask, N, e->cfg.obs_half ? 1 : 0);
  HIP_TRY(hipGetLastError());
  return 0;
}

}  // extern "C"
