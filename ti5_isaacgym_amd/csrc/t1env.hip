// t1env.hip -- MI355X (gfx950) kernels + C ABI for the T1 humanoid LeggedRobot.step() hot path.
//
// Per env step (t1env_step), four launches on the caller's stream, no host sync:
//   k_physics  : actions -> 10 x (PD torque with actuator lag + DR, dynamics substep, sensor-lag capture);
//                writes root/dof/rigid/contact/torques.  One env per lane, state in registers.
//   k_post_a   : base kinematics, command/ext-force callback, termination, 24 rewards (alphabetical),
//                episode sums, per-step extras reduction (legged_robot.py:458-489, 509-517, 654-680)
//   k_post_b   : masked reset_idx, compute_observations -> newest obs/priv frame, last_* bookkeeping
//                (legged_robot.py:490-502, t1_dh_stand_env.py:368-559)
//   shift      : 65 older frames of the 66-frame (and 3-frame critic) history shifted into the ping-pong
//                output buffer, lane per 4 floats, fully coalesced (the HBM-dominant part: ~26 KB per env
//                per step).  It does not depend on this step's physics, so it runs as extra workgroups of the
//                k_dynamics launch on the CUs the dynamics leaves idle (t1env_dynamics.hip); k_post_b, next
//                on the stream, writes the newest frame and zeroes the history rows of reset envs.
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
// history-shift workgroups appended to k_dynamics (128 threads).  A k_dynamics wave holds a whole SIMD's
// registers (1 wave/SIMD, 2 workgroups/CU), so the default fills exactly the workgroup slots the dynamics
// leaves free: 2 * CUs - dynamics workgroups (384 at 8192 envs on 256 CUs), at least MIN_SHIFT_BLOCKS.
constexpr int MIN_SHIFT_BLOCKS = 64;
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
  int shift_blocks;       // see MIN_SHIFT_BLOCKS; T1ENV_SHIFT_BLOCKS in the environment overrides (tuning)
  int shift_pending;      // phase A enqueued this step's history shift (phase B alone must run it)
  int step_timer;         // timing slot of the current step span (phase A start .. phase B end)
  unsigned* d_done;       // k_post_b block-completion counter (its last block finalises the extras)
  int16_t* d_hmax;        // coarse terrain height bound (Terrain::hmax), built by t1env_set_terrain
  float max_contact_radius;
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
  float* imu_dst = B.imu_hist + ((size_t)n * 2 + (ctr & 1u)) * 6;
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
// post-physics helpers
// =====================================================================================================
struct Phase {
  float sin_pos;
  float stance[2];
};

// copy K consecutive floats of one env's row into registers
template <int K, typename T>
__device__ __forceinline__ void ldrow(T (&d)[K], const T* s) {
#pragma unroll
  for (int i = 0; i < K; ++i) d[i] = s[i];
}
template <int K, typename T>
__device__ __forceinline__ void strow(T* d, const T (&s)[K]) {
#pragma unroll
  for (int i = 0; i < K; ++i) d[i] = s[i];
}

// _get_phase + _get_gait_phase (t1_dh_stand_env.py:80-107) on a phase counter already zeroed for standing envs
__device__ __forceinline__ float phase_value(const t1env_config& C, int64_t phase_len, float gait_start, bool stand) {
  const float dtf = (float)(C.sim_dt * C.decimation);
  float ph = ((float)phase_len * dtf) / C.cycle_time;
  ph = ph - floorf(ph);
  ph = (ph + gait_start) * (stand ? 0.0f : 1.0f);
  return ph;
}
__device__ __forceinline__ Phase gait_phase(float phase) {
  Phase p;
  p.sin_pos = sinf(TWO_PI_F * phase);
  p.stance[0] = p.sin_pos >= 0.0f ? 1.0f : 0.0f;
  p.stance[1] = p.sin_pos < 0.0f ? 1.0f : 0.0f;
  if (fabsf(p.sin_pos) < 0.1f) { p.stance[0] = 1.0f; p.stance[1] = 1.0f; }
  return p;
}
__device__ __forceinline__ bool is_stand(const t1env_config& C, const float* cmd) {
  return norm3(cmd[0], cmd[1], cmd[2]) <= C.stand_com_threshold;
}

// _resample_commands() (t1_dh_stand_env.py:126-177): every gait slot whose start equals the episode step
// redraws the command; returns whether cmd changed
__device__ __forceinline__ bool resample_commands_r(const t1env_config& C, const t1env_step_args& A, int64_t el,
                                                    const int32_t gt[3], float cmd[4], uint32_t genv, uint32_t ctr) {
  bool dirty = false;
  for (int i = 0; i < 3; ++i) {
    if (el != (int64_t)gt[i]) continue;
    dirty = true;
    const int kind = C.gait_kind[i];
    const float x = rand_float(A.cmd_ranges[0][0], A.cmd_ranges[0][1], C.seed, genv, ctr, SLOT_CMD_X);
    const float y = rand_float(A.cmd_ranges[1][0], A.cmd_ranges[1][1], C.seed, genv, ctr, SLOT_CMD_Y);
    const float z = rand_float(A.cmd_ranges[2][0], A.cmd_ranges[2][1], C.seed, genv, ctr, SLOT_CMD_YAW);
    if (kind == 0) { cmd[0] = x; cmd[1] = y; cmd[2] = z; }              // walk_omnidirectional
    else if (kind == 1) { cmd[0] = 0.0f; cmd[1] = 0.0f; cmd[2] = 0.0f; }  // stand
    else if (kind == 2) { cmd[0] = x; cmd[1] = 0.0f; cmd[2] = 0.0f; }     // walk_sagittal
    else if (kind == 3) { cmd[0] = 0.0f; cmd[1] = y; cmd[2] = 0.0f; }     // walk_lateral
    else { cmd[0] = 0.0f; cmd[1] = 0.0f; cmd[2] = z; }                    // rotate
  }
  return dirty;
}
__device__ __forceinline__ void resample_commands(const t1env_config& C, const t1env_buffers& B, const t1env_step_args& A,
                                                  int n, uint32_t genv, uint32_t ctr) {
  int32_t gt[3];
  float cmd[4];
  ldrow(gt, B.gait_time + n * 3);
  ldrow(cmd, B.commands + n * 4);
  if (resample_commands_r(C, A, B.episode_length_buf[n], gt, cmd, genv, ctr)) strow(B.commands + n * 4, cmd);
}

// base_lin_vel, base_ang_vel, projected_gravity, base_euler_xyz of a root state (legged_robot.py:469-477)
struct BaseQ {
  float lin[3], ang[3], grav[3], euler[3];
};
__device__ __forceinline__ void base_quantities_r(const float r[13], BaseQ& o) {
  const float q[4] = {r[3], r[4], r[5], r[6]};
  const float v[3] = {r[7], r[8], r[9]}, w[3] = {r[10], r[11], r[12]}, g[3] = {0.0f, 0.0f, -1.0f};
  quat_rotate_inverse(q, v, o.lin);
  quat_rotate_inverse(q, w, o.ang);
  quat_rotate_inverse(q, g, o.grav);
  euler_xyz(q, o.euler);
}
__device__ __forceinline__ void store_base_quantities(const t1env_buffers& B, int n, const BaseQ& o) {
  strow(B.base_lin_vel + n * 3, o.lin);
  strow(B.base_ang_vel + n * 3, o.ang);
  strow(B.projected_gravity + n * 3, o.grav);
  strow(B.base_euler_xyz + n * 3, o.euler);
}
__device__ __forceinline__ void base_quantities(const t1env_buffers& B, int n) {
  float r[13];
  ldrow(r, B.root_states + n * 13);
  BaseQ o;
  base_quantities_r(r, o);
  store_base_quantities(B, n, o);
}

// wave-level sum then one atomic per wave (extras reduction over reset envs)
__device__ __forceinline__ void wave_atomic_add(float* dst, float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if ((threadIdx.x & 63) == 0 && v != 0.0f) atomicAdd(dst, v);
}
// K wave sums at once: each butterfly round issues the K cross-lane moves back to back (one LDS-latency wait
// per round instead of one per value and round), then lane 0 adds the non-zero sums to dst[0..K)
template <int K>
__device__ __forceinline__ void wave_atomic_add_n(float* dst, float (&v)[K]) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    float t[K];
#pragma unroll
    for (int k = 0; k < K; ++k) t[k] = __shfl_xor(v[k], off, 64);
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] += t[k];
  }
  if ((threadIdx.x & 63) == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (v[k] != 0.0f) atomicAdd(dst + k, v[k]);
  }
}

// extras["episode"] of one step (legged_robot.py:560-569 via reset_idx): means over the envs reset this step
// into ring slot `slot`; a step without resets keeps the previous values, like the reference's extras dict.
// Run by one wave after every env's contribution to ep_accum is complete; zeroes ep_accum.
__device__ __forceinline__ void finalize_extras(const t1env_buffers& B, const t1env_config& C, int slot) {
  const int t = threadIdx.x & 63;
  const float cnt = atomicAdd(B.ep_accum + 24, 0.0f);  // device-scope read of the other blocks' atomics
  float* ex = B.extras + (size_t)slot * 32;
  const float* prev = B.extras + (size_t)((slot + T1ENV_EXTRAS_RING - 1) % T1ENV_EXTRAS_RING) * 32;
  if (t < 32) {
    float v = prev[t];
    if (cnt > 0.0f) {
      if (t < T1_NREW) v = (atomicAdd(B.ep_accum + t, 0.0f) / cnt) / C.episode_length_s;
      else if (t == 24) v = atomicAdd(B.ep_accum + 25, 0.0f) / (float)C.num_envs;
    }
    ex[t] = v;
  }
  __builtin_amdgcn_wave_barrier();
  if (t < 32) B.ep_accum[t] = 0.0f;
}


// =====================================================================================================
// post-physics phase A: callback, termination, rewards (legged_robot.py:469-489)
// =====================================================================================================
// Load-first: every input of the env is read into registers before the first store, so a wave has all its
// loads in flight at once.  Interleaving loads with the stores of results (the buffers may alias as far as the
// compiler knows) cost one memory round trip per access, and the kernel is latency-bound: 128 waves at 8192 envs.
__global__ __launch_bounds__(BLOCK) void k_post_a(const DynModel* __restrict__ Mp, const t1env_config* __restrict__ Cp,
                                                  t1env_buffers B, t1env_step_args A) {
  const int n0 = blockIdx.x * BLOCK + threadIdx.x;
  const t1env_config& C = *Cp;
  const DynModel& M = *Mp;
  const bool live = n0 < C.num_envs;
  const int n = live ? n0 : C.num_envs - 1;
  const uint32_t genv = (uint32_t)(C.env_offset + n);
  const uint32_t ctr = A.counter + 1u;  // common_step_counter += 1 happened before the callback
  const size_t N = (size_t)C.num_envs;
  // ---- inputs
  float root[13], dof[24], f0[13], f1[13], k0[2], k1[2], cfb[3], c0[3], c1[3];
  float a[12], la[12], lla[12], lrv[6], ldv[12], tq[12], ref[12], cmd[4], esum[T1_NREW];
  float at[2], fh[2], lfz[2], ef[3];
  uint8_t lc[2];
  int32_t gt[3];
  const float* rig = B.rigid_state + (size_t)n * 169;
  const float* cf = B.contact_forces + (size_t)n * 39;
  ldrow(root, B.root_states + n * 13);
  ldrow(dof, B.dof_state + (size_t)n * 24);
  ldrow(f0, rig + 6 * 13);
  ldrow(f1, rig + 12 * 13);
  ldrow(k0, rig + 4 * 13);
  ldrow(k1, rig + 10 * 13);
  ldrow(cfb, cf);
  ldrow(c0, cf + 6 * 3);
  ldrow(c1, cf + 12 * 3);
  ldrow(a, B.actions + n * 12);
  ldrow(la, B.last_actions + n * 12);
  ldrow(lla, B.last_last_actions + n * 12);
  ldrow(lrv, B.last_root_vel + n * 6);
  ldrow(ldv, B.last_dof_vel + n * 12);
  ldrow(tq, B.torques + n * 12);
  ldrow(ref, B.ref_dof_pos + n * 12);
  ldrow(cmd, B.commands + n * 4);
  ldrow(at, B.feet_air_time + n * 2);
  ldrow(fh, B.feet_height + n * 2);
  ldrow(lfz, B.last_feet_z + n * 2);
  ldrow(ef, B.ext_forces + n * 3);
  ldrow(lc, B.last_contacts + n * 2);
  ldrow(gt, B.gait_time + n * 3);
#pragma unroll
  for (int k = 0; k < T1_NREW; ++k) esum[k] = B.episode_sums[k * N + n];
  const int64_t el = B.episode_length_buf[n] + 1;
  int64_t pl = B.phase_length_buf[n] + 1;
  const float gstart = B.gait_start[n];
  // (lanes past num_envs shadow the last env: they compute but neither store nor contribute)
  // ---- base quantities (legged_robot.py:469-477) of the post-physics root state, feet euler angles
  BaseQ bq;
  base_quantities_r(root, bq);
  const float* blv = bq.lin;
  const float* bav = bq.ang;
  const float* pg = bq.grav;
  const float* be = bq.euler;
  float fe[6];
  {
    const float q0[4] = {f0[3], f0[4], f0[5], f0[6]}, q1[4] = {f1[3], f1[4], f1[5], f1[6]};
    euler_xyz(q0, fe);
    euler_xyz(q1, fe + 3);
  }
  // ---- _post_physics_step_callback (t1_dh_stand_env.py:179-215)
  const bool cmd_dirty = resample_commands_r(C, A, el, gt, cmd, genv, ctr);
  if (A.push_call) {  // _push_robots (t1:217-231): drawn every call (is_first_push reset is commented out)
    root[7] = rand_float(-C.push_vel_xy, C.push_vel_xy, C.seed, genv, ctr, SLOT_PUSH_VEL + 0);
    root[8] = rand_float(-C.push_vel_xy, C.push_vel_xy, C.seed, genv, ctr, SLOT_PUSH_VEL + 1);
    root[10] = rand_float(-C.push_ang, C.push_ang, C.seed, genv, ctr, SLOT_PUSH_ANG + 0);
    root[11] = rand_float(-C.push_ang, C.push_ang, C.seed, genv, ctr, SLOT_PUSH_ANG + 1);
    root[12] = rand_float(-C.push_ang, C.push_ang, C.seed, genv, ctr, SLOT_PUSH_ANG + 2);
  }
  float af[3] = {0.0f, 0.0f, 0.0f}, et[3];
  bool ext_store = true;
  if (A.ext_force_call) {  // _add_ext_force (t1:233-247)
    if (A.ext_force_first) {
      ef[0] = rand_float(-C.ext_force_max[0] / 2, C.ext_force_max[0], C.seed, genv, ctr, SLOT_EXT_FORCE + 0);
      ef[1] = rand_float(-C.ext_force_max[1], C.ext_force_max[1], C.seed, genv, ctr, SLOT_EXT_FORCE + 1);
      ef[2] = rand_float(-C.ext_force_max[2], C.ext_force_max[2], C.seed, genv, ctr, SLOT_EXT_FORCE + 2);
#pragma unroll
      for (int k = 0; k < 3; ++k)
        et[k] = rand_float(-C.ext_torque_max, C.ext_torque_max, C.seed, genv, ctr, SLOT_EXT_TORQUE + k);
    } else {
      const float st = is_stand(C, cmd) ? 1.0f : 0.0f;
      af[0] = ef[0] * st; af[1] = ef[1] * st; af[2] = ef[2] * st;
      ext_store = false;
    }
  } else {
    ef[0] = ef[1] = ef[2] = 0.0f;
    et[0] = et[1] = et[2] = 0.0f;
  }
  // ---- check_termination (legged_robot.py:509-517)
  const bool term = norm3(cfb[0], cfb[1], cfb[2]) > 1.0f;
  const bool tout = (float)el > C.max_episode_length;
  const bool do_reset = live && (term || tout);
  // ---- rewards (t1:576-935), alphabetical order
  const bool stand = is_stand(C, cmd);
  if (stand) pl = 0;  // _get_phase zeroes the phase counter of standing envs
  const Phase ph = gait_phase(phase_value(C, pl, gstart, stand));
  const float dtf = (float)(C.sim_dt * C.decimation);
  const bool contact0 = c0[2] > 5.0f, contact1 = c1[2] > 5.0f;
  float r[T1_NREW];
  {  // 0 action_smoothness
    float t1s = 0.0f, t2s = 0.0f, t3s = 0.0f;
    for (int j = 0; j < 12; ++j) {
      const float d1 = (la[j] - a[j]) * 1.0f;
      const float d2 = ((a[j] + lla[j]) - 2.0f * la[j]) * 1.0f;
      t1s += d1 * d1;
      t2s += d2 * d2;
      t3s += fabsf(a[j] * 1.0f);
    }
    r[0] = (t1s + t2s) + 0.05f * t3s;
  }
  {  // 1 base_acc (root velocity after a push, like the reference's root_states)
    float s = 0.0f;
    for (int i = 0; i < 6; ++i) { const float d = lrv[i] - root[7 + i]; s += d * d; }
    r[1] = expf(-sqrtf(s) * 3.0f);
  }
  {  // 2 base_height
    const float mh = (f0[2] * ph.stance[0] + f1[2] * ph.stance[1]) / (ph.stance[0] + ph.stance[1]);
    const float bh = root[2] - (mh - 0.05f);
    r[2] = expf(-fabsf(bh - C.base_height_target) * 100.0f);
  }
  r[3] = norm3(cfb[0], cfb[1], cfb[2]) > 0.1f ? 1.0f : 0.0f;  // 3 collision (penalised_contact_indices = base)
  {  // 4 default_joint_pos
    float jd[12], s = 0.0f;
    for (int j = 0; j < 12; ++j) { jd[j] = dof[2 * j] - M.default_dof_pos[j]; s += jd[j] * jd[j]; }
    float yr = norm3(jd[0], jd[1], jd[5]) + norm3(jd[6], jd[7], jd[11]);
    yr = clampf(yr - 0.1f, 0.0f, 50.0f);
    r[4] = expf(-yr * 100.0f) - 0.01f * sqrtf(s);
  }
  {  // 5 dof_acc, 6 dof_vel
    float s5 = 0.0f, s6 = 0.0f;
    for (int j = 0; j < 12; ++j) {
      const float d = (ldv[j] - dof[2 * j + 1]) / dtf;
      s5 += d * d;
      s6 += dof[2 * j + 1] * dof[2 * j + 1];
    }
    r[5] = s5;
    r[6] = s6;
  }
  {  // 7 feet_air_time (mutates feet_air_time, last_contacts)
    float sm0 = ph.stance[0], sm1 = ph.stance[1];
    if (norm3(cmd[0], cmd[1], cmd[2]) < 0.05f) { sm0 = 1.0f; sm1 = 1.0f; }
    const bool filt0 = contact0 || sm0 > 0.0f || lc[0];
    const bool filt1 = contact1 || sm1 > 0.0f || lc[1];
    lc[0] = contact0; lc[1] = contact1;
    const bool first0 = at[0] > 0.0f && filt0, first1 = at[1] > 0.0f && filt1;
    const float a0 = at[0] + dtf, a1 = at[1] + dtf;
    const float air0 = clampf(a0, 0.0f, 0.5f) * (first0 ? 1.0f : 0.0f);
    const float air1 = clampf(a1, 0.0f, 0.5f) * (first1 ? 1.0f : 0.0f);
    at[0] = a0 * (filt0 ? 0.0f : 1.0f);
    at[1] = a1 * (filt1 ? 0.0f : 1.0f);
    r[7] = air0 + air1;
  }
  {  // 8 feet_clearance (mutates feet_height, last_feet_z)
    const float z0 = f0[2], z1 = f1[2];
    const float h0 = fh[0] + (z0 - lfz[0]), h1 = fh[1] + (z1 - lfz[1]);
    lfz[0] = z0; lfz[1] = z1;
    const float sw0 = 1.0f - ph.stance[0], sw1 = 1.0f - ph.stance[1];
    const float rp0 = (h0 > C.target_feet_height && h0 < C.target_feet_height_max) ? 1.0f : 0.0f;
    const float rp1 = (h1 > C.target_feet_height && h1 < C.target_feet_height_max) ? 1.0f : 0.0f;
    r[8] = rp0 * sw0 + rp1 * sw1;
    fh[0] = h0 * (contact0 ? 0.0f : 1.0f);
    fh[1] = h1 * (contact1 ? 0.0f : 1.0f);
  }
  // 9 feet_contact_forces
  r[9] = clampf(norm3(c0[0], c0[1], c0[2]) - C.max_contact_force, 0.0f, 400.0f) +
         clampf(norm3(c1[0], c1[1], c1[2]) - C.max_contact_force, 0.0f, 400.0f);
  {  // 10 feet_contact_number
    float sm0 = ph.stance[0], sm1 = ph.stance[1];
    if (stand) { sm0 = 1.0f; sm1 = 1.0f; }
    const float q0 = ((contact0 ? 1.0f : 0.0f) == sm0) ? 1.0f : -0.3f;
    const float q1 = ((contact1 ? 1.0f : 0.0f) == sm1) ? 1.0f : -0.3f;
    r[10] = (q0 + q1) / 2.0f;
  }
  {  // 11 feet_distance, 15 knee_distance
    const float fd = norm2(f0[0] - f1[0], f0[1] - f1[1]);
    const float kd = norm2(k0[0] - k1[0], k0[1] - k1[1]);
    const float fmn = clampf(fd - C.foot_min_dist, -0.5f, 0.0f), fmx = clampf(fd - C.foot_max_dist, 0.0f, 0.5f);
    const float kmn = clampf(kd - C.knee_min_dist, -0.5f, 0.0f), kmx = clampf(kd - C.knee_max_dist, 0.0f, 0.5f);
    r[11] = (expf(-fabsf(fmn) * 100.0f) + expf(-fabsf(fmx) * 100.0f)) / 2.0f;
    r[15] = (expf(-fabsf(kmn) * 100.0f) + expf(-fabsf(kmx) * 100.0f)) / 2.0f;
  }
  {  // 12 feet_rotation
    const float rot = fe[1] * fe[1] + fe[4] * fe[4];
    const float x = rot / 1.0f;
    r[12] = 1.0f * expf(-(x * x));
  }
  {  // 13 foot_slip (rigid_state[..., 10:12] as in the reference)
    const float s0 = sqrtf(norm2(f0[10], f0[11])), s1 = sqrtf(norm2(f1[10], f1[11]));
    r[13] = s0 * (contact0 ? 1.0f : 0.0f) + s1 * (contact1 ? 1.0f : 0.0f);
  }
  {  // 14 joint_pos (ref_dof_pos from the previous compute_observations)
    float s = 0.0f;
    for (int j = 0; j < 12; ++j) {
      const float tgt = stand ? M.default_dof_pos[j] : ref[j];
      const float d = dof[2 * j] - tgt;
      s += d * d;
    }
    const float nr = sqrtf(s);
    r[14] = stand ? 1.0f : expf(-2.0f * nr) - 0.2f * clampf(nr, 0.0f, 0.5f);
  }
  {  // 16 low_speed
    const float sp = fabsf(blv[0]), cm = fabsf(cmd[0]);
    const bool low = sp < 0.5f * cm, high = sp > 1.2f * cm, ok = !(low || high);
    const bool mis = signf(blv[0]) != signf(cmd[0]);
    float v = 0.0f;
    if (low) v = -1.0f;
    if (high) v = 0.0f;
    if (ok) v = 1.2f;
    if (mis) v = -2.0f;
    r[16] = v * (fabsf(cmd[0]) > 0.05f ? 1.0f : 0.0f);
  }
  {  // 17 orientation
    const float qm = expf(-(fabsf(be[0]) + fabsf(be[1])) * 10.0f);
    const float o = expf(-norm2(pg[0], pg[1]) * 20.0f);
    r[17] = (qm + o) / 2.0f;
  }
  {  // 18 stand_still
    const int idx[8] = {0, 1, 2, 3, 5, 6, 7, 8};
    const float w[10] = {2.0f, 2.0f, 1.0f, 1.0f, 1.0f, 2.0f, 2.0f, 1.0f, 1.0f, 1.0f};
    float s = 0.0f;
    for (int k = 0; k < 8; ++k) {
      const float e = (dof[2 * idx[k]] - M.default_dof_pos[idx[k]]) * w[k];
      s += e * e;
    }
    const float e8 = fe[1] * w[8], e9 = fe[4] * w[9];
    s += e8 * e8;
    s += e9 * e9;
    r[18] = stand ? expf(-s) : 0.0f;
  }
  {  // 19 torques
    float s = 0.0f;
    for (int j = 0; j < 12; ++j) s += tq[j] * tq[j];
    r[19] = s;
  }
  {  // 20 track_vel_hard
    const float le = norm2(cmd[0] - blv[0], cmd[1] - blv[1]);
    const float ae = fabsf(cmd[2] - bav[2]);
    r[20] = (expf(-le * 10.0f) + expf(-ae * 10.0f)) / 2.0f - 0.2f * (le + ae);
  }
  {  // 21 tracking_ang_vel
    const float d = cmd[2] - bav[2];
    r[21] = stand ? expf(-fabsf(d) * (C.tracking_sigma * 2.0f)) : expf(-(d * d) * C.tracking_sigma);
  }
  {  // 22 tracking_lin_vel
    const float dx = cmd[0] - blv[0], dy = cmd[1] - blv[1];
    r[22] = stand ? expf(-(fabsf(dx) + fabsf(dy)) * (C.tracking_sigma * 2.0f))
                  : expf(-(dx * dx + dy * dy) * C.tracking_sigma);
  }
  {  // 23 vel_mismatch_exp
    const float lm = expf(-(blv[2] * blv[2]) * 10.0f);
    const float am = expf(-norm2(bav[0], bav[1]) * 5.0f);
    r[23] = (lm + am) / 2.0f;
  }
  float rew = 0.0f, contrib[T1_NREW];
  for (int k = 0; k < T1_NREW; ++k) {
    const float v = r[k] * C.reward_scales[k];
    rew = rew + v;
    esum[k] = esum[k] + v;
    contrib[k] = do_reset ? esum[k] : 0.0f;
  }
  if (C.only_positive_rewards) rew = fmaxf(rew, 0.0f);
  // ---- outputs
  if (live) {
    B.episode_length_buf[n] = el;
    B.phase_length_buf[n] = pl;
    store_base_quantities(B, n, bq);
    strow(B.feet_euler_xyz + n * 6, fe);
    if (cmd_dirty) strow(B.commands + n * 4, cmd);
    if (A.push_call) {
      float* rs = B.root_states + n * 13;
      rs[7] = root[7]; rs[8] = root[8]; rs[10] = root[10]; rs[11] = root[11]; rs[12] = root[12];
    }
    strow(B.applied_force + n * 3, af);
    if (ext_store) {
      strow(B.ext_forces + n * 3, ef);
      strow(B.ext_torques + n * 3, et);
    }
    B.reset_buf[n] = do_reset ? 1 : 0;
    B.time_out_buf[n] = tout ? 1 : 0;
    strow(B.last_contacts + n * 2, lc);
    strow(B.feet_air_time + n * 2, at);
    strow(B.feet_height + n * 2, fh);
    strow(B.last_feet_z + n * 2, lfz);
#pragma unroll
    for (int k = 0; k < T1_NREW; ++k) B.episode_sums[k * N + n] = esum[k];
    B.rew_buf[n] = rew;
  }
  // extras["episode"] means over reset envs: partial sums (finalised by k_post_b's last block)
  float part[T1_NREW + 1];
  for (int k = 0; k < T1_NREW; ++k) part[k] = contrib[k];
  part[T1_NREW] = do_reset ? 1.0f : 0.0f;
  wave_atomic_add_n(B.ep_accum, part);  // ep_accum[0..23] episode sums, [24] reset count
}

// =====================================================================================================
// reset_idx for one env (t1_dh_stand_env.py:483-559 + legged_robot.py:604-651, 732-783, 1076-1120, 1138-1158)
// =====================================================================================================
__device__ void reset_env(const DynModel& M, const t1env_config& C, const t1env_buffers& B, const t1env_step_args& A,
                          int n, uint32_t genv, uint32_t ctr, bool do_terrain) {
  const uint32_t seed = C.seed;
  if (do_terrain && C.terrain_curriculum) {  // _update_terrain_curriculum
    const float* r = B.root_states + n * 13;
    const float* o = B.env_origins + n * 3;
    const float dist = norm2(r[0] - o[0], r[1] - o[1]);
    const bool up = dist > C.env_length / 2.0f;
    const float* cmd = B.commands + n * 4;
    const bool down = (dist < norm2(cmd[0], cmd[1]) * (C.episode_length_s * 0.5f)) && !up;
    int lv = B.terrain_levels[n] + (up ? 1 : 0) - (down ? 1 : 0);
    const int rnd = rand_int(0, C.num_terrain_rows, seed, genv, ctr, SLOT_TERRAIN_LEVEL_RAND);
    lv = lv >= C.num_terrain_rows ? rnd : (lv < 0 ? 0 : lv);
    B.terrain_levels[n] = lv;
    const float* to = B.terrain_origins + ((size_t)lv * C.num_terrain_cols + B.terrain_types[n]) * 3;
    B.env_origins[n * 3 + 0] = to[0];
    B.env_origins[n * 3 + 1] = to[1];
    B.env_origins[n * 3 + 2] = to[2];
  }
  // _reset_dofs
  for (int j = 0; j < 12; ++j) {
    B.dof_state[n * 24 + 2 * j] =
        M.default_dof_pos[j] + rand_float(-C.reset_dof_range, C.reset_dof_range, seed, genv, ctr, SLOT_RESET_DOF + j);
    B.dof_state[n * 24 + 2 * j + 1] = 0.0f;
  }
  // _reset_root_states
  float* r = B.root_states + n * 13;
  for (int i = 0; i < 13; ++i) r[i] = M.base_init_state[i];
  for (int i = 0; i < 3; ++i) r[i] += B.env_origins[n * 3 + i];
  if (C.custom_origins) {
    const float p3 = C.reset_xy_range;
    r[0] += rand_float(-p3, p3, seed, genv, ctr, SLOT_RESET_ROOT_XY + 0);
    r[1] += rand_float(-p3, p3, seed, genv, ctr, SLOT_RESET_ROOT_XY + 1);
  }
  // randomize_dof_props (torque_multi is redrawn every substep anyway; its reset draw has no effect)
  for (int j = 0; j < 12; ++j) {
    B.motor_offsets[n * 12 + j] =
        rand_float(C.motor_offset_range[0], C.motor_offset_range[1], seed, genv, ctr, SLOT_DR_OFFSET + j);
    B.kp[n * 12 + j] = rand_float(C.kp_mult_range[0], C.kp_mult_range[1], seed, genv, ctr, SLOT_DR_KP + j) * M.p_gains[j];
    B.kd[n * 12 + j] = rand_float(C.kd_mult_range[0], C.kd_mult_range[1], seed, genv, ctr, SLOT_DR_KD + j) * M.d_gains[j];
    B.coulomb[n * 12 + j] = rand_float(C.coulomb_range[0], C.coulomb_range[1], seed, genv, ctr, SLOT_DR_COULOMB + j);
    B.viscous[n * 12 + j] = rand_float(C.viscous_range[0], C.viscous_range[1], seed, genv, ctr, SLOT_DR_VISCOUS + j);
    B.armature[n * 12 + j] =
        rand_float(C.armature_range[j][0], C.armature_range[j][1], seed, genv, ctr, SLOT_DR_ARMATURE + j);
  }
  // randomize_lag_props: zero the lag rings, redraw lag lengths
  for (int i = 0; i < 48; ++i) B.act_hist[(size_t)n * 48 + i] = 0.0f;
  for (int i = 0; i < 96; ++i) B.dof_hist[(size_t)n * 96 + i] = 0.0f;
  for (int i = 0; i < 12; ++i) B.imu_hist[(size_t)n * 12 + i] = 0.0f;
  B.lag_timestep[n] = rand_int(C.lag_range[0], C.lag_range[1] + 1, seed, genv, ctr, SLOT_LAG_ACTION);
  B.dof_lag_timestep[n] = rand_int(C.dof_lag_range[0], C.dof_lag_range[1] + 1, seed, genv, ctr, SLOT_LAG_DOF);
  B.imu_lag_timestep[n] = rand_int(C.imu_lag_range[0], C.imu_lag_range[1] + 1, seed, genv, ctr, SLOT_LAG_IMU);
  // buffers
  for (int j = 0; j < 12; ++j) {
    B.last_last_actions[n * 12 + j] = 0.0f;
    B.actions[n * 12 + j] = 0.0f;
    B.last_actions[n * 12 + j] = 0.0f;
    B.last_dof_vel[n * 12 + j] = 0.0f;
  }
  for (int i = 0; i < 6; ++i) B.last_root_vel[n * 6 + i] = 0.0f;
  B.feet_air_time[n * 2 + 0] = 0.0f;
  B.feet_air_time[n * 2 + 1] = 0.0f;
  B.episode_length_buf[n] = 0;
  B.phase_length_buf[n] = 0;
  B.reset_buf[n] = 1;
  B.gait_start[n] = (float)rand_int(0, 2, seed, genv, ctr, SLOT_GAIT_START) * 0.5f;
  // generate_gait_time (t1:109-124)
  float g[3];
  for (int i = 0; i < 3; ++i)
    g[i] = rand_float(C.gait_time_range[i][0], C.gait_time_range[i][1], seed, genv, ctr, SLOT_GAIT_TIME + i);
  const float s = (g[0] + g[1]) + g[2];
  const float f = C.max_episode_length / s;
  const float s0 = g[0] * f, s1 = g[1] * f;
  B.gait_time[n * 3 + 0] = 0;
  B.gait_time[n * 3 + 1] = (int32_t)(0.0f + s0);
  B.gait_time[n * 3 + 2] = (int32_t)((0.0f + s0) + s1);
  // episode sums are zeroed after the extras reduction; obs/critic history rows zeroed in the stack pass
  for (int k = 0; k < T1_NREW; ++k) B.episode_sums[(size_t)k * C.num_envs + n] = 0.0f;
  // base quantities of the reset env from the freshly written root state (t1:548-552)
  base_quantities(B, n);
}

// =====================================================================================================
// post-physics phase B: reset + observations (legged_robot.py:490-502, t1:368-481)
// =====================================================================================================
// the per-env inputs of compute_observations that reset_idx may rewrite (reloaded after a reset)
struct ObsIn {
  float cmd[4], dof[24], act[12], la[12], rv[6];
  BaseQ bq;
  int32_t gt[3];
  int64_t el, pl;
  float gstart;
  int dl, il;
};
__device__ __forceinline__ void load_obs_in(const t1env_buffers& B, int n, ObsIn& X) {
  ldrow(X.cmd, B.commands + n * 4);
  ldrow(X.dof, B.dof_state + (size_t)n * 24);
  ldrow(X.act, B.actions + n * 12);
  ldrow(X.la, B.last_actions + n * 12);
  const float* r = B.root_states + n * 13;
#pragma unroll
  for (int i = 0; i < 6; ++i) X.rv[i] = r[7 + i];
  ldrow(X.bq.lin, B.base_lin_vel + n * 3);
  ldrow(X.bq.ang, B.base_ang_vel + n * 3);
  ldrow(X.bq.euler, B.base_euler_xyz + n * 3);
  ldrow(X.gt, B.gait_time + n * 3);
  X.el = B.episode_length_buf[n];
  X.pl = B.phase_length_buf[n];
  X.gstart = B.gait_start[n];
  X.dl = B.dof_lag_timestep[n];
  X.il = B.imu_lag_timestep[n];
}

// Load-first like k_post_a: the inputs are read before any store; an env that resets this step rewrites its
// state in memory (reset_env) and reloads them.
__device__ __forceinline__ void post_b_env(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                           const t1env_step_args& A, int n, bool do_reset, bool any_reset) {
  const uint32_t genv = (uint32_t)(C.env_offset + n);
  const uint32_t ctr = A.counter + 1u;
  ObsIn X;
  load_obs_in(B, n, X);
  float ef[2], et[3], cfz[2];
  ldrow(ef, B.ext_forces + n * 3);
  ldrow(et, B.ext_torques + n * 3);
  cfz[0] = B.contact_forces[(size_t)n * 39 + 6 * 3 + 2];
  cfz[1] = B.contact_forces[(size_t)n * 39 + 12 * 3 + 2];
  const float fric = B.friction[n], mass = B.body_mass[n];
  if (do_reset) {
    reset_env(M, C, B, A, n, genv, ctr, true);
    load_obs_in(B, n, X);
  }
  if (any_reset && resample_commands_r(C, A, X.el, X.gt, X.cmd, genv, ctr)) strow(B.commands + n * 4, X.cmd);
  // lagged sensor samples (need the lag lengths loaded above)
  const float* ldp = B.dof_hist + ((size_t)n * 4 + ((A.counter - (uint32_t)(X.dl / 10)) & 3u)) * 24;
  const float* lip = B.imu_hist + ((size_t)n * 2 + ((A.counter - (uint32_t)(X.il / 10)) & 1u)) * 6;
  float ld[24], li[6];
  ldrow(ld, ldp);
  ldrow(li, lip);
  // ---- compute_observations
  const float* cmd = X.cmd;
  const float* dof = X.dof;
  const float* act = X.act;
  const bool stand = is_stand(C, cmd);
  if (stand) {  // _get_phase zeroes the phase counter of standing envs
    X.pl = 0;
    B.phase_length_buf[n] = 0;
  }
  const float phase = phase_value(C, X.pl, X.gstart, stand);
  // compute_ref_state (t1:250-274)
  const float sp = sinf(TWO_PI_F * phase);
  const float cp = cosf(TWO_PI_F * phase);
  float ref[12];
  {
    const float sl = sp > 0.0f ? 0.0f : sp;
    const float sr = sp < 0.0f ? 0.0f : sp;
    const float s1 = C.target_joint_pos_scale, s2 = 2.0f * C.target_joint_pos_scale;
    for (int j = 0; j < 12; ++j) ref[j] = 0.0f;
    ref[2] = sl * s1; ref[3] = -sl * s2; ref[4] = sl * s1;
    ref[8] = -sr * s1; ref[9] = sr * s2; ref[10] = -sr * s1;
    if (fabsf(sp) < 0.1f)
      for (int j = 0; j < 12; ++j) ref[j] = 0.0f;
    for (int j = 0; j < 12; ++j) ref[j] = ref[j] + M.default_dof_pos[j];
  }
  const Phase ph = gait_phase(phase);
  float* priv = B.priv_buf[A.obs_slot] + (size_t)n * (T1_NPRIV * T1_CHIST) + T1_NPRIV * (T1_CHIST - 1);
  float* obs = B.obs_buf[A.obs_slot] + (size_t)n * (T1_NOBS * T1_HIST) + T1_NOBS * (T1_HIST - 1);
  const float clipo = C.clip_obs;
  float cin[5] = {sp, cp, cmd[0] * C.lin_vel_obs_scale, cmd[1] * C.lin_vel_obs_scale, cmd[2] * C.ang_vel_obs_scale};
  {  // privileged frame (73)
    int k = 0;
    float v[T1_NPRIV];
    for (int i = 0; i < 5; ++i) v[k++] = cin[i];
    for (int j = 0; j < 12; ++j) v[k++] = (dof[2 * j] - M.default_dof_pos[j]) * C.dof_pos_obs_scale;
    for (int j = 0; j < 12; ++j) v[k++] = dof[2 * j + 1] * C.dof_vel_obs_scale;
    for (int j = 0; j < 12; ++j) v[k++] = act[j];
    for (int j = 0; j < 12; ++j) v[k++] = dof[2 * j] - ref[j];
    for (int i = 0; i < 3; ++i) v[k++] = X.bq.lin[i] * C.lin_vel_obs_scale;
    for (int i = 0; i < 3; ++i) v[k++] = X.bq.ang[i] * C.ang_vel_obs_scale;
    for (int i = 0; i < 3; ++i) v[k++] = X.bq.euler[i] * C.quat_obs_scale;
    v[k++] = ef[0] / (C.ext_force_max[0] + 0.1f);
    v[k++] = ef[1] / (C.ext_force_max[0] + 0.1f);
    for (int i = 0; i < 3; ++i) v[k++] = et[i] / (C.ext_torque_max + 0.1f);
    v[k++] = fric;
    v[k++] = mass / 30.0f;
    v[k++] = ph.stance[0];
    v[k++] = ph.stance[1];
    v[k++] = cfz[0] > 5.0f ? 1.0f : 0.0f;
    v[k++] = cfz[1] > 5.0f ? 1.0f : 0.0f;
    for (int i = 0; i < T1_NPRIV; ++i) priv[i] = clampf(v[i], -clipo, clipo);
  }
  {  // actor frame (47) from the lagged sensor rings + noise
    float v[T1_NOBS];
    int k = 0;
    for (int i = 0; i < 5; ++i) v[k++] = cin[i];
    for (int j = 0; j < 12; ++j) v[k++] = (ld[j] - M.default_dof_pos[j]) * C.dof_pos_obs_scale;
    for (int j = 0; j < 12; ++j) v[k++] = ld[12 + j] * C.dof_vel_obs_scale;
    for (int j = 0; j < 12; ++j) v[k++] = act[j];
    for (int i = 0; i < 3; ++i) v[k++] = li[i] * C.ang_vel_obs_scale;
    for (int i = 0; i < 3; ++i) v[k++] = li[3 + i] * C.quat_obs_scale;
    for (int i = 0; i < T1_NOBS; ++i) {
      const float u = uniform01(C.seed, genv, ctr, SLOT_OBS_NOISE + i);
      const float nz = ((2.0f * u - 1.0f) * C.noise_vec[i]) * C.noise_level;
      obs[i] = clampf(v[i] + nz, -clipo, clipo);
    }
  }
  strow(B.ref_dof_pos + n * 12, ref);
  // last_* (legged_robot.py:496-502)
  strow(B.last_last_actions + n * 12, X.la);
  strow(B.last_actions + n * 12, X.act);
  for (int j = 0; j < 12; ++j) B.last_dof_vel[n * 12 + j] = dof[2 * j + 1];
  strow(B.last_root_vel + n * 6, X.rv);
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
  if (C.terrain_curriculum && any_reset) wave_atomic_add(B.ep_accum + 25, live ? (float)B.terrain_levels[n] : 0.0f);
  // reset_idx zeroes the obs / critic history of the reset envs (t1:548-558): k_shift wrote the 65 (2) older
  // frames of every row, so the wave zeroes those of its reset envs here, one row at a time, coalesced
  uint64_t m = __ballot(do_reset);
  while (m) {
    const int l = __ffsll((unsigned long long)m) - 1;
    m &= m - 1;
    const size_t row = (size_t)blockIdx.x * BLOCK + l;
    float* o = B.obs_buf[A.obs_slot] + row * (T1_NOBS * T1_HIST);
    for (int c = threadIdx.x; c < T1_NOBS * (T1_HIST - 1); c += BLOCK) o[c] = 0.0f;
    float* p = B.priv_buf[A.obs_slot] + row * (T1_NPRIV * T1_CHIST);
    for (int c = threadIdx.x; c < T1_NPRIV * (T1_CHIST - 1); c += BLOCK) p[c] = 0.0f;
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

// extras finalisation for t1env_reset_all (one wave)
__global__ void k_finalize(t1env_buffers B, const t1env_config* __restrict__ Cp, int slot) {
  finalize_extras(B, *Cp, slot);
}

// terrain-level sum for extras["episode"]["terrain_level"] (only meaningful on reset steps)
__global__ __launch_bounds__(256) void k_terrain_level_sum(t1env_buffers B, const t1env_config* __restrict__ Cp) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const t1env_config& C = *Cp;
  const float v = (n < C.num_envs && C.terrain_curriculum && B.ep_accum[24] > 0.0f) ? (float)B.terrain_levels[n] : 0.0f;
  wave_atomic_add(B.ep_accum + 25, v);
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
__global__ __launch_bounds__(BLOCK) void k_reset_all(const DynModel* __restrict__ Mp, const t1env_config* __restrict__ Cp,
                                                     t1env_buffers B, t1env_step_args A) {
  const int n0 = blockIdx.x * BLOCK + threadIdx.x;
  const t1env_config& C = *Cp;
  const bool live = n0 < C.num_envs;
  const int n = live ? n0 : C.num_envs - 1;
  float contrib[T1_NREW];
  for (int k = 0; k < T1_NREW; ++k) contrib[k] = live ? B.episode_sums[(size_t)k * C.num_envs + n] : 0.0f;
  for (int k = 0; k < T1_NREW; ++k) wave_atomic_add(B.ep_accum + k, contrib[k]);
  wave_atomic_add(B.ep_accum + 24, live ? 1.0f : 0.0f);
  if (!live) return;
  const uint32_t genv = (uint32_t)(C.env_offset + n);
  reset_env(*Mp, C, B, A, n, genv, A.counter, true);
  resample_commands(C, B, A, n, genv, A.counter);
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
const char* t1env_version(void) { return "t1env-hip 0.1 (gfx950)"; }

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
      (err = hipMalloc(&e->d_done, sizeof(unsigned))) != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "t1env_create: hipMalloc: %s", hipGetErrorString(err));
    free(e);
    return (int)err;
  }
  HIP_TRY(hipMemcpy(e->d_model, &dm, sizeof(DynModel), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(e->d_cfg, cfg, sizeof(t1env_config), hipMemcpyHostToDevice));
  HIP_TRY(hipMemset(e->buf.ep_accum, 0, 32 * sizeof(float)));
  HIP_TRY(hipMemset(e->d_done, 0, sizeof(unsigned)));
  {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
        hipSuccess) cus = 256;
    const int free_slots = 2 * cus - (cfg->num_envs + 63) / 64;
    e->shift_blocks = free_slots > MIN_SHIFT_BLOCKS ? free_slots : MIN_SHIFT_BLOCKS;
    if (const char* sb = getenv("T1ENV_SHIFT_BLOCKS"))
      if (atoi(sb) > 0) e->shift_blocks = atoi(sb);
  }
  for (int b = 0; b < NB; ++b) e->max_contact_radius = fmaxf(e->max_contact_radius, dm.contact_radius[b]);
  *out = e;
  return 0;
}

int t1env_destroy(t1env* e) {
  if (!e) return 0;
  (void)hipFree(e->d_model);
  (void)hipFree(e->d_cfg);
  (void)hipFree(e->d_done);
  if (e->d_hmax) (void)hipFree(e->d_hmax);
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
                   N * T1_NOBS * T1_HIST, N * T1_NPRIV * T1_CHIST};
}

// the history shift as its own launch, in stream order (paths without k_dynamics)
static int launch_shift(t1env* e, const t1env_step_args* a, hipStream_t s) {
  const int t = t_begin(e, 3, s);
  hipLaunchKernelGGL(k_shift, dim3(SHIFT_BLOCKS), dim3(256), 0, s, shift_args(e, a));
  t_end(e, t, s);
  HIP_TRY(hipGetLastError());
  return 0;
}

static int launch_physics(t1env* e, const float* actions, const t1env_step_args* a, const t1env_injected* inj,
                          hipStream_t s) {
  if (a->obs_slot != 0 && a->obs_slot != 1) return fail(T1ENV_E_ARG, "obs_slot must be 0 or 1");
  const int N = e->cfg.num_envs;
  e->step_timer = t_begin(e, 5, s);
  int t = t_begin(e, 0, s);
  if (inj)
    hipLaunchKernelGGL(k_physics_injected, dim3(grid(N, BLOCK)), dim3(BLOCK), 0, s, e->d_model, e->d_cfg, e->buf,
                       actions, *a, *inj);
  else
    HIP_TRY((hipError_t)t1_launch_dynamics(e->d_model, e->d_cfg, e->buf, e->terrain, actions, *a, N,
                                           shift_args(e, a), e->shift_blocks, s));
  t_end(e, t, s);
  HIP_TRY(hipGetLastError());
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

int t1env_step(t1env* e, const float* actions, const t1env_step_args* a, void* stream) {
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
  hipLaunchKernelGGL(k_reset_all, dim3(grid(N, BLOCK)), dim3(BLOCK), 0, s, e->d_model, e->d_cfg, e->buf, *a);
  HIP_TRY(hipGetLastError());
  if (e->cfg.terrain_curriculum) {
    hipLaunchKernelGGL(k_terrain_level_sum, dim3(grid(N, 256)), dim3(256), 0, s, e->buf, e->d_cfg);
    HIP_TRY(hipGetLastError());
  }
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(64), 0, s, e->buf, e->d_cfg, (int)(a->counter % T1ENV_EXTRAS_RING));
  HIP_TRY(hipGetLastError());
  // every history row restarts from zeros: clear both ping-pong buffers (the next step shifts from either)
  for (int k = 0; k < 2; ++k) {
    HIP_TRY(hipMemsetAsync(e->buf.obs_buf[k], 0, sizeof(float) * (size_t)N * T1_NOBS * T1_HIST, s));
    HIP_TRY(hipMemsetAsync(e->buf.priv_buf[k], 0, sizeof(float) * (size_t)N * T1_NPRIV * T1_CHIST, s));
  }
  return 0;
}

}  // extern "C"
