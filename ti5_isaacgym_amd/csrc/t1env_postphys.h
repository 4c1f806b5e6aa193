// t1env_postphys.h -- post-physics device code (one env per lane), shared by the split kernels (t1env.hip:
// k_post_a / k_post_b, used on command-curriculum steps and for golden parity) and the fused epilogue of
// k_dynamics (t1env_dynamics.hip).  Included after t1env_device.h: no FMA contraction here (the float
// expressions keep the reference's op-by-op fp32 evaluation order).
#pragma once
#include "t1env_device.h"

namespace t1 {

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
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    if (el != (int64_t)gt[i]) continue;
    dirty = true;
    const int kind = C.gait_kind[i];
    const RngKey K = rng_key(C.seed, genv, ctr);
    const float x = rand_float(A.cmd_ranges[0][0], A.cmd_ranges[0][1], K, SLOT_CMD_X);
    const float y = rand_float(A.cmd_ranges[1][0], A.cmd_ranges[1][1], K, SLOT_CMD_Y);
    const float z = rand_float(A.cmd_ranges[2][0], A.cmd_ranges[2][1], K, SLOT_CMD_YAW);
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
// The wave sum of v, stored by lane 0 as an agent-scope (sc1) store: visible past the XCD's L2 once the store has
// completed (the fused step's per-workgroup partial extras, read by the last workgroup after its acquire fence)
__device__ __forceinline__ void wave_sum_store(float* dst, float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
// The same K wave sums stored to row[0..K) by lane 0 as agent-scope stores (no same-address atomics across
// workgroups).  Lane 0 stores them one by one: a lane-k-keeps-sum-k select chain is turned into a dynamically
// indexed array in scratch by the compiler.
template <int K>
__device__ __forceinline__ void wave_sum_store_n(float* row, float (&v)[K]) {
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
    for (int k = 0; k < K; ++k) __hip_atomic_store(row + k, v[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
// compiler knows) cost one memory round trip per access, and the pass is latency-bound (one lane per env).
// Called by a whole wave (the extras sums are wave reductions); lane = env n0 (lanes past num_envs shadow the
// last env).  Returns this env's reset decision.
// the inputs of post_a for one env (loaded by load_post_a_in in the split kernels, staged through LDS in the
// fused k_dyn4 epilogue); el / pl as stored, before this step's increment
struct PostAIn {
  float root[13], dof[24], f0[13], f1[13], k0[2], k1[2], cfb[3], c0[3], c1[3];
  float a[12], la[12], lla[12], lrv[6], ldv[12], tq[12], ref[12], cmd[4], esum[T1_NREW];
  float at[2], fh[2], lfz[2], ef[3], et[3];
  uint8_t lc[2];
  int32_t gt[3];
  int64_t el, pl;
  float gstart;
};
__device__ __forceinline__ void load_post_a_in(const t1env_buffers& B, size_t N, int n, PostAIn& X) {
  const float* rig = B.rigid_state + (size_t)n * 169;
  const float* cf = B.contact_forces + (size_t)n * 39;
  ldrow(X.root, B.root_states + n * 13);
  ldrow(X.dof, B.dof_state + (size_t)n * 24);
  ldrow(X.f0, rig + 6 * 13);
  ldrow(X.f1, rig + 12 * 13);
  ldrow(X.k0, rig + 4 * 13);
  ldrow(X.k1, rig + 10 * 13);
  ldrow(X.cfb, cf);
  ldrow(X.c0, cf + 6 * 3);
  ldrow(X.c1, cf + 12 * 3);
  ldrow(X.a, B.actions + n * 12);
  ldrow(X.la, B.last_actions + n * 12);
  ldrow(X.lla, B.last_last_actions + n * 12);
  ldrow(X.lrv, B.last_root_vel + n * 6);
  ldrow(X.ldv, B.last_dof_vel + n * 12);
  ldrow(X.tq, B.torques + n * 12);
  ldrow(X.ref, B.ref_dof_pos + n * 12);
  ldrow(X.cmd, B.commands + n * 4);
  ldrow(X.at, B.feet_air_time + n * 2);
  ldrow(X.fh, B.feet_height + n * 2);
  ldrow(X.lfz, B.last_feet_z + n * 2);
  ldrow(X.ef, B.ext_forces + n * 3);
  ldrow(X.et, B.ext_torques + n * 3);
  ldrow(X.lc, B.last_contacts + n * 2);
  ldrow(X.gt, B.gait_time + n * 3);
#pragma unroll
  for (int k = 0; k < T1_NREW; ++k) X.esum[k] = B.episode_sums[k * N + n];
  X.el = B.episode_length_buf[n];
  X.pl = B.phase_length_buf[n];
  X.gstart = B.gait_start[n];
}

// ---- _post_physics_step_callback (t1_dh_stand_env.py:179-215) on an env's registers: the commands redrawn at gait
// slots (el: the incremented episode step), pushes into root's velocities, the external force and torque; af = the
// force applied this step, ext_store = whether ef / et changed.  Returns whether the commands changed.
__device__ __forceinline__ bool post_callback(const t1env_config& C, const t1env_step_args& A, uint32_t genv,
                                              uint32_t ctr, RngKey K, int64_t el, const int32_t gt[3], float cmd[4],
                                              float root[13], float ef[3], float et[3], float af[3], bool& ext_store) {
  const bool cmd_dirty = resample_commands_r(C, A, el, gt, cmd, genv, ctr);
  if (A.push_call) {  // _push_robots (t1:217-231): drawn every call (is_first_push reset is commented out)
    root[7] = rand_float(-C.push_vel_xy, C.push_vel_xy, K, SLOT_PUSH_VEL + 0);
    root[8] = rand_float(-C.push_vel_xy, C.push_vel_xy, K, SLOT_PUSH_VEL + 1);
    root[10] = rand_float(-C.push_ang, C.push_ang, K, SLOT_PUSH_ANG + 0);
    root[11] = rand_float(-C.push_ang, C.push_ang, K, SLOT_PUSH_ANG + 1);
    root[12] = rand_float(-C.push_ang, C.push_ang, K, SLOT_PUSH_ANG + 2);
  }
  af[0] = af[1] = af[2] = 0.0f;
  ext_store = true;
  if (A.ext_force_call) {  // _add_ext_force (t1:233-247)
    if (A.ext_force_first) {
      ef[0] = rand_float(-C.ext_force_max[0] / 2, C.ext_force_max[0], K, SLOT_EXT_FORCE + 0);
      ef[1] = rand_float(-C.ext_force_max[1], C.ext_force_max[1], K, SLOT_EXT_FORCE + 1);
      ef[2] = rand_float(-C.ext_force_max[2], C.ext_force_max[2], K, SLOT_EXT_FORCE + 2);
#pragma unroll
      for (int k = 0; k < 3; ++k)
        et[k] = rand_float(-C.ext_torque_max, C.ext_torque_max, K, SLOT_EXT_TORQUE + k);
    } else {
      const float st = is_stand(C, cmd) ? 1.0f : 0.0f;
      af[0] = ef[0] * st; af[1] = ef[1] * st; af[2] = ef[2] * st;
      ext_store = false;
    }
  } else {
    ef[0] = ef[1] = ef[2] = 0.0f;
    et[0] = et[1] = et[2] = 0.0f;
  }
  return cmd_dirty;
}

// Called by a whole wave (the extras sums are wave reductions); lane = env n0 (lanes past num_envs shadow the
// last env).  Returns this env's reset decision; on return X holds the post-callback state (root after a push,
// resampled commands, incremented episode / phase counters, external force and torque) and bq the base
// quantities, which the fused epilogue hands to post_b without a reload.
// PART (fused k_dyn4 epilogue, two waves): POST_A_ALL runs everything (split kernels, one wave); POST_A_REWARDS
// runs the callback + termination prefix, the rewards and the reward-owned stores (rew, episode sums, feet
// state, extras sums) and zeroes the reward state of resetting envs itself; POST_A_STATE runs the same prefix
// and the state-owned stores (counters, base quantities, commands, push, external force, reset / time-out
// flags) for the wave that continues with post_b.  The prefix is deterministic, so both waves agree.
enum : int { POST_A_ALL = 0, POST_A_REWARDS = 1, POST_A_STATE = 2, POST_OBS_PRIV = 3, POST_OBS_ACTOR = 4 };
template <int PART = POST_A_ALL>
__device__ __forceinline__ bool post_a_core(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                            const t1env_step_args& A, int n0, PostAIn& X, BaseQ& bq,
                                            float* ep_row = nullptr) {
  const bool live = n0 < C.num_envs;
  const int n = live ? n0 : C.num_envs - 1;
  const uint32_t genv = (uint32_t)(C.env_offset + n);
  const uint32_t ctr = A.counter + 1u;  // common_step_counter += 1 happened before the callback
  const RngKey K = rng_key(C.seed, genv, ctr);
  const size_t N = (size_t)C.num_envs;
  float (&root)[13] = X.root;
  const float (&dof)[24] = X.dof;
  const float (&f0)[13] = X.f0;
  const float (&f1)[13] = X.f1;
  const float (&k0)[2] = X.k0;
  const float (&k1)[2] = X.k1;
  const float (&cfb)[3] = X.cfb;
  const float (&c0)[3] = X.c0;
  const float (&c1)[3] = X.c1;
  const float (&a)[12] = X.a;
  const float (&la)[12] = X.la;
  const float (&lla)[12] = X.lla;
  const float (&lrv)[6] = X.lrv;
  const float (&ldv)[12] = X.ldv;
  const float (&tq)[12] = X.tq;
  const float (&ref)[12] = X.ref;
  float (&cmd)[4] = X.cmd;
  float (&esum)[T1_NREW] = X.esum;
  float (&at)[2] = X.at;
  float (&fh)[2] = X.fh;
  float (&lfz)[2] = X.lfz;
  float (&ef)[3] = X.ef;
  float (&et)[3] = X.et;
  uint8_t (&lc)[2] = X.lc;
  const int32_t (&gt)[3] = X.gt;
  const int64_t el = X.el + 1;
  int64_t pl = X.pl + 1;
  const float gstart = X.gstart;
  // (lanes past num_envs shadow the last env: they compute but neither store nor contribute)
  // ---- base quantities (legged_robot.py:469-477) of the post-physics root state, feet euler angles
  base_quantities_r(root, bq);
  const float* blv = bq.lin;
  const float* bav = bq.ang;
  const float* pg = bq.grav;
  const float* be = bq.euler;
  float fe[6];
  if constexpr (PART != POST_A_STATE) {
    const float q0[4] = {f0[3], f0[4], f0[5], f0[6]}, q1[4] = {f1[3], f1[4], f1[5], f1[6]};
    euler_xyz(q0, fe);
    euler_xyz(q1, fe + 3);
  }
  T1_PROF_MARK(16);
  float af[3];
  bool ext_store;
  const bool cmd_dirty = post_callback(C, A, genv, ctr, K, el, gt, cmd, root, ef, et, af, ext_store);
  T1_PROF_MARK(17);
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
  if constexpr (PART != POST_A_STATE) {
    {  // 0 action_smoothness
      float t1s = 0.0f, t2s = 0.0f, t3s = 0.0f;
#pragma unroll
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
#pragma unroll
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
#pragma unroll
      for (int j = 0; j < 12; ++j) { jd[j] = dof[2 * j] - M.default_dof_pos[j]; s += jd[j] * jd[j]; }
      float yr = norm3(jd[0], jd[1], jd[5]) + norm3(jd[6], jd[7], jd[11]);
      yr = clampf(yr - 0.1f, 0.0f, 50.0f);
      r[4] = expf(-yr * 100.0f) - 0.01f * sqrtf(s);
    }
    {  // 5 dof_acc, 6 dof_vel
      float s5 = 0.0f, s6 = 0.0f;
#pragma unroll
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
#pragma unroll
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
#pragma unroll
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
#pragma unroll
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
  }
  T1_PROF_MARK(18);
  float rew = 0.0f, contrib[T1_NREW];
  if constexpr (PART != POST_A_STATE) {
#pragma unroll
    for (int k = 0; k < T1_NREW; ++k) {
      const float v = r[k] * C.reward_scales[k];
      rew = rew + v;
      esum[k] = esum[k] + v;
      contrib[k] = do_reset ? esum[k] : 0.0f;
    }
    if (C.only_positive_rewards) rew = fmaxf(rew, 0.0f);
  }
  T1_PROF_MARK(19);
  // ---- outputs
  if (live) {
    if constexpr (PART != POST_A_REWARDS) {
      B.episode_length_buf[n] = el;
      B.phase_length_buf[n] = pl;
      store_base_quantities(B, n, bq);
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
    }
    if constexpr (PART != POST_A_STATE) {
      strow(B.feet_euler_xyz + n * 6, fe);
      strow(B.last_contacts + n * 2, lc);
      strow(B.feet_height + n * 2, fh);
      strow(B.last_feet_z + n * 2, lfz);
      if constexpr (PART == POST_A_REWARDS) {  // reset_idx's zeroing of the reward state, done here (fused)
        const float keep = do_reset ? 0.0f : 1.0f;
        at[0] *= keep; at[1] *= keep;
#pragma unroll
        for (int k = 0; k < T1_NREW; ++k) B.episode_sums[k * N + n] = do_reset ? 0.0f : esum[k];
      } else {
#pragma unroll
        for (int k = 0; k < T1_NREW; ++k) B.episode_sums[k * N + n] = esum[k];
      }
      strow(B.feet_air_time + n * 2, at);
      B.rew_buf[n] = rew;
    }
  }
  if constexpr (PART != POST_A_STATE) {
    // extras["episode"] means over reset envs: partial sums (finalised by k_post_b's last block)
    float part[T1_NREW + 1];
#pragma unroll
    for (int k = 0; k < T1_NREW; ++k) part[k] = contrib[k];
    part[T1_NREW] = do_reset ? 1.0f : 0.0f;
    if (ep_row) {  // the fused step: this workgroup's partial row (FusedArgs::ep_part)
      if (__ballot(do_reset) != 0) {
        wave_sum_store_n(ep_row, part);
      } else if ((threadIdx.x & 63) == 0) {  // no env of the wave resets (most steps): the sums are all +0
#pragma unroll
        for (int k = 0; k <= T1_NREW; ++k) __hip_atomic_store(ep_row + k, 0.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else
      wave_atomic_add_n(B.ep_accum, part);  // ep_accum[0..23] episode sums, [24] reset count
  }
  X.el = el;
  X.pl = pl;
  return do_reset;
}

__device__ __forceinline__ bool post_a_env(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                           const t1env_step_args& A, int n0) {
  const int n = n0 < C.num_envs ? n0 : C.num_envs - 1;
  PostAIn X;
  load_post_a_in(B, (size_t)C.num_envs, n, X);
  BaseQ bq;
  return post_a_core(M, C, B, A, n0, X, bq);
}

// the per-env inputs of compute_observations that reset_idx may rewrite (reset_env writes a resetting env's new values into it)
struct ObsIn {
  float cmd[4], dof[24], act[12], la[12], rv[6];
  BaseQ bq;
  int32_t gt[3];
  int64_t el, pl;
  float gstart;
  int dl, il;
};

// =====================================================================================================
// reset_idx for one env (t1_dh_stand_env.py:483-559 + legged_robot.py:604-651, 732-783, 1076-1120, 1138-1158)
// =====================================================================================================
// The observation inputs of an env that reset_idx restarts, from its draws alone (the slots reset_env below draws
// them from): joint positions, zero actions, the initial root velocity and its base quantities (the root's position
// does not enter them), gait start and times, lag lengths; el = pl = 0.  cmd is left as it is.  The fused epilogue's
// observation waves take a resetting env's inputs from here while another wave stores its new state.
__device__ __forceinline__ void reset_obs_inputs(const DynModel& M, const t1env_config& C, RngKey K, ObsIn& X,
                                                 bool dof = true) {
  if (dof)  // _reset_dofs (dof = false: not drawn, for a caller that does not read them)
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      X.dof[2 * j] = M.default_dof_pos[j] + rand_float(-C.reset_dof_range, C.reset_dof_range, K, SLOT_RESET_DOF + j);
      X.dof[2 * j + 1] = 0.0f;
    }
#pragma unroll
  for (int j = 0; j < 12; ++j) { X.act[j] = 0.0f; X.la[j] = 0.0f; }
  float r[13];  // _reset_root_states without the origin / xy offsets (position only)
#pragma unroll
  for (int i = 0; i < 13; ++i) r[i] = M.base_init_state[i];
#pragma unroll
  for (int i = 0; i < 6; ++i) X.rv[i] = r[7 + i];
  base_quantities_r(r, X.bq);  // (t1:548-552) reads the quaternion and velocities only
  X.dl = rand_int(C.dof_lag_range[0], C.dof_lag_range[1] + 1, K, SLOT_LAG_DOF);
  X.il = rand_int(C.imu_lag_range[0], C.imu_lag_range[1] + 1, K, SLOT_LAG_IMU);
  X.gstart = (float)rand_int(0, 2, K, SLOT_GAIT_START) * 0.5f;
  float g[3];  // generate_gait_time (t1:109-124)
#pragma unroll
  for (int i = 0; i < 3; ++i)
    g[i] = rand_float(C.gait_time_range[i][0], C.gait_time_range[i][1], K, SLOT_GAIT_TIME + i);
  const float gs = (g[0] + g[1]) + g[2];
  const float f = C.max_episode_length / gs;
  const float s0 = g[0] * f, s1 = g[1] * f;
  X.gt[0] = 0;
  X.gt[1] = (int32_t)(0.0f + s0);
  X.gt[2] = (int32_t)((0.0f + s0) + s1);
  X.el = 0;
  X.pl = 0;
}

// zero_reward_state = false: the caller's reward pass zeroes feet_air_time and the episode sums itself (the fused
// epilogue, where that pass runs on another wave concurrently: post_a_core<POST_A_REWARDS>)
// (the new state's observation inputs: reset_obs_inputs, from the same draws, instead of reading back the rows just
// written -- one dependent memory round trip less)
// obs_elsewhere: the last_* rows are left to the wave that writes the observations (the fused epilogue's post_b
// stores them after the reset, with the values reset_obs_inputs gives; two waves storing one row would race)
// pos_cmd: the env's root position (x, y) and commands as they stand (the caller's registers) instead of memory
__device__ __forceinline__ void reset_env(const DynModel& M, const t1env_config& C, const t1env_buffers& B, const t1env_step_args& A,
                          int n, uint32_t genv, uint32_t ctr, bool do_terrain, bool zero_reward_state = true,
                          bool obs_elsewhere = false, const float* pos_cmd = nullptr) {
  const RngKey K = rng_key(C.seed, genv, ctr);
  float org[3];
  bool org_known = false;
  if (do_terrain && C.terrain_curriculum) {  // _update_terrain_curriculum
    const float* r = pos_cmd ? pos_cmd : B.root_states + n * 13;
    const float* o = B.env_origins + n * 3;
    const float dist = norm2(r[0] - o[0], r[1] - o[1]);
    const bool up = dist > C.env_length / 2.0f;
    const float* cmd = pos_cmd ? pos_cmd + 2 : B.commands + n * 4;
    const bool down = (dist < norm2(cmd[0], cmd[1]) * (C.episode_length_s * 0.5f)) && !up;
    int lv = B.terrain_levels[n] + (up ? 1 : 0) - (down ? 1 : 0);
    const int rnd = rand_int(0, C.num_terrain_rows, K, SLOT_TERRAIN_LEVEL_RAND);
    lv = lv >= C.num_terrain_rows ? rnd : (lv < 0 ? 0 : lv);
    B.terrain_levels[n] = lv;
    const float* to = B.terrain_origins + ((size_t)lv * C.num_terrain_cols + B.terrain_types[n]) * 3;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      org[i] = to[i];
      B.env_origins[n * 3 + i] = org[i];
    }
    org_known = true;
  }
  if (!org_known)
#pragma unroll
    for (int i = 0; i < 3; ++i) org[i] = B.env_origins[n * 3 + i];
  ObsIn R;
  reset_obs_inputs(M, C, K, R);
  // the new episode starts in the air as far as restitution is concerned (no contact episode carried over)
#pragma unroll
  for (int i = 0; i < NVIMP; ++i) B.contact_vimp[(size_t)n * NVIMP + i] = 0.0f;
  // _reset_dofs
#pragma unroll
  for (int j = 0; j < 24; ++j) B.dof_state[n * 24 + j] = R.dof[j];
  // _reset_root_states (in registers, then stored)
  float r[13];
#pragma unroll
  for (int i = 0; i < 13; ++i) r[i] = M.base_init_state[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) r[i] += org[i];
  if (C.custom_origins) {
    const float p3 = C.reset_xy_range;
    r[0] += rand_float(-p3, p3, K, SLOT_RESET_ROOT_XY + 0);
    r[1] += rand_float(-p3, p3, K, SLOT_RESET_ROOT_XY + 1);
  }
  strow(B.root_states + n * 13, r);
  // randomize_dof_props (torque_multi is redrawn every substep anyway; its reset draw has no effect)
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    B.motor_offsets[n * 12 + j] =
        rand_float(C.motor_offset_range[0], C.motor_offset_range[1], K, SLOT_DR_OFFSET + j);
    B.kp[n * 12 + j] = rand_float(C.kp_mult_range[0], C.kp_mult_range[1], K, SLOT_DR_KP + j) * M.p_gains[j];
    B.kd[n * 12 + j] = rand_float(C.kd_mult_range[0], C.kd_mult_range[1], K, SLOT_DR_KD + j) * M.d_gains[j];
    B.coulomb[n * 12 + j] = rand_float(C.coulomb_range[0], C.coulomb_range[1], K, SLOT_DR_COULOMB + j);
    B.viscous[n * 12 + j] = rand_float(C.viscous_range[0], C.viscous_range[1], K, SLOT_DR_VISCOUS + j);
    B.armature[n * 12 + j] =
        rand_float(C.armature_range[j][0], C.armature_range[j][1], K, SLOT_DR_ARMATURE + j);
  }
  // randomize_lag_props: zero the lag rings, redraw lag lengths
#ifndef T1_WHATIF_NO_RING_ZERO  // timing-only what-if build
#pragma unroll
  for (int i = 0; i < 48; ++i) B.act_hist[(size_t)n * 48 + i] = 0.0f;
#pragma unroll
  for (int i = 0; i < 96; ++i) B.dof_hist[(size_t)n * 96 + i] = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) B.imu_hist[(size_t)n * 16 + i] = 0.0f;
#endif
  B.lag_timestep[n] = rand_int(C.lag_range[0], C.lag_range[1] + 1, K, SLOT_LAG_ACTION);
  B.dof_lag_timestep[n] = R.dl;
  B.imu_lag_timestep[n] = R.il;
  // buffers
#pragma unroll
  for (int j = 0; j < 12; ++j) B.actions[n * 12 + j] = 0.0f;
  if (!obs_elsewhere) {
#pragma unroll
    for (int j = 0; j < 12; ++j) {
      B.last_last_actions[n * 12 + j] = 0.0f;
      B.last_actions[n * 12 + j] = 0.0f;
      B.last_dof_vel[n * 12 + j] = 0.0f;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) B.last_root_vel[n * 6 + i] = 0.0f;
  }
  if (zero_reward_state) {
    B.feet_air_time[n * 2 + 0] = 0.0f;
    B.feet_air_time[n * 2 + 1] = 0.0f;
  }
  B.episode_length_buf[n] = 0;
  B.phase_length_buf[n] = 0;
  B.reset_buf[n] = 1;
  B.gait_start[n] = R.gstart;
  strow(B.gait_time + n * 3, R.gt);
  // episode sums are zeroed after the extras reduction; obs/critic history rows zeroed in the stack pass
  if (zero_reward_state)
#pragma unroll
    for (int k = 0; k < T1_NREW; ++k) B.episode_sums[(size_t)k * C.num_envs + n] = 0.0f;
  // base quantities of the reset env from the fresh root state (t1:548-552)
  store_base_quantities(B, n, R.bq);
}

// the actor-frame noise of observation i (legged_robot.py compute_observations: (2 u - 1) * noise_vec * level, u keyed
// by the env's post-physics key)
__device__ __forceinline__ float obs_noise(const t1env_config& C, RngKey K, int i) {
  const float u = uniform01(K, SLOT_OBS_NOISE + i);
  return ((2.0f * u - 1.0f) * C.noise_vec[i]) * C.noise_level;
}

// =====================================================================================================
// post-physics phase B: reset + observations (legged_robot.py:490-502, t1:368-481)
// =====================================================================================================
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
// the rest of post_b's per-env inputs (reset_idx leaves them unchanged)
struct ObsExtra {
  float ef[2], et[3], cfz[2], fric, mass;
};
__device__ __forceinline__ void post_b_core(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                            const t1env_step_args& A, int n, bool do_reset, bool any_reset, ObsIn& X,
                                            const ObsExtra& E, bool zero_reward_state = true);
__device__ __forceinline__ void post_b_env(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                           const t1env_step_args& A, int n, bool do_reset, bool any_reset) {
  ObsIn X;
  load_obs_in(B, n, X);
  ObsExtra E;
  ldrow(E.ef, B.ext_forces + n * 3);
  ldrow(E.et, B.ext_torques + n * 3);
  E.cfz[0] = B.contact_forces[(size_t)n * 39 + 6 * 3 + 2];
  E.cfz[1] = B.contact_forces[(size_t)n * 39 + 12 * 3 + 2];
  E.fric = B.friction[n];
  E.mass = B.body_mass[n];
  post_b_core(M, C, B, A, n, do_reset, any_reset, X, E);
}

// compute_observations' gait terms (t1:250-274, 368-481): sin / cos of the phase, the reference joint positions and
// the stance masks of an env whose phase counter X.pl is already zeroed for standing
struct ObsPhase {
  float sp, cp, ref[12];
  Phase ph;
};
__device__ __forceinline__ void obs_phase(const DynModel& M, const t1env_config& C, const ObsIn& X, bool stand,
                                          ObsPhase& P) {
  const float phase = phase_value(C, X.pl, X.gstart, stand);
  // compute_ref_state (t1:250-274)
  P.sp = sinf(TWO_PI_F * phase);
  P.cp = cosf(TWO_PI_F * phase);
  const float sl = P.sp > 0.0f ? 0.0f : P.sp;
  const float sr = P.sp < 0.0f ? 0.0f : P.sp;
  const float s1 = C.target_joint_pos_scale, s2 = 2.0f * C.target_joint_pos_scale;
  float* ref = P.ref;
#pragma unroll
  for (int j = 0; j < 12; ++j) ref[j] = 0.0f;
  ref[2] = sl * s1; ref[3] = -sl * s2; ref[4] = sl * s1;
  ref[8] = -sr * s1; ref[9] = sr * s2; ref[10] = -sr * s1;
  if (fabsf(P.sp) < 0.1f)
#pragma unroll
    for (int j = 0; j < 12; ++j) ref[j] = 0.0f;
#pragma unroll
  for (int j = 0; j < 12; ++j) ref[j] = ref[j] + M.default_dof_pos[j];
  P.ph = gait_phase(phase);
}

// the newest frames: fp32, or rounded once to fp16 (round to nearest even, as torch's .half()) with obs_half
// privileged frame (73)
__device__ __forceinline__ void store_priv_frame(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                                 const t1env_step_args& A, int n, const ObsIn& X, const ObsExtra& E,
                                                 const ObsPhase& P) {
  const size_t priv_at = (size_t)n * (T1_NPRIV * T1_CHIST) + T1_NPRIV * (T1_CHIST - 1);
  float* priv = B.priv_buf[A.obs_slot] + priv_at;
  _Float16* priv_h = reinterpret_cast<_Float16*>(B.priv_buf[A.obs_slot]) + priv_at;
  const float clipo = C.clip_obs;
  const float* cmd = X.cmd;
  const float* dof = X.dof;
  int k = 0;
  float v[T1_NPRIV];
  v[k++] = P.sp;
  v[k++] = P.cp;
  v[k++] = cmd[0] * C.lin_vel_obs_scale;
  v[k++] = cmd[1] * C.lin_vel_obs_scale;
  v[k++] = cmd[2] * C.ang_vel_obs_scale;
#pragma unroll
  for (int j = 0; j < 12; ++j) v[k++] = (dof[2 * j] - M.default_dof_pos[j]) * C.dof_pos_obs_scale;
#pragma unroll
  for (int j = 0; j < 12; ++j) v[k++] = dof[2 * j + 1] * C.dof_vel_obs_scale;
#pragma unroll
  for (int j = 0; j < 12; ++j) v[k++] = X.act[j];
#pragma unroll
  for (int j = 0; j < 12; ++j) v[k++] = dof[2 * j] - P.ref[j];
#pragma unroll
  for (int i = 0; i < 3; ++i) v[k++] = X.bq.lin[i] * C.lin_vel_obs_scale;
#pragma unroll
  for (int i = 0; i < 3; ++i) v[k++] = X.bq.ang[i] * C.ang_vel_obs_scale;
#pragma unroll
  for (int i = 0; i < 3; ++i) v[k++] = X.bq.euler[i] * C.quat_obs_scale;
  v[k++] = E.ef[0] / (C.ext_force_max[0] + 0.1f);
  v[k++] = E.ef[1] / (C.ext_force_max[0] + 0.1f);
#pragma unroll
  for (int i = 0; i < 3; ++i) v[k++] = E.et[i] / (C.ext_torque_max + 0.1f);
  v[k++] = E.fric;
  v[k++] = E.mass / 30.0f;
  v[k++] = P.ph.stance[0];
  v[k++] = P.ph.stance[1];
  v[k++] = E.cfz[0] > 5.0f ? 1.0f : 0.0f;
  v[k++] = E.cfz[1] > 5.0f ? 1.0f : 0.0f;
  if (C.obs_half) {
#pragma unroll
    for (int i = 0; i < T1_NPRIV; ++i) priv_h[i] = (_Float16)clampf(v[i], -clipo, clipo);
  } else {
#pragma unroll
    for (int i = 0; i < T1_NPRIV; ++i) priv[i] = clampf(v[i], -clipo, clipo);
  }
}

// actor frame (47) from the lagged sensor samples (ld: joint positions / velocities, li: imu angular velocity and
// euler angles) + noise
__device__ __forceinline__ void store_actor_frame(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                                  const t1env_step_args& A, int n, RngKey K, const ObsIn& X,
                                                  const float ld[24], const float li[6], const ObsPhase& P) {
  const size_t obs_at = (size_t)n * (T1_NOBS * T1_HIST) + T1_NOBS * (T1_HIST - 1);
  float* obs = B.obs_buf[A.obs_slot] + obs_at;
  _Float16* obs_h = reinterpret_cast<_Float16*>(B.obs_buf[A.obs_slot]) + obs_at;
  const float clipo = C.clip_obs;
  const float* cmd = X.cmd;
  float v[T1_NOBS];
  int k = 0;
  v[k++] = P.sp;
  v[k++] = P.cp;
  v[k++] = cmd[0] * C.lin_vel_obs_scale;
  v[k++] = cmd[1] * C.lin_vel_obs_scale;
  v[k++] = cmd[2] * C.ang_vel_obs_scale;
#pragma unroll
  for (int j = 0; j < 12; ++j) v[k++] = (ld[j] - M.default_dof_pos[j]) * C.dof_pos_obs_scale;
#pragma unroll
  for (int j = 0; j < 12; ++j) v[k++] = ld[12 + j] * C.dof_vel_obs_scale;
#pragma unroll
  for (int j = 0; j < 12; ++j) v[k++] = X.act[j];
#pragma unroll
  for (int i = 0; i < 3; ++i) v[k++] = li[i] * C.ang_vel_obs_scale;
#pragma unroll
  for (int i = 0; i < 3; ++i) v[k++] = li[3 + i] * C.quat_obs_scale;
#pragma unroll
  for (int i = 0; i < T1_NOBS; ++i) {
#ifdef T1_WHATIF_NO_NOISE_DRAWS  // timing-only what-if build
    const float nz = 0.0f;
#else
    const float nz = obs_noise(C, K, i);
#endif
    v[i] = clampf(v[i] + nz, -clipo, clipo);
  }
  if (C.obs_half) {
#pragma unroll
    for (int i = 0; i < T1_NOBS; ++i) obs_h[i] = (_Float16)v[i];
  } else {
#pragma unroll
    for (int i = 0; i < T1_NOBS; ++i) obs[i] = v[i];
  }
}

// ref_dof_pos and last_* (legged_robot.py:496-502)
__device__ __forceinline__ void store_obs_last(const t1env_buffers& B, int n, const ObsIn& X, const float (&ref)[12]) {
  strow(B.ref_dof_pos + n * 12, ref);
  strow(B.last_last_actions + n * 12, X.la);
  strow(B.last_actions + n * 12, X.act);
#pragma unroll
  for (int j = 0; j < 12; ++j) B.last_dof_vel[n * 12 + j] = X.dof[2 * j + 1];
  strow(B.last_root_vel + n * 6, X.rv);
}

// the lagged sensor samples of an env (lags dl / il as they stand before this step's reset)
__device__ __forceinline__ void load_lagged(const t1env_buffers& B, const t1env_step_args& A, int n, int dl, int il,
                                            float (&ld)[24], float (&lraw)[8]) {
  const float* ldp = B.dof_hist + ((size_t)n * 4 + ((A.counter - (uint32_t)(dl / 10)) & 3u)) * 24;
  const float* lip = B.imu_hist + ((size_t)n * 2 + ((A.counter - (uint32_t)(il / 10)) & 1u)) * 8;
#ifdef T1_WHATIF_NO_LAG_LOADS  // timing-only what-if build: the lagged sensor samples not loaded
  (void)ldp;
  (void)lip;
#pragma unroll
  for (int i = 0; i < 24; ++i) ld[i] = 0.0f;
#pragma unroll
  for (int i = 0; i < 8; ++i) lraw[i] = 0.0f;
  lraw[3] = 1.0f;
#else
  ldrow(ld, ldp);
  ldrow(lraw, lip);
#endif
}

// X: the inputs as they stand after post_a (reloaded here after a reset)
__device__ __forceinline__ void post_b_core(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                            const t1env_step_args& A, int n, bool do_reset, bool any_reset, ObsIn& X,
                                            const ObsExtra& E, bool zero_reward_state) {
  const uint32_t genv = (uint32_t)(C.env_offset + n);
  const uint32_t ctr = A.counter + 1u;
  const RngKey K = rng_key(C.seed, genv, ctr);
  // lagged sensor samples, loaded before the reset: a resetting env's rings are zeroed by its reset, so its samples
  // are 0 whatever its new lag lengths (below); the others keep their lag lengths
  float ld[24], lraw[8], li[6];
  load_lagged(B, A, n, X.dl, X.il, ld, lraw);
  if (do_reset) {
    reset_env(M, C, B, A, n, genv, ctr, true, zero_reward_state);
    reset_obs_inputs(M, C, K, X);
#pragma unroll
    for (int i = 0; i < 24; ++i) ld[i] = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) lraw[i] = 0.0f;
  }
  T1_PROF_MARK(20);
  if (any_reset && resample_commands_r(C, A, X.el, X.gt, X.cmd, genv, ctr)) strow(B.commands + n * 4, X.cmd);
  imu_sample(lraw, li);
  // ---- compute_observations
  const bool stand = is_stand(C, X.cmd);
  if (stand) {  // _get_phase zeroes the phase counter of standing envs
    X.pl = 0;
    B.phase_length_buf[n] = 0;
  }
  ObsPhase P;
  obs_phase(M, C, X, stand, P);
  T1_PROF_MARK(21);
  store_priv_frame(M, C, B, A, n, X, E, P);
  T1_PROF_MARK(22);
  store_actor_frame(M, C, B, A, n, K, X, ld, li, P);
  T1_PROF_MARK(23);
  store_obs_last(B, n, X, P.ref);
}

}  // namespace t1
