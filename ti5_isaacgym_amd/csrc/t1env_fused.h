// t1env_fused.h -- the parts of the step kernels shared by k_dyn4 (t1env_dynamics.hip, 64 envs per workgroup) and
// k_dyn5 (t1env_dyn5.hip, 32 envs per workgroup): per-leg setup, the fused epilogue (post-physics of a workgroup's
// envs from LDS-staged inputs), the rigid-state and contact-force reports and the extras finaliser.  Templated on
// NE, the envs of one workgroup; LDS rows are [value][env] (conflict-free).  Included after t1env_postphys.h (no FMA
// contraction: the report and post-physics keep the reference's fp32 evaluation order).
#pragma once
#include "t1env_device.h"
#include "t1env_internal.h"
#include "t1env_postphys.h"

namespace t1 {

constexpr int SHIFT_UNIT = 8;  // rows per shift/zeroing unit (a multiple of 4: unit boundaries are 16-B aligned)
constexpr int K_SHANK = 3, K_FOOT = 5;
static_assert(T1_LEG_CONTACT_MASK == ((1 << K_SHANK) | (1 << K_FOOT)), "the step kernels assume shank + foot contacts");
constexpr int XCH = 27;  // Sym6 (21) + rhs (6)

// ---- the in-launch history shift's reset-row handoff (k_dyn4: the shift runs in other workgroups, possibly on
// another XCD).  Handoff word of a shift unit: [epoch tag : 22][reset mask : 8][dynamics done : 1][shift done : 1].
// Set `bits` (state bits and, from the dynamics side, the mask) for this epoch; returns the new word.  The word is
// complete when both state bits are set; the party whose update completes it zeroes the unit's reset rows.
constexpr uint32_t HANDOFF_SHIFT = 1u, HANDOFF_DYN = 2u;
__device__ __forceinline__ uint32_t unit_handoff(uint32_t* word, uint32_t epoch, uint32_t bits) {
  const uint32_t tag = (epoch & 0x3fffffu) << 10;
  uint32_t old = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    const uint32_t nw = ((old & ~0x3ffu) == tag ? old : tag) | bits;
    if (__hip_atomic_compare_exchange_strong(word, &old, nw, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT))
      return nw;
  }
}
__device__ __forceinline__ bool handoff_complete(uint32_t w) { return (w & 3u) == 3u; }

// zero the history rows of unit u flagged in its handoff word
__device__ __forceinline__ void zero_unit_resets(const ShiftArgs& S, int u, uint32_t word, int t0, int stride) {
  uint32_t bits = (word >> 2) & 0xffu;
  while (bits) {
    const int r = __ffs(bits) - 1;
    bits &= bits - 1;
    zero_history_row(S, (int64_t)u * SHIFT_UNIT + r, t0, stride);
  }
}

// After post-physics: the reset rows of the workgroup's NE envs.  INWG (k_dyn5): the workgroup shifted its own rows
// earlier in the launch, so it zeroes its reset rows itself (the shift's stores completed before the epilogue
// barrier); likewise when the shift ran as its own launch before this one (FA.shift_done).  Otherwise (k_dyn4) each
// of the workgroup's shift units is handed off with its 8-bit reset mask.
template <int NE, bool INWG>
__device__ __forceinline__ void epilogue_handoff(const t1env_config& C, const ShiftArgs& S, const FusedArgs& FA, int lane,
                                                 bool do_reset, bool active) {
  const int N = C.num_envs;
  const unsigned long long m = __ballot(do_reset && active);
  if (INWG || FA.shift_done) {
    unsigned long long todo = m;
    while (todo) {
      const int l = __ffsll(todo) - 1;
      todo &= todo - 1;
      zero_history_row(S, (int64_t)blockIdx.x * NE + l, lane, 64);
    }
    return;
  }
  // ---- reset rows: hand off each of the workgroup's shift units with its 8-bit reset mask
  const int units = (N + SHIFT_UNIT - 1) / SHIFT_UNIT;
  const int u = blockIdx.x * (NE / SHIFT_UNIT) + lane;
  uint32_t w = 0;
  if (lane < NE / SHIFT_UNIT && u < units)
    w = unit_handoff(FA.unit_state + u, FA.epoch, HANDOFF_DYN | ((uint32_t)(m >> (lane * SHIFT_UNIT)) & 0xffu) << 2);
  uint64_t todo = __ballot(handoff_complete(w));
  while (todo) {
    const int l = __ffsll((unsigned long long)todo) - 1;
    todo &= todo - 1;
    zero_unit_resets(S, blockIdx.x * (NE / SHIFT_UNIT) + l, __shfl(w, l, 64), lane, 64);
  }
}

// The finaliser: every dynamics workgroup stored one row of partial sums (FusedArgs::ep_part, agent-scope stores
// completed before its counter increment); the last one sums the rows in a fixed order after an acquire fence (no
// same-address atomics: 25 per workgroup into one row cost 3.6% of the step, r02ar).  Lane l reads the float4 l % 8 of
// rows l / 8, l / 8 + 8, ...; the 8 lanes of a float4 are then summed across the wave.
__device__ __forceinline__ void epilogue_finalize_parts(const t1env_config& C, const t1env_buffers& B,
                                                        const t1env_step_args& A, const FusedArgs& FA, int dyn_blocks,
                                                        int lane) {
#ifdef T1_WHATIF_NO_FINALIZE  // timing-only what-if build: no completion counter, no extras
  return;
#endif
  unsigned prev = 0;
  // Ordering: the increment is RELAXED and no release fence precedes it.  What orders the ep_part rows
  // before it is gfx950 hardware behaviour, not the HIP memory model: every row element is a relaxed agent-scope
  // store (global_store ... sc1, which writes through past this XCD's L2 and drops the line), every storing wave ran
  // s_waitcnt vmcnt(0) after its stores and joined the barrier before lane 0's agent-scope atomic add; the workgroup
  // whose add returns dyn_blocks - 1 then reads the rows after an agent acquire (buffer_inv sc1).  That is the
  // hand-off MI355X_MICROARCH.md measures safe on gfx950 / ROCm 7.2 ("one lane of each storing workgroup ... an
  // agent-scope atomic add", sc1 stores); an agent release here would be buffer_wbl2 sc1 per workgroup, ~1.7-6.5 us
  // on the step's tail (same guide).  Porting this off gfx950 needs __ATOMIC_RELEASE on the add.
  if (lane == 0) prev = __hip_atomic_fetch_add(FA.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  prev = __shfl(prev, 0, 64);
  if (prev != (unsigned)dyn_blocks - 1u) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  static_assert(EP_PART_ROW == 32, "8 float4 per row");
  const float4* P = reinterpret_cast<const float4*>(FA.ep_part);
  const int q = lane & 7;
  float4 s = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  // loads in flight per lane: 32 covers 256 workgroups in one memory round trip (8 took four, serialised at the very
  // end of the launch); each lane still adds its rows in row order, so the sums do not depend on BATCH
  constexpr int BATCH = 32;
  for (int r0 = lane >> 3; r0 < dyn_blocks; r0 += 8 * BATCH) {
    float4 v[BATCH];
#pragma unroll
    for (int j = 0; j < BATCH; ++j) {
      const int r = r0 + 8 * j;
      v[j] = r < dyn_blocks ? P[(size_t)r * 8 + q] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
#pragma unroll
    for (int j = 0; j < BATCH; ++j) { s.x += v[j].x; s.y += v[j].y; s.z += v[j].z; s.w += v[j].w; }
  }
#pragma unroll
  for (int off = 8; off < 64; off <<= 1) {
    s.x += __shfl_xor(s.x, off, 64); s.y += __shfl_xor(s.y, off, 64);
    s.z += __shfl_xor(s.z, off, 64); s.w += __shfl_xor(s.w, off, 64);
  }
  // sum t (t < 32) sits in component t % 4 of lane t / 4
  const int src = (lane & 31) >> 2;
  const float c0 = __shfl(s.x, src, 64), c1 = __shfl(s.y, src, 64), c2 = __shfl(s.z, src, 64), c3 = __shfl(s.w, src, 64);
  const int c = lane & 3;
  const float mine = c == 0 ? c0 : c == 1 ? c1 : c == 2 ? c2 : c3;
  const float cnt = __shfl(mine, 24, 64);    // reset count
  const float lvl = __shfl(mine, 25, 64);    // terrain-level sum
  const int slot = (int)((A.counter + 1u) % T1ENV_EXTRAS_RING);
  float* ex = B.extras + (size_t)slot * 32;
  const float* prevx = B.extras + (size_t)((slot + T1ENV_EXTRAS_RING - 1) % T1ENV_EXTRAS_RING) * 32;
  if (lane < 32) {  // finalize_extras' formulas
    float v = prevx[lane];
    if (cnt > 0.0f) {
      if (lane < T1_NREW) v = (mine / cnt) / C.episode_length_s;
      else if (lane == 24) v = lvl / (float)C.num_envs;
    }
    ex[lane] = v;
  }
  if (lane == 0) __hip_atomic_store(FA.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// per-leg setup shared by the step kernels: clipped actions into the step's action slot, sensor-lag capture
// slots, per-env parameters, base state and the leg's joint state
struct LegSetup {
  int lag, s_dof, s_imu;
  float* dof_dst;
  float* imu_dst;
};
__device__ __forceinline__ LegSetup leg_setup(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                              const float* __restrict__ actions, uint32_t ctr, int n, bool active,
                                              int j0, BaseParams<float>& PB, LegParams<float>& PL,
                                              BaseState<float>& sb, float q[NLEG], float qd[NLEG]) {
  if (active) {  // actions = clip(actions); push the scaled action into this step's history slot
    float* slot = B.act_hist + ((size_t)n * 4 + (ctr & 3u)) * 12;
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      const float a = fminf(fmaxf(actions[n * 12 + j0 + k], -C.clip_actions), C.clip_actions);
      B.actions[n * 12 + j0 + k] = a;
      slot[j0 + k] = a * C.action_scale;
    }
  }
  LegSetup L;
  L.lag = B.lag_timestep[n];
  L.s_dof = 9 - B.dof_lag_timestep[n] % 10;
#ifdef T1_MUTANT_CAPTURE  // mutation check of tests/test_gpu_product_parity.py only (tools/gpu): capture a substep early
  L.s_dof = L.s_dof > 0 ? L.s_dof - 1 : 0;
#endif
  L.s_imu = 9 - B.imu_lag_timestep[n] % 10;
  L.dof_dst = B.dof_hist + ((size_t)n * 4 + (ctr & 3u)) * 24;
  L.imu_dst = B.imu_hist + ((size_t)n * 2 + (ctr & 1u)) * 8;
  load_base_params(M, B, n, PB);
  load_leg_params(M, B, n, j0, PL);
  load_base_state(M, PB, B.root_states + (size_t)n * 13, sb);
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    q[k] = B.dof_state[n * 24 + 2 * (j0 + k)];
    qd[k] = B.dof_state[n * 24 + 2 * (j0 + k) + 1];
  }
  return L;
}

// fused epilogue staging (post-physics inputs of the workgroup's envs in LDS):
//   epi (EPI_N rows): the state post-physics reads that the step has not changed, prefetched with coalesced
//        row loads by the helper waves while the leg waves run the dynamics
//   fresh (FR_N rows): this step's dynamics outputs, from registers
enum : int {
  E_LA = 0, E_LLA = 12, E_LRV = 24, E_LDV = 30, E_REF = 42, E_CMD = 54, E_AT = 58, E_FH = 60, E_LFZ = 62,
  E_EF = 64, E_ET = 67, E_GT = 70, E_EL = 73, E_PL = 75, E_GS = 77, E_LC = 78, E_FRIC = 80, E_MASS = 81,
  E_DL = 82, E_IL = 83, E_ESUM = 84, EPI_N = 84 + T1_NREW
};
enum : int {
  F_ROOT = 0, F_DOF = 13, F_TQ = 37, F_F0 = 49, F_F1 = 62, F_K0 = 75, F_K1 = 77, F_CFB = 79, F_C0 = 82, F_C1 = 85,
  FR_N = 88
};

// ---- epilogue staging by NT threads (t in [0, NT)) for the NE envs of the workgroup.  Rows [nb, nb + nv) of the
// env buffers; a row-major source is read as one contiguous run (consecutive threads, consecutive words:
// coalesced) and transposed into [value][env].  All loads of a thread are issued before the first LDS write
// (stage_ld for every source, then stage_st), so the staging costs one memory latency.
template <int NE, int NT, int L> constexpr int stage_n() { return (NE * L + NT - 1) / NT; }
template <typename T> __device__ __forceinline__ float stage_bits(T v) {
  if constexpr (sizeof(T) == 4) return __builtin_bit_cast(float, v);
  else return __int_as_float((int)v);
}
template <int NE, int NT, int L, typename T>
__device__ __forceinline__ void stage_ld(const T* __restrict__ src, int nb, int nv, int t, float (&v)[stage_n<NE, NT, L>()]) {
  const T* base = src + (size_t)nb * L;
#pragma unroll
  for (int i = 0; i < stage_n<NE, NT, L>(); ++i) {
    const int e = t + NT * i;
    v[i] = e < nv * L ? stage_bits(base[e]) : 0.0f;
  }
}
template <int NE, int NT, int L>
__device__ __forceinline__ void stage_st(float (*dst)[NE], int nv, int t, const float (&v)[stage_n<NE, NT, L>()]) {
#pragma unroll
  for (int i = 0; i < stage_n<NE, NT, L>(); ++i) {
    const int e = t + NT * i;
    if (e < nv * L) dst[e % L][e / L] = v[i];
  }
}
// the staged values of one thread between its loads and its LDS writes (epi_stage_load / epi_stage_store)
template <int NE, int NT> struct EpiStage {
  static constexpr int NES = (T1_NREW * NE + NT - 1) / NT;
  float la[stage_n<NE, NT, 12>()], lla[stage_n<NE, NT, 12>()], lrv[stage_n<NE, NT, 6>()], ldv[stage_n<NE, NT, 12>()];
  float ref[stage_n<NE, NT, 12>()], cmd[stage_n<NE, NT, 4>()], at[stage_n<NE, NT, 2>()], fh[stage_n<NE, NT, 2>()];
  float lfz[stage_n<NE, NT, 2>()], ef[stage_n<NE, NT, 3>()], et[stage_n<NE, NT, 3>()], gt[stage_n<NE, NT, 3>()];
  float el[stage_n<NE, NT, 2>()], pl[stage_n<NE, NT, 2>()], gs[stage_n<NE, NT, 1>()], lc[stage_n<NE, NT, 2>()];
  float fr[stage_n<NE, NT, 1>()], ms[stage_n<NE, NT, 1>()], dl[stage_n<NE, NT, 1>()], il[stage_n<NE, NT, 1>()];
  float es[NES];
};
template <int NE, int NT>
__device__ __forceinline__ void epi_stage_load(const t1env_buffers& B, int N, int nb, int t, EpiStage<NE, NT>& V) {
  const int nv = N - nb < NE ? N - nb : NE;
  stage_ld<NE, NT, 12>(B.last_actions, nb, nv, t, V.la);
  stage_ld<NE, NT, 12>(B.last_last_actions, nb, nv, t, V.lla);
  stage_ld<NE, NT, 6>(B.last_root_vel, nb, nv, t, V.lrv);
  stage_ld<NE, NT, 12>(B.last_dof_vel, nb, nv, t, V.ldv);
  stage_ld<NE, NT, 12>(B.ref_dof_pos, nb, nv, t, V.ref);
  stage_ld<NE, NT, 4>(B.commands, nb, nv, t, V.cmd);
  stage_ld<NE, NT, 2>(B.feet_air_time, nb, nv, t, V.at);
  stage_ld<NE, NT, 2>(B.feet_height, nb, nv, t, V.fh);
  stage_ld<NE, NT, 2>(B.last_feet_z, nb, nv, t, V.lfz);
  stage_ld<NE, NT, 3>(B.ext_forces, nb, nv, t, V.ef);
  stage_ld<NE, NT, 3>(B.ext_torques, nb, nv, t, V.et);
  stage_ld<NE, NT, 3>(B.gait_time, nb, nv, t, V.gt);
  stage_ld<NE, NT, 2>(reinterpret_cast<const uint32_t*>(B.episode_length_buf), nb, nv, t, V.el);
  stage_ld<NE, NT, 2>(reinterpret_cast<const uint32_t*>(B.phase_length_buf), nb, nv, t, V.pl);
  stage_ld<NE, NT, 1>(B.gait_start, nb, nv, t, V.gs);
  stage_ld<NE, NT, 2>(B.last_contacts, nb, nv, t, V.lc);
  stage_ld<NE, NT, 1>(B.friction, nb, nv, t, V.fr);
  stage_ld<NE, NT, 1>(B.body_mass, nb, nv, t, V.ms);
  stage_ld<NE, NT, 1>(B.dof_lag_timestep, nb, nv, t, V.dl);
  stage_ld<NE, NT, 1>(B.imu_lag_timestep, nb, nv, t, V.il);
#pragma unroll
  for (int i = 0; i < EpiStage<NE, NT>::NES; ++i) {  // episode_sums is [reward][env]: already row-contiguous
    const int e = t + NT * i;
    V.es[i] = e < T1_NREW * nv ? B.episode_sums[(size_t)(e / nv) * N + nb + e % nv] : 0.0f;
  }
}
template <int NE, int NT>
__device__ __forceinline__ void epi_stage_store(int N, int nb, int t, const EpiStage<NE, NT>& V, float (*E)[NE]) {
  const int nv = N - nb < NE ? N - nb : NE;
  stage_st<NE, NT, 12>(E + E_LA, nv, t, V.la);
  stage_st<NE, NT, 12>(E + E_LLA, nv, t, V.lla);
  stage_st<NE, NT, 6>(E + E_LRV, nv, t, V.lrv);
  stage_st<NE, NT, 12>(E + E_LDV, nv, t, V.ldv);
  stage_st<NE, NT, 12>(E + E_REF, nv, t, V.ref);
  stage_st<NE, NT, 4>(E + E_CMD, nv, t, V.cmd);
  stage_st<NE, NT, 2>(E + E_AT, nv, t, V.at);
  stage_st<NE, NT, 2>(E + E_FH, nv, t, V.fh);
  stage_st<NE, NT, 2>(E + E_LFZ, nv, t, V.lfz);
  stage_st<NE, NT, 3>(E + E_EF, nv, t, V.ef);
  stage_st<NE, NT, 3>(E + E_ET, nv, t, V.et);
  stage_st<NE, NT, 3>(E + E_GT, nv, t, V.gt);
  stage_st<NE, NT, 2>(E + E_EL, nv, t, V.el);
  stage_st<NE, NT, 2>(E + E_PL, nv, t, V.pl);
  stage_st<NE, NT, 1>(E + E_GS, nv, t, V.gs);
  stage_st<NE, NT, 2>(E + E_LC, nv, t, V.lc);
  stage_st<NE, NT, 1>(E + E_FRIC, nv, t, V.fr);
  stage_st<NE, NT, 1>(E + E_MASS, nv, t, V.ms);
  stage_st<NE, NT, 1>(E + E_DL, nv, t, V.dl);
  stage_st<NE, NT, 1>(E + E_IL, nv, t, V.il);
#pragma unroll
  for (int i = 0; i < EpiStage<NE, NT>::NES; ++i) {
    const int e = t + NT * i;
    if (e < T1_NREW * nv) E[E_ESUM + e / nv][e % nv] = V.es[i];
  }
}
template <int NE, int NT>
__device__ __forceinline__ void stage_epilogue_inputs(const t1env_buffers& B, int N, int nb, int t, float (*E)[NE]) {
  EpiStage<NE, NT> V;
  epi_stage_load<NE, NT>(B, N, nb, t, V);
  epi_stage_store<NE, NT>(N, nb, t, V, E);
}

// The fused step's post-physics for the NE envs of one workgroup, run by four waves after the epilogue barrier (lane =
// env; lanes >= NE shadow an env of the workgroup and store nothing), every input from LDS (fresh outputs FR, staged
// state E, the clipped actions in ACT0 (joints 0-5) / ACT1 (joints 6-11)).  This function is the two post_a waves:
// both run post_a's callback + termination prefix; PART = POST_A_REWARDS then the 24 rewards, their stores and extras
// sums and the reset rows, POST_A_STATE the state stores, reset_idx of the resetting envs (their new state, commands
// redrawn) and the terrain-level sum.  The observations are the other two waves' (fused_epilogue_obs).  After one
// barrier the rewards wave signals completion (the extras finaliser).
template <int PART, int NE, bool INWG>
__device__ __forceinline__ void fused_epilogue_staged(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                                      const t1env_step_args& A, const ShiftArgs& S,
                                                      const FusedArgs& FA, int dyn_blocks, int lane,
                                                      const float (*E)[NE], const float (*FR)[NE],
                                                      const float (*ACT0)[NE], const float (*ACT1)[NE]) {
  const int N = C.num_envs;
  const int e = lane % NE;  // the LDS column (lanes >= NE read a valid column and are inactive)
  const int n0 = lane < NE ? (int)blockIdx.x * NE + lane : N;
  const bool active = n0 < N;
  const int n = active ? n0 : N - 1;
  PostAIn X;
#pragma unroll
  for (int i = 0; i < 13; ++i) X.root[i] = FR[F_ROOT + i][e];
#pragma unroll
  for (int i = 0; i < 24; ++i) X.dof[i] = FR[F_DOF + i][e];
#pragma unroll
  for (int i = 0; i < 13; ++i) { X.f0[i] = FR[F_F0 + i][e]; X.f1[i] = FR[F_F1 + i][e]; }
#pragma unroll
  for (int i = 0; i < 2; ++i) { X.k0[i] = FR[F_K0 + i][e]; X.k1[i] = FR[F_K1 + i][e]; }
#pragma unroll
  for (int i = 0; i < 3; ++i) { X.cfb[i] = FR[F_CFB + i][e]; X.c0[i] = FR[F_C0 + i][e]; X.c1[i] = FR[F_C1 + i][e]; }
#pragma unroll
  for (int i = 0; i < 12; ++i) X.tq[i] = FR[F_TQ + i][e];
#pragma unroll
  for (int k = 0; k < NLEG; ++k) { X.a[k] = ACT0[k][e]; X.a[NLEG + k] = ACT1[k][e]; }
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    X.la[i] = E[E_LA + i][e]; X.lla[i] = E[E_LLA + i][e];
    X.ldv[i] = E[E_LDV + i][e]; X.ref[i] = E[E_REF + i][e];
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) X.lrv[i] = E[E_LRV + i][e];
#pragma unroll
  for (int i = 0; i < 4; ++i) X.cmd[i] = E[E_CMD + i][e];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    X.at[i] = E[E_AT + i][e]; X.fh[i] = E[E_FH + i][e]; X.lfz[i] = E[E_LFZ + i][e];
    X.lc[i] = (uint8_t)__float_as_int(E[E_LC + i][e]);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    X.ef[i] = E[E_EF + i][e]; X.et[i] = E[E_ET + i][e];
    X.gt[i] = __float_as_int(E[E_GT + i][e]);
  }
#pragma unroll
  for (int k = 0; k < T1_NREW; ++k) X.esum[k] = E[E_ESUM + k][e];
  X.el = (int64_t)(((uint64_t)(uint32_t)__float_as_int(E[E_EL + 1][e]) << 32) |
                   (uint32_t)__float_as_int(E[E_EL][e]));
  X.pl = (int64_t)(((uint64_t)(uint32_t)__float_as_int(E[E_PL + 1][e]) << 32) |
                   (uint32_t)__float_as_int(E[E_PL][e]));
  X.gstart = E[E_GS][e];
  BaseQ bq;
  float* const ep_row = FA.ep_part + (size_t)blockIdx.x * EP_PART_ROW;  // this workgroup's partial extras sums
#ifdef T1_WHATIF_EPI_NO_POSTA  // timing-only what-if build: no post_a (no rewards, termination, callback)
  const bool do_reset = false;
  base_quantities_r(X.root, bq);
  if (PART == POST_A_REWARDS && lane < 25)  // the finaliser still sums every row (agent-scope stores, as wave_sum_store)
    __hip_atomic_store(ep_row + lane, 0.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  const bool do_reset = post_a_core<PART>(M, C, B, A, n0, X, bq, PART == POST_A_REWARDS ? ep_row : nullptr);
#endif
  T1_PROF_MARK(13);
  if constexpr (PART == POST_A_REWARDS) {
    epilogue_handoff<NE, INWG>(C, S, FA, lane, do_reset, active);
    __builtin_amdgcn_s_waitcnt(0);  // this wave's atomics (extras sums) complete
    __syncthreads();                // E2: the state wave's terrain-level sum complete
    epilogue_finalize_parts(C, B, A, FA, dyn_blocks, lane);
    T1_PROF_MARK(15);
    return;
  }
  if (active && do_reset) {  // reset_idx (post_b's first half): the new state; the observation waves take its inputs
    const uint32_t genv = (uint32_t)(C.env_offset + n);
    const uint32_t ctr = A.counter + 1u;
    const float pos_cmd[4] = {X.root[0], X.root[1], X.cmd[0], X.cmd[1]};
    reset_env(M, C, B, A, n, genv, ctr, true, /*zero_reward_state=*/false, /*obs_elsewhere=*/true, pos_cmd);
    ObsIn O;  // the new gait times (the reset's draws again), then the commands redrawn at the new episode's start
#pragma unroll
    for (int i = 0; i < 4; ++i) O.cmd[i] = X.cmd[i];
    reset_obs_inputs(M, C, rng_key(C.seed, genv, ctr), O, /*dof=*/false);
    if (resample_commands_r(C, A, O.el, O.gt, O.cmd, genv, ctr)) strow(B.commands + n * 4, O.cmd);
  }
  T1_PROF_MARK(14);
  // the terrain-level sum reads the levels reset_idx may just have changed
  wave_sum_store(ep_row + 25, (C.custom_origins && active) ? (float)B.terrain_levels[n] : 0.0f);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();  // E2
  T1_PROF_MARK(15);
}

// The fused step's observation writers (the helper waves after the epilogue barrier): PART = POST_OBS_PRIV the
// privileged frame, ref_dof_pos and the last_* rows, POST_OBS_ACTOR the actor frame (post_b's compute_observations,
// legged_robot.py:490-502, t1:368-481).  Each wave runs the part of post_a's callback + termination prefix it needs on
// the same LDS inputs (deterministic: the values the state wave computes) and takes a resetting env's new inputs from
// its reset draws (reset_obs_inputs), so neither waits for the state wave's stores; none of their rows is written by
// another wave.  No wave-wide operations: lanes without an env leave at once.
template <int PART, int NE>
__device__ __forceinline__ void fused_epilogue_obs(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                                   const t1env_step_args& A, int lane, const float (*E)[NE],
                                                   const float (*FR)[NE], const float (*ACT0)[NE],
                                                   const float (*ACT1)[NE]) {
  static_assert(PART == POST_OBS_PRIV || PART == POST_OBS_ACTOR, "an observation part");
  constexpr bool PRIV = PART == POST_OBS_PRIV;
  const int e = lane % NE;
  const int n = (int)blockIdx.x * NE + lane;
  if (lane >= NE || n >= C.num_envs) return;
  const uint32_t genv = (uint32_t)(C.env_offset + n);
  const uint32_t ctr = A.counter + 1u;
  const RngKey K = rng_key(C.seed, genv, ctr);
  float ld[24], lraw[8];
  if constexpr (!PRIV)  // issued first: the lagged samples are the actor wave's only memory reads
    load_lagged(B, A, n, __float_as_int(E[E_DL][e]), __float_as_int(E[E_IL][e]), ld, lraw);
  ObsIn O;
#pragma unroll
  for (int i = 0; i < 4; ++i) O.cmd[i] = E[E_CMD + i][e];
#pragma unroll
  for (int i = 0; i < 3; ++i) O.gt[i] = __float_as_int(E[E_GT + i][e]);
  const int64_t el = (int64_t)(((uint64_t)(uint32_t)__float_as_int(E[E_EL + 1][e]) << 32) |
                               (uint32_t)__float_as_int(E[E_EL][e])) + 1;
  const int64_t pl = (int64_t)(((uint64_t)(uint32_t)__float_as_int(E[E_PL + 1][e]) << 32) |
                               (uint32_t)__float_as_int(E[E_PL][e])) + 1;
  O.gstart = E[E_GS][e];
#pragma unroll
  for (int i = 0; i < 24; ++i) O.dof[i] = FR[F_DOF + i][e];
#pragma unroll
  for (int k = 0; k < NLEG; ++k) { O.act[k] = ACT0[k][e]; O.act[NLEG + k] = ACT1[k][e]; }
  ObsExtra Ex;
  if constexpr (PRIV) {  // post_a's prefix: base quantities of the step's root state, then the callback
    float root[13], ef[3], et[3], af[3];
#pragma unroll
    for (int i = 0; i < 13; ++i) root[i] = FR[F_ROOT + i][e];
#pragma unroll
    for (int i = 0; i < 3; ++i) { ef[i] = E[E_EF + i][e]; et[i] = E[E_ET + i][e]; }
#pragma unroll
    for (int i = 0; i < 12; ++i) O.la[i] = E[E_LA + i][e];
    base_quantities_r(root, O.bq);
    bool ext_store;
    post_callback(C, A, genv, ctr, K, el, O.gt, O.cmd, root, ef, et, af, ext_store);
#pragma unroll
    for (int i = 0; i < 6; ++i) O.rv[i] = root[7 + i];
    Ex.ef[0] = ef[0]; Ex.ef[1] = ef[1];
#pragma unroll
    for (int i = 0; i < 3; ++i) Ex.et[i] = et[i];
    Ex.cfz[0] = FR[F_C0 + 2][e]; Ex.cfz[1] = FR[F_C1 + 2][e];
    Ex.fric = E[E_FRIC][e];
    Ex.mass = E[E_MASS][e];
  } else {
    resample_commands_r(C, A, el, O.gt, O.cmd, genv, ctr);  // the only part of the callback the actor frame reads
  }
  // check_termination (legged_robot.py:509-517), as post_a_core
  const bool term = norm3(FR[F_CFB][e], FR[F_CFB + 1][e], FR[F_CFB + 2][e]) > 1.0f;
  const bool tout = (float)el > C.max_episode_length;
  const bool do_reset = term || tout;
  O.el = el;
  O.pl = is_stand(C, O.cmd) ? 0 : pl;  // post_a's _get_phase zeroing (the state wave stores it)
  if (do_reset) {
    reset_obs_inputs(M, C, K, O, /*dof=*/PRIV);
    resample_commands_r(C, A, O.el, O.gt, O.cmd, genv, ctr);
    if constexpr (!PRIV) {
#pragma unroll
      for (int i = 0; i < 24; ++i) ld[i] = 0.0f;
#pragma unroll
      for (int i = 0; i < 8; ++i) lraw[i] = 0.0f;
    }
  }
  const bool stand = is_stand(C, O.cmd);
  if (stand) O.pl = 0;
  ObsPhase P;
  obs_phase(M, C, O, stand, P);
  if constexpr (PRIV) {
    store_priv_frame(M, C, B, A, n, O, Ex, P);
    store_obs_last(B, n, O, P.ref);
  } else {
    float li[6];
    imu_sample(lraw, li);
    store_actor_frame(M, C, B, A, n, K, O, ld, li, P);
  }
}

// the Gym root-state row (pos, quat xyzw, COM linear velocity, angular velocity; world) of the internal base state
// (base-origin velocity): the report's root and the substep log's root rows
__device__ __forceinline__ void root_row(const DynModel& M, const BaseParams<float>& PB, const BaseState<float>& sb,
                                         const BaseFrame<float>& F, float body[13]) {
  const V3<float> c0 = base_com(M, PB, F.R0);
  const V3<float> vcom = v3<float>(sb.vo[0], sb.vo[1], sb.vo[2]) + cross(v3<float>(sb.w[0], sb.w[1], sb.w[2]), c0);
  const float r[13] = {sb.pos[0], sb.pos[1], sb.pos[2], sb.quat[0], sb.quat[1], sb.quat[2], sb.quat[3],
                       vcom.x, vcom.y, vcom.z, sb.w[0], sb.w[1], sb.w[2]};
#pragma unroll
  for (int i = 0; i < 13; ++i) body[i] = r[i];
}

// The leg wave's part of the report: its bodies' rigid states (and the root for leg 0), zeroed contact rows of its
// bodies without contact points; the helper evaluates the contact forces of the shank, foot (and the base box,
// leg 0).  FR (fused step): this step's outputs post-physics reads are also written to LDS rows (column e).
template <int NE>
__device__ __forceinline__ void leg_report_rigid(const DynModel& M, const t1env_buffers& B, const BaseParams<float>& PB,
                                                 const BaseState<float>& sb, const BaseFrame<float>& F,
                                                 const float q[NLEG], const float qd[NLEG], int n, int leg, bool active,
                                                 int e, float (*FR)[NE]) {
  float* rig = B.rigid_state + (size_t)n * 169;
  float* cf = B.contact_forces + (size_t)n * 39;
  if (leg == 0) {
    float body[13];
    root_row(M, PB, sb, F, body);
    if (active)
#pragma unroll
      for (int i = 0; i < 13; ++i) { B.root_states[(size_t)n * 13 + i] = body[i]; rig[i] = body[i]; }
    if (FR)
#pragma unroll
      for (int i = 0; i < 13; ++i) FR[F_ROOT + i][e] = body[i];
  }
  BodyState<float> Bk[NLEG];
  leg_fk(M, leg, F.R0, q, Bk);
  float V[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) V[i] = F.V0[i];
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    const int b = 1 + 6 * leg + k;
    float S6[6];
    motion_subspace(M, b, Bk[k], S6);
#pragma unroll
    for (int i = 0; i < 6; ++i) V[i] += S6[i] * qd[k];
    const V3<float> c = Bk[k].p + mul(Bk[k].Rot, v3<float>(M.com[b][0], M.com[b][1], M.com[b][2]));
    const V3<float> om{V[0], V[1], V[2]};
    const V3<float> vc = v3<float>(V[3], V[4], V[5]) + cross(om, c);
    float qb[4];
    mat_to_quat(Bk[k].Rot, qb);
    const float out[13] = {Bk[k].p.x + F.abs.x, Bk[k].p.y + F.abs.y, Bk[k].p.z + F.abs.z, qb[0], qb[1], qb[2], qb[3],
                           vc.x, vc.y, vc.z, om.x, om.y, om.z};
    if (FR) {
      if (k == K_FOOT)
#pragma unroll
        for (int i = 0; i < 13; ++i) FR[(leg == 0 ? F_F0 : F_F1) + i][e] = out[i];
      if (k == K_SHANK) { FR[(leg == 0 ? F_K0 : F_K1)][e] = out[0]; FR[(leg == 0 ? F_K0 : F_K1) + 1][e] = out[1]; }
    }
    if (!active) continue;
#pragma unroll
    for (int i = 0; i < 13; ++i) rig[b * 13 + i] = out[i];
    if (k != K_SHANK && k != K_FOOT) { cf[b * 3 + 0] = 0.0f; cf[b * 3 + 1] = 0.0f; cf[b * 3 + 2] = 0.0f; }
  }
}

// the contact-force report from the poses the helper computes itself from the end-of-step state: terrain forces plus
// the self-contact forces fself of the shank / foot
// (vt: the restitution set points of the shank, foot and base half; the base box's whole report uses the larger of
// its two halves')
template <int NE>
__device__ __forceinline__ void helper_report_contacts_at(const DynModel& M, const Terrain& T, const t1env_buffers& B,
                                                          const BaseFrame<float>& F, const BodyKin<float> (&Kc)[2],
                                                          const V3<float> (&fself)[2], int n, int leg, float mu,
                                                          const float (&vt)[3], float vt_base, int e, bool active,
                                                          float (*FR)[NE]) {
  float* cf = B.contact_forces + (size_t)n * 39;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int b = 1 + 6 * leg + (s == 0 ? K_SHANK : K_FOOT);
    const V3<float> f = body_contact_force(M, T, b, Kc[s].Rb, Kc[s].p, F.abs, Kc[s].V, mu, vt[s]) + fself[s];
    if (active) { cf[b * 3 + 0] = f.x; cf[b * 3 + 1] = f.y; cf[b * 3 + 2] = f.z; }
    if (FR && s == 1) {
      const int r = leg == 0 ? F_C0 : F_C1;
      FR[r][e] = f.x; FR[r + 1][e] = f.y; FR[r + 2][e] = f.z;
    }
  }
  if (leg == 0) {
    const V3<float> f = body_contact_force(M, T, 0, F.R0, v3<float>(0, 0, 0), F.abs, F.V0, mu, vt_base);
    if (active) { cf[0] = f.x; cf[1] = f.y; cf[2] = f.z; }
    if (FR) { FR[F_CFB][e] = f.x; FR[F_CFB + 1][e] = f.y; FR[F_CFB + 2][e] = f.z; }
  }
}

}  // namespace t1
