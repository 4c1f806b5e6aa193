// t1env_dynamics.hip -- the env step's main launch: the decimation loop with the articulated-body solver
// (legged_robot.py:399-434 + Isaac Gym simulate()), the history shift, and in the fused step post-physics.
// Its own translation unit because it is compiled at -O1 (build.py; -O2/-O3 measure the same since round 2 and are
// correct too (tests/test_gpu_opt_levels.py runs the -O3 build through the fp64 dynamics check and the product replay).
#include <hip/hip_runtime.h>

// -DT1_PHASE_PROF (tools/prof_dynamics_phases.py): lane 0 of every dynamics wave accumulates shader-clock
// deltas between T1_PROF_MARK points into per-phase buckets; never part of the product build.
#ifdef T1_PHASE_PROF
constexpr int T1_NPROF = 24, T1_PROF_WAVES = 4;
__device__ unsigned long long g_t1_prof[T1_PROF_WAVES][T1_NPROF];
__shared__ unsigned long long t1_prof_acc[T1_PROF_WAVES][T1_NPROF + 1];  // [wave][bucket], last = previous mark
// a stamp is one asm statement (s_memtime + its lgkmcnt wait) fenced by scheduling barriers, so the compiler
// cannot move work across it (cdna_hip_programming.md, In-kernel stamps); profiling build only
__device__ __forceinline__ unsigned long long t1_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) :: "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ void t1_prof_mark(int i) {
  const int w = threadIdx.x / 64;
  const unsigned long long now = t1_stamp();
  if ((threadIdx.x & 63) == 0) {
    t1_prof_acc[w][i] += now - t1_prof_acc[w][T1_NPROF];
    t1_prof_acc[w][T1_NPROF] = now;
  }
}
__device__ __forceinline__ void t1_prof_begin() {
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    for (int i = 0; i < T1_NPROF; ++i) t1_prof_acc[w][i] = 0;
    t1_prof_acc[w][T1_NPROF] = t1_stamp();
  }
}
__device__ __forceinline__ void t1_prof_end() {
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0)
    for (int i = 0; i < T1_NPROF; ++i) atomicAdd(&g_t1_prof[w][i], t1_prof_acc[w][i]);
}
#define T1_PROF_MARK(i) t1_prof_mark(i)
#define T1_PROF_BEGIN() t1_prof_begin()
#define T1_PROF_END() t1_prof_end()
#else
#define T1_PROF_BEGIN() ((void)0)
#define T1_PROF_END() ((void)0)
#endif

#include "t1env_device.h"
#include "t1env_internal.h"
#include "t1env_postphys.h"

using namespace t1;

// ---------------------------------------------------------------------------------------------------
// The launch: ceil(N/64) dynamics workgroups of 64 envs, then history-shift workgroups (blockIdx >= dyn_blocks,
// t1env_device.h).  The dynamics fill at most half the CUs at 8192 envs, so the HBM-bound shift streams on the rest
// of the chip inside the same launch -- no second stream, no cross-stream events on the step path.
//
//   k_dyn4 (4 waves / 64 envs): waves 0/1 are the leg waves -- wave 0 runs every env's left leg, wave 1 the right
//     leg (the leg index is wave-uniform, so model reads are scalar loads) -- running the articulated-body passes
//     without contact (leg_forward_nc / leg_backward_nc); waves 2/3 are their contact helpers: from the substep
//     state the leg waves publish they compute the shank / foot contact terms (terrain and self-collision) while
//     the leg wave runs its passes, then the base-box contact terms while the leg wave folds the contact terms in
//     (leg_apply_contacts) and eliminates its leg into a 27-float base-block contribution.  The contributions meet
//     in LDS and both leg waves solve the 6x6 base system redundantly, so the base state stays bit-identical in
//     both.  Three barriers per substep; all four SIMDs of the CU work on the same 64 envs.  (Round 1's 2-wave
//     k_dynamics, with contacts inside the leg waves, ran 34 % slower and was retired in round 3.)
//
// FUSED (t1env_step on every step that needs no host decision between the phases): the whole env step is
// one launch.  After its dynamics, wave 0 of each dynamics workgroup runs post-physics for its 64 envs
// (t1env_postphys.h post_a_env + post_b_env: rewards, termination, reset_idx, observations, newest history
// frame), and the last dynamics workgroup to finish finalises the extras.  Two things had to change for that:
//   * reset_idx's "resample commands of every env if any env reset" has no global dependency here: for an env
//     that did not reset, the second resample repeats post_a's (same episode step, same keyed draws), so each
//     env needs only its own reset flag;
//   * zeroing the history rows of reset envs must follow the shift of those rows, which other workgroups do
//     concurrently.  The shift is cut into units of SHIFT_UNIT rows, and each unit has a handoff word
//     (epoch-tagged): the shift workgroup sets bit 0 once the unit is shifted, the dynamics workgroup sets
//     bit 1 together with the unit's 8-bit reset mask.  Whoever sets the second bit zeroes the unit's reset
//     rows.  Nobody waits for anybody, so no dispatch order or residency is assumed.  The shift writes these
//     rows with agent-coherent sc1 stores (t1env_device.h store4), so once they have completed (s_waitcnt) no
//     dirty copy is left in any L2 and the zeros, written later by either party, land last --
//     placement-independent, and without an L2 write-back fence (buffer_wbl2 per unit cost the concurrently
//     running dynamics ~8 %).
// ---------------------------------------------------------------------------------------------------
// The contact helper waves compute the shank / foot poses themselves from the substep state the leg waves publish
// after integrating (leg_contact_kinematics), so their contact terms start in parallel with the leg's forward pass
// (+2.5 % env-steps/s at 8192 envs, r02ab); with self-collision on, each helper also computes the other leg's
// contact-body kinematics from that leg's published state.

constexpr int DYN_ENVS = 64;
constexpr int D4_BLOCK = 4 * DYN_ENVS;
constexpr int XCH = 27;  // Sym6 (21) + rhs (6)
constexpr int SHIFT_UNIT = 8;  // rows per shift/zeroing unit (a multiple of 4: unit boundaries are 16-B aligned)
// chunks per lane in flight in the in-launch shift: the shift workgroups run one wave per SIMD on the CUs the dynamics
// leave idle, so they need deep per-lane batches (r02u: 8 -> 16 took the shift alone from 114 to 106 us at 8192 envs)
#ifndef T1_FUSED_SHIFT_UNROLL
#define T1_FUSED_SHIFT_UNROLL 16
#endif
static_assert(DYN_ENVS % SHIFT_UNIT == 0, "a dynamics workgroup owns whole shift units");

// Handoff word of a shift unit: [epoch tag : 22][reset mask : 8][dynamics done : 1][shift done : 1].  Set
// `bits` (state bits and, from the dynamics side, the mask) for this epoch; returns the new word.  The word
// is complete when both state bits are set; the party whose update completes it zeroes the unit's reset rows.
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

// A history-shift workgroup (j of nsw) of BS threads; `words` is LDS scratch of >= BS uint32.
template <bool FUSED, int BS>
__device__ __forceinline__ void shift_workgroup(const ShiftArgs& S, const FusedArgs& FA, int N, int j, int nsw,
                                                uint32_t* words, int delay) {
  if (delay > 0) {  // let the dynamics workgroups' prologue loads go first (wave-uniform; the 100 MHz real-time clock)
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (uint64_t)delay) __builtin_amdgcn_s_sleep(32);
  }
  if constexpr (!FUSED) {
    shift_history(S, (int64_t)j * BS + threadIdx.x, (int64_t)nsw * BS);
  } else {
    // a contiguous run of units per workgroup, shifted as one flat row range: each lane keeps
    // T1_FUSED_SHIFT_UNROLL x 32 B of loads in flight, enough for HBM rate from one workgroup per CU on the CUs
    // the dynamics leave idle (a per-unit loop re-starts its unrolled batches every 8 rows and wastes their tails)
    const int units = (N + SHIFT_UNIT - 1) / SHIFT_UNIT;
    const int per = (units + nsw - 1) / nsw;
    const int u0 = j * per < units ? j * per : units, u1 = u0 + per < units ? u0 + per : units;
    const int mine = u1 - u0;  // units of this workgroup
#ifndef T1_WHATIF_NO_SHIFT  // timing-only what-if build: the history is not shifted (handoff and zeroing kept)
    if (mine > 0) {
      const int64_t r0 = (int64_t)u0 * SHIFT_UNIT, r1 = (int64_t)u1 * SHIFT_UNIT < N ? (int64_t)u1 * SHIFT_UNIT : N;
      shift_rows_range_sc1<T1_FUSED_SHIFT_UNROLL>(S, r0, r1, threadIdx.x, BS);
    }
#endif
    // every lane's sc1 stores complete (visible at agent scope) before any handoff
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    for (int k0 = 0; k0 < mine; k0 += BS) {
      const int k = k0 + (int)threadIdx.x;
      if (k < mine) words[threadIdx.x] = unit_handoff(FA.unit_state + u0 + k, FA.epoch, HANDOFF_SHIFT);
      __syncthreads();
      const int cnt = mine - k0 < BS ? mine - k0 : BS;
      for (int i = 0; i < cnt; ++i)
        if (handoff_complete(words[i])) zero_unit_resets(S, u0 + k0 + i, words[i], threadIdx.x, BS);
      __syncthreads();
    }
  }
}

// after post-physics: the terrain-level sum, the reset-row handoff and the extras finalisation
__device__ __forceinline__ void epilogue_handoff(const t1env_config& C, const ShiftArgs& S, const FusedArgs& FA, int lane,
                                                 bool do_reset, bool active) {
  const int N = C.num_envs;
  const unsigned long long m = __ballot(do_reset && active);
  if (FA.shift_done) {  // the shift completed before this launch (stream order): zero the reset rows now
    unsigned long long todo = m;
    while (todo) {
      const int l = __ffsll(todo) - 1;
      todo &= todo - 1;
      zero_history_row(S, (int64_t)blockIdx.x * DYN_ENVS + l, lane, DYN_ENVS);
    }
    return;
  }
  // ---- reset rows: hand off each of the workgroup's shift units with its 8-bit reset mask
  const int units = (N + SHIFT_UNIT - 1) / SHIFT_UNIT;
  const int u = blockIdx.x * (DYN_ENVS / SHIFT_UNIT) + lane;
  uint32_t w = 0;
  if (lane < DYN_ENVS / SHIFT_UNIT && u < units)
    w = unit_handoff(FA.unit_state + u, FA.epoch, HANDOFF_DYN | ((uint32_t)(m >> (lane * SHIFT_UNIT)) & 0xffu) << 2);
  uint64_t todo = __ballot(handoff_complete(w));
  while (todo) {
    const int l = __ffsll((unsigned long long)todo) - 1;
    todo &= todo - 1;
    zero_unit_resets(S, blockIdx.x * (DYN_ENVS / SHIFT_UNIT) + l, __shfl(w, l, 64), lane, DYN_ENVS);
  }
}
// k_dyn4's finaliser: every dynamics workgroup stored one row of partial sums (FusedArgs::ep_part, agent-scope
// stores completed before its counter increment); the last one sums the rows in a fixed order after an acquire
// fence (no same-address atomics: 25 per workgroup into one row cost 3.6% of the step, r02ar).  Lane l reads the
// float4 l % 8 of rows l / 8, l / 8 + 8, ...; the 8 lanes of a float4 are then summed across the wave.
__device__ __forceinline__ void epilogue_finalize_parts(const t1env_config& C, const t1env_buffers& B,
                                                        const t1env_step_args& A, const FusedArgs& FA, int dyn_blocks,
                                                        int lane) {
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
  constexpr int BATCH = 8;  // loads in flight per lane
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

// per-leg setup shared by both kernels: clipped actions into the step's action slot, sensor-lag capture
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


// ---------------------------------------------------------------------------------------------------
// k_dyn4: 4 waves per 64 envs (see the top of the file).  Per substep, leg wave | contact helper wave:
//   forward pass, publishing the base frame and the shank / foot poses       |
//   S1 -------------------------------------------------------------------------------------------------
//   PD torques, backward pass without contact                                 | shank + foot contact terms
//   S2 -------------------------------------------------------------------------------------------------
//   contact terms folded in (leg_apply_contacts), elimination, base block     | base-box contact terms
//   S3 -------------------------------------------------------------------------------------------------
//   base solve (4 contributions), back-substitution, integration             | (waits for the next poses)
// The leg wave stages its PD constants and the action ring in LDS once per step, and captures the lagged
// sensor samples into LDS (written to the rings once after the loop): in the loop it touches global memory
// only for the terrain.
// LDS per workgroup (floats, [value][env]: every access is a conflict-free row):
//   pose[leg] (POSE_N): base frame R0 (9) abs (3) V0 (6), then shank / foot R (9) p (3) V (6)
//   ct[leg]   (CT_N):   shank C (21) c (6), foot C (21) c (6)
//   xch[4]:             base-block contributions: legs 0, 1 (leg waves), base-box contacts 0, 1 (helpers)
// Each region is written and read in disjoint barrier intervals (pose: written before S1, read S1..S3;
// ct: written S1..S2, read S2..S3; xch: written S2..S3, read after S3, rewritten after the next S2).
// ---------------------------------------------------------------------------------------------------
constexpr int POSE_F = 18, POSE_B = 18, POSE_N = POSE_F + 2 * POSE_B;
constexpr int CT_N = 2 * XCH;
constexpr int CAP_N = 2 * NLEG + 8 + NLEG;  // dof capture (q, qd of the leg), IMU capture (raw, leg 0), actions
constexpr int CAP_ACT = 2 * NLEG + 8;
// fused epilogue staging (post-physics inputs of the workgroup's 64 envs in LDS):
//   epi (EPI_N rows): the state post-physics reads that the step has not changed, prefetched with coalesced
//        row loads by the helper waves while the leg waves run the last substep
//   fresh (FR_N rows, in the ct region once the loop is over): this step's dynamics outputs, from registers
enum : int {
  E_LA = 0, E_LLA = 12, E_LRV = 24, E_LDV = 30, E_REF = 42, E_CMD = 54, E_AT = 58, E_FH = 60, E_LFZ = 62,
  E_EF = 64, E_ET = 67, E_GT = 70, E_EL = 73, E_PL = 75, E_GS = 77, E_LC = 78, E_FRIC = 80, E_MASS = 81,
  E_DL = 82, E_IL = 83, E_ESUM = 84, EPI_N = 84 + T1_NREW
};
enum : int {
  F_ROOT = 0, F_DOF = 13, F_TQ = 37, F_F0 = 49, F_F1 = 62, F_K0 = 75, F_K1 = 77, F_CFB = 79, F_C0 = 82, F_C1 = 85,
  FR_N = 88
};
constexpr int K_SHANK = 3, K_FOOT = 5;
static_assert(T1_LEG_CONTACT_MASK == ((1 << K_SHANK) | (1 << K_FOOT)), "k_dyn4 assumes shank + foot contact bodies");

struct Dyn4Lds {
  float pose[2][POSE_N][DYN_ENVS];
  float ct[2][CT_N][DYN_ENVS];
  float xch[4][XCH][DYN_ENVS];
  PdStage<DYN_ENVS> pd[2];
  float cap[2][CAP_N][DYN_ENVS];
  float epi[EPI_N][DYN_ENVS];
  float vib[2][DYN_ENVS];  // the base-box halves' end-of-step restitution episodes (helpers, for the report)
  int xflag[2];            // helper h's self-collision bodies of the current (sub)step published (helper_signal)
  float vis[2][DYN_ENVS];  // the shanks' end-of-step restitution episodes (leg waves, for the helpers' report)
};
static_assert(FR_N <= 2 * CT_N, "the fresh outputs fit the contact-term region");

__device__ __forceinline__ void lds_put_m3(float (*dst)[DYN_ENVS], int lane, const M3<float>& R) {
#pragma unroll
  for (int i = 0; i < 9; ++i) dst[i][lane] = R.m[i];
}
__device__ __forceinline__ M3<float> lds_get_m3(const float (*src)[DYN_ENVS], int lane) {
  M3<float> R;
#pragma unroll
  for (int i = 0; i < 9; ++i) R.m[i] = src[i][lane];
  return R;
}
__device__ __forceinline__ void lds_put_sym(float (*dst)[DYN_ENVS], int lane, const Sym6<float>& A, const float g[6]) {
#pragma unroll
  for (int i = 0; i < 21; ++i) dst[i][lane] = A.a[i];
#pragma unroll
  for (int i = 0; i < 6; ++i) dst[21 + i][lane] = g[i];
}
__device__ __forceinline__ void lds_get_sym(const float (*src)[DYN_ENVS], int lane, Sym6<float>& A, float g[6]) {
#pragma unroll
  for (int i = 0; i < 21; ++i) A.a[i] = src[i][lane];
#pragma unroll
  for (int i = 0; i < 6; ++i) g[i] = src[21 + i][lane];
}

constexpr int32_t T1_NO_BOUND = 0x7fffffff;  // bound_height() = +inf: the body is always evaluated


// a contact body's terrain terms (from its pose held in registers) added to its self-contact terms (Cc, cc), then
// published to LDS for the leg wave's fold-in
__device__ __forceinline__ void body_terms_at(const DynModel& M, const Terrain& T, const BodyKin<float>& K, int lane,
                                              int b, V3<float> abs, float mu, float e, float& vimp, float dt,
                                              Sym6<float>& Cc, float (&cc)[6], float (*dst)[DYN_ENVS], int32_t bound) {
  body_contact_fixed<T1_POINTS_PER_BODY>(M, T, K.p.z + abs.z - M.contact_radius[b], bound, M.contact_start[b], K.Rb,
                                         K.p, abs, K.V, mu, e, vimp, dt, Cc, cc);
  lds_put_sym(dst, lane, Cc, cc);
}
// The substep state each leg wave publishes for the helpers: base pos, quat, omega, v_O, and the leg's q, qd -- rows
// of the leg's pose region, written after integration, read by the helpers between S1 and S2 (and after R1).
enum : int { ST_POS = 0, ST_QUAT = 3, ST_W = 7, ST_VO = 10, ST_Q = 13, ST_QD = 19, ST_N = 25 };
static_assert(ST_N <= POSE_N, "the substep state fits the pose rows");
#ifdef T1_WHATIF_NO_SELF  // timing-only what-if build: the self-collision code compiled out of k_dyn4
#define T1_SELF_CODE 0
#else
#define T1_SELF_CODE 1
#endif
// a helper's kinematics of one published state: the base frame and the contact bodies of leg `leg` (own state P)
__device__ __forceinline__ void helper_kinematics(const DynModel& M, const float (*P)[DYN_ENVS], int lane, int leg,
                                                  BaseFrame<float>& F, BodyKin<float> (&Ko)[2]) {
  BaseState<float> sb;
  float qh[NLEG], qdh[NLEG];
#pragma unroll
  for (int i = 0; i < 3; ++i) { sb.pos[i] = P[ST_POS + i][lane]; sb.w[i] = P[ST_W + i][lane]; sb.vo[i] = P[ST_VO + i][lane]; }
#pragma unroll
  for (int i = 0; i < 4; ++i) sb.quat[i] = P[ST_QUAT + i][lane];
#pragma unroll
  for (int k = 0; k < NLEG; ++k) { qh[k] = P[ST_Q + k][lane]; qdh[k] = P[ST_QD + k][lane]; }
  base_frame(sb, F);
  leg_body_kinematics(M, F, qh, qdh, leg, Ko);
}
__device__ __forceinline__ void publish_state(float (*P)[DYN_ENVS], int lane, const BaseState<float>& sb,
                                              const float q[NLEG], const float qd[NLEG]) {
#pragma unroll
  for (int i = 0; i < 3; ++i) { P[ST_POS + i][lane] = sb.pos[i]; P[ST_W + i][lane] = sb.w[i]; P[ST_VO + i][lane] = sb.vo[i]; }
#pragma unroll
  for (int i = 0; i < 4; ++i) P[ST_QUAT + i][lane] = sb.quat[i];
#pragma unroll
  for (int k = 0; k < NLEG; ++k) { P[ST_Q + k][lane] = q[k]; P[ST_QD + k][lane] = qd[k]; }
}

// ---- fused-epilogue staging by the two helper waves (STAGE_NT threads).  Rows [nb, nb + nv) of the workgroup;
// a row-major source is read as one contiguous run (consecutive threads, consecutive words: coalesced) and
// transposed into [value][env].  All loads of a thread are issued before the first LDS write (stage_ld for
// every source, then stage_st), so the staging costs one memory latency.
constexpr int STAGE_NT = 2 * DYN_ENVS;
template <int L> constexpr int stage_n() { return (DYN_ENVS * L + STAGE_NT - 1) / STAGE_NT; }
template <typename T> __device__ __forceinline__ float stage_bits(T v) {
  if constexpr (sizeof(T) == 4) return __builtin_bit_cast(float, v);
  else return __int_as_float((int)v);
}
template <int L, typename T>
__device__ __forceinline__ void stage_ld(const T* __restrict__ src, int nb, int nv, int t, float (&v)[stage_n<L>()]) {
  const T* base = src + (size_t)nb * L;
#pragma unroll
  for (int i = 0; i < stage_n<L>(); ++i) {
    const int e = t + STAGE_NT * i;
    v[i] = e < nv * L ? stage_bits(base[e]) : 0.0f;
  }
}
template <int L>
__device__ __forceinline__ void stage_st(float (*dst)[DYN_ENVS], int nv, int t, const float (&v)[stage_n<L>()]) {
#pragma unroll
  for (int i = 0; i < stage_n<L>(); ++i) {
    const int e = t + STAGE_NT * i;
    if (e < nv * L) dst[e % L][e / L] = v[i];
  }
}
// the staged values of one helper thread between its loads and its LDS writes (epi_stage_load / epi_stage_store)
constexpr int EPI_NES = (T1_NREW * DYN_ENVS + STAGE_NT - 1) / STAGE_NT;
struct EpiStage {
  float la[stage_n<12>()], lla[stage_n<12>()], lrv[stage_n<6>()], ldv[stage_n<12>()], ref[stage_n<12>()];
  float cmd[stage_n<4>()], at[stage_n<2>()], fh[stage_n<2>()], lfz[stage_n<2>()], ef[stage_n<3>()];
  float et[stage_n<3>()], gt[stage_n<3>()], el[stage_n<2>()], pl[stage_n<2>()], gs[stage_n<1>()], lc[stage_n<2>()];
  float fr[stage_n<1>()], ms[stage_n<1>()], dl[stage_n<1>()], il[stage_n<1>()];
  float es[EPI_NES];
};
__device__ __forceinline__ void epi_stage_load(const t1env_buffers& B, int N, int nb, int t, EpiStage& V) {
  const int nv = N - nb < DYN_ENVS ? N - nb : DYN_ENVS;
  stage_ld<12>(B.last_actions, nb, nv, t, V.la);
  stage_ld<12>(B.last_last_actions, nb, nv, t, V.lla);
  stage_ld<6>(B.last_root_vel, nb, nv, t, V.lrv);
  stage_ld<12>(B.last_dof_vel, nb, nv, t, V.ldv);
  stage_ld<12>(B.ref_dof_pos, nb, nv, t, V.ref);
  stage_ld<4>(B.commands, nb, nv, t, V.cmd);
  stage_ld<2>(B.feet_air_time, nb, nv, t, V.at);
  stage_ld<2>(B.feet_height, nb, nv, t, V.fh);
  stage_ld<2>(B.last_feet_z, nb, nv, t, V.lfz);
  stage_ld<3>(B.ext_forces, nb, nv, t, V.ef);
  stage_ld<3>(B.ext_torques, nb, nv, t, V.et);
  stage_ld<3>(B.gait_time, nb, nv, t, V.gt);
  stage_ld<2>(reinterpret_cast<const uint32_t*>(B.episode_length_buf), nb, nv, t, V.el);
  stage_ld<2>(reinterpret_cast<const uint32_t*>(B.phase_length_buf), nb, nv, t, V.pl);
  stage_ld<1>(B.gait_start, nb, nv, t, V.gs);
  stage_ld<2>(B.last_contacts, nb, nv, t, V.lc);
  stage_ld<1>(B.friction, nb, nv, t, V.fr);
  stage_ld<1>(B.body_mass, nb, nv, t, V.ms);
  stage_ld<1>(B.dof_lag_timestep, nb, nv, t, V.dl);
  stage_ld<1>(B.imu_lag_timestep, nb, nv, t, V.il);
#pragma unroll
  for (int i = 0; i < EPI_NES; ++i) {  // episode_sums is [reward][env]: already row-contiguous
    const int e = t + STAGE_NT * i;
    V.es[i] = e < T1_NREW * nv ? B.episode_sums[(size_t)(e / nv) * N + nb + e % nv] : 0.0f;
  }
}
__device__ __forceinline__ void epi_stage_store(int N, int nb, int t, const EpiStage& V, float (*E)[DYN_ENVS]) {
  const int nv = N - nb < DYN_ENVS ? N - nb : DYN_ENVS;
  stage_st<12>(E + E_LA, nv, t, V.la);
  stage_st<12>(E + E_LLA, nv, t, V.lla);
  stage_st<6>(E + E_LRV, nv, t, V.lrv);
  stage_st<12>(E + E_LDV, nv, t, V.ldv);
  stage_st<12>(E + E_REF, nv, t, V.ref);
  stage_st<4>(E + E_CMD, nv, t, V.cmd);
  stage_st<2>(E + E_AT, nv, t, V.at);
  stage_st<2>(E + E_FH, nv, t, V.fh);
  stage_st<2>(E + E_LFZ, nv, t, V.lfz);
  stage_st<3>(E + E_EF, nv, t, V.ef);
  stage_st<3>(E + E_ET, nv, t, V.et);
  stage_st<3>(E + E_GT, nv, t, V.gt);
  stage_st<2>(E + E_EL, nv, t, V.el);
  stage_st<2>(E + E_PL, nv, t, V.pl);
  stage_st<1>(E + E_GS, nv, t, V.gs);
  stage_st<2>(E + E_LC, nv, t, V.lc);
  stage_st<1>(E + E_FRIC, nv, t, V.fr);
  stage_st<1>(E + E_MASS, nv, t, V.ms);
  stage_st<1>(E + E_DL, nv, t, V.dl);
  stage_st<1>(E + E_IL, nv, t, V.il);
#pragma unroll
  for (int i = 0; i < EPI_NES; ++i) {
    const int e = t + STAGE_NT * i;
    if (e < T1_NREW * nv) E[E_ESUM + e / nv][e % nv] = V.es[i];
  }
}
__device__ __forceinline__ void stage_epilogue_inputs(const t1env_buffers& B, int N, int nb, int t,
                                                      float (*E)[DYN_ENVS]) {
  EpiStage V;
  epi_stage_load(B, N, nb, t, V);
  epi_stage_store(N, nb, t, V, E);
}

// The fused step's post-physics for one k_dyn4 workgroup, run by the two leg waves: every input from LDS (fresh
// outputs, staged state, the actions in the capture rows).  Both waves run post_a's callback + termination
// prefix; wave 0 (PART = POST_A_REWARDS) then the 24 rewards, their stores and extras sums and the reset-row
// handoff, wave 1 (POST_A_STATE) the state stores, post_b (reset_idx, observations, newest history frame) and
// the terrain-level sum.  After one barrier wave 0 signals completion (the extras finaliser).
template <int PART>
__device__ __forceinline__ void fused_epilogue_staged(const DynModel& M, const t1env_config& C, const t1env_buffers& B,
                                                      const t1env_step_args& A, const ShiftArgs& S,
                                                      const FusedArgs& FA, int dyn_blocks, int lane,
                                                      const float (*E)[DYN_ENVS], const float (*FR)[DYN_ENVS],
                                                      const float (*cap0)[DYN_ENVS], const float (*cap1)[DYN_ENVS]) {
  const int N = C.num_envs;
  const int n0 = blockIdx.x * DYN_ENVS + lane;
  const bool active = n0 < N;
  const int n = active ? n0 : N - 1;
  PostAIn X;
#pragma unroll
  for (int i = 0; i < 13; ++i) X.root[i] = FR[F_ROOT + i][lane];
#pragma unroll
  for (int i = 0; i < 24; ++i) X.dof[i] = FR[F_DOF + i][lane];
#pragma unroll
  for (int i = 0; i < 13; ++i) { X.f0[i] = FR[F_F0 + i][lane]; X.f1[i] = FR[F_F1 + i][lane]; }
#pragma unroll
  for (int i = 0; i < 2; ++i) { X.k0[i] = FR[F_K0 + i][lane]; X.k1[i] = FR[F_K1 + i][lane]; }
#pragma unroll
  for (int i = 0; i < 3; ++i) { X.cfb[i] = FR[F_CFB + i][lane]; X.c0[i] = FR[F_C0 + i][lane]; X.c1[i] = FR[F_C1 + i][lane]; }
#pragma unroll
  for (int i = 0; i < 12; ++i) X.tq[i] = FR[F_TQ + i][lane];
#pragma unroll
  for (int k = 0; k < NLEG; ++k) { X.a[k] = cap0[CAP_ACT + k][lane]; X.a[NLEG + k] = cap1[CAP_ACT + k][lane]; }
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    X.la[i] = E[E_LA + i][lane]; X.lla[i] = E[E_LLA + i][lane];
    X.ldv[i] = E[E_LDV + i][lane]; X.ref[i] = E[E_REF + i][lane];
  }
#pragma unroll
  for (int i = 0; i < 6; ++i) X.lrv[i] = E[E_LRV + i][lane];
#pragma unroll
  for (int i = 0; i < 4; ++i) X.cmd[i] = E[E_CMD + i][lane];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    X.at[i] = E[E_AT + i][lane]; X.fh[i] = E[E_FH + i][lane]; X.lfz[i] = E[E_LFZ + i][lane];
    X.lc[i] = (uint8_t)__float_as_int(E[E_LC + i][lane]);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    X.ef[i] = E[E_EF + i][lane]; X.et[i] = E[E_ET + i][lane];
    X.gt[i] = __float_as_int(E[E_GT + i][lane]);
  }
#pragma unroll
  for (int k = 0; k < T1_NREW; ++k) X.esum[k] = E[E_ESUM + k][lane];
  X.el = (int64_t)(((uint64_t)(uint32_t)__float_as_int(E[E_EL + 1][lane]) << 32) |
                   (uint32_t)__float_as_int(E[E_EL][lane]));
  X.pl = (int64_t)(((uint64_t)(uint32_t)__float_as_int(E[E_PL + 1][lane]) << 32) |
                   (uint32_t)__float_as_int(E[E_PL][lane]));
  X.gstart = E[E_GS][lane];
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
    epilogue_handoff(C, S, FA, lane, do_reset, active);
    __builtin_amdgcn_s_waitcnt(0);  // this wave's atomics (extras sums) complete
    __syncthreads();                // E2: wave 1's terrain-level sum complete
    epilogue_finalize_parts(C, B, A, FA, dyn_blocks, lane);
    T1_PROF_MARK(15);
    return;
  }
  if (active) {
    ObsIn O;
#pragma unroll
    for (int i = 0; i < 4; ++i) O.cmd[i] = X.cmd[i];
#pragma unroll
    for (int i = 0; i < 24; ++i) O.dof[i] = X.dof[i];
#pragma unroll
    for (int i = 0; i < 12; ++i) { O.act[i] = X.a[i]; O.la[i] = X.la[i]; }
#pragma unroll
    for (int i = 0; i < 6; ++i) O.rv[i] = X.root[7 + i];
    O.bq = bq;
#pragma unroll
    for (int i = 0; i < 3; ++i) O.gt[i] = X.gt[i];
    O.el = X.el;
    O.pl = X.pl;
    O.gstart = X.gstart;
    O.dl = __float_as_int(E[E_DL][lane]);
    O.il = __float_as_int(E[E_IL][lane]);
    ObsExtra Ex;
    Ex.ef[0] = X.ef[0]; Ex.ef[1] = X.ef[1];
#pragma unroll
    for (int i = 0; i < 3; ++i) Ex.et[i] = X.et[i];
    Ex.cfz[0] = X.c0[2]; Ex.cfz[1] = X.c1[2];
    Ex.fric = E[E_FRIC][lane];
    Ex.mass = E[E_MASS][lane];
#ifndef T1_WHATIF_EPI_NO_POSTB  // timing-only what-if build: no reset / observations
    post_b_core(M, C, B, A, n, do_reset, do_reset, O, Ex, /*zero_reward_state=*/false);
#endif
  }
  T1_PROF_MARK(14);
  // the terrain-level sum reads the levels reset_idx may just have changed
  wave_sum_store(ep_row + 25, (C.custom_origins && active) ? (float)B.terrain_levels[n] : 0.0f);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();  // E2
  T1_PROF_MARK(15);
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

// k_dyn4's report, split between the waves: the leg wave writes its bodies' rigid states (and the root for
// leg 0), zeros the contact rows of its bodies without contact points, and publishes the end-of-step base frame
// and contact-body poses; after a barrier the helper evaluates the contact forces of the shank, foot (and the
// base box, leg 0) -- the height queries and point forces that dominate the report.
// FR (fused step): this step's outputs post-physics reads are also written to LDS rows (every lane)
__device__ __forceinline__ void leg_report_rigid(const DynModel& M, const t1env_buffers& B, const BaseParams<float>& PB,
                                                 const BaseState<float>& sb, const BaseFrame<float>& F,
                                                 const float q[NLEG], const float qd[NLEG], int n, int leg, bool active,
                                                 float (*P)[DYN_ENVS], int lane, float (*FR)[DYN_ENVS]) {
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
      for (int i = 0; i < 13; ++i) FR[F_ROOT + i][lane] = body[i];
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
    if (P && (k == K_SHANK || k == K_FOOT)) {
      float (*D)[DYN_ENVS] = P + POSE_F + (k == K_FOOT ? POSE_B : 0);
      lds_put_m3(D, lane, Bk[k].Rot);
      D[9][lane] = Bk[k].p.x; D[10][lane] = Bk[k].p.y; D[11][lane] = Bk[k].p.z;
#pragma unroll
      for (int i = 0; i < 6; ++i) D[12 + i][lane] = V[i];
    }
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
        for (int i = 0; i < 13; ++i) FR[(leg == 0 ? F_F0 : F_F1) + i][lane] = out[i];
      if (k == K_SHANK) { FR[(leg == 0 ? F_K0 : F_K1)][lane] = out[0]; FR[(leg == 0 ? F_K0 : F_K1) + 1][lane] = out[1]; }
    }
    if (!active) continue;
#pragma unroll
    for (int i = 0; i < 13; ++i) rig[b * 13 + i] = out[i];
    if (k != K_SHANK && k != K_FOOT) { cf[b * 3 + 0] = 0.0f; cf[b * 3 + 1] = 0.0f; cf[b * 3 + 2] = 0.0f; }
  }
}

// Self-collision needs the other leg's shank / foot too: each helper publishes its own bodies' capsules and velocities
// (rows SB_ROW.. of its leg's pose region, unused by the state) and the two helpers meet at an LDS flag -- a barrier of
// the two helper waves only (the leg waves run their backward pass meanwhile), instead of each helper recomputing the
// other leg's kinematics.  The flags count (sub)steps, so they never need resetting within a launch; a helper
// overwrites its rows only after the next S1, after the other has read them (before S2).
constexpr int SB_ROW = ST_N, SB_N = 12;  // per body: capsule ends p (3), q (3), spatial velocity (6)
static_assert(SB_ROW + 2 * SB_N <= POSE_N, "the self-collision bodies fit the pose rows");
__device__ __forceinline__ void publish_self_bodies(float (*P)[DYN_ENVS], int lane, const SelfBody<float> (&O)[2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    float (*D)[DYN_ENVS] = P + SB_ROW + s * SB_N;
    D[0][lane] = O[s].cap.p.x; D[1][lane] = O[s].cap.p.y; D[2][lane] = O[s].cap.p.z;
    D[3][lane] = O[s].cap.q.x; D[4][lane] = O[s].cap.q.y; D[5][lane] = O[s].cap.q.z;
#pragma unroll
    for (int i = 0; i < 6; ++i) D[6 + i][lane] = O[s].V[i];
  }
}
__device__ __forceinline__ void read_self_bodies(const DynModel& M, const float (*P)[DYN_ENVS], int lane, int leg,
                                                 SelfBody<float> (&X)[2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const float (*D)[DYN_ENVS] = P + SB_ROW + s * SB_N;
    X[s].cap.p = v3<float>(D[0][lane], D[1][lane], D[2][lane]);
    X[s].cap.q = v3<float>(D[3][lane], D[4][lane], D[5][lane]);
    X[s].cap.r = M.self_cap[leg][s].r;
#pragma unroll
    for (int i = 0; i < 6; ++i) X[s].V[i] = D[6 + i][lane];
  }
}
__device__ __forceinline__ void helper_signal(int* flag, int v, int lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // this wave's row stores before the flag
  if (lane == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void helper_wait(const int* flag, int v) {
  while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < v) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
// both helpers' self-collision bodies of (sub)step `tick` (1, 2, ...): O from this helper's kinematics, X the other's
__device__ __forceinline__ void exchange_self_bodies(const DynModel& M, Dyn4Lds& lds, int lane, int leg, int tick,
                                                     const BodyKin<float> (&Ko)[2], SelfBody<float> (&O)[2],
                                                     SelfBody<float> (&X)[2]) {
#pragma unroll
  for (int s = 0; s < 2; ++s) O[s] = self_body(M, leg, s, Ko[s]);
  publish_self_bodies(lds.pose[leg], lane, O);
  helper_signal(&lds.xflag[leg], tick, lane);
  helper_wait(&lds.xflag[1 - leg], tick);
  read_self_bodies(M, lds.pose[1 - leg], lane, 1 - leg, X);
}
// the contact-force report from the poses the helper computes itself from the end-of-step state: terrain forces plus
// the self-contact forces fself of the shank / foot
// (vt: the restitution set points of the shank, foot and base half; the base box's whole report uses the larger of
// its two halves', the other half's being the other helper's)
__device__ __forceinline__ void helper_report_contacts_at(const DynModel& M, const Terrain& T, const t1env_buffers& B,
                                                          const BaseFrame<float>& F, const BodyKin<float> (&Kc)[2],
                                                          const V3<float> (&fself)[2], int n, int leg, float mu,
                                                          const float (&vt)[3], float vt_base, int lane, bool active,
                                                          float (*FR)[DYN_ENVS]) {
  float* cf = B.contact_forces + (size_t)n * 39;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int b = 1 + 6 * leg + (s == 0 ? K_SHANK : K_FOOT);
    const V3<float> f = body_contact_force(M, T, b, Kc[s].Rb, Kc[s].p, F.abs, Kc[s].V, mu, vt[s]) + fself[s];
    if (active) { cf[b * 3 + 0] = f.x; cf[b * 3 + 1] = f.y; cf[b * 3 + 2] = f.z; }
    if (FR && s == 1) {
      const int r = leg == 0 ? F_C0 : F_C1;
      FR[r][lane] = f.x; FR[r + 1][lane] = f.y; FR[r + 2][lane] = f.z;
    }
  }
  if (leg == 0) {
    const V3<float> f = body_contact_force(M, T, 0, F.R0, v3<float>(0, 0, 0), F.abs, F.V0, mu, vt_base);
    if (active) { cf[0] = f.x; cf[1] = f.y; cf[2] = f.z; }
    if (FR) { FR[F_CFB][lane] = f.x; FR[F_CFB + 1][lane] = f.y; FR[F_CFB + 2][lane] = f.z; }
  }
}

// The substep log (tests only: t1env_substep_log; LG.root == nullptr when off) -- each leg wave writes its joints'
// torques and post-substep (q, qd), leg wave 0 the post-substep root row.  A run-time switch, not a template
// parameter: the logged and the product step are the same code object, so the log cannot change the arithmetic
// (r03: a separate LOG instantiation differed from the product's by up to 2.5e-5 in obs, compiler contraction).
template <bool HF, bool FUSED>
#ifdef T1_DYN4_WAVES_PER_EU1  // A/B: tell the scheduler one wave per SIMD is the target (it is, by registers)
#define T1_DYN4_ATTR __attribute__((amdgpu_waves_per_eu(1, 1)))
#else
#define T1_DYN4_ATTR
#endif
__global__ __launch_bounds__(D4_BLOCK) T1_DYN4_ATTR void k_dyn4(const DynModel* __restrict__ Mp, const t1env_config* __restrict__ Cp,
                                                   t1env_buffers B, Terrain Tin, const float* __restrict__ actions,
                                                   t1env_step_args A, ShiftArgs S, int dyn_blocks, FusedArgs FA,
                                                   SubLog LG, int shift_delay) {
  __shared__ Dyn4Lds lds;
  if ((int)blockIdx.x >= dyn_blocks) {
    shift_workgroup<FUSED, D4_BLOCK>(S, FA, Cp->num_envs, blockIdx.x - dyn_blocks, gridDim.x - dyn_blocks,
                                     reinterpret_cast<uint32_t*>(&lds.xch[0][0][0]), shift_delay);
    return;
  }
  Terrain T = Tin;
  T.type = HF ? 2 : 0;
  const t1env_config& C = *Cp;
  const DynModel& M = *Mp;
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / DYN_ENVS);
  const int leg = wave & 1;
  const bool helper = wave >= 2;
  T1_PROF_BEGIN();
  const int lane = threadIdx.x % DYN_ENVS;
  const int N = C.num_envs;
  const bool active = (int)(blockIdx.x * DYN_ENVS) + lane < N;
  const int n = active ? blockIdx.x * DYN_ENVS + lane : N - 1;  // inactive lanes shadow a valid env, never store
  const float dt = C.sim_dt;
  if (helper) {
    // ---------------- contact helper of leg `leg`
    const float mu = 0.5f * (B.friction[n] + M.ground_friction);  // robot shape vs ground (PhysX average)
    const float mu_self = B.friction[n];                          // robot shape vs robot shape
    const float e_self = B.restitution[n];
    const float e = ground_restitution(M, e_self);
    int cb, ce;
    base_contact_range(M, leg, cb, ce);
    const float (*P)[DYN_ENVS] = lds.pose[leg];
    // this helper's restitution episodes: its leg's shank, foot and base-box half (include/t1env.h contact_vimp)
    float* const vimp_row = B.contact_vimp + (size_t)n * NVIMP;
    if (lane == 0) lds.xflag[leg] = 0;  // before the first S1; the other helper first reads it after that barrier
    float vi_ft = vimp_row[vimp_foot(leg)], vi_b = vimp_row[vimp_base(leg)];
    T1_PROF_MARK(10);
    // the epilogue's inputs the step does not change, staged while the leg waves set up and run the first
    // forward pass (nothing writes them before the epilogue)
    // (staging in the helpers' first S2..S1 idle window instead measured +5% per step: profiles/r03h_ab.txt)
    if constexpr (FUSED) stage_epilogue_inputs(B, N, blockIdx.x * DYN_ENVS, (int)threadIdx.x - 2 * DYN_ENVS, lds.epi);
    for (int sub = 0; sub < C.decimation; ++sub) {
      T1_PROF_MARK(7);
      __syncthreads();  // S1: the substep states published
      T1_PROF_MARK(8);
      BaseFrame<float> F;
      BodyKin<float> Ko[2];
      helper_kinematics(M, P, lane, leg, F, Ko);
      SelfBody<float> Os[2], Xs[2];
      if (T1_SELF_CODE && M.self_collisions) exchange_self_bodies(M, lds, lane, leg, sub + 1, Ko, Os, Xs);
      T1_PROF_MARK(20);
      const V3<float> abs = F.abs;
      const int32_t bound_base = terrain_bound_raw_any(T, abs.x, abs.y);
      Sym6<float> Cs[2];
      float cs[2][6];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        sym_zero(Cs[i]);
#pragma unroll
        for (int j = 0; j < 6; ++j) cs[i][j] = 0.0f;
      }
      // the foot's terrain queries go out first; the self-contact terms run while its height loads are in flight
      body_contact_query_apply<T1_POINTS_PER_BODY>(M, T, M.contact_start[1 + 6 * leg + K_FOOT], Ko[1].Rb, Ko[1].p, abs,
                                                   Ko[1].V, mu, e, vi_ft, dt, Cs[1], cs[1], [&] {
        if (T1_SELF_CODE && M.self_collisions) self_terms_bodies(M, leg, Os, Xs, mu_self, dt, Cs, cs);
        T1_PROF_MARK(21);
      });
      lds_put_sym(lds.ct[leg] + XCH, lane, Cs[1], cs[1]);
      lds_put_sym(lds.ct[leg], lane, Cs[0], cs[0]);  // the shank's self terms (its terrain terms: the leg wave's)
      T1_PROF_MARK(3);
      __syncthreads();  // S2: contact terms published
      T1_PROF_MARK(11);
      {  // base-box contact share of this leg, straight into the base system
        Sym6<float> Cb;
        float gw[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        sym_zero(Cb);
        body_contact_fixed<T1_POINTS_PER_BODY / 2>(M, T, F.abs.z - M.contact_radius[0], bound_base, cb, F.R0,
                                                   v3<float>(0, 0, 0), F.abs, F.V0, mu, e, vi_b, dt, Cb, gw);
#pragma unroll
        for (int i = 0; i < 6; ++i) gw[i] = -gw[i];
        lds_put_sym(lds.xch[2 + leg], lane, Cb, gw);
      }
      T1_PROF_MARK(5);
      __syncthreads();  // S3: base system complete
      T1_PROF_MARK(12);
    }
    T1_PROF_MARK(7);
    lds.vib[leg][lane] = vi_b;
    if (active) { vimp_row[vimp_foot(leg)] = vi_ft; vimp_row[vimp_base(leg)] = vi_b; }
    __syncthreads();  // R1: the end-of-step states published
    T1_PROF_MARK(8);
    float (*FR)[DYN_ENVS] = FUSED ? reinterpret_cast<float (*)[DYN_ENVS]>(&lds.ct[0][0][0]) : nullptr;
    {  // the contact-force report beside the leg wave's rigid-state report
      BaseFrame<float> F;
      BodyKin<float> Ko[2];
      helper_kinematics(M, P, lane, leg, F, Ko);
      V3<float> fself[2] = {v3<float>(0.0f, 0.0f, 0.0f), v3<float>(0.0f, 0.0f, 0.0f)};
      if (T1_SELF_CODE && M.self_collisions) {
        SelfBody<float> Os[2], Xs[2];
        exchange_self_bodies(M, lds, lane, leg, C.decimation + 1, Ko, Os, Xs);
        self_forces_bodies(M, leg, Os, Xs, mu_self, fself);
      }
      const float vt[3] = {restitution_target(M, e, lds.vis[leg][lane]), restitution_target(M, e, vi_ft),
                           restitution_target(M, e, vi_b)};
      const float vt_o = restitution_target(M, e, lds.vib[1 - leg][lane]);  // the other base half (leg 0 reports)
      const float vt_base = vt_o > vt[2] ? vt_o : vt[2];
      helper_report_contacts_at(M, T, B, F, Ko, fself, n, leg, mu, vt, vt_base, lane, active, FR);
    }
    T1_PROF_MARK(11);
    if constexpr (FUSED) __syncthreads();  // the epilogue barrier
    T1_PROF_END();
    return;
  }
  // ---------------- leg wave
  const int j0 = 6 * leg;
  const uint32_t genv = (uint32_t)(C.env_offset + n);
  const uint32_t ctr = A.counter;
  const RngKey K = rng_key(C.seed, genv, ctr);
  BaseParams<float> PB;
  LegParams<float> PL;
  BaseState<float> sb;
  float q[NLEG], qd[NLEG], tau[NLEG];
  const LegSetup L = leg_setup(M, C, B, actions, ctr, n, active, j0, PB, PL, sb, q, qd);
  const V3<float> ef = v3<float>(B.applied_force[n * 3 + 0], B.applied_force[n * 3 + 1], B.applied_force[n * 3 + 2]);
  PdStage<DYN_ENVS>& PD = lds.pd[leg];
  pd_stage(B, n, j0, lane, PD);  // this step's action slot was written by leg_setup (same lane)
  float (*P)[DYN_ENVS] = lds.pose[leg];
  float (*CAP)[DYN_ENVS] = lds.cap[leg];
  if constexpr (FUSED)  // the clipped actions, for the epilogue
#pragma unroll
    for (int k = 0; k < NLEG; ++k)
      CAP[CAP_ACT + k][lane] = fminf(fmaxf(actions[n * 12 + j0 + k], -C.clip_actions), C.clip_actions);
  // the shank's terrain contact is this wave's (its forward pass has the shank's pose; the helper, the critical path
  // before S2, keeps the foot and the self-contacts): restitution episode, combined friction / restitution
  float vi_sh = B.contact_vimp[(size_t)n * NVIMP + vimp_shank(leg)];
  const float e_g = ground_restitution(M, PB.restitution);
  T1_PROF_MARK(10);
  publish_state(P, lane, sb, q, qd);  // the helpers start each substep from the state (their own kinematics)
  for (int sub = 0; sub < C.decimation; ++sub) {
    T1_PROF_MARK(7);
    __syncthreads();  // S1: the substep state published
    T1_PROF_MARK(8);
    BaseFrame<float> F;
    base_frame(sb, F);
    LegPass<float> st;
    leg_forward_nc<T1_LEG_CONTACT_MASK>(M, PL, F, q, qd, leg, dt, st,
                                        [&](auto kc, const M3<float>& Rk, V3<float> pk, const float* V) {
      if constexpr (decltype(kc)::value == K_SHANK) {
        // the shank's terrain terms, stashed in this leg's base-block rows (free between S1 and S2) until the fold-in
        const int b = 1 + 6 * leg + K_SHANK;
        Sym6<float> Ct;
        float ct6[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        sym_zero(Ct);
        const int32_t bnd = terrain_bound_raw_any(T, pk.x + F.abs.x, pk.y + F.abs.y);
        body_contact_fixed<T1_POINTS_PER_BODY>(M, T, pk.z + F.abs.z - M.contact_radius[b], bnd, M.contact_start[b], Rk,
                                               pk, F.abs, V, PB.friction, e_g, vi_sh, dt, Ct, ct6);
        lds_put_sym(lds.xch[leg], lane, Ct, ct6);
      }
    });
    T1_PROF_MARK(1);
    pd_torques_staged(M, C, PD, lane, K, ctr, sub, L.lag, j0, q, qd, tau);
    T1_PROF_MARK(0);
    LegBlock<float> lb;
    Sym6<float> Ab;
    float g6[6] = {0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    sym_zero(Ab);
    leg_backward_nc(M, PL, q, qd, leg, dt, st, lb, Ab, g6);
    T1_PROF_MARK(2);
    // the base block needs no contact term: built while the helpers finish theirs (the leg waits at S2)
    Sym6<float> Ac;
    float r[6];
    base_block(M, PB, F, sub == 0 ? ef : v3<float>(0, 0, 0), dt, Ac, r);
#pragma unroll
    for (int i = 0; i < 6; ++i) r[i] = -r[i];
    T1_PROF_MARK(6);
    __syncthreads();  // S2
    T1_PROF_MARK(11);
    {
      Sym6<float> Csh, Cft;
      float csh[6], cft[6];
      lds_get_sym(lds.ct[leg], lane, Csh, csh);  // the helper's self terms of the shank
      {
        Sym6<float> Ct;
        float ct6[6];
        lds_get_sym(lds.xch[leg], lane, Ct, ct6);  // plus this wave's terrain terms of it
#pragma unroll
        for (int i = 0; i < 21; ++i) Csh.a[i] += Ct.a[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) csh[i] += ct6[i];
      }
      lds_get_sym(lds.ct[leg] + XCH, lane, Cft, cft);
      leg_apply_contacts<K_SHANK, K_FOOT>(Csh, csh, Cft, cft, tau, dt, st, lb, Ab, g6);
#ifdef T1_WHATIF_FOLD2  // timing-only: the fold-in and elimination run twice (second result scaled by 0 and added)
      {
        LegBlock<float> lb2 = lb;
        Sym6<float> Ab2 = Ab;
        float g2[6], rb2[6];
        for (int i = 0; i < 6; ++i) g2[i] = g6[i];
        leg_apply_contacts<K_SHANK, K_FOOT>(Csh, csh, Cft, cft, tau, dt, st, lb2, Ab2, g2);
        for (int i = 0; i < 6; ++i) rb2[i] = -g2[i];
        eliminate_leg(lb2, Ab2, rb2);
        for (int i = 0; i < 21; ++i) Ab.a[i] += 0.0f * Ab2.a[i];
        for (int i = 0; i < 6; ++i) g6[i] += 0.0f * rb2[i];
      }
#endif
    }
    float rb[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) rb[i] = -g6[i];
    eliminate_leg(lb, Ab, rb);
    lds_put_sym(lds.xch[leg], lane, Ab, rb);
    T1_PROF_MARK(4);
    __syncthreads();  // S3
    T1_PROF_MARK(12);
#pragma unroll
    for (int l = 0; l < 4; ++l) {
#pragma unroll
      for (int i = 0; i < 21; ++i) Ac.a[i] += lds.xch[l][i][lane];
#pragma unroll
      for (int i = 0; i < 6; ++i) r[i] += lds.xch[l][21 + i][lane];
    }
    solve_base(Ac, r);
    float dq[NLEG];
    backsub_leg(lb, r, dq);
    integrate_base(sb, r, dt);
    integrate_leg(M, leg, q, qd, dq, dt);
    T1_PROF_MARK(9);
#ifdef T1_WHATIF_NO_LOG  // timing-only what-if build: the substep-log branch compiled out
    if (false) {
#else
    if (LG.root != nullptr) {  // wave-uniform (a kernel argument)
#endif
      if (active) {
        const size_t row = (size_t)sub * N + n;
#pragma unroll
        for (int k = 0; k < NLEG; ++k) {
          LG.torque[row * 12 + j0 + k] = tau[k];
          LG.dof[row * 24 + 2 * (j0 + k)] = q[k];
          LG.dof[row * 24 + 2 * (j0 + k) + 1] = qd[k];
        }
        if (leg == 0) {
          BaseFrame<float> FL;
          base_frame(sb, FL);
          float body[13];
          root_row(M, PB, sb, FL, body);
#pragma unroll
          for (int i = 0; i < 13; ++i) LG.root[row * 13 + i] = body[i];
        }
      }
    }
    if (sub == L.s_dof) {
#pragma unroll
      for (int k = 0; k < NLEG; ++k) { CAP[k][lane] = q[k]; CAP[NLEG + k][lane] = qd[k]; }
    }
    if (leg == 0 && sub == L.s_imu) {
#pragma unroll
      for (int i = 0; i < 4; ++i) CAP[2 * NLEG + i][lane] = sb.quat[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) CAP[2 * NLEG + 4 + i][lane] = sb.w[i];
    }
    publish_state(P, lane, sb, q, qd);  // the helper read the previous one before S2; after the last substep: the
                                        // end-of-step state its contact-force report starts from
  }
  lds.vis[leg][lane] = vi_sh;  // the shank's episode for the helper's contact-force report
  if (active) B.contact_vimp[(size_t)n * NVIMP + vimp_shank(leg)] = vi_sh;
  __syncthreads();  // R1: the end-of-step state published (the helpers compute the contact forces meanwhile)
  T1_PROF_MARK(7);
  if (active) {
    if (L.s_dof < C.decimation) {  // the sensor-lag samples captured in the loop
#pragma unroll
      for (int k = 0; k < NLEG; ++k) { L.dof_dst[j0 + k] = CAP[k][lane]; L.dof_dst[12 + j0 + k] = CAP[NLEG + k][lane]; }
    }
    if (leg == 0 && L.s_imu < C.decimation) {
      const float quat[4] = {CAP[2 * NLEG][lane], CAP[2 * NLEG + 1][lane], CAP[2 * NLEG + 2][lane], CAP[2 * NLEG + 3][lane]};
      const float w[3] = {CAP[2 * NLEG + 4][lane], CAP[2 * NLEG + 5][lane], CAP[2 * NLEG + 6][lane]};
      capture_imu(quat, w, L.imu_dst);
    }
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      B.dof_state[n * 24 + 2 * (j0 + k)] = q[k];
      B.dof_state[n * 24 + 2 * (j0 + k) + 1] = qd[k];
      B.torques[n * 12 + j0 + k] = tau[k];
    }
  }
  float (*FR)[DYN_ENVS] = FUSED ? reinterpret_cast<float (*)[DYN_ENVS]>(&lds.ct[0][0][0]) : nullptr;
  if constexpr (FUSED) {
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      FR[F_DOF + 2 * (j0 + k)][lane] = q[k];
      FR[F_DOF + 2 * (j0 + k) + 1][lane] = qd[k];
      FR[F_TQ + j0 + k][lane] = tau[k];
    }
  }
  {
    BaseFrame<float> F;
    base_frame(sb, F);
    leg_report_rigid(M, B, PB, sb, F, q, qd, n, leg, active, nullptr, lane, FR);
  }
  T1_PROF_MARK(11);
  if constexpr (FUSED) {
    __syncthreads();  // all four waves: every output of the workgroup is in memory
    T1_PROF_MARK(12);
    if (leg == 0)
      fused_epilogue_staged<POST_A_REWARDS>(M, C, B, A, S, FA, dyn_blocks, lane, lds.epi, FR, lds.cap[0], lds.cap[1]);
    else
      fused_epilogue_staged<POST_A_STATE>(M, C, B, A, S, FA, dyn_blocks, lane, lds.epi, FR, lds.cap[0], lds.cap[1]);
  }
  T1_PROF_END();
}

int t1_dyn_waves_default() { return 4; }

constexpr int MIN_SHIFT_BLOCKS = 64;
bool t1_shift_prelaunch(int num_envs, const DynLaunch& cfg) {
  if (cfg.shift_blocks < 0) return true;   // forced stand-alone shift (tuning: T1ENV_SHIFT_BLOCKS=-1)
  if (cfg.shift_blocks > 0) return false;  // explicit shift-workgroup count (tuning)
  const int dyn_blocks = (num_envs + DYN_ENVS - 1) / DYN_ENVS;
  return cfg.cus - dyn_blocks < MIN_SHIFT_BLOCKS;
}

int t1_launch_dynamics(const DynModel* d_model, const t1env_config* d_cfg, const t1env_buffers& B, const Terrain& T,
                       const float* actions, const t1env_step_args& A, int num_envs, const ShiftArgs& S,
                       const DynLaunch& cfg, const FusedArgs* fused, hipStream_t s, bool shift_prelaunched,
                       const SubLog* log) {
  const int dyn_blocks = (num_envs + DYN_ENVS - 1) / DYN_ENVS;
  // history-shift workgroups: the workgroup slots the dynamics leave free (a k_dyn4 wave holds a whole SIMD's
  // registers: one workgroup per CU), at least MIN_SHIFT_BLOCKS; none when the caller ran the shift as its own
  // launch (t1_shift_prelaunch)
  int shift_blocks = cfg.shift_blocks > 0 ? cfg.shift_blocks : cfg.cus - dyn_blocks;
  if (shift_blocks < MIN_SHIFT_BLOCKS) shift_blocks = MIN_SHIFT_BLOCKS;
  if (shift_prelaunched) shift_blocks = 0;
  // the shift's delayed start only where it has slack: as many shift workgroups as dynamics ones (N <= 8192 on 256 CUs)
  const int shift_delay = shift_blocks >= dyn_blocks ? cfg.shift_delay : 0;
  const FusedArgs FA = fused ? *fused : FusedArgs{};
  const SubLog LG = log ? *log : SubLog{};
  const dim3 grid(dyn_blocks + shift_blocks);
  const bool hf = T.type != 0;
  if (log && !fused) return (int)hipErrorInvalidValue;  // the substep log: fused steps only (the caller checks)
#define T1_LAUNCH(HF, FU) \
  hipLaunchKernelGGL((k_dyn4<HF, FU>), grid, dim3(D4_BLOCK), 0, s, d_model, d_cfg, B, T, actions, A, S, dyn_blocks, FA, LG, \
                     shift_delay)
  if (fused) { if (hf) T1_LAUNCH(true, true); else T1_LAUNCH(false, true); }
  else { if (hf) T1_LAUNCH(true, false); else T1_LAUNCH(false, false); }
#undef T1_LAUNCH
  return (int)hipGetLastError();
}

#ifdef T1_PHASE_PROF
// profiling build only: summed clock deltas per [wave][bucket] since the last reset
extern "C" int t1env_debug_phase_cycles(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t1_prof), sizeof(g_t1_prof));
  if (e == hipSuccess && reset) {
    static const unsigned long long zero[T1_PROF_WAVES][T1_NPROF] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_t1_prof), zero, sizeof(zero));
  }
  return (int)e;
}
#endif
