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
#include "t1env_fused.h"

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
// chunks per lane in flight in the in-launch shift: the shift workgroups run one wave per SIMD on the CUs the dynamics
// leave idle, so they need deep per-lane batches (r02u: 8 -> 16 took the shift alone from 114 to 106 us at 8192 envs)
#ifndef T1_FUSED_SHIFT_UNROLL
#define T1_FUSED_SHIFT_UNROLL 16
#endif
static_assert(DYN_ENVS % SHIFT_UNIT == 0, "a dynamics workgroup owns whole shift units");

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
    if constexpr (FUSED) stage_epilogue_inputs<DYN_ENVS, 2 * DYN_ENVS>(B, N, blockIdx.x * DYN_ENVS, (int)threadIdx.x - 2 * DYN_ENVS, lds.epi);
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
      helper_report_contacts_at<DYN_ENVS>(M, T, B, F, Ko, fself, n, leg, mu, vt, vt_base, lane, active, FR);
    }
    T1_PROF_MARK(11);
    if constexpr (FUSED) {
      __syncthreads();  // the epilogue barrier
      if (leg == 0)
        fused_epilogue_obs<POST_OBS_PRIV, DYN_ENVS>(M, C, B, A, lane, lds.epi, FR, lds.cap[0] + CAP_ACT,
                                                    lds.cap[1] + CAP_ACT);
      else
        fused_epilogue_obs<POST_OBS_ACTOR, DYN_ENVS>(M, C, B, A, lane, lds.epi, FR, lds.cap[0] + CAP_ACT,
                                                     lds.cap[1] + CAP_ACT);
    }
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
    leg_report_rigid<DYN_ENVS>(M, B, PB, sb, F, q, qd, n, leg, active, lane, FR);
  }
  T1_PROF_MARK(11);
  if constexpr (FUSED) {
    __syncthreads();  // all four waves: every output of the workgroup is in memory
    T1_PROF_MARK(12);
    if (leg == 0)
      fused_epilogue_staged<POST_A_REWARDS, DYN_ENVS, false>(M, C, B, A, S, FA, dyn_blocks, lane, lds.epi, FR,
                                                              lds.cap[0] + CAP_ACT, lds.cap[1] + CAP_ACT);
    else
      fused_epilogue_staged<POST_A_STATE, DYN_ENVS, false>(M, C, B, A, S, FA, dyn_blocks, lane, lds.epi, FR,
                                                            lds.cap[0] + CAP_ACT, lds.cap[1] + CAP_ACT);
  }
  T1_PROF_END();
}

// k_dyn6 at 8192 trimesh envs (one round of 32-env workgroups on 256 CUs): 0.127 ms, k_dyn5 0.141, k_dyn4 0.150.
// Above one round k_dyn6's rounds still beat k_dyn4's 64-env workgroups with fp32 histories (r05full: 16384 trimesh
// 0.247 vs 0.268 ms, 32768 hf + push 0.485 vs 0.519), but not with fp16 histories, where k_dyn4's stand-alone shift
// launch halves and k_dyn4's 64 envs per workgroup are the better throughput (r05cfg5: 32768 hf + push 0.437 vs 0.471,
// 16384 0.216 vs 0.240).  T1ENV_DYN_KERNEL=4|5|6 overrides (A/B).
int t1_dyn_waves_default(int num_envs, int cus, bool obs_half) {
  return obs_half && (num_envs + 31) / 32 > cus ? 4 : 6;
}

constexpr int MIN_SHIFT_BLOCKS = 64;
bool t1_shift_prelaunch(int num_envs, const DynLaunch& cfg) {
  if (cfg.waves >= 5) return false;        // k_dyn5 / k_dyn6: every workgroup shifts its own rows
  if (cfg.shift_blocks < 0) return true;   // forced stand-alone shift (tuning: T1ENV_SHIFT_BLOCKS=-1)
  if (cfg.shift_blocks > 0) return false;  // explicit shift-workgroup count (tuning)
  const int dyn_blocks = (num_envs + DYN_ENVS - 1) / DYN_ENVS;
  return cfg.cus - dyn_blocks < MIN_SHIFT_BLOCKS;
}

int t1_launch_dynamics(const DynModel* d_model, const t1env_config* d_cfg, const t1env_buffers& B, const Terrain& T,
                       const float* actions, const t1env_step_args& A, int num_envs, const ShiftArgs& S,
                       const DynLaunch& cfg, const FusedArgs* fused, hipStream_t s, bool shift_prelaunched,
                       const SubLog* log) {
  if (cfg.waves == 6) return t1_launch_dyn6(d_model, d_cfg, B, T, actions, A, num_envs, S, fused, s, log);
  if (cfg.waves == 5)  // the shift in the workgroup (d5_shift 0) or the caller's concurrent k_shift5 launch (1)
    return t1_launch_dyn5(d_model, d_cfg, B, T, actions, A, num_envs, S, fused, s, log, cfg.d5_shift == 0);
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
