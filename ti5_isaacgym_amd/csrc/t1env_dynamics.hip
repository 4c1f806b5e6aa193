// t1env_dynamics.hip -- k_dynamics, the decimation loop with the articulated-body solver (legged_robot.py:
// 399-434 + Isaac Gym simulate()).  Its own translation unit because it is compiled at -O1 (build.py): at
// -O2/-O3 the optimiser produced wrong dynamics for this kernel (GPU one-step error far above fp32 against
// the host fp64 replica, tests/test_gpu_dynamics.py) while -O1 is both correct and faster (no scratch).
#include <hip/hip_runtime.h>

// -DT1_PHASE_PROF (tools/prof_dynamics_phases.py): lane 0 of every dynamics wave accumulates shader-clock
// deltas between T1_PROF_MARK points into per-phase buckets; never part of the product build.
#ifdef T1_PHASE_PROF
constexpr int T1_NPROF = 16;
__device__ unsigned long long g_t1_prof[2][T1_NPROF];
__shared__ unsigned long long t1_prof_acc[2][T1_NPROF + 1];  // [wave][bucket], last = previous mark
__device__ __forceinline__ void t1_prof_mark(int i) {
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    const unsigned long long now = clock64();
    t1_prof_acc[w][i] += now - t1_prof_acc[w][T1_NPROF];
    t1_prof_acc[w][T1_NPROF] = now;
  }
}
#define T1_PROF_MARK(i) t1_prof_mark(i)
#endif

#include "t1env_device.h"
#include "t1env_internal.h"
#include "t1env_postphys.h"

using namespace t1;

// ---------------------------------------------------------------------------------------------------
// k_dynamics: the decimation loop with the articulated-body solver.  A workgroup owns 64 envs and runs
// them on two waves: wave 0 handles every env's left leg, wave 1 the right leg (the leg index is
// wave-uniform, so all model reads are scalar loads).  Per substep each wave eliminates its leg into a
// 27-float base-block contribution (t1_dynamics.h leg_contribution), the two contributions meet in LDS
// (double-buffered by substep parity -> one barrier per substep), and both waves solve the 6x6 base system
// redundantly, so the base state stays bit-identical in both without further exchange.
//
// Workgroups past the dynamics grid (blockIdx >= dyn_blocks) run the history shift instead
// (t1env_device.h shift_history).  The dynamics waves fill at most half the CUs at 8192 envs, so the
// HBM-bound shift streams on the rest of the chip inside the same launch -- no second stream, no
// cross-stream events on the step path.  The dynamics workgroups have the lower ids, so they are dispatched
// first.
//
// FUSED (t1env_step on every step that needs no host decision between the phases): the whole env step is this
// one launch.  After its dynamics, wave 0 of each dynamics workgroup runs post-physics for its 64 envs
// (t1env_postphys.h post_a_env + post_b_env: rewards, termination, reset_idx, observations, newest history
// frame), and the last dynamics workgroup to finish finalises the extras.  Two things had to change for that:
//   * reset_idx's "resample commands of every env if any env reset" has no global dependency here: for an env
//     that did not reset, the second resample repeats post_a's (same episode step, same keyed draws), so each
//     env needs only its own reset flag;
//   * zeroing the history rows of reset envs must follow the shift of those rows, which other workgroups do
//     concurrently.  The shift is cut into units of SHIFT_UNIT rows, and each unit has a handoff word
//     (epoch-tagged): the shift workgroup sets bit 0 once the unit is shifted and written back, the dynamics
//     workgroup sets bit 1 together with the unit's 8-bit reset mask.  Whoever sets the second bit zeroes the
//     unit's reset rows.  Nobody waits for anybody, so no dispatch order or residency is assumed.
//     The shift writes these rows with agent-coherent sc1 stores (t1env_device.h store4), so once they have
//     completed (s_waitcnt) no dirty copy is left in any L2 and the zeros, written later by either party, land
//     last -- placement-independent, and without an L2 write-back fence (buffer_wbl2 per unit cost the
//     concurrently running dynamics ~8 %).
// ---------------------------------------------------------------------------------------------------
constexpr int DYN_ENVS = 64;
constexpr int DYN_BLOCK = 2 * DYN_ENVS;
constexpr int XCH = 27;  // Sym6 (21) + rhs (6)
constexpr int SHIFT_UNIT = 8;  // rows per shift/zeroing unit (a multiple of 4: unit boundaries are 16-B aligned)
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

// HF: height-field terrain (mesh heightfield/trimesh) or plane; one instantiation each so the contact code
// of the other terrain kind is folded away (it is uniform per launch).
template <bool HF, bool FUSED>
__global__ __launch_bounds__(DYN_BLOCK) void k_dynamics(const DynModel* __restrict__ Mp,
                                                        const t1env_config* __restrict__ Cp, t1env_buffers B,
                                                        Terrain Tin, const float* __restrict__ actions,
                                                        t1env_step_args A, ShiftArgs S, int dyn_blocks,
                                                        FusedArgs FA) {
  __shared__ float xch[2][2][XCH][DYN_ENVS];  // [substep parity][leg][value][env]
  if ((int)blockIdx.x >= dyn_blocks) {
    const int j = blockIdx.x - dyn_blocks, nsw = gridDim.x - dyn_blocks;
    if constexpr (!FUSED) {
      shift_history(S, (int64_t)j * DYN_BLOCK + threadIdx.x, (int64_t)nsw * DYN_BLOCK);
    } else {
      const int N = Cp->num_envs;
      const int units = (N + SHIFT_UNIT - 1) / SHIFT_UNIT;
      uint32_t* words = reinterpret_cast<uint32_t*>(&xch[0][0][0][0]);  // LDS: handoff results of this WG
      for (int u = j; u < units; u += nsw) {
        const int64_t r0 = (int64_t)u * SHIFT_UNIT, r1 = r0 + SHIFT_UNIT < N ? r0 + SHIFT_UNIT : N;
        shift_rows_range_sc1(S, r0, r1, threadIdx.x, DYN_BLOCK);
      }
      // every lane's sc1 stores complete (visible at agent scope) before any handoff
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      const int mine = units > j ? (units - j + nsw - 1) / nsw : 0;  // units of this workgroup
      for (int k0 = 0; k0 < mine; k0 += DYN_BLOCK) {
        const int k = k0 + (int)threadIdx.x;
        if (k < mine) words[threadIdx.x] = unit_handoff(FA.unit_state + j + k * nsw, FA.epoch, HANDOFF_SHIFT);
        __syncthreads();
        const int cnt = mine - k0 < DYN_BLOCK ? mine - k0 : DYN_BLOCK;
        for (int i = 0; i < cnt; ++i)
          if (handoff_complete(words[i])) zero_unit_resets(S, j + (k0 + i) * nsw, words[i], threadIdx.x, DYN_BLOCK);
        __syncthreads();
      }
    }
    return;
  }
  Terrain T = Tin;
  T.type = HF ? 2 : 0;
  const t1env_config& C = *Cp;
  const DynModel& M = *Mp;
  const int leg = __builtin_amdgcn_readfirstlane((int)threadIdx.x / DYN_ENVS);
#ifdef T1_PHASE_PROF
  if ((threadIdx.x & 63) == 0) {
    for (int i = 0; i < T1_NPROF; ++i) t1_prof_acc[leg][i] = 0;
    t1_prof_acc[leg][T1_NPROF] = clock64();
  }
#endif
  const int lane = threadIdx.x % DYN_ENVS;
  const int N = C.num_envs;
  const bool active = (int)(blockIdx.x * DYN_ENVS) + lane < N;
  const int n = active ? blockIdx.x * DYN_ENVS + lane : N - 1;  // inactive lanes shadow a valid env, never store
  const int j0 = 6 * leg;
  const uint32_t genv = (uint32_t)(C.env_offset + n);
  const uint32_t ctr = A.counter;
  // actions = clip(actions); push the scaled action into this step's history slot
  if (active) {
    float* slot = B.act_hist + ((size_t)n * 4 + (ctr & 3u)) * 12;
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      const float a = fminf(fmaxf(actions[n * 12 + j0 + k], -C.clip_actions), C.clip_actions);
      B.actions[n * 12 + j0 + k] = a;
      slot[j0 + k] = a * C.action_scale;
    }
  }
  const int lag = B.lag_timestep[n];
  const int s_dof = 9 - B.dof_lag_timestep[n] % 10, s_imu = 9 - B.imu_lag_timestep[n] % 10;
  float* dof_dst = B.dof_hist + ((size_t)n * 4 + (ctr & 3u)) * 24;
  float* imu_dst = B.imu_hist + ((size_t)n * 2 + (ctr & 1u)) * 6;
  const float dt = C.sim_dt;
  BaseParams<float> PB;
  LegParams<float> PL;
  load_base_params(M, B, n, PB);
  load_leg_params(M, B, n, j0, PL);
  BaseState<float> sb;
  load_base_state(M, PB, B.root_states + (size_t)n * 13, sb);
  float q[NLEG], qd[NLEG], tau[NLEG];
#pragma unroll
  for (int k = 0; k < NLEG; ++k) {
    q[k] = B.dof_state[n * 24 + 2 * (j0 + k)];
    qd[k] = B.dof_state[n * 24 + 2 * (j0 + k) + 1];
  }
  const V3<float> ef = v3<float>(B.applied_force[n * 3 + 0], B.applied_force[n * 3 + 1], B.applied_force[n * 3 + 2]);
  T1_PROF_MARK(10);
  for (int sub = 0; sub < C.decimation; ++sub) {
    T1_PROF_MARK(7);
    pd_torques<NLEG>(M, C, B, n, genv, ctr, sub, lag, j0, q, qd, tau);
    BaseFrame<float> F;
    base_frame(sb, F);
    T1_PROF_MARK(0);
    LegBlock<float> lb;
    {
      Sym6<float> Ab;
      float rb[6];
      leg_contribution<T1_LEG_CONTACT_MASK>(M, T, PB, PL, F, q, qd, tau, leg, dt, lb, Ab, rb);
      float* X = &xch[sub & 1][leg][0][lane];
#pragma unroll
      for (int i = 0; i < 21; ++i) X[i * DYN_ENVS] = Ab.a[i];
#pragma unroll
      for (int i = 0; i < 6; ++i) X[(21 + i) * DYN_ENVS] = rb[i];
    }
    Sym6<float> Ac;
    float r[6];
    base_block(M, PB, F, sub == 0 ? ef : v3<float>(0, 0, 0), dt, Ac, r);
#pragma unroll
    for (int i = 0; i < 6; ++i) r[i] = -r[i];
    T1_PROF_MARK(6);
    __syncthreads();
    T1_PROF_MARK(8);
#pragma unroll
    for (int l = 0; l < 2; ++l) {
      const float* Y = &xch[sub & 1][l][0][lane];
#pragma unroll
      for (int i = 0; i < 21; ++i) Ac.a[i] += Y[i * DYN_ENVS];
#pragma unroll
      for (int i = 0; i < 6; ++i) r[i] += Y[(21 + i) * DYN_ENVS];
    }
    solve_base(Ac, r);
    float dq[NLEG];
    backsub_leg(lb, r, dq);
    integrate_base(sb, r, dt);
    integrate_leg(M, leg, q, qd, dq, dt);
    T1_PROF_MARK(9);
    if (active && sub == s_dof) {
#pragma unroll
      for (int k = 0; k < NLEG; ++k) { dof_dst[j0 + k] = q[k]; dof_dst[12 + j0 + k] = qd[k]; }
    }
    if (active && leg == 0 && sub == s_imu) capture_imu(sb.quat, sb.w, imu_dst);
  }
  T1_PROF_MARK(7);
  if (active) {
    BaseFrame<float> F;
    base_frame(sb, F);
    DevWriter W{B.root_states + (size_t)n * 13, B.rigid_state + (size_t)n * 169, B.contact_forces + (size_t)n * 39};
    if (leg == 0) report_base(M, T, PB, sb, F, W);
    report_leg(M, T, PB.friction, F, q, qd, leg, W);
#pragma unroll
    for (int k = 0; k < NLEG; ++k) {
      B.dof_state[n * 24 + 2 * (j0 + k)] = q[k];
      B.dof_state[n * 24 + 2 * (j0 + k) + 1] = qd[k];
      B.torques[n * 12 + j0 + k] = tau[k];
    }
  }
  T1_PROF_MARK(11);
  if constexpr (FUSED) {
    __syncthreads();  // both legs' outputs are in memory (same workgroup: visible after the barrier)
    T1_PROF_MARK(12);
#ifdef T1_PHASE_PROF
    if (leg != 0 && (threadIdx.x & 63) == 0)
      for (int i = 0; i < T1_NPROF; ++i) atomicAdd(&g_t1_prof[leg][i], t1_prof_acc[leg][i]);
#endif
    if (leg != 0) return;
    // ---- post-physics of the workgroup's 64 envs on wave 0 (t1env_postphys.h; same code as k_post_a/b)
    const int n0 = blockIdx.x * DYN_ENVS + lane;
    const bool do_reset = post_a_env(M, C, B, A, n0);
    T1_PROF_MARK(13);
    if (active) post_b_env(M, C, B, A, n, do_reset, do_reset);
    T1_PROF_MARK(14);
    if (C.terrain_curriculum) wave_atomic_add(B.ep_accum + 25, active ? (float)B.terrain_levels[n] : 0.0f);
    // ---- reset rows: hand off each of the workgroup's shift units with its 8-bit reset mask
    const unsigned long long m = __ballot(do_reset && active);
    const int units = (N + SHIFT_UNIT - 1) / SHIFT_UNIT;
    const int u = blockIdx.x * (DYN_ENVS / SHIFT_UNIT) + lane;
    uint32_t w = 0;
    if (lane < DYN_ENVS / SHIFT_UNIT && u < units)
      w = unit_handoff(FA.unit_state + u, FA.epoch,
                       HANDOFF_DYN | ((uint32_t)(m >> (lane * SHIFT_UNIT)) & 0xffu) << 2);
    uint64_t todo = __ballot(handoff_complete(w));
    while (todo) {
      const int l = __ffsll((unsigned long long)todo) - 1;
      todo &= todo - 1;
      zero_unit_resets(S, blockIdx.x * (DYN_ENVS / SHIFT_UNIT) + l, __shfl(w, l, 64), lane, DYN_ENVS);
    }
    // ---- the last dynamics workgroup to finish finalises the step's extras.  Only atomics cross workgroups
    // here (the ep_accum sums and this counter; agent-scope atomics are performed past the L2s), so waiting for
    // this wave's atomics to complete orders them before the increment; the finaliser reads ep_accum through
    // atomics as well.
    __builtin_amdgcn_s_waitcnt(0);
    unsigned prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add(FA.done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    prev = __shfl(prev, 0, 64);
    if (prev == (unsigned)dyn_blocks - 1u) {
      finalize_extras(B, C, (int)((A.counter + 1u) % T1ENV_EXTRAS_RING));
      if (lane == 0) __hip_atomic_store(FA.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    T1_PROF_MARK(15);
  }
#ifdef T1_PHASE_PROF
  if ((threadIdx.x & 63) == 0 && (!FUSED || leg == 0))
    for (int i = 0; i < T1_NPROF; ++i) atomicAdd(&g_t1_prof[leg][i], t1_prof_acc[leg][i]);
#endif
}

int t1_launch_dynamics(const DynModel* d_model, const t1env_config* d_cfg, const t1env_buffers& B, const Terrain& T,
                       const float* actions, const t1env_step_args& A, int num_envs, const ShiftArgs& S,
                       int shift_blocks, const FusedArgs* fused, hipStream_t s) {
  const int dyn_blocks = (num_envs + DYN_ENVS - 1) / DYN_ENVS;
  const dim3 grid(dyn_blocks + shift_blocks), block(DYN_BLOCK);
  const FusedArgs FA = fused ? *fused : FusedArgs{};
  if (fused) {
    if (T.type == 0)
      hipLaunchKernelGGL((k_dynamics<false, true>), grid, block, 0, s, d_model, d_cfg, B, T, actions, A, S, dyn_blocks, FA);
    else
      hipLaunchKernelGGL((k_dynamics<true, true>), grid, block, 0, s, d_model, d_cfg, B, T, actions, A, S, dyn_blocks, FA);
  } else if (T.type == 0) {
    hipLaunchKernelGGL((k_dynamics<false, false>), grid, block, 0, s, d_model, d_cfg, B, T, actions, A, S, dyn_blocks, FA);
  } else {
    hipLaunchKernelGGL((k_dynamics<true, false>), grid, block, 0, s, d_model, d_cfg, B, T, actions, A, S, dyn_blocks, FA);
  }
  return (int)hipGetLastError();
}

#ifdef T1_PHASE_PROF
// profiling build only: summed clock deltas per [wave = leg][bucket] since the last reset
extern "C" int t1env_debug_phase_cycles(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_t1_prof), sizeof(g_t1_prof));
  if (e == hipSuccess && reset) {
    static const unsigned long long zero[2][T1_NPROF] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_t1_prof), zero, sizeof(zero));
  }
  return (int)e;
}
#endif
