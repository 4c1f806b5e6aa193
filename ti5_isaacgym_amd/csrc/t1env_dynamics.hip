// t1env_dynamics.hip -- k_dynamics, the decimation loop with the articulated-body solver (legged_robot.py:
// 399-434 + Isaac Gym simulate()).  Its own translation unit because it is compiled at -O1 (build.py): at
// -O2/-O3 the optimiser produced wrong dynamics for this kernel (GPU one-step error far above fp32 against
// the host fp64 replica, tests/test_gpu_dynamics.py) while -O1 is both correct and faster (no scratch).
#include <hip/hip_runtime.h>

#include "t1env_device.h"
#include "t1env_internal.h"

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
// ---------------------------------------------------------------------------------------------------
constexpr int DYN_ENVS = 64;
constexpr int DYN_BLOCK = 2 * DYN_ENVS;
constexpr int XCH = 27;  // Sym6 (21) + rhs (6)

// HF: height-field terrain (mesh heightfield/trimesh) or plane; one instantiation each so the contact code
// of the other terrain kind is folded away (it is uniform per launch).
template <bool HF>
__global__ __launch_bounds__(DYN_BLOCK) void k_dynamics(const DynModel* __restrict__ Mp,
                                                        const t1env_config* __restrict__ Cp, t1env_buffers B,
                                                        Terrain Tin, const float* __restrict__ actions,
                                                        t1env_step_args A, ShiftArgs S, int dyn_blocks) {
  __shared__ float xch[2][2][XCH][DYN_ENVS];  // [substep parity][leg][value][env]
  if ((int)blockIdx.x >= dyn_blocks) {
    const int64_t stride = (int64_t)(gridDim.x - dyn_blocks) * DYN_BLOCK;
    shift_history(S, (int64_t)(blockIdx.x - dyn_blocks) * DYN_BLOCK + threadIdx.x, stride);
    return;
  }
  Terrain T = Tin;
  T.type = HF ? 2 : 0;
  const t1env_config& C = *Cp;
  const DynModel& M = *Mp;
  const int leg = __builtin_amdgcn_readfirstlane((int)threadIdx.x / DYN_ENVS);
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
  for (int sub = 0; sub < C.decimation; ++sub) {
    pd_torques<NLEG>(M, C, B, n, genv, ctr, sub, lag, j0, q, qd, tau);
    BaseFrame<float> F;
    base_frame(sb, F);
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
    __syncthreads();
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
    if (active && sub == s_dof) {
#pragma unroll
      for (int k = 0; k < NLEG; ++k) { dof_dst[j0 + k] = q[k]; dof_dst[12 + j0 + k] = qd[k]; }
    }
    if (active && leg == 0 && sub == s_imu) capture_imu(sb.quat, sb.w, imu_dst);
  }
  if (!active) return;
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

int t1_launch_dynamics(const DynModel* d_model, const t1env_config* d_cfg, const t1env_buffers& B, const Terrain& T,
                       const float* actions, const t1env_step_args& A, int num_envs, const ShiftArgs& S,
                       int shift_blocks, hipStream_t s) {
  const int dyn_blocks = (num_envs + DYN_ENVS - 1) / DYN_ENVS;
  const dim3 grid(dyn_blocks + shift_blocks), block(DYN_BLOCK);
  if (T.type == 0)
    hipLaunchKernelGGL(k_dynamics<false>, grid, block, 0, s, d_model, d_cfg, B, T, actions, A, S, dyn_blocks);
  else
    hipLaunchKernelGGL(k_dynamics<true>, grid, block, 0, s, d_model, d_cfg, B, T, actions, A, S, dyn_blocks);
  return (int)hipGetLastError();
}
