// t1env_internal.h -- entry points shared between the library's translation units (not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/t1env.h"
#include "t1_dynamics.h"

#include "t1env_device.h"

// state of the fused step (k_dynamics with post-physics in its epilogue, t1env_dynamics.hip)
struct FusedArgs {
  unsigned* done;                  // dynamics-workgroup completion counter (the last one finalises the extras)
  uint32_t* unit_state;            // per shift unit: epoch-tagged handoff word (reset mask inside)
  uint32_t epoch;                  // launch number (unique per fused step)
  int32_t shift_done;              // 1: the history shift ran as its own launch before this one (large N):
                                   //    the epilogue zeroes its reset rows directly, no handoff
  float* ep_part;                  // k_dyn4: per dynamics workgroup one row of EP_PART_ROW partial extras sums
                                   //    ([0,24) episode sums over reset envs, [24] reset count, [25] terrain levels)
};
constexpr int EP_PART_ROW = 32;

// substep log of the fused k_dyn4 (t1env_substep_log; all null = off)
struct SubLog {
  float* root;
  float* dof;
  float* torque;
};

// default delayed start of the in-launch history-shift workgroups (100 MHz ticks; DynLaunch::shift_delay): 30 us, so
// the dynamics workgroups' prologue loads do not queue behind the shift's stream.  At 8192 trimesh envs 2,000-4,000
// ticks measured -0.6..-0.8% per step against 0 (profiles/r03g_shift_grid.txt); applied only while the shift has at
// least as many workgroups as the dynamics (its ~104 us then ends well before the ~160 us dynamics)
constexpr int T1_SHIFT_DELAY_DEFAULT = 3000;

// launch shape of the dynamics kernel
struct DynLaunch {
  int waves;         // 6: k_dyn6 (t1env_dyn6.hip: 32 envs per workgroup, eight role waves, two per SIMD), 5: k_dyn5
                     //    (t1env_dyn5.hip: 32 envs per workgroup, four roles, in-workgroup history shift), 4: k_dyn4
                     //    (64 envs per workgroup, leg + contact helper waves); t1_dyn_waves_default picks k_dyn6
                     //    (k_dyn4 for fp16 histories above one round), T1ENV_DYN_KERNEL=4|5|6 overrides
  int cus;           // compute units of the device (default history-shift grid)
  int shift_blocks;  // > 0: history-shift workgroups override (tuning)
  int shift_delay;   // in-launch shift workgroups start this many 100 MHz ticks late (T1ENV_SHIFT_DELAY; 0 = at once)
  int d5_shift;      // k_dyn5's history shift: 0 = in the workgroup through LDS-DMA (default), 1 = a concurrent launch
                     // on a second stream (k_shift5; T1ENV_D5_SHIFT=1, A/B: the same step time, r04e)
  int d4_shift;      // k_dyn4's history shift where the dynamics fill the CUs (t1_shift_prelaunch, config 5): 1 = a
                     // concurrent launch on a second stream beside the dynamics (k_shift4c, the default), 0 = its own
                     // launch ahead of them in stream order (T1ENV_D4_SHIFT=0, A/B)
};
int t1_dyn_waves_default(int num_envs, int cus, bool obs_half);

// dynamics launch (t1env_dynamics.hip) plus history-shift workgroups running the shift S; fused != nullptr:
// the whole step (post-physics in the epilogue).  shift_prelaunched: the caller already enqueued the shift as
// its own launch (no shift workgroups).  log: the substep log (fused k_dyn4 only).  Returns a hipError_t.
int t1_launch_dynamics(const t1::DynModel* d_model, const t1env_config* d_cfg, const t1env_buffers& B,
                       const t1::Terrain& T, const float* actions, const t1env_step_args& A, int num_envs,
                       const t1::ShiftArgs& S, const DynLaunch& cfg, const FusedArgs* fused, hipStream_t s,
                       bool shift_prelaunched = false, const SubLog* log = nullptr);
// Whether the history shift should run as its own launch ahead of the dynamics: the dynamics workgroups (one
// per CU for k_dyn4: 148 KB of LDS) leave fewer than MIN_SHIFT_BLOCKS CUs idle, and shift workgroups of the
// dynamics launch would each hold a whole CU's LDS for a small slice of the 26 KB/env stream.
bool t1_shift_prelaunch(int num_envs, const DynLaunch& cfg);
// k_dyn5 (t1env_dyn5.hip): the same contract as t1_launch_dynamics; each workgroup shifts its own history rows
int t1_launch_dyn5(const t1::DynModel* d_model, const t1env_config* d_cfg, const t1env_buffers& B, const t1::Terrain& T,
                   const float* actions, const t1env_step_args& A, int num_envs, const t1::ShiftArgs& S,
                   const FusedArgs* fused, hipStream_t s, const SubLog* log, bool inwg_shift);
// k_dyn6 (t1env_dyn6.hip): k_dyn5's roles on eight waves (two per SIMD), the same contract; each workgroup shifts its own
// history rows
int t1_launch_dyn6(const t1::DynModel* d_model, const t1env_config* d_cfg, const t1env_buffers& B, const t1::Terrain& T,
                   const float* actions, const t1env_step_args& A, int num_envs, const t1::ShiftArgs& S,
                   const FusedArgs* fused, hipStream_t s, const SubLog* log);
// k_dyn5's history shift as its own launch (k_shift5), for a second stream beside k_dyn5 (d5_shift = 1); fused: the
// unit handoff with the fused epilogue, else plain (k_post_b zeroes the reset rows)
// beside4: the k_dyn4 form (k_shift4c, <= 72 registers per lane so a wave fits beside a k_dyn4 wave on its SIMD)
int t1_launch_shift5(const t1::ShiftArgs& S, const FusedArgs* fused, int num_envs, int cus, hipStream_t s,
                     bool beside4 = false);
