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
};

// launch shape of the dynamics kernel
struct DynLaunch {
  int waves;         // 4: k_dyn4 (leg waves + contact helper waves, default), 2: k_dynamics
  int cus;           // compute units of the device (default history-shift grid)
  int shift_blocks;  // > 0: history-shift workgroups override (tuning)
};
int t1_dyn_waves_default();

// dynamics launch (t1env_dynamics.hip) plus history-shift workgroups running the shift S; fused != nullptr:
// the whole step (post-physics in the epilogue).  Returns a hipError_t.
int t1_launch_dynamics(const t1::DynModel* d_model, const t1env_config* d_cfg, const t1env_buffers& B,
                       const t1::Terrain& T, const float* actions, const t1env_step_args& A, int num_envs,
                       const t1::ShiftArgs& S, const DynLaunch& cfg, const FusedArgs* fused, hipStream_t s);
