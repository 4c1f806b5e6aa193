// t1_model_conv.h -- t1env_model (C ABI) -> DynModel (kernel layout); shared by the HIP library and the CPU
// build of the dynamics (oracle/dyn_cpu.cpp).
#pragma once
#include <math.h>
#include <string.h>

#include "../../include/t1env.h"
#include "t1_dynamics.h"

namespace t1 {

// returns nullptr on success, else a static error message
inline const char* make_dyn_model(const t1env_model* model, DynModel* dm) {
  memset(dm, 0, sizeof(*dm));
  if (model->n_contact > T1_MAXC || model->n_contact > 48) return "too many contact points";
  for (int b = 0; b < NB; ++b)
    if (model->contact_count[b] < 0 || model->contact_start[b] < 0 ||
        model->contact_start[b] + model->contact_count[b] > model->n_contact)
      return "contact_start/contact_count out of range";
  for (int b = 0; b < NB; ++b) {
    int ax = -1;
    float sg = 1.0f;
    for (int k = 0; k < 3; ++k) {
      const float v = model->joint_axis[b][k];
      if (fabsf(fabsf(v) - 1.0f) < 1e-6f) { ax = k; sg = v > 0 ? 1.0f : -1.0f; }
      else if (fabsf(v) > 1e-6f && b > 0) return "joint axes must be +-x/y/z";
    }
    if (b > 0 && ax < 0) return "missing joint axis";
    if (b > 0 && model->parent[b] != (b == 1 || b == 7 ? 0 : b - 1))
      return "body order must be base, left leg chain, right leg chain";
    dm->axis_idx[b] = ax < 0 ? 0 : ax;
    dm->axis_sign[b] = sg;
    for (int k = 0; k < 3; ++k) {
      dm->joint_offset[b][k] = model->joint_offset[b][k];
      dm->com[b][k] = model->com[b][k];
    }
    dm->mass[b] = model->mass[b];
    for (int k = 0; k < 6; ++k) dm->inertia[b][k] = model->inertia[b][k];
    dm->contact_start[b] = model->contact_start[b];
    dm->contact_count[b] = model->contact_count[b];
  }
  for (int j = 0; j < ND; ++j) {
    dm->q_lower[j] = model->q_lower[j]; dm->q_upper[j] = model->q_upper[j];
    dm->vel_limit[j] = model->vel_limit[j]; dm->torque_limit[j] = model->torque_limit[j];
    dm->default_dof_pos[j] = model->default_dof_pos[j]; dm->p_gains[j] = model->p_gains[j];
    dm->d_gains[j] = model->d_gains[j];
  }
  for (int c = 0; c < model->n_contact; ++c)
    for (int k = 0; k < 3; ++k) dm->contact_point[c][k] = model->contact_point[c][k];
  for (int b = 0; b < NB; ++b) {
    float r2 = 0.0f;
    for (int c = dm->contact_start[b]; c < dm->contact_start[b] + dm->contact_count[b]; ++c) {
      const float* p = dm->contact_point[c];
      const float d = p[0] * p[0] + p[1] * p[1] + p[2] * p[2];
      r2 = d > r2 ? d : r2;
    }
    dm->contact_radius[b] = sqrtf(r2) * 1.0001f + 1e-6f;  // rounded up: the bound must be conservative
  }
  dm->k_contact = model->k_contact; dm->d_contact = model->d_contact; dm->friction_vs = model->friction_vs;
  dm->k_limit = model->k_limit; dm->d_limit = model->d_limit; dm->gravity = model->gravity;
  dm->ground_friction = model->ground_friction; dm->ground_restitution = model->ground_restitution;
  for (int i = 0; i < 13; ++i) dm->base_init_state[i] = model->base_init_state[i];
  dm->self_collisions = model->self_collisions != 0;
  for (int i = 0; i < 4; ++i) {
    SelfCapsule& c = dm->self_cap[i / 2][i % 2];
    float len2 = 0.0f;
    for (int k = 0; k < 3; ++k) {
      c.a[k] = model->self_capsule[i][k];
      c.b[k] = model->self_capsule[i][3 + k];
      len2 += (c.b[k] - c.a[k]) * (c.b[k] - c.a[k]);
    }
    c.r = model->self_capsule[i][6];
    if (dm->self_collisions && !(c.r > 0.0f && len2 > 1e-8f))
      return "self_capsule needs a positive radius and two distinct segment ends";
  }
  dm->bounce_threshold = model->bounce_threshold;
  if (!(dm->bounce_threshold >= 0.0f)) return "bounce_threshold must be >= 0";
  return nullptr;
}

// The HIP kernel compiles the T1 layout in (t1_dynamics.h): joint axes T1_LEG_AXIS, and contact points on the
// base box and, on each leg, the shank (k=3) and the foot (k=5), T1_POINTS_PER_BODY each; none elsewhere.
inline const char* check_fixed_contact_layout(const DynModel& dm) {
  if (dm.contact_count[0] != T1_POINTS_PER_BODY) return "base must carry 8 contact points";
  for (int leg = 0; leg < 2; ++leg)
    for (int k = 0; k < NLEG; ++k)
      if (dm.axis_idx[1 + 6 * leg + k] != T1_LEG_AXIS[k]) return "leg joint axes must be z, x, y, y, y, x (T1)";
  for (int leg = 0; leg < 2; ++leg)
    for (int k = 0; k < NLEG; ++k) {
      const bool has = (T1_LEG_CONTACT_MASK >> k) & 1;
      if (dm.contact_count[1 + 6 * leg + k] != (has ? T1_POINTS_PER_BODY : 0))
        return "leg contact points must be 8 on the shank and the foot and none elsewhere";
    }
  return nullptr;
}

}  // namespace t1
