// dyn_cpu.cpp -- CPU (g++/OpenMP) build of the product dynamics header, TEST INFRASTRUCTURE.
//
// PhysX has no oracle (closed binary, absent), so physics parity is unpinned; this build exists to
//  (1) check the GPU fp32 dynamics against the same algorithm in fp64 on the host,
//  (2) expose the solver's accelerations to the independent numpy formulation in oracle/dynamics_ref.py,
//  (3) serve as the physics half of bench.py's cpu_baseline ("port": oracle numpy post-physics + this).
#include <omp.h>
#include <stdint.h>
#include <string.h>

#include "../ti5_isaacgym_amd/csrc/t1_model_conv.h"
#include "../ti5_isaacgym_amd/csrc/t1_dyn5.h"

using namespace t1;

namespace {
template <typename R>
void load(const DynModel& M, int n, const float* root, const float* dof, const float* body_mass,
          const float* link_scale, const float* com_disp, const float* armature, const float* friction,
          const float* restitution, const float* vimp, EnvParams<R>& P, EnvState<R>& s) {
  P.base.mass = body_mass[n];
  P.base.inertia_scale = P.base.mass / R(M.mass[0]);
  for (int k = 0; k < 3; ++k) P.base.com_disp[k] = com_disp[n * 3 + k];
  P.base.friction = R(0.5) * (R(friction[n]) + R(M.ground_friction));
  P.base.self_friction = R(friction[n]);
  P.base.restitution = restitution ? R(restitution[n]) : R(0);
  for (int j = 0; j < ND; ++j) {
    LegParams<R>& L = P.leg[j / 6];
    L.mass[j % 6] = R(M.mass[1 + j]) * link_scale[n * 12 + j];
    L.inertia_scale[j % 6] = link_scale[n * 12 + j];
    L.armature[j % 6] = armature[n * 12 + j];
  }
  const float* r = root + (size_t)n * 13;
  for (int i = 0; i < 3; ++i) s.pos[i] = r[i];
  for (int i = 0; i < 4; ++i) s.quat[i] = r[3 + i];
  M3<R> R0 = quat_to_mat(s.quat[0], s.quat[1], s.quat[2], s.quat[3]);
  V3<R> c0 = base_com(M, P.base, R0);
  V3<R> w = v3<R>(r[10], r[11], r[12]);
  V3<R> vo = v3<R>(r[7], r[8], r[9]) - cross(w, c0);
  s.w[0] = w.x; s.w[1] = w.y; s.w[2] = w.z; s.vo[0] = vo.x; s.vo[1] = vo.y; s.vo[2] = vo.z;
  for (int j = 0; j < ND; ++j) { s.q[j] = dof[(size_t)n * 24 + 2 * j]; s.qd[j] = dof[(size_t)n * 24 + 2 * j + 1]; }
  for (int i = 0; i < NVIMP; ++i) s.vimp[i] = vimp ? R(vimp[(size_t)n * NVIMP + i]) : R(0);
}

template <typename R> struct Writer {
  float* rootp; float* rigidp; float* contactp;
  void root(const R* v) { for (int i = 0; i < 13; ++i) rootp[i] = (float)v[i]; }
  void rigid(int b, const R* v) { if (rigidp) for (int i = 0; i < 13; ++i) rigidp[b * 13 + i] = (float)v[i]; }
  void contact(int b, V3<R> f) { if (contactp) { contactp[b * 3] = (float)f.x; contactp[b * 3 + 1] = (float)f.y; contactp[b * 3 + 2] = (float)f.z; } }
};

template <typename R>
int substep_batch(const t1env_model* model, int N, float* root, float* dof, const float* tau, const float* body_mass,
                  const float* link_scale, const float* com_disp, const float* armature, const float* friction,
                  const float* restitution, float* vimp, const float* ext_force, float dt, int nsub, const int16_t* hf,
                  int rows, int cols, float hs, float vs, float border, int mesh, float* rigid, float* contact,
                  int mode) {
  DynModel M;
  if (make_dyn_model(model, &M)) return -1;
  Terrain T = make_terrain(hf, rows, cols, mesh, hs, vs, border);
#pragma omp parallel for schedule(static)
  for (int n = 0; n < N; ++n) {
    EnvParams<R> P;
    EnvState<R> s;
    load<R>(M, n, root, dof, body_mass, link_scale, com_disp, armature, friction, restitution, vimp, P, s);
    R t[ND];
    for (int j = 0; j < ND; ++j) t[j] = tau[(size_t)n * 12 + j];
    for (int k = 0; k < nsub; ++k) {
      V3<R> ef = (ext_force && k == 0) ? v3<R>(ext_force[n * 3], ext_force[n * 3 + 1], ext_force[n * 3 + 2]) : v3<R>(0, 0, 0);
      if (mode == 2) substep_roles(M, T, P, s, t, ef, R(dt));  // k_dyn5's role composition
      else if (mode == 3) substep_roles6(M, T, P, s, t, ef, R(dt));  // k_dyn6's
      else substep(M, T, P, s, t, ef, R(dt), mode == 1);
    }
    Writer<R> W{root + (size_t)n * 13, rigid ? rigid + (size_t)n * 169 : nullptr, contact ? contact + (size_t)n * 39 : nullptr};
    report(M, T, P, s, W);
    for (int j = 0; j < ND; ++j) { dof[(size_t)n * 24 + 2 * j] = (float)s.q[j]; dof[(size_t)n * 24 + 2 * j + 1] = (float)s.qd[j]; }
    if (vimp)
      for (int i = 0; i < NVIMP; ++i) vimp[(size_t)n * NVIMP + i] = (float)s.vimp[i];
  }
  return 0;
}
}  // namespace

extern "C" {
// Advance N envs by nsub substeps with constant joint torques (root: Gym layout, COM velocity).
// flags: bit 0 = fp64, bit 1 = the k_dyn4 split composition (compute_delta_split) instead of compute_delta,
// bit 2 = k_dyn5's role composition (compute_delta_roles, t1_dyn5.h), bit 3 = k_dyn6's (compute_delta_roles6).
// restitution: the envs' shape restitution (null: 0); vimp: (N, 6) restitution episodes of the contact bodies, read
// and updated (null: none carried across calls).
int t1dyn_substeps(const t1env_model* model, int N, int flags, float* root, float* dof, const float* tau,
                   const float* body_mass, const float* link_scale, const float* com_disp, const float* armature,
                   const float* friction, const float* restitution, float* vimp, const float* ext_force, float dt, int nsub,
                   const int16_t* hf, int rows, int cols, float hs, float vs, float border, int mesh, float* rigid,
                   float* contact) {
  const int mode = (flags & 8) ? 3 : ((flags & 4) ? 2 : ((flags & 2) ? 1 : 0));
  return (flags & 1) ? substep_batch<double>(model, N, root, dof, tau, body_mass, link_scale, com_disp, armature,
                                             friction, restitution, vimp, ext_force, dt, nsub, hf, rows, cols, hs, vs, border,
                                             mesh, rigid, contact, mode)
                     : substep_batch<float>(model, N, root, dof, tau, body_mass, link_scale, com_disp, armature,
                                            friction, restitution, vimp, ext_force, dt, nsub, hf, rows, cols, hs, vs, border,
                                            mesh, rigid, contact, mode);
}

// Solver accelerations in fp64 for one env with internal state (pos, quat, w, v_O, q, qd): returns
// udot = [omega_dot, a_O (classical, base origin), qdd] (no contact if the robot is airborne).
int t1dyn_accel(const t1env_model* model, const double* mass, const double* inertia_scale, const double* com_disp,
                const double* armature, const double* state /* 3+4+3+3+12+12 */, const double* tau, double* udot) {
  DynModel M;
  if (make_dyn_model(model, &M)) return -1;
  Terrain T = make_terrain(nullptr, 0, 0, 0, 0.1f, 0.005f, 0.0f);
  EnvParams<double> P;
  P.base.mass = mass[0];
  P.base.inertia_scale = inertia_scale[0];
  for (int k = 0; k < 3; ++k) P.base.com_disp[k] = com_disp[k];
  P.base.friction = 0.5;
  P.base.self_friction = 0.5;
  P.base.restitution = 0.0;
  for (int j = 0; j < ND; ++j) {
    P.leg[j / 6].mass[j % 6] = mass[1 + j];
    P.leg[j / 6].inertia_scale[j % 6] = inertia_scale[1 + j];
    P.leg[j / 6].armature[j % 6] = armature[j];
  }
  EnvState<double> s;
  for (int i = 0; i < 3; ++i) s.pos[i] = state[i];
  for (int i = 0; i < 4; ++i) s.quat[i] = state[3 + i];
  for (int i = 0; i < 3; ++i) { s.w[i] = state[7 + i]; s.vo[i] = state[10 + i]; }
  for (int j = 0; j < ND; ++j) { s.q[j] = state[13 + j]; s.qd[j] = state[25 + j]; }
  for (int i = 0; i < NVIMP; ++i) s.vimp[i] = 0.0;
  double d[18];
  compute_delta(M, T, P, s, tau, v3<double>(0, 0, 0), 1.0, d);
  V3<double> w{s.w[0], s.w[1], s.w[2]}, v{s.vo[0], s.vo[1], s.vo[2]};
  V3<double> a = v3<double>(d[3], d[4], d[5]) + cross(w, v);
  udot[0] = d[0]; udot[1] = d[1]; udot[2] = d[2]; udot[3] = a.x; udot[4] = a.y; udot[5] = a.z;
  for (int j = 0; j < ND; ++j) udot[6 + j] = d[6 + j];
  return 0;
}

int t1dyn_num_threads(void) { return omp_get_max_threads(); }
// the OpenMP thread count of the calling thread's parallel regions (bench.py's CPU baseline sets it explicitly instead
// of inheriting OMP_NUM_THREADS; each shard thread of oracle/cpu_env.py ShardedCpuT1Env sets its own share)
void t1dyn_set_num_threads(int n) { if (n > 0) omp_set_num_threads(n); }
}
