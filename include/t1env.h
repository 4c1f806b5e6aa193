/*
 * t1env.h -- C ABI of the MI355X-native T1 humanoid env hot path (libt1env_hip.so).
 *
 * This is the lower drop-in boundary of SURVEY.md §8(b): it replaces the Isaac Gym tensor API + PhysX
 * calls that the reference makes on the LeggedRobot.step() path:
 *
 *   t1env_create        <- gym.create_sim / load_asset / create_env / create_actor / prepare_sim and the
 *                          acquire_*_tensor + gymtorch.wrap_tensor views
 *                          (legged_robot.py:121-154, 1244-1417; base_task.py:80-82)
 *   t1env_step          <- the whole body of LeggedRobot.step(): decimation loop of _compute_torques +
 *                          set_dof_actuation_force_tensor + simulate + refresh_* + lag pushes
 *                          (legged_robot.py:387-448, 1019-1074), then post_physics_step
 *                          (legged_robot.py:458-506; t1_dh_stand_env.py:179-215, 368-559, 576-935)
 *   t1env_reset_all     <- LeggedRobot.reset()'s reset_idx(arange(N)) (legged_robot.py:450-455,
 *                          t1_dh_stand_env.py:483-559) incl. set_dof_state_tensor_indexed /
 *                          set_actor_root_state_tensor_indexed (legged_robot.py:1088, 1118)
 *   t1env_set_terrain   <- gym.add_ground / add_heightfield / add_triangle_mesh (legged_robot.py:1172-1237)
 *   t1env_step_injected <- test hook: step() with simulate() replaced by caller-provided physics states
 *                          (how obs/reward parity is pinned against the reference, tests/golden/)
 *
 * Conventions: every pointer in t1env_buffers is DEVICE memory owned by the caller (the Python host
 * layer allocates torch tensors and passes data_ptr()); the library never allocates per step and never
 * synchronises the stream inside t1env_step.  All calls return 0 on success, a positive hipError_t on a
 * HIP failure, or a negative T1ENV_E* code for argument errors; t1env_last_error() describes the last one.
 * `stream` is a hipStream_t passed as void* so the header needs no HIP include.
 */
#ifndef T1ENV_H
#define T1ENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define T1_NB 13          /* rigid bodies after collapse_fixed_joints */
#define T1_ND 12          /* revolute DOF = actions */
#define T1_MAXC 48        /* contact candidate points */
#define T1_NOBS 47        /* num_single_obs */
#define T1_NPRIV 73       /* single_num_privileged_obs */
#define T1_HIST 66        /* frame_stack */
#define T1_CHIST 3        /* c_frame_stack */
#define T1_NREW 24        /* active reward terms, alphabetical order */

#define T1ENV_EXTRAS_RING 64  /* steps an extras["episode"] view stays valid (the runner logs every 24) */

#define T1ENV_E_ARG (-1)
#define T1ENV_E_SHAPE (-2)
#define T1ENV_E_STATE (-3)

/* Robot + solver description (host memory, copied at create).  Filled by ti5_isaacgym_amd/utils/urdf.py. */
typedef struct t1env_model {
  float joint_offset[T1_NB][3]; /* joint frame origin in parent body frame (body b >= 1) */
  float joint_axis[T1_NB][3];   /* revolute axis, body frame */
  int32_t parent[T1_NB];
  float mass[T1_NB];            /* nominal mass (base = collapsed upper body) */
  float com[T1_NB][3];          /* COM, body frame */
  float inertia[T1_NB][6];      /* about COM, body frame: xx yy zz xy xz yz */
  float q_lower[T1_ND], q_upper[T1_ND], vel_limit[T1_ND], torque_limit[T1_ND];
  float default_dof_pos[T1_ND], p_gains[T1_ND], d_gains[T1_ND];
  int32_t contact_start[T1_NB], contact_count[T1_NB];
  float contact_point[T1_MAXC][3];
  int32_t n_contact;
  /* compliant-contact / limit solver constants */
  float k_contact, d_contact, friction_vs, k_limit, d_limit, gravity;
  float ground_friction, ground_restitution;
  float base_init_state[13];    /* pos(3) quat xyzw(4) linvel(3) angvel(3) -- cfg.init_state */
  /* self-collision (asset.self_collisions = 0: enabled, t1_dh_stand_config.py:51) between the legs' contact bodies:
   * the shank collision boxes (t1.urdf:265-272, 625-632) and the feet's ankle-roll STL hulls (t1.urdf:390-398,
   * 750-758) as capsules along their long axes (utils/urdf.py self_capsules), each in its link frame: segment end a (3),
   * end b (3), radius (1); order left shank, left foot, right shank, right foot.  Restitution acts above
   * bounce_threshold (sim.physx.bounce_threshold_velocity, t1_dh_stand_config.py:171) with the per-env coefficient of
   * DR (restitution_range, :185). */
  int32_t self_collisions;      /* 1: enabled */
  float self_capsule[4][7];
  float bounce_threshold;       /* [m/s] */
} t1env_model;

/* Scalar config (DHT1StandCfg values that shape the step; see t1_dh_stand_config.py). */
typedef struct t1env_config {
  int32_t num_envs;        /* envs on this rank */
  int32_t env_offset;      /* global id of env 0 (multi-GPU sharding; RNG + terrain_types use it) */
  int32_t num_envs_total;  /* envs over all ranks */
  uint32_t seed;
  float sim_dt;            /* 0.001 */
  int32_t decimation;      /* 10 */
  float action_scale, clip_actions, clip_obs;
  float max_episode_length;     /* ceil(24 / dt) = 2400 */
  float episode_length_s;
  float cycle_time, stand_com_threshold, target_joint_pos_scale;
  float noise_level;
  float noise_vec[T1_NOBS];
  float reward_scales[T1_NREW]; /* already multiplied by dt, alphabetical order */
  int32_t only_positive_rewards;
  float base_height_target, foot_min_dist, foot_max_dist, knee_min_dist, knee_max_dist;
  float target_feet_height, target_feet_height_max, tracking_sigma, max_contact_force;
  float gait_time_range[3][2];  /* per gait slot (walk_omni, stand, walk_omni) */
  int32_t gait_kind[3];         /* 0 = walk_omnidirectional, 1 = stand, 2 = walk_sagittal, 3 = walk_lateral, 4 = rotate */
  float ext_force_max[3], ext_torque_max;
  float push_vel_xy, push_ang;
  int32_t lag_range[2], dof_lag_range[2], imu_lag_range[2];
  float torque_mult_range[2], motor_offset_range[2], kp_mult_range[2], kd_mult_range[2];
  float coulomb_range[2], viscous_range[2], armature_range[T1_ND][2];
  float reset_dof_range;        /* +-0.1 */
  int32_t terrain_curriculum;   /* mesh in (heightfield, trimesh) and curriculum */
  float platform, env_length;   /* terrain platform [m], terrain_length [m] */
  int32_t num_terrain_rows, num_terrain_cols;
  float lin_vel_obs_scale, ang_vel_obs_scale, dof_pos_obs_scale, dof_vel_obs_scale, quat_obs_scale;
  /* creation-time domain randomisation (legged_robot.py:692-730, 786-824) and origins (:1477-1512) */
  int32_t dr_base_mass, dr_link_mass, dr_com, dr_friction;
  float added_mass_range[2], link_mass_range[2], com_range[3][2], friction_range[2], restitution_range[2];
  int32_t custom_origins;       /* terrain origins (heightfield/trimesh) instead of a grid */
  int32_t max_init_terrain_level;
  float reset_xy_range;         /* custom origins: +- platform/3 (curriculum) or terrain_length/2 */
  /* 1: obs_buf / priv_buf hold fp16 (BASELINE config 5's fp16 state storage: the 66/3-frame histories, ~85% of
   * the step's bytes, are stored, shifted and returned as fp16; every value is computed in fp32 and rounded once,
   * round-to-nearest-even).  0: fp32 (DHT1StandCfg). */
  int32_t obs_half;
} t1env_config;

/* Device buffers (caller-owned).  Shapes follow the reference's tensors. */
typedef struct t1env_buffers {
  float* root_states;       /* (N,13) pos, quat xyzw, COM lin vel (world), ang vel (world) */
  float* dof_state;         /* (N,12,2) pos, vel */
  float* rigid_state;       /* (N,13,13) */
  float* contact_forces;    /* (N,13,3) net contact force, world */
  float* obs_buf[2];        /* ping-pong (N,3102); step k writes obs_buf[k & 1]; fp16 data when cfg.obs_half */
  float* priv_buf[2];       /* ping-pong (N,219); fp16 data when cfg.obs_half */
  float* rew_buf;           /* (N,) */
  uint8_t* reset_buf;       /* (N,) bool */
  uint8_t* time_out_buf;    /* (N,) bool */
  int64_t* episode_length_buf;  /* (N,) */
  int64_t* phase_length_buf;    /* (N,) */
  float* commands;          /* (N,4) */
  float* torques;           /* (N,12) last substep */
  float* actions;           /* (N,12) clipped actions of this step (zeroed for reset envs) */
  float* last_actions;      /* (N,12) */
  float* last_last_actions; /* (N,12) */
  float* last_dof_vel;      /* (N,12) */
  float* last_root_vel;     /* (N,6) */
  float* base_lin_vel;      /* (N,3) */
  float* base_ang_vel;      /* (N,3) */
  float* projected_gravity; /* (N,3) */
  float* base_euler_xyz;    /* (N,3) */
  float* feet_euler_xyz;    /* (N,2,3) */
  float* feet_air_time;     /* (N,2) */
  uint8_t* last_contacts;   /* (N,2) bool */
  float* feet_height;       /* (N,2) */
  float* last_feet_z;       /* (N,2) */
  float* ref_dof_pos;       /* (N,12) */
  int32_t* gait_time;       /* (N,3) */
  float* gait_start;        /* (N,) */
  float* ext_forces;        /* (N,3) */
  float* ext_torques;       /* (N,3) */
  float* applied_force;     /* (N,3) base force for the next simulate (ENV_SPACE) */
  float* episode_sums;      /* (24,N) */
  float* kp;                /* (N,12) randomized_p_gains */
  float* kd;                /* (N,12) randomized_d_gains */
  float* motor_offsets;     /* (N,12) */
  float* coulomb;           /* (N,12) randomized_joint_coulomb */
  float* viscous;           /* (N,12) randomized_joint_viscous */
  float* armature;          /* (N,12) joint_armatures */
  float* friction;          /* (N,)  env_frictions */
  float* restitution;       /* (N,) */
  float* body_mass;         /* (N,)  base mass incl. payload */
  float* link_mass_scale;   /* (N,12) link mass multipliers (bodies 1..12) */
  float* com_disp;          /* (N,3) base COM displacement */
  int32_t* lag_timestep;    /* (N,) */
  int32_t* dof_lag_timestep;/* (N,) */
  int32_t* imu_lag_timestep;/* (N,) */
  float* act_hist;          /* (N,4,12) scaled actions of the last 4 env steps (ring by step) */
  float* dof_hist;          /* (N,4,24) lagged (q, qd) samples, ring by step */
  float* imu_hist;          /* (N,2,8) lagged IMU samples (raw base quat xyzw, world ang vel, pad), ring by step */
  float* env_origins;       /* (N,3) */
  int32_t* terrain_levels;  /* (N,) */
  int32_t* terrain_types;   /* (N,) */
  float* terrain_origins;   /* (rows, cols, 3) */
  float* extras;            /* (T1ENV_EXTRAS_RING, 32) ring of extras["episode"]: [0,24) rew_<name> means, [24]
                               terrain level mean.  A step with args.counter = c writes slot (c+1) % RING
                               (t1env_reset_all: c % RING); a step without resets carries the previous slot */
  float* ep_accum;          /* (32,) per-step reduction scratch: [0,24) sums over reset envs, [24] count,
                               [25] terrain level sum; zeroed by the library */
  float* contact_vimp;      /* (N,6) restitution episodes of the contact bodies (left shank, left foot, right shank,
                               right foot, base-box halves of the left / right leg): the approach speed a body's
                               current terrain contact began with, 0 when it touches nothing; zeroed at reset
                               (physics state PhysX keeps inside its contact cache) */
} t1env_buffers;

/* Per-step host-side schedule (no device->host sync needed to build it). */
typedef struct t1env_step_args {
  uint32_t counter;        /* common_step_counter BEFORE this step's increment */
  int32_t obs_slot;        /* which ping-pong buffer this step writes (0/1) */
  int32_t ext_force_call;  /* 1: _add_ext_force() runs this step; 0: forces zeroed */
  int32_t ext_force_first; /* is_first_add_force at that call */
  int32_t push_call;       /* 1: _push_robots() runs this step (push_robots cfg) */
  float cmd_ranges[3][2];  /* lin_vel_x, lin_vel_y, ang_vel_yaw (curriculum may widen x) */
} t1env_step_args;

/* Injected physics (tests): per-substep states replacing simulate(). */
typedef struct t1env_injected {
  const float* root;       /* (decimation, N, 13) */
  const float* dof;        /* (decimation, N, 12, 2) */
  const float* rigid;      /* (N, 13, 13) state after the last substep */
  const float* contact;    /* (N, 13, 3) */
  float* torque_log;       /* (decimation, N, 12) out: torques sent per substep, or NULL */
} t1env_injected;

/* Substep log of the product step (tests): what the dynamics kernel handed to each substep's post-simulate code,
 * in the Gym layouts the reference's Python sees after refresh_*_tensor (legged_robot.py:405-434).  With a log set,
 * t1env_step's fused launch (k_dyn4, the product kernel) also writes, for every substep s:
 *   root[s]   (decimation, N, 13) root state after substep s (pos, quat xyzw, COM lin vel, ang vel; world),
 *             before post-physics (pushes, resets) -- root[decimation-1] is what post-physics starts from
 *   dof[s]    (decimation, N, 12, 2) dof state after substep s
 *   torque[s] (decimation, N, 12) the torques _compute_torques produced for substep s
 * rigid_state / contact_forces are the end-of-step values already (post-physics never writes them).  Replaying
 * these states through the oracle's injected-physics step re-derives the PD torques, lag captures, observations
 * and rewards of the product kernel (tests/test_gpu_product_parity.py).  log = NULL switches it off.  Only the
 * fused step logs: while a log is set, t1env_step on a split step and t1env_step_physics_and_rewards fail
 * (T1ENV_E_STATE) rather than leave substeps unlogged. */
typedef struct t1env_substep_log {
  float* root;
  float* dof;
  float* torque;
} t1env_substep_log;

typedef struct t1env t1env;

int t1env_create(const t1env_model* model, const t1env_config* cfg, const t1env_buffers* bufs, t1env** out);
int t1env_destroy(t1env* env);
/* Creation-time state: DR draws (payload, link masses, COM, friction/restitution buckets), terrain levels /
 * types / env origins, initial lag lengths and gait phase offset, start pose (legged_robot.py:1259-1417,
 * 116-349; t1_dh_stand_env.py:562-569).  env_origins must already hold the grid origins for plane terrain. */
int t1env_init(t1env* env, void* stream);
int t1env_set_terrain(t1env* env, const int16_t* heights_dev, int32_t rows, int32_t cols, float horizontal_scale,
                      float vertical_scale, float border_size, int32_t mesh_type /* 0 plane, 1 hf, 2 trimesh */);
/* reset_idx(arange(N)); counter = common_step_counter (RNG key). */
int t1env_reset_all(t1env* env, const t1env_step_args* args, void* stream);
/* reset_idx(env_ids) between steps (t1_dh_stand_env.py:483-559): mask (N,) uint8 device, nonzero = reset.  The same
 * per-env reset as a step's, keyed by args->counter = common_step_counter; extras slot counter % RING gets the
 * means over the masked envs; every frame of the masked envs' obs / critic history rows is zeroed in ping-pong
 * buffer args->obs_slot (the one holding the current observations, which the next step shifts from).  The
 * command curriculum (legged_robot.py:1160-1169) is the caller's, as for t1env_reset_all. */
int t1env_reset_idx(t1env* env, const uint8_t* mask, const t1env_step_args* args, void* stream);
/* Phase A of post-physics ends with the per-env reset decision; curriculum steps (counter+1) % 2400 == 0
 * need the host to read ep_accum between the phases, so the step is exposed in two halves:
 *   t1env_step_physics_and_rewards  -> physics, post_a (callback, termination, rewards, extras reduction)
 *   t1env_step_reset_and_observe    -> post_b (reset_idx of flagged envs, observations, newest history frame)
 * The 65 older history frames are shifted by extra workgroups of phase A's dynamics launch (it reads only the
 * previous step's buffer, so it overlaps the dynamics on the CUs they leave idle); post_b follows in stream
 * order.  Everything runs on the caller's stream: no internal streams or events.
 * t1env_step() runs both back to back (no host sync). */
int t1env_step(t1env* env, const float* actions, const t1env_step_args* args, void* stream);
int t1env_step_physics_and_rewards(t1env* env, const float* actions, const t1env_step_args* args, void* stream);
int t1env_step_reset_and_observe(t1env* env, const t1env_step_args* args, void* stream);
int t1env_step_injected(t1env* env, const float* actions, const t1env_step_args* args, const t1env_injected* inj,
                        void* stream);
/* Height scan (terrain.measure_heights = True; inactive in DHT1StandCfg).  With it on, a step
 * runs the split sequence with the scan between the phases, as the reference orders it:
 *   t1env_step_physics_and_rewards -> t1env_measure_heights -> t1env_step_reset_and_observe -> t1env_critic_heights
 * t1env_measure_heights replaces LeggedRobot._get_heights (legged_robot.py:1551-1587, called from the callback,
 *   t1_dh_stand_env.py:190-191): measured (N, npts) from the post-physics, pre-reset base pose in root_states and
 *   points (npts, 2) = the base-frame (x, y) of _init_height_points (legged_robot.py:1535-1549); zeros on a plane.
 * t1env_critic_heights replaces the critic-history concatenation (t1_dh_stand_env.py:466-468, 548-558):
 *   out (N, 3, 73 + npts), frame f = [priv_buf[obs_slot] frame f | heights frame f]; heights frames 0-1 = prev
 *   frames 1-2 (zero for envs reset this step), frame 2 = clip(root_z - 0.5 - measured, -1, 1) * scale, all
 *   clipped to +-clip_obs.  prev = the previous step's out (zeroed by the caller at reset_all). */
int t1env_measure_heights(t1env* env, const float* points, int32_t npts, float* measured, void* stream);
int t1env_critic_heights(t1env* env, int32_t obs_slot, int32_t npts, float scale, const float* measured,
                         const float* prev, float* out, void* stream);
/* t1env_step runs the whole step as ONE launch by default (fused): the history shift and post-physics ride in
 * the dynamics kernel (post-physics in its epilogue).  enable = 0 makes t1env_step run the split sequence
 * (physics_and_rewards + reset_and_observe) instead; both give the same buffers.  The split entry points are
 * unaffected (they are what command-curriculum steps use). */
int t1env_set_fused(t1env* env, int32_t enable);
int t1env_set_substep_log(t1env* env, const t1env_substep_log* log);
/* Per-kernel timing with HIP events recorded around every launch (bench.py's live roofline).  Ids:
 * 0 k_dynamics incl. its history-shift workgroups (or the injected-physics kernel), 1 k_post_a, 2 k_post_b (its
 * last block also finalises the extras), 3 stand-alone k_shift (injected physics or phase B without phase A),
 * 4 unused, 5 the whole step (phase A start .. phase B end).  get_timing synchronises and returns summed milliseconds and launch counts per id since
 * the last enable. */
#define T1ENV_NTIMERS 6
/* enable: bit 0 = record events from now on; bit 1 = keep (do not clear) the events recorded so far */
int t1env_set_timing(t1env* env, int32_t enable);
int t1env_get_timing(t1env* env, double* ms /* [T1ENV_NTIMERS] */, int32_t* launches /* [T1ENV_NTIMERS] */);
const char* t1env_last_error(void);
const char* t1env_version(void);

#ifdef __cplusplus
}
#endif
#endif /* T1ENV_H */
