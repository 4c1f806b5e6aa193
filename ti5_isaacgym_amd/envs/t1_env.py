"""T1DHStandEnv on MI355X: the reference's env API over the HIP hot path (libt1env_hip.so).

Upper drop-in boundary: constructor signature of the reference
(``cfg, sim_params, physics_engine, sim_device, headless``; humanoid/envs/t1/t1_dh_stand_env.py:72),
``step`` / ``reset`` / ``get_observations`` / ``get_privileged_observations`` and the attributes the DH PPO
runner and play.py read (num_envs, num_obs, num_short_obs, num_privileged_obs, num_actions,
max_episode_length, episode_length_buf (writable), obs/priv/rew/reset buffers, extras, root_states,
dof_pos/dof_vel, rigid_state, contact_forces, commands, torques, base_lin_vel/ang_vel, feet_indices, cfg).

All per-env state lives in device tensors owned here; ``step`` enqueues the HIP kernels on the current
stream and returns without a host sync (the only syncs: the command curriculum check, once per 2400
steps, and ``reset()``).  Differences in buffer semantics vs the reference (documented in DESIGN.md):
  * obs/priv are two ping-pong buffers; the tensor returned by step k stays valid through step k+1
    (the reference allocates a fresh tensor per step; DHPPO only keeps one step back).
  * extras["episode"] values are 0-d views into a 64-step ring the library writes (no per-step copy).
"""
import math

import numpy as np
import torch

from .. import _lib
from ..algo.vec_env import VecEnv
from ..utils.helpers import class_to_dict
from ..utils.terrain import Terrain
from ..utils.urdf import load_model, self_capsules

REWARD_NAMES = sorted(["action_smoothness", "base_acc", "base_height", "collision", "default_joint_pos", "dof_acc",
                       "dof_vel", "feet_air_time", "feet_clearance", "feet_contact_forces", "feet_contact_number",
                       "feet_distance", "feet_rotation", "foot_slip", "joint_pos", "knee_distance", "low_speed",
                       "orientation", "stand_still", "torques", "track_vel_hard", "tracking_ang_vel",
                       "tracking_lin_vel", "vel_mismatch_exp"])
GAIT_KINDS = {"walk_omnidirectional": 0, "stand": 1, "walk_sagittal": 2, "walk_lateral": 3, "rotate": 4}

# Solver constants of the compliant contact / soft limit model (PhysX TGS is unpinned).
EXTRAS_RING = 64  # include/t1env.h T1ENV_EXTRAS_RING
SOLVER = dict(k_contact=1.0e5, d_contact=1.5e3, friction_vs=0.01, k_limit=2.0e4, d_limit=200.0, gravity=9.81)


class _SimDt:
    def __init__(self, dt):
        self.dt = dt


def _ptr(t):
    return t.data_ptr()


def build_model(cfg, urdf_path=None):
    """LeggedRobotCfg + URDF -> (t1env_model ctypes struct, model table, default pose, kp, kd).

    Mirrors _create_envs / _process_dof_props / _init_buffers (legged_robot.py:225-234, 1171-1262): dof
    limits scaled by cfg.safety, PD gains by substring match of the dof names."""
    tab = load_model(urdf_path)
    m = _lib.Model()
    for b in range(13):
        for k in range(3):
            m.joint_offset[b][k] = tab["joint_offset"][b][k]
            m.joint_axis[b][k] = tab["joint_axis"][b][k]
            m.com[b][k] = tab["com"][b][k]
        m.parent[b] = tab["parent"][b]
        m.mass[b] = tab["mass"][b]
        for k in range(6):
            m.inertia[b][k] = tab["inertia"][b][k]
        m.contact_start[b] = tab["contact_start"][b]
        m.contact_count[b] = tab["contact_count"][b]
    lim = np.asarray(tab["limits"])
    default = np.array([cfg.init_state.default_joint_angles[n] for n in tab["dof_names"]], np.float32)
    kp = np.zeros(12, np.float32)
    kd = np.zeros(12, np.float32)
    for i, n in enumerate(tab["dof_names"]):   # substring match, legged_robot.py:225-234
        for key in cfg.control.stiffness:
            if key in n:
                kp[i] = cfg.control.stiffness[key]
                kd[i] = cfg.control.damping[key]
    safety = getattr(cfg, "safety", None)
    pos_k = safety.pos_limit if safety else 1.0
    vel_k = safety.vel_limit if safety else 1.0
    tq_k = safety.torque_limit if safety else 1.0
    for j in range(12):
        m.q_lower[j], m.q_upper[j] = lim[j, 0] * pos_k, lim[j, 1] * pos_k
        m.vel_limit[j] = lim[j, 3] * vel_k
        m.torque_limit[j] = np.float32(lim[j, 2]) * np.float32(tq_k)
        m.default_dof_pos[j], m.p_gains[j], m.d_gains[j] = default[j], kp[j], kd[j]
    pts = tab["contact_point"]
    m.n_contact = len(pts)
    for c, p in enumerate(pts):
        for k in range(3):
            m.contact_point[c][k] = p[k]
    for k, v in SOLVER.items():
        setattr(m, k, v)
    m.gravity = -float(cfg.sim.gravity[2]) if hasattr(cfg.sim, "gravity") else 9.81
    m.ground_friction = cfg.terrain.static_friction
    m.ground_restitution = cfg.terrain.restitution
    init = list(cfg.init_state.pos) + list(cfg.init_state.rot) + list(cfg.init_state.lin_vel) + \
        list(cfg.init_state.ang_vel)
    for i in range(13):
        m.base_init_state[i] = init[i]
    # asset.self_collisions is Isaac Gym's bitwise filter: 0 enables self-collision (t1_dh_stand_config.py:51)
    set_self_collision(m, tab, enabled=int(cfg.asset.self_collisions) == 0,
                       bounce_threshold=cfg.sim.physx.bounce_threshold_velocity)
    return m, tab, default, kp, kd


def set_self_collision(m, tab, enabled=True, bounce_threshold=0.5):
    """The model's self-collision capsules (utils/urdf.py self_capsules: left shank, left foot, right shank, right
    foot) and the restitution bounce threshold (sim.physx.bounce_threshold_velocity, t1_dh_stand_config.py:171)."""
    m.self_collisions = int(bool(enabled))
    for i, cap in enumerate(self_capsules(tab)):
        for k in range(7):
            m.self_capsule[i][k] = cap[k]
    m.bounce_threshold = float(bounce_threshold)


def check_supported(cfg):
    """Configuration switches the HIP path does not implement raise here, before any device work."""
    dr = cfg.domain_rand
    if dr.add_ext_force and dr.ext_torque_max != 0:
        # the reference applies the drawn torques to the base too (apply_torques, t1_dh_stand_env.py:243-247); the
        # HIP dynamics applies the base force only (ext_torque_max = 0 in DHT1StandCfg, t1_dh_stand_config.py:201)
        raise NotImplementedError("domain_rand.ext_torque_max != 0: external base torques are not applied by the HIP "
                                  "dynamics (t1_dh_stand uses 0)")


class T1DHStandEnv(VecEnv):
    def __init__(self, cfg, sim_params=None, physics_engine=None, sim_device="cuda:0", headless=True,
                 env_offset=0, num_envs_total=None, urdf_path=None):
        check_supported(cfg)
        lib = _lib.load()
        self.cfg = cfg
        self.sim_params = sim_params if sim_params is not None else _SimDt(cfg.sim.dt)
        self.physics_engine = physics_engine
        self.headless = headless
        self.device = torch.device(sim_device)
        if self.device.type != "cuda":
            raise RuntimeError("T1DHStandEnv runs on the HIP device only (sim_device='cuda:<i>'); "
                               "the CPU oracle lives in oracle/ and is test infrastructure")
        self.sim_device = sim_device
        e = cfg.env
        self.num_envs = N = int(e.num_envs)
        self.num_obs = int(e.num_observations)
        self.num_short_obs = int(e.num_single_obs * e.short_frame_stack)
        self.num_privileged_obs = int(e.num_privileged_obs)
        self.num_actions = int(e.num_actions)
        self.num_single_obs = int(e.num_single_obs)
        # the actor observation is frame_stack frames of num_single_obs, shifted one frame per step and zeroed at
        # reset (t1_dh_stand_env.py:368-481, 548-558): the runner's rollout storage keeps frames (algo/rollout.py)
        self.obs_frame_history = (self.num_single_obs, int(e.frame_stack))
        if (self.num_single_obs, e.single_num_privileged_obs, e.frame_stack, e.c_frame_stack, self.num_actions) != \
                (_lib.NOBS, _lib.NPRIV, _lib.HIST, _lib.CHIST, _lib.ND):
            raise ValueError("the HIP kernels are specialised for the t1_dh_stand layout (47 x 66 obs, 73 x 3 priv)")
        # height scan (inactive in DHT1StandCfg): 187 heights per critic frame, t1env_measure_heights /
        # t1env_critic_heights between and after the split step phases
        self.measure_heights = bool(cfg.terrain.measure_heights)
        sd = getattr(cfg.env, "state_dtype", "fp32")
        if sd not in ("fp32", "fp16"):
            raise ValueError(f"cfg.env.state_dtype must be 'fp32' or 'fp16', got {sd!r}")
        self.obs_dtype = torch.float16 if sd == "fp16" else torch.float32
        if self.obs_dtype == torch.float16 and self.measure_heights:
            raise NotImplementedError("fp16 histories (state_dtype='fp16') with measure_heights=True")
        self.env_offset = int(env_offset)
        self.num_envs_total = int(num_envs_total) if num_envs_total is not None else N
        self.dt = cfg.control.decimation * self.sim_params.dt
        self.max_episode_length_s = cfg.env.episode_length_s
        self.max_episode_length = np.ceil(self.max_episode_length_s / self.dt)
        self.obs_scales = cfg.normalization.obs_scales
        if cfg.terrain.mesh_type not in ("heightfield", "trimesh"):
            cfg.terrain.curriculum = False
        self.mesh_type = cfg.terrain.mesh_type
        self.command_ranges = class_to_dict(cfg.commands.ranges)
        dr = cfg.domain_rand
        self.push_interval = np.ceil(dr.push_interval_s / self.dt)
        self.ext_force_interval = np.ceil(dr.ext_force_interval_s / self.dt)
        scales = {k: v for k, v in class_to_dict(cfg.rewards.scales).items() if v != 0}
        unknown = set(scales) - set(REWARD_NAMES)
        if unknown:
            raise NotImplementedError(f"reward terms without a HIP kernel: {sorted(unknown)}")
        self.reward_scales = {k: v * self.dt for k, v in scales.items()}
        self.reward_names = [k for k in REWARD_NAMES if k in self.reward_scales]
        self.common_step_counter = 0
        self.is_first_add_force = True
        self.is_first_push = True
        self.init_done = False
        self._alloc(N)
        self._model = self._build_model(urdf_path)
        self._terrain = None
        self._setup_terrain()
        self._cfg = self._build_config()
        self._bufs = self._build_buffers()
        handle = _lib.C.c_void_p()
        _lib.check(lib.t1env_create(_lib.C.byref(self._model), _lib.C.byref(self._cfg), _lib.C.byref(self._bufs),
                                    _lib.C.byref(handle)), "t1env_create")
        self._handle = handle
        self._lib = lib
        if self._terrain is not None:
            hf = self.height_samples
            _lib.check(lib.t1env_set_terrain(handle, _ptr(hf), hf.shape[0], hf.shape[1], self.cfg.terrain.horizontal_scale,
                                             self.cfg.terrain.vertical_scale, float(self.cfg.terrain.border_size),
                                             2 if self.mesh_type == "trimesh" else 1), "t1env_set_terrain")
        _lib.check(lib.t1env_init(handle, self._stream()), "t1env_init")
        self.extras = {}
        self._ep_dicts = None
        self._slot = 0
        self.init_done = True

    # ------------------------------------------------------------------------------------------- setup
    def _alloc(self, N):
        d, f, i64, i32, b = self.device, torch.float32, torch.int64, torch.int32, torch.bool
        z = lambda *s, dtype=f: torch.zeros(*s, dtype=dtype, device=d)  # noqa: E731
        self.root_states = z(N, 13)
        self.dof_state = z(N * 12, 2)
        self.rigid_state = z(N, 13, 13)
        self.contact_forces = z(N, 13, 3)
        # obs / critic histories: fp32 (the reference's), or fp16 storage with cfg.env.state_dtype = "fp16"
        # (BASELINE config 5; computed in fp32, rounded once; the runner's RolloutStorage converts on copy)
        h = self.obs_dtype
        self._obs = [z(N, self.num_obs, dtype=h), z(N, self.num_obs, dtype=h)]
        self._priv = [z(N, self.num_privileged_obs, dtype=h), z(N, self.num_privileged_obs, dtype=h)]
        self.rew_buf = z(N)
        self.reset_buf = torch.ones(N, dtype=b, device=d)
        self.time_out_buf = z(N, dtype=b)
        self._episode_length_buf = z(N, dtype=i64)
        self.phase_length_buf = z(N, dtype=i64)
        self.commands = z(N, 4)
        for name in ("torques", "actions", "last_actions", "last_last_actions", "last_dof_vel", "ref_dof_pos",
                     "randomized_p_gains", "randomized_d_gains", "motor_offsets", "randomized_joint_coulomb",
                     "randomized_joint_viscous", "joint_armatures", "link_mass_scale"):
            setattr(self, name, z(N, 12))
        self.last_root_vel = z(N, 6)
        for name in ("base_lin_vel", "base_ang_vel", "projected_gravity", "base_euler_xyz", "ext_forces",
                     "ext_torques", "applied_force", "com_displacements", "env_origins"):
            setattr(self, name, z(N, 3))
        self.feet_euler_xyz = z(N, 2, 3)
        self.feet_air_time, self.feet_height, self.last_feet_z = z(N, 2), z(N, 2), z(N, 2)
        self.last_contacts = z(N, 2, dtype=b)
        self.gait_time = z(N, 3, dtype=i32)
        self.gait_start = z(N)
        self._episode_sums = z(len(REWARD_NAMES), N)
        self.episode_sums = {k: self._episode_sums[i] for i, k in enumerate(REWARD_NAMES) if k in self.reward_scales}
        self.env_frictions, self.restitution_coeffs, self.body_mass = z(N, 1), z(N, 1), z(N, 1)
        self.lag_timestep, self.dof_lag_timestep, self.imu_lag_timestep = z(N, dtype=i32), z(N, dtype=i32), z(N, dtype=i32)
        self._act_hist, self._dof_hist, self._imu_hist = z(N, 4, 12), z(N, 4, 24), z(N, 2, 8)
        self.terrain_levels, self.terrain_types = z(N, dtype=i32), z(N, dtype=i32)
        self.terrain_origins = z(1, 1, 3)
        self._extras_ring = torch.full((EXTRAS_RING, 32), float("nan"), device=d)
        self.contact_vimp = z(N, 6)   # restitution episodes of the contact bodies (include/t1env.h)
        self._ep_accum = z(32)
        # views mirroring the reference's attribute names
        self.dof_pos = self.dof_state.view(N, 12, 2)[..., 0]
        self.dof_vel = self.dof_state.view(N, 12, 2)[..., 1]
        self.base_quat = self.root_states[:, 3:7]
        self.torque_multi = torch.ones(N, 12, device=d)
        self.measured_heights = 0      # legged_robot.py:210
        if self.measure_heights:
            t = self.cfg.terrain
            gx, gy = np.meshgrid(np.array(t.measured_points_x, np.float32), np.array(t.measured_points_y, np.float32),
                                 indexing="ij")                      # _init_height_points (legged_robot.py:1535-1549)
            pts = np.stack([gx.ravel(), gy.ravel()], 1)
            self.num_height_points = pts.shape[0]
            self._height_pts = torch.tensor(pts, device=d).contiguous()
            self.height_points = torch.zeros(N, self.num_height_points, 3, device=d)
            self.height_points[:, :, :2] = self._height_pts
            self.measured_heights = z(N, self.num_height_points)
            w = self.cfg.env.c_frame_stack * (self.cfg.env.single_num_privileged_obs + self.num_height_points)
            self._priv_ext = [z(N, w), z(N, w)]

    def _build_model(self, urdf_path):
        cfg = self.cfg
        m, tab, default, kp, kd = build_model(cfg, urdf_path)
        self.dof_names = tab["dof_names"]
        self.body_names = tab["body_names"]
        self.num_dof = self.num_dofs = 12
        self.num_bodies = 13
        d = self.device
        self.default_dof_pos = torch.tensor(default, device=d).unsqueeze(0)
        self.default_joint_pd_target = self.default_dof_pos.clone()
        self.p_gains = torch.tensor(kp, device=d)
        self.d_gains = torch.tensor(kd, device=d)
        self.torque_limits = torch.tensor([m.torque_limit[j] for j in range(12)], device=d)
        self.dof_pos_limits = torch.tensor([[m.q_lower[j], m.q_upper[j]] for j in range(12)], device=d)
        self.dof_vel_limits = torch.tensor([m.vel_limit[j] for j in range(12)], device=d)
        names = self.body_names
        idx = lambda sub: torch.tensor([names.index(n) for n in names if sub in n], dtype=torch.long, device=d)  # noqa
        self.feet_indices = idx(cfg.asset.foot_name)
        self.knee_indices = idx(cfg.asset.knee_name)
        self.termination_contact_indices = torch.cat([idx(s) for s in cfg.asset.terminate_after_contacts_on])
        self.penalised_contact_indices = torch.cat([idx(s) for s in cfg.asset.penalize_contacts_on])
        if self.feet_indices.tolist() != [6, 12] or self.knee_indices.tolist() != [4, 10] or \
                self.termination_contact_indices.tolist() != [0] or self.penalised_contact_indices.tolist() != [0]:
            raise ValueError("the HIP reward/termination kernels assume feet [6,12], knees [4,10], base [0]")
        return m

    def _setup_terrain(self):
        cfg = self.cfg.terrain
        N, d = self.num_envs, self.device
        if self.mesh_type in ("heightfield", "trimesh"):
            self._terrain = Terrain(cfg, self.num_envs_total)
            self.terrain = self._terrain
            self.height_samples = torch.tensor(self._terrain.heightsamples, dtype=torch.int16, device=d)
            self.terrain_origins = torch.tensor(self._terrain.env_origins, dtype=torch.float32, device=d)
            self.custom_origins = True
        elif self.mesh_type == "plane":
            self.custom_origins = False
            nc = np.floor(np.sqrt(self.num_envs_total))
            nr = np.ceil(self.num_envs_total / nc)
            xx, yy = np.meshgrid(np.arange(nr), np.arange(nc), indexing="ij")
            g = np.arange(N) + self.env_offset
            org = np.zeros((N, 3), np.float32)
            org[:, 0] = self.cfg.env.env_spacing * xx.flatten()[g]
            org[:, 1] = self.cfg.env.env_spacing * yy.flatten()[g]
            self.env_origins.copy_(torch.from_numpy(org))
        else:
            raise ValueError("Terrain mesh type not recognised. Allowed types are [None, plane, heightfield, trimesh]")

    def _build_config(self):
        cfg = self.cfg
        c = _lib.Config()
        dr = cfg.domain_rand
        c.num_envs, c.env_offset, c.num_envs_total = self.num_envs, self.env_offset, self.num_envs_total
        c.seed = int(getattr(cfg, "seed", 5)) & 0xFFFFFFFF
        c.sim_dt, c.decimation = self.sim_params.dt, cfg.control.decimation
        c.action_scale = cfg.control.action_scale
        c.clip_actions, c.clip_obs = cfg.normalization.clip_actions, cfg.normalization.clip_observations
        c.max_episode_length, c.episode_length_s = float(self.max_episode_length), float(cfg.env.episode_length_s)
        c.cycle_time = cfg.rewards.cycle_time
        c.stand_com_threshold = cfg.commands.stand_com_threshold
        c.target_joint_pos_scale = cfg.rewards.target_joint_pos_scale
        c.noise_level = cfg.noise.noise_level if cfg.noise.add_noise else 0.0
        ns, os_ = cfg.noise.noise_scales, self.obs_scales
        nv = np.zeros(47, np.float32)      # _get_noise_scale_vec (t1_dh_stand_env.py:326-357)
        nv[5:17] = ns.dof_pos * os_.dof_pos
        nv[17:29] = ns.dof_vel * os_.dof_vel
        nv[41:44] = ns.ang_vel * os_.ang_vel
        nv[44:47] = ns.quat * os_.quat
        self.noise_scale_vec = torch.tensor(nv, device=self.device)
        for i in range(47):
            c.noise_vec[i] = nv[i]
        for i, k in enumerate(REWARD_NAMES):
            c.reward_scales[i] = self.reward_scales.get(k, 0.0)
        r = cfg.rewards
        c.only_positive_rewards = int(r.only_positive_rewards)
        for k in ("base_height_target", "foot_min_dist", "foot_max_dist", "knee_min_dist", "knee_max_dist",
                  "target_feet_height", "target_feet_height_max", "tracking_sigma", "max_contact_force"):
            setattr(c, k, getattr(r, k))
        gait = cfg.commands.gait
        if len(gait) != 3:
            raise NotImplementedError("the HIP command scheduler supports exactly 3 gait slots")
        for i, g in enumerate(gait):
            c.gait_kind[i] = GAIT_KINDS[g]
            c.gait_time_range[i][0], c.gait_time_range[i][1] = cfg.commands.gait_time_range[g]
        c.ext_force_max[0], c.ext_force_max[1], c.ext_force_max[2] = dr.ext_force_max_x, dr.ext_force_max_y, dr.ext_force_max_z
        c.ext_torque_max = dr.ext_torque_max
        c.push_vel_xy, c.push_ang = dr.max_push_vel_xy, dr.max_push_ang_vel
        if getattr(dr, "add_dof_pos_vel_lag", False) or dr.randomize_lag_timesteps_perstep or \
                dr.randomize_dof_lag_timesteps_perstep or dr.randomize_imu_lag_timesteps_perstep:
            raise NotImplementedError("per-step lag redraws / split pos-vel lag are not on the t1_dh_stand path")

        def lag(flag, rnd, rng):
            if not flag:
                return (0, 0)
            return tuple(rng) if rnd else (rng[1], rng[1])
        c.lag_range[0], c.lag_range[1] = lag(dr.add_lag, dr.randomize_lag_timesteps, dr.lag_timesteps_range)
        c.dof_lag_range[0], c.dof_lag_range[1] = lag(dr.add_dof_lag, dr.randomize_dof_lag_timesteps, dr.dof_lag_timesteps_range)
        c.imu_lag_range[0], c.imu_lag_range[1] = lag(dr.add_imu_lag, dr.randomize_imu_lag_timesteps, dr.imu_lag_timesteps_range)

        def rng(flag, r_, one):
            return tuple(r_) if flag else (one, one)
        c.torque_mult_range[:] = rng(dr.randomize_torque, dr.torque_multiplier_range, 1.0)
        c.motor_offset_range[:] = rng(dr.randomize_motor_offset, dr.motor_offset_range, 0.0)
        c.kp_mult_range[:] = rng(dr.randomize_gains, dr.stiffness_multiplier_range, 1.0)
        c.kd_mult_range[:] = rng(dr.randomize_gains, dr.damping_multiplier_range, 1.0)
        c.coulomb_range[:] = rng(dr.randomize_coulomb_friction, dr.joint_coulomb_range, 0.0)
        c.viscous_range[:] = rng(dr.randomize_coulomb_friction, dr.joint_viscous_range, 0.0)
        for j in range(12):
            if dr.randomize_joint_armature:
                rr = getattr(dr, f"joint_{j + 1}_armature_range") if dr.randomize_joint_armature_each_joint \
                    else dr.joint_armature_range
            else:
                rr = (0.0, 0.0)
            c.armature_range[j][0], c.armature_range[j][1] = rr
        c.reset_dof_range = 0.1
        c.terrain_curriculum = int(bool(cfg.terrain.curriculum) and self.custom_origins)
        c.platform = float(getattr(cfg.terrain, "platform", 3.0))
        c.env_length = float(cfg.terrain.terrain_length)
        c.num_terrain_rows = int(cfg.terrain.num_rows)
        c.num_terrain_cols = int(cfg.terrain.num_cols)
        c.lin_vel_obs_scale, c.ang_vel_obs_scale = os_.lin_vel, os_.ang_vel
        c.dof_pos_obs_scale, c.dof_vel_obs_scale, c.quat_obs_scale = os_.dof_pos, os_.dof_vel, os_.quat
        c.dr_base_mass, c.dr_link_mass = int(dr.randomize_base_mass), int(dr.randomize_link_mass)
        c.dr_com, c.dr_friction = int(dr.randomize_com), int(dr.randomize_friction)
        c.added_mass_range[:] = dr.added_mass_range
        c.link_mass_range[:] = dr.added_link_mass_range
        for k in range(3):
            c.com_range[k][0], c.com_range[k][1] = dr.com_displacement_range[k]
        c.friction_range[:] = dr.friction_range
        c.restitution_range[:] = dr.restitution_range
        c.custom_origins = int(self.custom_origins)
        c.max_init_terrain_level = int(cfg.terrain.max_init_terrain_level if cfg.terrain.curriculum
                                       else cfg.terrain.num_rows - 1)
        c.reset_xy_range = (c.platform / 3 if cfg.terrain.curriculum else cfg.terrain.terrain_length / 2) \
            if self.custom_origins else 0.0
        c.obs_half = int(self.obs_dtype == torch.float16)
        self.max_terrain_level = cfg.terrain.num_rows
        return c

    def _build_buffers(self):
        b = _lib.Buffers()
        P = _lib.C.cast
        fp, u8p, i32p, i64p = _lib.fp, _lib.u8p, _lib.i32p, _lib.i64p
        m = {
            "root_states": self.root_states, "dof_state": self.dof_state, "rigid_state": self.rigid_state,
            "contact_forces": self.contact_forces, "rew_buf": self.rew_buf, "reset_buf": self.reset_buf,
            "time_out_buf": self.time_out_buf, "episode_length_buf": self._episode_length_buf,
            "phase_length_buf": self.phase_length_buf, "commands": self.commands, "torques": self.torques,
            "actions": self.actions, "last_actions": self.last_actions, "last_last_actions": self.last_last_actions,
            "last_dof_vel": self.last_dof_vel, "last_root_vel": self.last_root_vel, "base_lin_vel": self.base_lin_vel,
            "base_ang_vel": self.base_ang_vel, "projected_gravity": self.projected_gravity,
            "base_euler_xyz": self.base_euler_xyz, "feet_euler_xyz": self.feet_euler_xyz,
            "feet_air_time": self.feet_air_time, "last_contacts": self.last_contacts, "feet_height": self.feet_height,
            "last_feet_z": self.last_feet_z, "ref_dof_pos": self.ref_dof_pos, "gait_time": self.gait_time,
            "gait_start": self.gait_start, "ext_forces": self.ext_forces, "ext_torques": self.ext_torques,
            "applied_force": self.applied_force, "episode_sums": self._episode_sums, "kp": self.randomized_p_gains,
            "kd": self.randomized_d_gains, "motor_offsets": self.motor_offsets, "coulomb": self.randomized_joint_coulomb,
            "viscous": self.randomized_joint_viscous, "armature": self.joint_armatures, "friction": self.env_frictions,
            "restitution": self.restitution_coeffs, "body_mass": self.body_mass, "link_mass_scale": self.link_mass_scale,
            "com_disp": self.com_displacements, "lag_timestep": self.lag_timestep,
            "dof_lag_timestep": self.dof_lag_timestep, "imu_lag_timestep": self.imu_lag_timestep,
            "act_hist": self._act_hist, "dof_hist": self._dof_hist, "imu_hist": self._imu_hist,
            "env_origins": self.env_origins, "terrain_levels": self.terrain_levels, "terrain_types": self.terrain_types,
            "terrain_origins": self.terrain_origins, "extras": self._extras_ring, "ep_accum": self._ep_accum,
            "contact_vimp": self.contact_vimp,
        }
        types = dict(_lib.BUFFER_FIELDS)
        for name, t in m.items():
            assert t.is_contiguous() and t.device == self.device, name
            setattr(b, name, P(t.data_ptr(), types[name]))
        for k in range(2):
            b.obs_buf[k] = P(self._obs[k].data_ptr(), fp)
            b.priv_buf[k] = P(self._priv[k].data_ptr(), fp)
        self._keepalive = m
        return b

    # ------------------------------------------------------------------------------------------- API
    @property
    def episode_length_buf(self):
        return self._episode_length_buf

    @episode_length_buf.setter
    def episode_length_buf(self, v):   # the runner rebinds it (dh_on_policy_runner.py:101): copy in place
        self._episode_length_buf.copy_(torch.as_tensor(v, device=self.device).to(torch.int64))

    @property
    def obs_buf(self):
        return self._obs[self._slot ^ 1]

    @property
    def privileged_obs_buf(self):
        if self.measure_heights:   # (N, 3 * (73 + 187)): the critic history with heights
            return self._priv_ext[self._slot ^ 1]
        return self._priv[self._slot ^ 1]

    def get_observations(self):
        return self.obs_buf

    def get_privileged_observations(self):
        return self.privileged_obs_buf

    def _stream(self):
        return _lib.C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _schedule(self):
        """Host-side callback schedule for this step (t1_dh_stand_env.py:193-215): no device data needed."""
        dr = self.cfg.domain_rand
        ctr_post = self.common_step_counter + 1
        ext_call = ext_first = push_call = 0
        if dr.add_ext_force:
            i = min(int(ctr_post / dr.add_update_step), len(dr.add_duration) - 1)
            if ctr_post % self.ext_force_interval <= dr.add_duration[i] / self.dt:
                ext_call, ext_first = 1, int(self.is_first_add_force)
                self.is_first_add_force = False
            else:
                self.is_first_add_force = True
        if dr.push_robots:
            i = min(int(ctr_post / dr.update_step), len(dr.push_duration) - 1)
            if ctr_post % self.push_interval <= dr.push_duration[i] / self.dt:
                push_call = 1
            else:
                self.is_first_push = True
        return ext_call, ext_first, push_call

    def _args(self, counter, ext_call=0, ext_first=0, push_call=0):
        a = _lib.StepArgs()
        a.counter = counter & 0xFFFFFFFF
        a.obs_slot = self._slot
        a.ext_force_call, a.ext_force_first, a.push_call = ext_call, ext_first, push_call
        for i, k in enumerate(("lin_vel_x", "lin_vel_y", "ang_vel_yaw")):
            a.cmd_ranges[i][0], a.cmd_ranges[i][1] = self.command_ranges[k]
        return a

    def _command_curriculum(self, sums, count):
        """update_command_curriculum (legged_robot.py:1160-1169), evaluated on the host once per episode length."""
        if not self.cfg.commands.curriculum or "tracking_lin_vel" not in self.reward_scales:
            return
        if torch.distributed.is_available() and torch.distributed.is_initialized() and \
                torch.distributed.get_world_size() > 1:
            # sharded envs: the mean runs over every rank's resetting envs, so all ranks keep
            # identical command ranges; every rank calls this at the same step counter
            dev = self.device if torch.distributed.get_backend() == "nccl" else torch.device("cpu")
            t = torch.tensor([sums, count], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(t)
            sums, count = float(t[0]), float(t[1])
        if count <= 0:
            return
        if sums / count / self.max_episode_length > 0.8 * self.reward_scales["tracking_lin_vel"]:
            r = self.command_ranges["lin_vel_x"]
            r[0] = float(np.clip(r[0] - 0.25, -self.cfg.commands.max_curriculum / 2, 0.0))
            r[1] = float(np.clip(r[1] + 0.5, 0.0, self.cfg.commands.max_curriculum))

    def step(self, actions, _injected=None):
        """LeggedRobot.step (legged_robot.py:387-448) + T1 overrides; returns the reference's 5-tuple."""
        if actions.device != self.device or actions.dtype != torch.float32 or not actions.is_contiguous():
            actions = actions.to(self.device, torch.float32).contiguous()
        if actions.shape != (self.num_envs, self.num_actions):
            raise ValueError(f"actions must be ({self.num_envs}, {self.num_actions}), got {tuple(actions.shape)}")
        if self.cfg.env.use_ref_actions:
            raise NotImplementedError("use_ref_actions=True is not on the t1_dh_stand path")
        lib, h, s = self._lib, self._handle, self._stream()
        ext_call, ext_first, push_call = self._schedule()
        a = self._args(self.common_step_counter, ext_call, ext_first, push_call)
        ctr_post = self.common_step_counter + 1
        needs_curriculum = self.cfg.commands.curriculum and ctr_post % self.max_episode_length == 0
        if _injected is None and not needs_curriculum and not self.measure_heights:
            _lib.check(lib.t1env_step(h, _ptr(actions), _lib.C.byref(a), s), "t1env_step")
        else:
            if _injected is None:
                _lib.check(lib.t1env_step_physics_and_rewards(h, _ptr(actions), _lib.C.byref(a), s), "physics")
            else:
                _lib.check(lib.t1env_step_injected(h, _ptr(actions), _lib.C.byref(a), _lib.C.byref(_injected), s),
                           "t1env_step_injected")
            if self.measure_heights:   # the callback's _get_heights, before reset_idx (t1_dh_stand_env.py:190)
                _lib.check(lib.t1env_measure_heights(h, _ptr(self._height_pts), self.num_height_points,
                                                     _ptr(self.measured_heights), s), "t1env_measure_heights")
            if needs_curriculum:
                idx = REWARD_NAMES.index("tracking_lin_vel")
                acc = self._ep_accum.cpu()
                self._command_curriculum(float(acc[idx]), float(acc[24]))
                a = self._args(self.common_step_counter, ext_call, ext_first, push_call)
            _lib.check(lib.t1env_step_reset_and_observe(h, _lib.C.byref(a), s), "t1env_step_reset_and_observe")
            if self.measure_heights:
                _lib.check(lib.t1env_critic_heights(h, self._slot, self.num_height_points,
                                                    float(self.obs_scales.height_measurements),
                                                    _ptr(self.measured_heights), _ptr(self._priv_ext[self._slot ^ 1]),
                                                    _ptr(self._priv_ext[self._slot]), s), "t1env_critic_heights")
        self.common_step_counter += 1
        self._slot ^= 1
        self._fill_extras(self.common_step_counter % EXTRAS_RING)
        return self.obs_buf, self.privileged_obs_buf, self.rew_buf, self.reset_buf, self.extras

    def _fill_extras(self, slot):
        """extras["episode"] for the ring slot the library just wrote (0-d views, valid for EXTRAS_RING steps --
        the runner logs every num_steps_per_env = 24); the dicts are built once, a step only picks one."""
        if self._ep_dicts is None:
            self._ep_dicts = []
            for r in range(EXTRAS_RING):
                ex = self._extras_ring[r]
                ep = {"rew_" + k: ex[REWARD_NAMES.index(k)] for k in self.reward_names}
                if self.mesh_type == "trimesh":
                    ep["terrain_level"] = ex[24]
                self._ep_dicts.append(ep)
        ep = self._ep_dicts[slot]
        if self.cfg.commands.curriculum:
            ep["max_command_x"] = self.command_ranges["lin_vel_x"][1]
        self.extras["episode"] = ep
        if self.cfg.env.send_timeouts:
            self.extras["time_outs"] = self.time_out_buf

    def reset_idx_all(self):
        """reset_idx(arange(num_envs)) (t1_dh_stand_env.py:483-559)."""
        if self.cfg.commands.curriculum and self.common_step_counter % self.max_episode_length == 0 and \
                "tracking_lin_vel" in self.episode_sums:
            self._command_curriculum(float(self.episode_sums["tracking_lin_vel"].sum()), float(self.num_envs))
        a = self._args(self.common_step_counter)
        _lib.check(self._lib.t1env_reset_all(self._handle, _lib.C.byref(a), self._stream()), "t1env_reset_all")
        if self.measure_heights:   # reset_idx clears the critic history deque (t1_dh_stand_env.py:548-558)
            for t in self._priv_ext:
                t.zero_()
        self._fill_extras(self.common_step_counter % EXTRAS_RING)

    def reset_idx(self, env_ids):
        """reset_idx(env_ids) between steps (t1_dh_stand_env.py:483-559): the same per-env reset as a step's, keyed by
        common_step_counter; extras["episode"] = means over env_ids.  The cleared history rows are zeroed in the
        buffer the next step shifts from, i.e. in place in the current obs_buf / privileged_obs_buf (the
        reference's stacked obs_buf keeps the old rows until the next step)."""
        ids = torch.as_tensor(env_ids, device=self.device, dtype=torch.long).flatten()
        if ids.numel() == 0:
            return
        if self.cfg.commands.curriculum and self.common_step_counter % self.max_episode_length == 0 and \
                "tracking_lin_vel" in self.episode_sums:
            self._command_curriculum(float(self.episode_sums["tracking_lin_vel"][ids].sum()), float(ids.numel()))
        mask = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
        mask[ids] = 1
        a = self._args(self.common_step_counter)
        a.obs_slot = self._slot ^ 1   # the buffer holding the current observations
        _lib.check(self._lib.t1env_reset_idx(self._handle, _ptr(mask), _lib.C.byref(a), self._stream()),
                   "t1env_reset_idx")
        if self.measure_heights:
            self._priv_ext[self._slot ^ 1][ids] = 0.0
        self._fill_extras(self.common_step_counter % EXTRAS_RING)

    def reset(self):
        """LeggedRobot.reset (legged_robot.py:450-455)."""
        self.reset_idx_all()
        obs, priv, _, _, _ = self.step(torch.zeros(self.num_envs, self.num_actions, device=self.device))
        return obs, priv

    def set_fused(self, enable=True):
        """t1env_step as one fused launch (default) or the split kernel sequence (same results; tests)."""
        _lib.check(self._lib.t1env_set_fused(self._handle, int(bool(enable))), "t1env_set_fused")

    def set_substep_log(self, enable=True):
        """Test hook (t1env_set_substep_log): every following fused step also writes its per-substep root / dof
        states and torques to ``self.substep_log`` = dict(root (dec, N, 13), dof (dec, N, 12, 2), torque (dec, N, 12)),
        the states the reference's post-simulate code would see.  Split steps (command curriculum, height scan)
        raise while it is on."""
        if not enable:
            _lib.check(self._lib.t1env_set_substep_log(self._handle, None), "t1env_set_substep_log")
            self.substep_log = None
            return
        dec, N, d = self.cfg.control.decimation, self.num_envs, self.device
        self.substep_log = dict(root=torch.zeros(dec, N, 13, device=d), dof=torch.zeros(dec, N, 12, 2, device=d),
                                torque=torch.zeros(dec, N, 12, device=d))
        lg = _lib.SubstepLog()
        for k, t in self.substep_log.items():
            setattr(lg, k, _lib.C.cast(t.data_ptr(), _lib.fp))
        _lib.check(self._lib.t1env_set_substep_log(self._handle, _lib.C.byref(lg)), "t1env_set_substep_log")

    def set_timing(self, enable=True, reset=True):
        """Record HIP events around every kernel launch (bench.py's live per-kernel timing).  reset=False keeps
        the events recorded so far (bench.py samples every k-th step)."""
        _lib.check(self._lib.t1env_set_timing(self._handle, int(enable) | (0 if reset else 2)), "t1env_set_timing")

    def get_timing(self):
        names = ["k_dynamics", "k_post_a", "k_post_b", "k_shift", "unused", "step"]  # include/t1env.h timers
        ms = (_lib.C.c_double * len(names))()
        n = (_lib.C.c_int32 * len(names))()
        _lib.check(self._lib.t1env_get_timing(self._handle, ms, n), "t1env_get_timing")
        return {k: {"ms": ms[i], "launches": n[i]} for i, k in enumerate(names)}

    def render(self, sync_frame_time=True):
        return None

    def set_camera(self, position, lookat):
        return None

    def close(self):
        if getattr(self, "_handle", None) is not None:
            self._lib.t1env_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
