"""CPU restatement (numpy, fp32) of the reference's ``T1DHStandEnv.step()`` hot path.

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the CPU baseline -- never as the product path.

Follows, function by function (file:line in /root/reference):
  LeggedRobot.step                      humanoid/envs/base/legged_robot.py:387-448
  LeggedRobot._compute_torques          legged_robot.py:1019-1074
  sensor lag pushes                     legged_robot.py:412-434
  LeggedRobot.post_physics_step         legged_robot.py:458-506
  get_euler_xyz_tensor                  legged_robot.py:27-53
  T1._post_physics_step_callback        humanoid/envs/t1/t1_dh_stand_env.py:179-215
  T1._add_ext_force / _push_robots      t1_dh_stand_env.py:217-247
  LeggedRobot.check_termination         legged_robot.py:509-517
  LeggedRobot.compute_reward            legged_robot.py:654-680 (24 _reward_* in t1_dh_stand_env.py:576-935)
  T1.reset_idx                          t1_dh_stand_env.py:483-559 (+ legged_robot.py:604-651, 732-783,
                                        1076-1120, 1138-1169)
  T1.compute_observations               t1_dh_stand_env.py:368-481 (+ _get_phase 80-92, compute_ref_state
                                        250-274, _get_gait_phase 95-107, generate_gait_time 109-124)
  height scan (measure_heights=True;    legged_robot.py:1535-1587 (_init_height_points, _get_heights),
    inactive in DHT1StandCfg)           utils/math.py:8-12 (quat_apply_yaw), t1_dh_stand_env.py:190-191,
                                        466-468 (callback, critic-obs concatenation)
Physics (Isaac Gym ``simulate``) is not part of the oracle: it is injected through ``physics(g, torques,
state)`` so the same oracle serves the injected-state parity tests and the CPU baseline (with the CPU
build of the dynamics plugged in).  Random draws come from oracle/rng.py (see its docstring).
Constants are the DHT1StandCfg defaults (humanoid/envs/t1/t1_dh_stand_config.py) unless overridden.
"""
import numpy as np

from . import rng as R

f32 = np.float32
PI = np.pi

# ---- DHT1StandCfg constants (t1_dh_stand_config.py) -------------------------------------------------
NUM_ACTIONS = 12
NUM_BODIES = 13
FRAME_STACK = 66          # :10
C_FRAME_STACK = 3         # :12
NUM_SINGLE_OBS = 47       # :15
SINGLE_PRIV = 73          # :21
DECIMATION = 10           # :155
SIM_DT = 0.001            # :160
DT = DECIMATION * SIM_DT  # legged_robot.py:96
EPISODE_S = 24            # :30
MAX_EPISODE_LEN = float(np.ceil(EPISODE_S / DT))  # legged_robot.py:109 -> 2400
ACTION_SCALE = 0.5        # :153
CLIP_ACTIONS = 100.0      # :426
CLIP_OBS = 100.0          # :424
Q0 = np.array([0, 0, -0.3, 0.6, -0.3, 0] * 2, dtype=f32)           # :124-141
KP = np.array([50, 70, 90, 120, 50, 30] * 2, dtype=f32)            # :147-148
KD = np.array([5, 7, 9, 12, 5, 3] * 2, dtype=f32)                  # :149-150
EFFORT = np.array([102, 102, 267, 267, 80, 40, 102, 102, 267, 267, 80, 40.2], dtype=f32)  # t1.urdf limits
TORQUE_LIMITS = (EFFORT * f32(0.85)).astype(f32)                    # legged_robot.py:849, cfg safety :40
FEET = (6, 12)
KNEES = (4, 10)
BASE = 0
OBS_SCALES = dict(lin_vel=2.0, ang_vel=1.0, dof_pos=1.0, dof_vel=0.05, quat=1.0)  # :412-419
NOISE_LEVEL = 1.5         # :113
CYCLE_TIME = 0.8          # :370
STAND_THRESH = 0.05       # :339
GAIT = ("walk_omnidirectional", "stand", "walk_omnidirectional")   # :327
GAIT_RANGE = {"walk_omnidirectional": (4, 6), "stand": (2, 3)}     # :329-334
EXT_FORCE_MAX = (600.0, 400.0, 5.0)   # :197-199
EXT_TORQUE_MAX = 0.0                  # :200
EXT_INTERVAL = float(np.ceil(4 / DT))     # legged_robot.py:113 -> 400
ADD_UPDATE_STEP = 4000 * 24               # :202
ADD_DURATION = (0.0, 0.05, 0.1, 0.15)     # :203
PUSH_INTERVAL_S = 6                       # :190 (push_robots = False by default, :188)
PUSH_UPDATE_STEP = 2500 * 24              # :191
PUSH_DURATION = (0, 0.05, 0.1, 0.15, 0.2, 0.25, 0.3)  # :192
MAX_PUSH_VEL_XY = 0.2                     # :193
MAX_PUSH_ANG_VEL = 0.2                    # :194
ARMATURE_RANGE = [(0.15 * 0.8, 0.15 * 1.2), (0.15 * 0.8, 0.15 * 1.2), (3.6 * 0.5, 3.6 * 1.0),
                  (3.6 * 0.5, 3.6 * 1.0), (0.1 * 0.5, 0.1 * 1.1), (0.028 * 0.5, 0.028 * 1.5)] * 2  # :273-285
REWARD_SCALES = dict(joint_pos=4, feet_clearance=1, feet_contact_number=1.2, feet_air_time=1, foot_slip=-0.5,
                     feet_distance=0.2, knee_distance=0.2, feet_rotation=0.8, feet_contact_forces=-0.01,
                     tracking_lin_vel=1.5, tracking_ang_vel=0.8, vel_mismatch_exp=0.5, low_speed=0.2,
                     track_vel_hard=0.5, default_joint_pos=1, orientation=1, base_height=0.2, base_acc=0.2,
                     action_smoothness=-0.03, torques=-2e-7, dof_vel=-2e-5, dof_acc=-5e-7, collision=-1,
                     stand_still=2.5)    # :383-410
REWARD_NAMES = sorted(REWARD_SCALES)    # class_to_dict iterates dir() -> alphabetical (helpers.py:18)
BASE_MASS = 23.644        # base_link 9.999 + collapsed upper body 13.645 (t1.urdf)
HEIGHT_X = [round(-0.8 + 0.1 * i, 1) for i in range(17)]   # legged_robot_config.py:29
HEIGHT_Y = [round(-0.5 + 0.1 * i, 1) for i in range(11)]   # legged_robot_config.py:30
NUM_HEIGHT = len(HEIGHT_X) * len(HEIGHT_Y)                  # 187 (legged_robot_config.py:36)
HEIGHT_OBS_SCALE = 5.0    # obs_scales.height_measurements (t1_dh_stand_config.py:424)


def euler_xyz(q):
    """get_euler_xyz_tensor (legged_robot.py:27-53) on (..., 4) xyzw float32 quaternions."""
    qx, qy, qz, qw = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    sinr = f32(2.0) * (qw * qx + qy * qz)
    cosr = qw * qw - qx * qx - qy * qy + qz * qz
    roll = np.arctan2(sinr, cosr)
    sinp = f32(2.0) * (qw * qy - qz * qx)
    pitch = np.where(np.abs(sinp) >= 1, np.abs(f32(PI / 2)) * np.sign(sinp), np.arcsin(np.clip(sinp, -1, 1)))
    siny = f32(2.0) * (qw * qz + qx * qy)
    cosy = qw * qw + qx * qx - qy * qy - qz * qz
    yaw = np.arctan2(siny, cosy)
    e = np.stack([np.mod(roll, f32(2 * PI)), np.mod(pitch.astype(f32), f32(2 * PI)), np.mod(yaw, f32(2 * PI))], -1)
    e = e.astype(f32)
    return np.where(e > PI, e - f32(2 * PI), e).astype(f32)


def quat_rotate_inverse(q, v):
    """isaacgym.torch_utils.quat_rotate_inverse (third party, parity unpinned)."""
    qw = q[:, 3:4]
    qv = q[:, :3]
    a = v * (f32(2.0) * qw ** 2 - f32(1.0))
    b = np.cross(qv, v) * qw * f32(2.0)
    c = qv * np.sum(qv * v, axis=1, keepdims=True) * f32(2.0)
    return (a - b + c).astype(f32)


def height_points():
    """_init_height_points (legged_robot.py:1535-1549): torch.meshgrid(x, y) ('ij') flattened -> (187, 2) base-frame
    (x, y), point k = ix * 11 + iy."""
    gx, gy = np.meshgrid(np.array(HEIGHT_X, f32), np.array(HEIGHT_Y, f32), indexing="ij")
    return np.stack([gx.ravel(), gy.ravel()], 1).astype(f32)


def get_heights(base_pos, base_quat, pts, height_samples, horizontal_scale, vertical_scale, border_size):
    """_get_heights (legged_robot.py:1551-1587) for all envs on a height field: the points rotated by the base yaw
    (quat_apply_yaw, utils/math.py:8-12: roll/pitch components zeroed, normalised, quat_apply), offset by the base
    position and the border, truncated (`.long()`) to samples, clipped to [0, rows-2] x [0, cols-2], min of the
    sample and its +x and +y neighbours, times vertical_scale.  fp32 as the reference computes it."""
    q = base_quat.astype(f32).copy()
    q[:, :2] = 0
    q = (q / np.maximum(_norm(q)[:, None], f32(1e-9))).astype(f32)            # torch_utils.normalize
    n, m = q.shape[0], pts.shape[0]
    v = np.zeros((n, m, 3), f32)
    v[:, :, :2] = pts[None]
    xyz = np.broadcast_to(q[:, None, :3], v.shape)
    t = (np.cross(xyz, v) * f32(2)).astype(f32)                                 # torch_utils.quat_apply
    p = (v + q[:, None, 3:4] * t + np.cross(xyz, t)).astype(f32)
    p = (p + base_pos[:, None, :3].astype(f32)).astype(f32)
    p = (p + f32(border_size)).astype(f32)
    p = np.trunc(p / f32(horizontal_scale)).astype(np.int64)
    rows, cols = height_samples.shape
    px = np.clip(p[..., 0], 0, rows - 2)
    py = np.clip(p[..., 1], 0, cols - 2)
    hs = height_samples
    h = np.minimum(np.minimum(hs[px, py], hs[px + 1, py]), hs[px, py + 1])
    return (h.astype(f32) * f32(vertical_scale)).astype(f32)


def _norm(x, axis=-1):
    return np.sqrt(np.sum(x * x, axis=axis)).astype(f32)


class T1Oracle:
    """Numpy mirror of T1DHStandEnv's state and step.  ``physics(g, torques, st)`` must return
    (root (N,13), dof (N,12,2), rigid (N,13,13), contact (N,13,3)) after global substep g."""

    def __init__(self, num_envs, seed=5, mesh_type="plane", terrain=None, env_offset=0, reduce_fn=None,
                 measure_heights=False, push_robots=False, push_interval_s=PUSH_INTERVAL_S, terrain_curriculum=True):
        """reduce_fn: sharded runs only -- (sum, count) -> (sum, count) over all ranks, so the command
        curriculum sees the same mean as an unsharded run.  measure_heights: the height scan
        (inactive in DHT1StandCfg): 187 heights appended to every critic frame (260 per frame).  push_robots /
        push_interval_s: domain_rand.push_robots (off in DHT1StandCfg, on in BASELINE config 5).  terrain_curriculum:
        cfg.terrain.curriculum (on in DHT1StandCfg; off: levels drawn over every row, no level updates, start xy
        within terrain_length / 2, legged_robot.py:1103-1108, 1487)."""
        N = num_envs
        self.N, self.seed, self.env_offset = N, int(seed), int(env_offset)
        self.reduce_fn = reduce_fn
        self.ids = np.arange(N, dtype=np.int64) + env_offset
        self.mesh_type = mesh_type
        self.custom_origins = mesh_type in ("heightfield", "trimesh")   # legged_robot.py:1481-1482
        self.curriculum = self.custom_origins and bool(terrain_curriculum)  # legged_robot.py:104-105
        self.command_ranges = dict(lin_vel_x=[-0.5, 0.5], lin_vel_y=[-0.5, 0.5], ang_vel_yaw=[-0.5, 0.5])
        self.reward_scales = {k: v * DT for k, v in REWARD_SCALES.items()}   # legged_robot.py:357-364
        self.noise_vec = np.zeros(NUM_SINGLE_OBS, f32)                       # t1_dh_stand_env.py:326-357
        self.noise_vec[5:17] = f32(0.02 * OBS_SCALES["dof_pos"])
        self.noise_vec[17:29] = f32(1.5 * OBS_SCALES["dof_vel"])
        self.noise_vec[41:44] = f32(0.2 * OBS_SCALES["ang_vel"])
        self.noise_vec[44:47] = f32(0.1 * OBS_SCALES["quat"])
        self.common_step_counter = 0
        self._key_salt = 0         # R.BETWEEN_STEP_SALT while reset_idx runs between steps
        self.substep_counter = 0
        self.push_robots = bool(push_robots)
        self.push_interval = float(np.ceil(push_interval_s / DT))          # legged_robot.py:112
        # creation-time DR (legged_robot.py:692-730, 786-824, 852-885)
        self.payload = R.rand_float(-2.5, 2.5, seed, self.ids, 0, R.SLOT_PAYLOAD)
        self.body_mass = (f32(BASE_MASS) + self.payload).astype(f32)
        bucket = R.randint(0, 256, seed, self.ids, 0, R.SLOT_FRICTION_BUCKET)
        fr_b = R.rand_float(0.2, 1.3, seed, np.arange(256), 0, R.SLOT_FRICTION_VALUE)
        re_b = R.rand_float(0.0, 0.4, seed, np.arange(256), 0, R.SLOT_RESTITUTION_VALUE)
        self.friction = fr_b[bucket]
        self.restitution = re_b[bucket]
        self.link_mass_scale = np.stack([R.rand_float(0.9, 1.1, seed, self.ids, 0, R.SLOT_LINK_MASS + b)
                                         for b in range(12)], 1)
        self.com_disp = np.stack([R.rand_float(-0.05, 0.05, seed, self.ids, 0, R.SLOT_COM + k) for k in range(3)], 1)
        # terrain origins (legged_robot.py:1477-1512)
        self.env_origins = np.zeros((N, 3), f32)
        if self.custom_origins:
            t = terrain
            self.num_rows, self.num_cols = t["terrain_origins"].shape[:2]
            self.terrain_origins = t["terrain_origins"].astype(f32)
            self.env_length = float(t.get("env_length", 8.0))
            self.platform = float(t.get("platform", 3.0))
            max_init = int(t.get("max_init_terrain_level", 5)) if self.curriculum else self.num_rows - 1  # :1486-1487
            self.terrain_levels = R.randint(0, max_init + 1, seed, self.ids, 0, R.SLOT_TERRAIN_LEVEL_INIT)
            n_total = int(t.get("num_envs_total", N))
            self.terrain_types = np.floor(self.ids / (n_total / self.num_cols)).astype(np.int64)
            self.max_terrain_level = self.num_rows
            self.env_origins[:] = self.terrain_origins[self.terrain_levels, self.terrain_types]
        else:
            nc = np.floor(np.sqrt(N))
            nr = np.ceil(N / nc)
            xx, yy = np.meshgrid(np.arange(nr), np.arange(nc), indexing="ij")
            self.env_origins[:, 0] = 3.0 * xx.flatten()[:N]
            self.env_origins[:, 1] = 3.0 * yy.flatten()[:N]
        # sim state (Gym tensors)
        self.root = np.zeros((N, 13), f32)
        self.root[:, 6] = 1.0
        # start pose (legged_robot.py:1380-1383): origin + U(-1,1) xy jitter; Gym reports it after prepare_sim
        self.root[:, 0:3] = self.env_origins
        self.root[:, 0] += R.rand_float(-1.0, 1.0, seed, self.ids, 0, R.SLOT_START_XY + 0)
        self.root[:, 1] += R.rand_float(-1.0, 1.0, seed, self.ids, 0, R.SLOT_START_XY + 1)
        self.dof = np.zeros((N, 12, 2), f32)
        self.rigid = np.zeros((N, 13, 13), f32)
        self.rigid[:, :, 6] = 1.0
        self.contact = np.zeros((N, 13, 3), f32)
        # buffers (legged_robot.py:116-349, base_task.py:55-74, t1_dh_stand_env.py:72-77, 562-569)
        z = lambda *s: np.zeros(s, f32)  # noqa: E731
        self.obs_buf = z(N, FRAME_STACK * NUM_SINGLE_OBS)
        self.measure_heights = bool(measure_heights)
        self.priv_width = SINGLE_PRIV + (NUM_HEIGHT if self.measure_heights else 0)
        self.terrain = terrain
        self.height_points = height_points()
        self.measured_heights = z(N, NUM_HEIGHT)
        self.priv_buf = z(N, C_FRAME_STACK * self.priv_width)
        self.obs_hist = z(N, FRAME_STACK, NUM_SINGLE_OBS)
        self.priv_hist = z(N, C_FRAME_STACK, self.priv_width)
        self.rew_buf = z(N)
        self.reset_buf = np.ones(N, bool)
        self.time_out_buf = np.zeros(N, bool)
        self.episode_length_buf = np.zeros(N, np.int64)
        self.phase_length_buf = np.zeros(N, np.int64)
        self.gait_time = np.zeros((N, 3), np.int32)
        self.gait_start = R.randint(0, 2, seed, self.ids, 0, R.SLOT_GAIT_START).astype(f32) * f32(0.5)
        self.torques = z(N, 12)
        self.actions, self.last_actions, self.last_last_actions = z(N, 12), z(N, 12), z(N, 12)
        self.last_dof_vel = z(N, 12)
        self.last_root_vel = z(N, 6)
        self.commands = z(N, 4)
        self.feet_air_time = z(N, 2)
        self.last_contacts = np.zeros((N, 2), bool)
        self.feet_height = z(N, 2)
        self.last_feet_z = z(N, 2)
        self.ref_dof_pos = z(N, 12)
        self.ext_forces, self.ext_torques = z(N, 3), z(N, 3)
        self.rand_push_force, self.rand_push_torque = z(N, 3), z(N, 3)
        self.is_first_add_force = True
        self.base_quat = self.root[:, 3:7].copy()
        self.base_lin_vel = quat_rotate_inverse(self.base_quat, self.root[:, 7:10])
        self.base_ang_vel = quat_rotate_inverse(self.base_quat, self.root[:, 10:13])
        self.gravity = np.tile(np.array([0, 0, -1], f32), (N, 1))
        self.projected_gravity = quat_rotate_inverse(self.base_quat, self.gravity)
        self.base_euler_xyz = euler_xyz(self.base_quat)
        self.feet_euler_xyz = euler_xyz(self.rigid[:, FEET, 3:7])
        self.lag_buffer = z(N, 12, 31)
        self.dof_lag_buffer = z(N, 24, 31)
        self.imu_lag_buffer = z(N, 6, 11)
        self.lag_timestep = R.randint(0, 31, seed, self.ids, 0, R.SLOT_LAG_ACTION)
        self.dof_lag_timestep = R.randint(0, 31, seed, self.ids, 0, R.SLOT_LAG_DOF)
        self.imu_lag_timestep = R.randint(0, 11, seed, self.ids, 0, R.SLOT_LAG_IMU)
        self.episode_sums = {k: z(N) for k in REWARD_NAMES}
        # randomize_dof_props at creation runs before p_gains exist -> randomized gains are 0
        self.kp_r, self.kd_r = z(N, 12), z(N, 12)
        self.motor_offsets, self.coulomb, self.viscous = z(N, 12), z(N, 12), z(N, 12)
        self.armature = z(N, 12)
        self.torque_multi = np.ones((N, 12), f32)
        self.extras = {}
        self.applied_force = z(N, 13, 3)
        self.force_pending = False

    # ---------------------------------------------------------------- random helpers
    def _key_ctr(self):
        return self.common_step_counter | self._key_salt

    def _rf(self, lo, hi, ids, slot, ctr=None):
        return R.rand_float(lo, hi, self.seed, ids + self.env_offset, self._key_ctr() if ctr is None else ctr, slot)

    def _ri(self, lo, hi, ids, slot):
        return R.randint(lo, hi, self.seed, ids + self.env_offset, self._key_ctr(), slot)

    # ---------------------------------------------------------------- step
    def step(self, actions, physics):
        """legged_robot.py:387-448"""
        self.actions = np.clip(actions.astype(f32), -CLIP_ACTIONS, CLIP_ACTIONS)
        self.torque_log = []
        for sub in range(DECIMATION):
            self.torques = self._compute_torques(self.actions, sub)
            self.torque_log.append(self.torques.copy())
            root, dof, rigid, contact = physics(self.substep_counter, self.torques, self)
            self.substep_counter += 1
            self.root[:], self.dof[:], self.rigid[:], self.contact[:] = root, dof, rigid, contact
            self.force_pending = False
            # dof lag push (legged_robot.py:412-418)
            self.dof_lag_buffer[:, :, 1:] = self.dof_lag_buffer[:, :, :30].copy()
            self.dof_lag_buffer[:, :, 0] = np.concatenate([self.dof[:, :, 0], self.dof[:, :, 1]], 1)
            # imu lag push (legged_robot.py:428-434)
            self.base_quat = self.root[:, 3:7].copy()
            self.base_ang_vel = quat_rotate_inverse(self.base_quat, self.root[:, 10:13])
            self.base_euler_xyz = euler_xyz(self.base_quat)
            self.imu_lag_buffer[:, :, 1:] = self.imu_lag_buffer[:, :, :10].copy()
            self.imu_lag_buffer[:, :, 0] = np.concatenate([self.base_ang_vel, self.base_euler_xyz], 1)
        self.post_physics_step()
        self.obs_buf = np.clip(self.obs_buf, -CLIP_OBS, CLIP_OBS)
        self.priv_buf = np.clip(self.priv_buf, -CLIP_OBS, CLIP_OBS)
        return self.obs_buf, self.priv_buf, self.rew_buf, self.reset_buf, self.extras

    def reset(self, physics):
        """legged_robot.py:450-455.  After the first step the draws take the between-step key domain: the plain
        counter would repeat the draws of every env the last step reset (t1env.hip k_reset_all)."""
        self.reset_idx(np.arange(self.N), between_steps=self.common_step_counter > 0)
        self.step(np.zeros((self.N, 12), f32), physics)
        return self.obs_buf, self.priv_buf

    def _compute_torques(self, actions, sub):
        """legged_robot.py:1019-1074"""
        a_s = (actions * f32(ACTION_SCALE)).astype(f32)
        self.lag_buffer[:, :, 1:] = self.lag_buffer[:, :, :30].copy()
        self.lag_buffer[:, :, 0] = a_s
        lagged = self.lag_buffer[np.arange(self.N), :, self.lag_timestep]
        tq = self.kp_r * (lagged + Q0 - self.dof[:, :, 0] + self.motor_offsets) - self.kd_r * self.dof[:, :, 1] \
            - self.viscous * self.dof[:, :, 1] - self.coulomb * np.sign(self.dof[:, :, 1])
        self.torque_multi = np.stack([self._rf(0.8, 1.2, np.arange(self.N), R.SLOT_TORQUE_MULT + sub * 12 + j)
                                      for j in range(12)], 1)
        tq = (tq * self.torque_multi).astype(f32)
        return np.clip(tq, -TORQUE_LIMITS, TORQUE_LIMITS).astype(f32)

    def post_physics_step(self):
        """legged_robot.py:458-506"""
        self.episode_length_buf += 1
        self.common_step_counter += 1
        self.base_quat = self.root[:, 3:7].copy()
        self.base_lin_vel = quat_rotate_inverse(self.base_quat, self.root[:, 7:10])
        self.base_ang_vel = quat_rotate_inverse(self.base_quat, self.root[:, 10:13])
        self.projected_gravity = quat_rotate_inverse(self.base_quat, self.gravity)
        self.base_euler_xyz = euler_xyz(self.base_quat)
        self.feet_euler_xyz = euler_xyz(self.rigid[:, FEET, 3:7])
        self._callback()
        self._check_termination()
        self._compute_reward()
        env_ids = np.nonzero(self.reset_buf)[0]
        self.reset_idx(env_ids)
        self.compute_observations()
        self.last_last_actions = self.last_actions.copy()
        self.last_actions = self.actions.copy()
        self.last_dof_vel = self.dof[:, :, 1].copy()
        self.last_root_vel = self.root[:, 7:13].copy()

    # ---------------------------------------------------------------- callback (t1:179-215)
    def _stand(self):
        return _norm(self.commands[:, :3], 1) <= STAND_THRESH

    def _resample_commands(self):
        """t1_dh_stand_env.py:126-136 (+ walk_omnidirectional 170-177, stand 138-144)"""
        for i, name in enumerate(GAIT):
            ids = np.nonzero(self.episode_length_buf == self.gait_time[:, i])[0]
            if len(ids) == 0:
                continue
            if name == "stand":
                self.commands[ids, 0:3] = 0.0
            else:
                cr = self.command_ranges
                self.commands[ids, 0] = self._rf(cr["lin_vel_x"][0], cr["lin_vel_x"][1], ids, R.SLOT_CMD_X)
                self.commands[ids, 1] = self._rf(cr["lin_vel_y"][0], cr["lin_vel_y"][1], ids, R.SLOT_CMD_Y)
                self.commands[ids, 2] = self._rf(cr["ang_vel_yaw"][0], cr["ang_vel_yaw"][1], ids, R.SLOT_CMD_YAW)

    def _get_heights(self):
        """legged_robot.py:1551-1587 on the post-physics (pre-reset) base pose; zeros on a plane (:1564-1565)."""
        if self.mesh_type == "plane":
            return np.zeros((self.N, NUM_HEIGHT), f32)
        t = self.terrain
        return get_heights(self.root[:, :3], self.root[:, 3:7], self.height_points, t["height_samples"],
                           t["horizontal_scale"], t["vertical_scale"], t["border_size"])

    def _callback(self):
        self.phase_length_buf += 1
        self._resample_commands()
        if self.measure_heights:                                 # t1_dh_stand_env.py:190-191
            self.measured_heights = self._get_heights()
        if self.push_robots:                                     # t1_dh_stand_env.py:193-202
            i = min(int(self.common_step_counter / PUSH_UPDATE_STEP), len(PUSH_DURATION) - 1)
            if self.common_step_counter % self.push_interval <= PUSH_DURATION[i] / DT:
                self._push_robots()
            else:
                self.rand_push_force[:] = 0
                self.rand_push_torque[:] = 0
        i = int(self.common_step_counter / ADD_UPDATE_STEP)
        i = min(i, len(ADD_DURATION) - 1)
        duration = ADD_DURATION[i] / DT
        if self.common_step_counter % EXT_INTERVAL <= duration:
            self._add_ext_force()
        else:
            self.ext_forces[:] = 0
            self.ext_torques[:] = 0
            self.is_first_add_force = True

    def _push_robots(self):
        """t1_dh_stand_env.py:217-231: root linear velocity xy U(+-0.2) and angular velocity U(+-0.2) of EVERY env,
        redrawn on every call (`is_first_push = False` is commented out, :227), written into the root state the
        next simulate() starts from (set_actor_root_state_tensor, :230).  The base quantities of this step were
        taken before the callback, so only the root state (base_acc, last_root_vel, the next step) sees it."""
        allids = np.arange(self.N)
        self.rand_push_force[:, :2] = np.stack([self._rf(-MAX_PUSH_VEL_XY, MAX_PUSH_VEL_XY, allids, R.SLOT_PUSH_VEL + k)
                                                for k in range(2)], 1)
        self.rand_push_torque = np.stack([self._rf(-MAX_PUSH_ANG_VEL, MAX_PUSH_ANG_VEL, allids, R.SLOT_PUSH_ANG + k)
                                          for k in range(3)], 1)
        self.root[:, 7:9] = self.rand_push_force[:, :2]
        self.root[:, 10:13] = self.rand_push_torque

    def _add_ext_force(self):
        """t1_dh_stand_env.py:233-247: forces drawn on the first call, applied (base, standing envs only)
        from the second call on, for the next simulate()."""
        allids = np.arange(self.N)
        apply = np.zeros((self.N, 13, 3), f32)
        if self.is_first_add_force:
            fx = self._rf(-EXT_FORCE_MAX[0] / 2, EXT_FORCE_MAX[0], allids, R.SLOT_EXT_FORCE + 0)
            fy = self._rf(-EXT_FORCE_MAX[1], EXT_FORCE_MAX[1], allids, R.SLOT_EXT_FORCE + 1)
            fz = self._rf(-EXT_FORCE_MAX[2], EXT_FORCE_MAX[2], allids, R.SLOT_EXT_FORCE + 2)
            self.ext_forces = np.stack([fx, fy, fz], 1)
            self.ext_torques = np.stack([self._rf(-EXT_TORQUE_MAX, EXT_TORQUE_MAX, allids, R.SLOT_EXT_TORQUE + k)
                                         for k in range(3)], 1)
        if not self.is_first_add_force:
            st = self._stand()
            apply[:, 0, :] = self.ext_forces * st[:, None]
        self.is_first_add_force = False
        self.applied_force = apply
        self.force_pending = True

    def _check_termination(self):
        """legged_robot.py:509-517"""
        self.reset_buf = np.any(_norm(self.contact[:, [BASE], :], -1) > 1, axis=1)
        self.time_out_buf = self.episode_length_buf > MAX_EPISODE_LEN
        self.reset_buf |= self.time_out_buf

    # ---------------------------------------------------------------- phase helpers (t1:80-107, 250-274)
    def _get_phase(self):
        stand = self._stand()
        self.phase_length_buf[stand] = 0
        ph = (self.phase_length_buf.astype(f32) * f32(DT)) / f32(CYCLE_TIME)
        ph = (ph - np.floor(ph)).astype(f32)
        return ((ph + self.gait_start) * (~stand)).astype(f32)

    def _get_gait_phase(self):
        s = np.sin(f32(2 * PI) * self._get_phase()).astype(f32)
        m = np.zeros((self.N, 2), f32)
        m[:, 0] = s >= 0
        m[:, 1] = s < 0
        m[np.abs(s) < 0.1] = 1
        return m

    def _compute_ref_state(self):
        s = np.sin(f32(2 * PI) * self._get_phase()).astype(f32)
        sl, sr = s.copy(), s.copy()
        ref = np.zeros((self.N, 12), f32)
        sl[sl > 0] = 0
        ref[:, 2] = sl * f32(0.3)
        ref[:, 3] = -sl * f32(0.6)
        ref[:, 4] = sl * f32(0.3)
        sr[sr < 0] = 0
        ref[:, 8] = -sr * f32(0.3)
        ref[:, 9] = sr * f32(0.6)
        ref[:, 10] = -sr * f32(0.3)
        ref[np.abs(s) < 0.1] = 0
        self.ref_dof_pos = (ref + Q0).astype(f32)

    # ---------------------------------------------------------------- rewards (t1:576-935)
    def _compute_reward(self):
        """legged_robot.py:654-680: scale*dt, alphabetical order, clip >= 0."""
        self.rew_terms = {}
        rew = np.zeros(self.N, f32)
        for name in REWARD_NAMES:
            r = (getattr(self, "_r_" + name)().astype(f32) * f32(self.reward_scales[name])).astype(f32)
            self.rew_terms[name] = r
            rew = (rew + r).astype(f32)
            self.episode_sums[name] = (self.episode_sums[name] + r).astype(f32)
        self.rew_buf = np.maximum(rew, 0).astype(f32)

    def _contact(self):
        return self.contact[:, FEET, 2] > 5.0

    def _r_joint_pos(self):
        pos_target = self.ref_dof_pos.copy()
        st = self._stand()
        pos_target[st] = Q0
        diff = self.dof[:, :, 0] - pos_target
        n = _norm(diff, 1)
        r = np.exp(f32(-2) * n) - f32(0.2) * np.clip(n, 0, 0.5)
        r[st] = 1.0
        return r

    def _dist_reward(self, idx, dmin, dmax):
        p = self.rigid[:, idx, :2]
        d = _norm(p[:, 0] - p[:, 1], 1)
        a = np.clip(d - f32(dmin), -0.5, 0)
        b = np.clip(d - f32(dmax), 0, 0.5)
        return (np.exp(-np.abs(a) * f32(100)) + np.exp(-np.abs(b) * f32(100))) / f32(2)

    def _r_feet_distance(self):
        return self._dist_reward(FEET, 0.15, 0.45)

    def _r_knee_distance(self):
        return self._dist_reward(KNEES, 0.12, 0.35)

    def _r_foot_slip(self):
        c = self._contact()
        sp = _norm(self.rigid[:, FEET, 10:12], 2)
        return np.sum(np.sqrt(sp) * c, 1)

    def _r_feet_air_time(self):
        c = self._contact()
        sm = self._get_gait_phase()
        sm[_norm(self.commands[:, :3], 1) < 0.05] = 1
        cf = c | (sm > 0) | self.last_contacts
        self.last_contacts = c
        first = (self.feet_air_time > 0) & cf
        self.feet_air_time = (self.feet_air_time + f32(DT)).astype(f32)
        air = np.clip(self.feet_air_time, 0, 0.5) * first
        self.feet_air_time = (self.feet_air_time * (~cf)).astype(f32)
        return np.sum(air, 1)

    def _r_feet_contact_number(self):
        c = self._contact()
        sm = self._get_gait_phase()
        sm[self._stand()] = 1
        return np.mean(np.where(c == (sm > 0), f32(1), f32(-0.3)), 1)

    def _r_orientation(self):
        qm = np.exp(-np.sum(np.abs(self.base_euler_xyz[:, :2]), 1) * f32(10))
        o = np.exp(-_norm(self.projected_gravity[:, :2], 1) * f32(20))
        return (qm + o) / f32(2)

    def _r_feet_contact_forces(self):
        return np.sum(np.clip(_norm(self.contact[:, FEET, :], -1) - f32(500), 0, 400), 1)

    def _r_default_joint_pos(self):
        jd = self.dof[:, :, 0] - Q0
        yr = _norm(jd[:, [0, 1, 5]], 1) + _norm(jd[:, [6, 7, 11]], 1)
        yr = np.clip(yr - f32(0.1), 0, 50)
        return np.exp(-yr * f32(100)) - f32(0.01) * _norm(jd, 1)

    def _r_base_height(self):
        sm = self._get_gait_phase()
        mh = np.sum(self.rigid[:, FEET, 2] * sm, 1) / np.sum(sm, 1)
        bh = self.root[:, 2] - (mh - f32(0.05))
        return np.exp(-np.abs(bh - f32(0.965)) * f32(100))

    def _r_base_acc(self):
        return np.exp(-_norm(self.last_root_vel - self.root[:, 7:13], 1) * f32(3))

    def _r_vel_mismatch_exp(self):
        lm = np.exp(-np.square(self.base_lin_vel[:, 2]) * f32(10))
        am = np.exp(-_norm(self.base_ang_vel[:, :2], 1) * f32(5.0))
        return (lm + am) / f32(2.0)

    def _r_track_vel_hard(self):
        le = _norm(self.commands[:, :2] - self.base_lin_vel[:, :2], 1)
        ae = np.abs(self.commands[:, 2] - self.base_ang_vel[:, 2])
        return (np.exp(-le * f32(10)) + np.exp(-ae * f32(10))) / f32(2.0) - f32(0.2) * (le + ae)

    def _r_tracking_lin_vel(self):
        st = self._stand()
        d = self.commands[:, :2] - self.base_lin_vel[:, :2]
        rs = np.exp(-np.sum(d * d, 1) * f32(5))
        ra = np.exp(-np.sum(np.abs(d), 1) * f32(5 * 2))
        return np.where(st, ra, rs)

    def _r_tracking_ang_vel(self):
        st = self._stand()
        d = self.commands[:, 2] - self.base_ang_vel[:, 2]
        return np.where(st, np.exp(-np.abs(d) * f32(10)), np.exp(-(d * d) * f32(5)))

    def _r_feet_clearance(self):
        c = self._contact()
        fz = self.rigid[:, FEET, 2]
        self.feet_height = (self.feet_height + (fz - self.last_feet_z)).astype(f32)
        self.last_feet_z = fz.copy()
        sw = f32(1) - self._get_gait_phase()
        rp = (self.feet_height > 0.02) & (self.feet_height < 0.08)
        r = np.sum(rp * sw, 1)
        self.feet_height = (self.feet_height * (~c)).astype(f32)
        return r

    def _r_low_speed(self):
        sp = np.abs(self.base_lin_vel[:, 0])
        cm = np.abs(self.commands[:, 0])
        low = sp < f32(0.5) * cm
        high = sp > f32(1.2) * cm
        ok = ~(low | high)
        mis = np.sign(self.base_lin_vel[:, 0]) != np.sign(self.commands[:, 0])
        r = np.zeros(self.N, f32)
        r[low] = -1.0
        r[high] = 0.0
        r[ok] = 1.2
        r[mis] = -2.0
        return r * (np.abs(self.commands[:, 0]) > 0.05)

    def _r_torques(self):
        return np.sum(np.square(self.torques), 1)

    def _r_dof_vel(self):
        return np.sum(np.square(self.dof[:, :, 1]), 1)

    def _r_dof_acc(self):
        return np.sum(np.square((self.last_dof_vel - self.dof[:, :, 1]) / f32(DT)), 1)

    def _r_collision(self):
        return np.sum((_norm(self.contact[:, [BASE], :], -1) > 0.1).astype(f32), 1)

    def _r_action_smoothness(self):
        d1 = self.last_actions - self.actions
        d2 = self.actions + self.last_last_actions - f32(2) * self.last_actions
        return np.sum(d1 * d1, 1) + np.sum(d2 * d2, 1) + f32(0.05) * np.sum(np.abs(self.actions), 1)

    def _r_stand_still(self):
        st = self._stand()
        idx = [0, 1, 2, 3, 5, 6, 7, 8]
        w = np.array([2, 2, 1, 1, 1, 2, 2, 1, 1, 1], f32)
        err = np.concatenate([self.dof[:, idx, 0] - Q0[idx], self.feet_euler_xyz[:, :, 1]], 1) * w
        r = np.exp(-np.sum(err * err, 1))
        return np.where(st, r, f32(0))

    def _r_feet_rotation(self):
        rot = np.sum(np.square(self.feet_euler_xyz[:, :, 1]), 1)
        return np.exp(-np.square(rot / f32(1)))

    # ---------------------------------------------------------------- reset (t1:483-559)
    def _widen_commands(self):
        cr = self.command_ranges["lin_vel_x"]
        cr[0] = float(np.clip(cr[0] - 0.25, -1.5 / 2, 0.0))
        cr[1] = float(np.clip(cr[1] + 0.5, 0.0, 1.5))

    def reset_idx(self, env_ids, between_steps=False):
        """t1_dh_stand_env.py:483-559.  between_steps: called by the user between two steps (not by
        post_physics_step / reset()): the draws take the between-step key domain (oracle/rng.py BETWEEN_STEP_SALT)."""
        if between_steps:
            self._key_salt = R.BETWEEN_STEP_SALT
            try:
                return self.reset_idx(env_ids)
            finally:
                self._key_salt = 0
        curriculum_step = self.common_step_counter % MAX_EPISODE_LEN == 0
        if self.reduce_fn is not None and curriculum_step:
            # sharded: every rank takes part, also with no local resets (the mean is over all ranks' resets)
            s, c = self.reduce_fn(float(np.sum(self.episode_sums["tracking_lin_vel"][env_ids], dtype=np.float64)),
                                  float(len(env_ids)))
            if c > 0 and s / c / MAX_EPISODE_LEN > 0.8 * self.reward_scales["tracking_lin_vel"]:
                self._widen_commands()
        if len(env_ids) == 0:
            return
        if self.curriculum:
            self._update_terrain_curriculum(env_ids)
        if self.reduce_fn is None and curriculum_step:      # command curriculum (legged_robot.py:1160-1169)
            if np.mean(self.episode_sums["tracking_lin_vel"][env_ids]) / MAX_EPISODE_LEN > \
                    0.8 * self.reward_scales["tracking_lin_vel"]:
                self._widen_commands()
        n = len(env_ids)
        # _reset_dofs (legged_robot.py:1076-1090)
        self.dof[env_ids, :, 0] = Q0 + np.stack([self._rf(-0.1, 0.1, env_ids, R.SLOT_RESET_DOF + j)
                                                 for j in range(12)], 1)
        self.dof[env_ids, :, 1] = 0.0
        # _reset_root_states (legged_robot.py:1092-1120)
        init = np.array([0, 0, 1.1, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0], f32)
        self.root[env_ids] = init
        self.root[env_ids, :3] += self.env_origins[env_ids]
        if self.custom_origins:
            p3 = self.platform / 3 if self.curriculum else self.env_length / 2
            self.root[env_ids, 0] += self._rf(-p3, p3, env_ids, R.SLOT_RESET_ROOT_XY + 0)
            self.root[env_ids, 1] += self._rf(-p3, p3, env_ids, R.SLOT_RESET_ROOT_XY + 1)
        # randomize_dof_props (legged_robot.py:732-783)
        rf = lambda lo, hi, s: np.stack([self._rf(lo, hi, env_ids, s + j) for j in range(12)], 1)  # noqa: E731
        self.torque_multi[env_ids] = rf(0.8, 1.2, R.SLOT_DR_TORQUE)
        self.motor_offsets[env_ids] = rf(-0.035, 0.035, R.SLOT_DR_OFFSET)
        self.kp_r[env_ids] = rf(0.8, 1.2, R.SLOT_DR_KP) * KP
        self.kd_r[env_ids] = rf(0.8, 1.2, R.SLOT_DR_KD) * KD
        self.coulomb[env_ids] = rf(0.1, 1.0, R.SLOT_DR_COULOMB)
        self.viscous[env_ids] = rf(0.1, 0.9, R.SLOT_DR_VISCOUS)
        for j in range(12):
            lo, hi = ARMATURE_RANGE[j]
            self.armature[env_ids, j] = self._rf(lo, hi, env_ids, R.SLOT_DR_ARMATURE + j)
        # randomize_lag_props (legged_robot.py:604-651)
        self.lag_buffer[env_ids] = 0
        self.lag_timestep[env_ids] = self._ri(0, 31, env_ids, R.SLOT_LAG_ACTION)
        self.dof_lag_buffer[env_ids] = 0
        self.dof_lag_timestep[env_ids] = self._ri(0, 31, env_ids, R.SLOT_LAG_DOF)
        self.imu_lag_buffer[env_ids] = 0
        self.imu_lag_timestep[env_ids] = self._ri(0, 11, env_ids, R.SLOT_LAG_IMU)
        # buffers
        for b in (self.last_last_actions, self.actions, self.last_actions, self.last_dof_vel, self.last_root_vel,
                  self.feet_air_time):
            b[env_ids] = 0
        self.episode_length_buf[env_ids] = 0
        self.phase_length_buf[env_ids] = 0
        self.reset_buf[env_ids] = True
        self.gait_start[env_ids] = self._ri(0, 2, env_ids, R.SLOT_GAIT_START).astype(f32) * f32(0.5)
        self._generate_gait_time(env_ids)
        self._resample_commands()
        ep = {}
        for k in REWARD_NAMES:
            ep["rew_" + k] = f32(np.mean(self.episode_sums[k][env_ids]) / EPISODE_S)
            self.episode_sums[k][env_ids] = 0
        if self.mesh_type == "trimesh":
            ep["terrain_level"] = f32(np.mean(self.terrain_levels.astype(f32)))
        ep["max_command_x"] = self.command_ranges["lin_vel_x"][1]
        self.extras["episode"] = ep
        self.extras["time_outs"] = self.time_out_buf
        # recompute base quantities of the reset envs (t1:548-554); rigid/contact stay stale
        q = self.root[env_ids, 3:7]
        self.base_quat[env_ids] = q
        self.base_euler_xyz = euler_xyz(self.base_quat)
        self.projected_gravity[env_ids] = quat_rotate_inverse(q, self.gravity[env_ids])
        self.base_lin_vel[env_ids] = quat_rotate_inverse(q, self.root[env_ids, 7:10])
        self.base_ang_vel[env_ids] = quat_rotate_inverse(q, self.root[env_ids, 10:13])
        self.feet_euler_xyz = euler_xyz(self.rigid[:, FEET, 3:7])
        self.obs_hist[env_ids] = 0
        self.priv_hist[env_ids] = 0

    def _generate_gait_time(self, env_ids):
        """t1_dh_stand_env.py:109-124"""
        r = np.stack([self._rf(GAIT_RANGE[g][0], GAIT_RANGE[g][1], env_ids, R.SLOT_GAIT_TIME + i)
                      for i, g in enumerate(GAIT)], 1).astype(f32)
        s = ((r[:, 0] + r[:, 1]) + r[:, 2]).astype(f32)
        sc = (r * (f32(MAX_EPISODE_LEN) / s)[:, None]).astype(f32)
        sc[:, 1:] = sc[:, :-1].copy()
        sc[:, 0] = 0
        self.gait_time[env_ids] = np.cumsum(sc, 1, dtype=f32).astype(np.int32)

    def _update_terrain_curriculum(self, env_ids):
        """legged_robot.py:1138-1158"""
        d = _norm(self.root[env_ids, :2] - self.env_origins[env_ids, :2], 1)
        up = d > self.env_length / 2
        down = (d < _norm(self.commands[env_ids, :2], 1) * f32(EPISODE_S * 0.5)) & ~up
        lv = self.terrain_levels[env_ids] + up.astype(np.int64) - down.astype(np.int64)
        rnd = self._ri(0, self.max_terrain_level, env_ids, R.SLOT_TERRAIN_LEVEL_RAND)
        lv = np.where(lv >= self.max_terrain_level, rnd, np.maximum(lv, 0))
        self.terrain_levels[env_ids] = lv
        self.env_origins[env_ids] = self.terrain_origins[lv, self.terrain_types[env_ids]]

    # ---------------------------------------------------------------- observations (t1:368-481)
    def compute_observations(self):
        phase = self._get_phase()
        self._compute_ref_state()
        sin_p = np.sin(f32(2 * PI) * phase).astype(f32)
        cos_p = np.cos(f32(2 * PI) * phase).astype(f32)
        stance = self._get_gait_phase()
        cmask = self._contact().astype(f32)
        cmd_in = np.concatenate([sin_p[:, None], cos_p[:, None],
                                 self.commands[:, :3] * np.array([2, 2, 1], f32)], 1)
        q, dq = self.dof[:, :, 0], self.dof[:, :, 1]
        pf = self.ext_forces[:, :2] / f32(EXT_FORCE_MAX[0] + 0.1)
        pt = self.ext_torques / f32(EXT_TORQUE_MAX + 0.1)
        priv = np.concatenate([cmd_in, q - Q0, dq * f32(0.05), self.actions, q - self.ref_dof_pos,
                               self.base_lin_vel * f32(2), self.base_ang_vel * f32(1),
                               self.base_euler_xyz * f32(1), pf, pt, self.friction[:, None],
                               (self.body_mass / f32(30.0))[:, None], stance, cmask], 1).astype(f32)
        if self.measure_heights:                                 # t1_dh_stand_env.py:466-468
            hts = np.clip(self.root[:, 2:3] - f32(0.5) - self.measured_heights, -1, 1) * f32(HEIGHT_OBS_SCALE)
            priv = np.concatenate([priv, hts.astype(f32)], 1)
        ar = np.arange(self.N)
        lq = self.dof_lag_buffer[ar, :12, self.dof_lag_timestep]
        ldq = self.dof_lag_buffer[ar, 12:, self.dof_lag_timestep]
        limu = self.imu_lag_buffer[ar, :, self.imu_lag_timestep]
        obs = np.concatenate([cmd_in, (lq - Q0) * f32(1), ldq * f32(0.05), self.actions, limu[:, :3] * f32(1),
                              limu[:, 3:] * f32(1)], 1).astype(f32)
        u = np.stack([R.uniform(self.seed, self.ids, self.common_step_counter, R.SLOT_OBS_NOISE + j)
                      for j in range(NUM_SINGLE_OBS)], 1)
        obs = (obs + (f32(2) * u - f32(1)) * self.noise_vec * f32(NOISE_LEVEL)).astype(f32)
        self.obs_hist = np.concatenate([self.obs_hist[:, 1:], obs[:, None]], 1)
        self.priv_hist = np.concatenate([self.priv_hist[:, 1:], priv[:, None]], 1)
        self.obs_buf = self.obs_hist.reshape(self.N, -1).copy()
        self.priv_buf = self.priv_hist.reshape(self.N, -1).copy()
