"""Generate golden vectors by running the REFERENCE's own env code (this container only).

    python tests/golden/gen_golden.py            # writes tests/golden/*.npz

The reference (/root/reference/humanoid/envs/**) is imported behind the test-only isaacgym stand-in
(tests/golden/harness): FakeGym injects physics states from tests/golden/synth.py, and every random draw
site of the reference is routed through the shared counter RNG (oracle/rng.py, hook in harness/draws.py).
The fixtures hold inputs (actions, overrides, seeds) and the reference's outputs; nothing from the
reference's source is stored.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refenv  # noqa: E402

refenv.setup_paths()
import torch  # noqa: E402

import synth  # noqa: E402

SYNTH_SEED = 11

REWARD_NAMES = sorted(["joint_pos", "feet_clearance", "feet_contact_number", "feet_air_time", "foot_slip",
                       "feet_distance", "knee_distance", "feet_rotation", "feet_contact_forces",
                       "tracking_lin_vel", "tracking_ang_vel", "vel_mismatch_exp", "low_speed",
                       "track_vel_hard", "default_joint_pos", "orientation", "base_height", "base_acc",
                       "action_smoothness", "torques", "dof_vel", "dof_acc", "collision", "stand_still"])


def _np(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy().copy()
    return np.asarray(x).copy()


def make_provider(env, num_envs, seed):
    def provider(tensors, g):
        root, dof, rigid, contact = synth.state(seed, num_envs, g, _np(env.env_origins))
        tensors["root"][:] = torch.from_numpy(root)
        tensors["dof"][:] = torch.from_numpy(dof.reshape(num_envs * 12, 2))
        tensors["rigid"][:] = torch.from_numpy(rigid.reshape(num_envs * 13, 13))
        tensors["contact"][:] = torch.from_numpy(contact.reshape(num_envs * 13, 3))
    return provider


def snapshot(env):
    s = {}
    for k in ["commands", "feet_air_time", "feet_height", "ref_dof_pos", "phase_length_buf",
              "episode_length_buf", "gait_time", "gait_start", "dof_lag_timestep", "imu_lag_timestep",
              "lag_timestep", "randomized_p_gains", "randomized_d_gains", "motor_offsets",
              "randomized_joint_coulomb", "randomized_joint_viscous", "joint_armatures", "torque_multi",
              "ext_forces", "ext_torques", "last_actions", "last_last_actions", "actions", "last_dof_vel",
              "last_root_vel", "last_contacts", "root_states", "env_origins", "base_lin_vel", "base_ang_vel",
              "projected_gravity", "base_euler_xyz", "feet_euler_xyz"]:
        s[k] = _np(getattr(env, k))
    s["dof_state"] = _np(env.dof_state).reshape(env.num_envs, 12, 2)
    lfz = env.last_feet_z
    s["last_feet_z"] = _np(lfz) if isinstance(lfz, torch.Tensor) else np.full((env.num_envs, 2), lfz, np.float32)
    s["episode_sums"] = np.stack([_np(env.episode_sums[n]) for n in REWARD_NAMES])
    if env.cfg.terrain.measure_heights:
        s["measured_heights"] = _np(env.measured_heights)
    return s


def run(name, num_envs=16, mesh_type="plane", n_steps=10, cfg_hook=None, after_reset=None, act_scale=0.5,
        mid_reset=None, cfg_keys=None):
    """mid_reset = (t, env_ids): the reference's reset_idx(env_ids) called between step t and step t + 1.
    cfg_keys: config values the scenario's cfg_hook changed, stored as cfg_<key> so the replays set the same."""
    env, cfg, gym = refenv.make_env(num_envs, mesh_type, cfg_hook)
    assert list(env.reward_names) == REWARD_NAMES, env.reward_names
    gym.provider = make_provider(env, num_envs, SYNTH_SEED)
    out = {"num_envs": np.int64(num_envs), "synth_seed": np.int64(SYNTH_SEED), "seed": np.int64(cfg.seed),
           "mesh_type": np.array(mesh_type)}
    for k, v in (cfg_keys or {}).items():
        out["cfg_" + k] = np.asarray(v)
    init = {
        "env_frictions": _np(env.env_frictions), "body_mass": _np(env.body_mass),
        "payload_masses": _np(env.payload_masses), "link_masses": _np(env.link_masses),
        "com_displacements": _np(env.com_displacements), "restitution": _np(env.restitution_coeffs),
        "env_origins": _np(env.env_origins), "default_dof_pos": _np(env.default_dof_pos),
        "torque_limits": _np(env.torque_limits), "dof_pos_limits": _np(env.dof_pos_limits),
        "dof_vel_limits": _np(env.dof_vel_limits), "p_gains": _np(env.p_gains), "d_gains": _np(env.d_gains),
        "noise_scale_vec": _np(env.noise_scale_vec),
    }
    if mesh_type in ("trimesh", "heightfield"):
        init["terrain_levels"] = _np(env.terrain_levels)
        init["terrain_types"] = _np(env.terrain_types)
        init["terrain_origins"] = _np(env.terrain_origins)
        init["height_samples"] = _np(env.height_samples).astype(np.int16)
        if cfg.terrain.measure_heights:
            tc = cfg.terrain
            init["terrain_scales"] = np.array([tc.horizontal_scale, tc.vertical_scale, tc.border_size], np.float64)
    for k, v in init.items():
        out["init_" + k] = v
    # --- reset(): reset_idx(all) + step(zeros) --------------------------------------------------
    n_torque = len(gym.torque_log)
    obs, priv = env.reset()
    rec = [dict(snapshot(env), obs=_np(env.obs_buf), priv=_np(env.privileged_obs_buf), rew=_np(env.rew_buf),
                reset=_np(env.reset_buf), time_out=_np(env.time_out_buf),
                torques=np.stack([_np(t).reshape(num_envs, 12) for t in gym.torque_log[n_torque:]]),
                counter=np.int64(env.common_step_counter))]
    overrides = {}
    if after_reset is not None:
        overrides = after_reset(env) or {}
    for k, v in overrides.items():
        out["override_" + k] = _np(v)
    gen = np.random.default_rng(1234)
    actions = (act_scale * gen.standard_normal((n_steps, num_envs, 12))).astype(np.float32)
    actions[:, 0, :] = 0.0     # one env with exact-zero actions
    actions[min(2, n_steps - 1), 1, 3] = 150.0   # exercises clip_actions = 100
    out["actions"] = actions
    if mid_reset is not None:
        out["mid_reset_step"] = np.int64(mid_reset[0])
        out["mid_reset_ids"] = np.asarray(mid_reset[1], np.int64)
    for t in range(n_steps):
        n_torque, n_force = len(gym.torque_log), len(gym.force_log)
        env.step(torch.from_numpy(actions[t]).clone())
        forces = gym.force_log[n_force:]
        ep = env.extras.get("episode", {})
        ep_vals = np.array([float(ep.get("rew_" + n, np.nan)) for n in REWARD_NAMES], np.float32)
        r = dict(snapshot(env), obs=_np(env.obs_buf), priv=_np(env.privileged_obs_buf), rew=_np(env.rew_buf),
                 reset=_np(env.reset_buf), time_out=_np(env.time_out_buf),
                 torques=np.stack([_np(t_).reshape(num_envs, 12) for t_ in gym.torque_log[n_torque:]]),
                 counter=np.int64(env.common_step_counter),
                 applied_force=(_np(forces[-1][0]) if forces else np.zeros((num_envs, 13, 3), np.float32)),
                 force_applied=np.bool_(len(forces) > 0),
                 extras_episode=ep_vals,
                 extras_max_command_x=np.float32(ep.get("max_command_x", np.nan)),
                 extras_terrain_level=np.float32(ep.get("terrain_level", np.nan)))
        rec.append(r)
        if mid_reset is not None and t == mid_reset[0]:
            import draws   # the between-step key domain (oracle/rng.py BETWEEN_STEP_SALT)
            draws.CTR_SALT = draws.R.BETWEEN_STEP_SALT
            try:
                env.reset_idx(torch.tensor(mid_reset[1], dtype=torch.long))
            finally:
                draws.CTR_SALT = 0
    keys = sorted(set().union(*[r.keys() for r in rec[1:]]))
    for k in keys:
        vals = [r.get(k) for r in rec]
        if vals[0] is None:
            vals[0] = np.zeros_like(vals[1])
        arr = np.stack([np.asarray(v) for v in vals])
        if k == "obs":  # newest frame every step; the full (N, 3102) buffer only for the last step
            out["obs_full_last"] = arr[-1]
            arr = arr[:, :, -47:]
        out["step_" + k] = arr
    path = os.path.join(HERE, f"{name}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {os.path.getsize(path) / 1e6:.2f} MB, resets per step "
          f"{[int(r['reset'].sum()) for r in rec]}")
    return out


def plane16_overrides(env):
    el = env.episode_length_buf
    gt = env.gait_time.long()
    el[0:4] = gt[0:4, 1] - 3       # walk -> stand transition at step 3
    el[4:6] = gt[4:6, 2] - 2       # stand -> walk transition at step 2
    el[6:8] = 2397                 # time-out reset at step 4
    return {"episode_length_buf": el.clone()}


def events16_overrides(env):
    # command curriculum (counter % 2400 == 0 on a reset step) + ext-force application window
    env.common_step_counter = 2 * 96000 - 3     # crosses 96000*2 (=2400*80): duration index 2 (0.1 s)
    el = env.episode_length_buf
    el[0:6] = 2398                 # time out exactly at counter 192000 -> curriculum evaluated
    env.episode_sums["tracking_lin_vel"][:] = 2400 * 0.02   # mean/2400 > 0.8*scale -> widen x range
    gt = env.gait_time.long()
    el[6:9] = gt[6:9, 1] - 1       # standing envs get the applied force
    return {"episode_length_buf": el.clone(), "common_step_counter": np.int64(env.common_step_counter),
            "episode_sums_tracking_lin_vel": env.episode_sums["tracking_lin_vel"].clone()}


def trimesh_hook(cfg):
    cfg.terrain.num_rows = 6
    cfg.terrain.num_cols = 4
    cfg.terrain.border_size = 5


def trimesh_nocurr_hook(cfg):
    # trimesh with the terrain curriculum off: levels over every row, no level updates, start xy over the whole
    # sub-terrain, and extras["episode"]["terrain_level"] still reported (t1_dh_stand_env.py:535-536)
    trimesh_hook(cfg)
    cfg.terrain.curriculum = False


def trimesh_overrides(env):
    el = env.episode_length_buf
    el[0:8] = 2399                 # time out at step 2 -> terrain curriculum on reset
    el[8:12] = 2397                # and at step 4
    return {"episode_length_buf": el.clone()}


def heights_hook(cfg):
    # the inactive height scan (legged_robot.py:1535-1587, t1_dh_stand_env.py:190-191,466-468) switched on
    # on rough / sloped sub-terrains (the default proportions give only flat and rough-flat columns at 4 cols)
    trimesh_hook(cfg)
    cfg.terrain.measure_heights = True
    cfg.terrain.terrain_proportions = [0.0, 0.25, 0.25, 0.25, 0.25, 0.0, 0.0, 0.0, 0.0, 0.0]


PUSH_INTERVAL_S = 0.03   # push_interval = 3 steps: pushes at counters 3, 6, 9 (duration index 0 -> counter % 3 == 0)


def push_hook(cfg):
    # BASELINE config 5's push perturbation (t1_dh_stand_env.py:193-202, 217-231), off in DHT1StandCfg (:188)
    cfg.domain_rand.push_robots = True
    cfg.domain_rand.push_interval_s = PUSH_INTERVAL_S


SCENARIOS = {
    "plane16": lambda: run("plane16", 16, "plane", 10, after_reset=plane16_overrides),
    "events16": lambda: run("events16", 16, "plane", 14, after_reset=events16_overrides),
    "config1_64": lambda: run("config1_64", 64, "plane", 2),
    "trimesh16": lambda: run("trimesh16", 16, "trimesh", 6, cfg_hook=trimesh_hook, after_reset=trimesh_overrides),
    "resetidx16": lambda: run("resetidx16", 16, "trimesh", 6, cfg_hook=trimesh_hook, mid_reset=(2, [1, 4, 9, 15])),
    "heights16": lambda: run("heights16", 16, "trimesh", 6, cfg_hook=heights_hook, after_reset=trimesh_overrides),
    "trimesh_nocurr16": lambda: run("trimesh_nocurr16", 16, "trimesh", 6, cfg_hook=trimesh_nocurr_hook,
                                    after_reset=trimesh_overrides, cfg_keys={"terrain_curriculum": 0}),
    "push16": lambda: run("push16", 16, "plane", 10, cfg_hook=push_hook, after_reset=plane16_overrides,
                          cfg_keys={"push_interval_s": PUSH_INTERVAL_S}),
}

if __name__ == "__main__":
    for name in sys.argv[1:] or list(SCENARIOS):
        SCENARIOS[name]()
