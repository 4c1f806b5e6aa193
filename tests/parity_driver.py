"""Drive the HIP env with injected physics through a golden scenario and compare with the reference.

The reference outputs (tests/golden/*.npz) were produced by the reference's own env code running on the
same synthetic physics states (tests/golden/synth.py) with the same counter-RNG draws.  Tolerance: 1e-4
relative with a 1e-6 absolute floor (golden_util.RTOL / ATOL), exact for bool / integer buffers.
"""
import copy

import numpy as np
import torch

import synth
from golden_util import assert_close, load, torque_atol, measures_heights, mid_reset, push_interval_s, terrain_curriculum

REWARD_NAMES = sorted(["joint_pos", "feet_clearance", "feet_contact_number", "feet_air_time", "foot_slip",
                       "feet_distance", "knee_distance", "feet_rotation", "feet_contact_forces",
                       "tracking_lin_vel", "tracking_ang_vel", "vel_mismatch_exp", "low_speed",
                       "track_vel_hard", "default_joint_pos", "orientation", "base_height", "base_acc",
                       "action_smoothness", "torques", "dof_vel", "dof_acc", "collision", "stand_still"])


def make_env_for(fx, device="cuda:0"):
    from ti5_isaacgym_amd import make_t1_env

    name_hook = None
    heights = measures_heights(fx)
    push = push_interval_s(fx)
    if str(fx["mesh_type"]) == "trimesh":
        def name_hook(cfg):
            cfg.terrain.num_rows, cfg.terrain.num_cols, cfg.terrain.border_size = 6, 4, 5
            cfg.terrain.curriculum = terrain_curriculum(fx)   # gen_golden.trimesh_nocurr_hook
            if heights:   # gen_golden.heights_hook
                cfg.terrain.measure_heights = True
                cfg.terrain.terrain_proportions = [0.0, 0.25, 0.25, 0.25, 0.25, 0.0, 0.0, 0.0, 0.0, 0.0]
    if push is not None:   # gen_golden.push_hook
        def name_hook(cfg):
            cfg.domain_rand.push_robots = True
            cfg.domain_rand.push_interval_s = push
    env = make_t1_env(num_envs=int(fx["num_envs"]), mesh_type=str(fx["mesh_type"]), seed=int(fx["seed"]),
                      device=device, cfg_hook=name_hook)
    if heights:
        # the scan samples the field: run it on the reference's own height samples, so this scenario does not
        # depend on the terrain generator (tests/test_terrain.py pins that one against the same fixture)
        from ti5_isaacgym_amd import _lib
        hf = torch.from_numpy(fx["init_height_samples"]).to(env.device)
        assert hf.shape == env.height_samples.shape
        env.height_samples.copy_(hf)
        # and its origins (rough / sloped sub-terrains: the origin z follows the random samples)
        env.terrain_origins.copy_(torch.from_numpy(fx["init_terrain_origins"]).to(env.device))
        env.env_origins.copy_(torch.from_numpy(fx["init_env_origins"]).to(env.device))
        tc = env.cfg.terrain
        _lib.check(env._lib.t1env_set_terrain(env._handle, env.height_samples.data_ptr(), hf.shape[0], hf.shape[1],
                                              tc.horizontal_scale, tc.vertical_scale, float(tc.border_size), 2),
                   "t1env_set_terrain")
    return env


class Injector:
    """Builds the t1env_injected struct for one env step from synth states."""

    def __init__(self, env, seed):
        self.env, self.seed, self.g = env, seed, 0

    def next(self):
        from ti5_isaacgym_amd import _lib
        env = self.env
        n = env.num_envs
        origins = env.env_origins.cpu().numpy()
        roots, dofs = [], []
        for s in range(10):
            r, d, rig, con = synth.state(self.seed, n, self.g + s, origins)
            roots.append(r)
            dofs.append(d)
        self.g += 10
        dev = env.device
        self._keep = [torch.from_numpy(np.stack(roots)).to(dev), torch.from_numpy(np.stack(dofs)).to(dev),
                      torch.from_numpy(rig).to(dev), torch.from_numpy(con).to(dev),
                      torch.zeros(10, n, 12, device=dev)]
        inj = _lib.Injected()
        P = _lib.C.cast
        inj.root, inj.dof, inj.rigid, inj.contact, inj.torque_log = [P(t.data_ptr(), _lib.fp) for t in self._keep]
        return inj

    @property
    def torque_log(self):
        return self._keep[4]


def snapshot(env):
    n = env.num_envs
    ex = env.extras.get("episode", {})
    return dict(
        obs=env.obs_buf[:, -47:].cpu().numpy(), priv=env.privileged_obs_buf.cpu().numpy(),
        rew=env.rew_buf.cpu().numpy(), reset=env.reset_buf.cpu().numpy(), time_out=env.time_out_buf.cpu().numpy(),
        commands=env.commands.cpu().numpy(), gait_time=env.gait_time.cpu().numpy(),
        ref_dof_pos=env.ref_dof_pos.cpu().numpy(), feet_air_time=env.feet_air_time.cpu().numpy(),
        feet_height=env.feet_height.cpu().numpy(), episode_length_buf=env.episode_length_buf.cpu().numpy(),
        ext_forces=env.ext_forces.cpu().numpy(), env_origins=env.env_origins.cpu().numpy(),
        root_states=env.root_states.cpu().numpy(), dof_state=env.dof_state.view(n, 12, 2).cpu().numpy(),
        episode_sums=np.stack([env.episode_sums[k].cpu().numpy() for k in REWARD_NAMES]),
        extras_episode=np.array([float(ex["rew_" + k]) for k in REWARD_NAMES], np.float32) if ex else None,
        max_command_x=ex.get("max_command_x") if ex else None,
        terrain_level=float(ex["terrain_level"]) if ex and "terrain_level" in ex else None,
        applied_force=env.applied_force.cpu().numpy(),
        full_obs=env.obs_buf.cpu().numpy(), gait_start=env.gait_start.cpu().numpy(),
        dof_lag=env.dof_lag_timestep.cpu().numpy(), imu_lag=env.imu_lag_timestep.cpu().numpy(),
        lag=env.lag_timestep.cpu().numpy(), kp=env.randomized_p_gains.cpu().numpy(),
        armature=env.joint_armatures.cpu().numpy(),
        measured_heights=env.measured_heights.cpu().numpy() if env.measure_heights else None)


def run_parity(name, max_steps=None, device="cuda:0", check=True):
    fx = load(name)
    env = make_env_for(fx, device)
    assert_close("env_frictions", env.env_frictions.cpu().numpy(), fx["init_env_frictions"])
    assert_close("body_mass", env.body_mass.cpu().numpy(), fx["init_body_mass"])
    # creation-time DR of k_init vs the reference's randomize_rigid_body_props / _process_rigid_shape_props
    # (legged_robot.py:692-730, 786-824)
    assert_close("link_masses", env.link_mass_scale.cpu().numpy(), fx["init_link_masses"].reshape(-1, 12))
    assert_close("com_displacements", env.com_displacements.cpu().numpy(), fx["init_com_displacements"])
    assert_close("restitution", env.restitution_coeffs.cpu().numpy(), fx["init_restitution"].reshape(-1, 1))
    if "init_terrain_levels" in fx:
        np.testing.assert_array_equal(env.terrain_levels.cpu().numpy(), fx["init_terrain_levels"])
        np.testing.assert_array_equal(env.terrain_types.cpu().numpy(), fx["init_terrain_types"])
        assert_close("env_origins_init", env.env_origins.cpu().numpy(), fx["init_env_origins"])
    inj = Injector(env, int(fx["synth_seed"]))
    # reset(): reset_idx(all) + step(zeros) with injected physics
    env.reset_idx_all()
    env.step(torch.zeros(env.num_envs, 12, device=env.device), _injected=inj.next())
    outs = [dict(snapshot(env), torques=inj.torque_log.cpu().numpy())]
    if "override_episode_length_buf" in fx:
        env.episode_length_buf = torch.from_numpy(fx["override_episode_length_buf"])
    if "override_common_step_counter" in fx:
        env.common_step_counter = int(fx["override_common_step_counter"])
    if "override_episode_sums_tracking_lin_vel" in fx:
        env.episode_sums["tracking_lin_vel"].copy_(torch.from_numpy(fx["override_episode_sums_tracking_lin_vel"]))
    steps = fx["actions"].shape[0] if max_steps is None else min(max_steps, fx["actions"].shape[0])
    for t in range(steps):
        env.step(torch.from_numpy(fx["actions"][t]).to(env.device), _injected=inj.next())
        outs.append(dict(snapshot(env), torques=inj.torque_log.cpu().numpy()))
        ids = mid_reset(fx, t)
        if ids is not None:   # the reference's reset_idx(env_ids) between two steps
            env.reset_idx(torch.from_numpy(ids))
    if check:
        compare(name, fx, outs)
    return env, outs


def compare(name, fx, outs):
    for t, s in enumerate(outs):
        ctx = f" [{name} step {t}]"
        np.testing.assert_array_equal(s["reset"], fx["step_reset"][t], err_msg="reset" + ctx)
        np.testing.assert_array_equal(s["time_out"], fx["step_time_out"][t], err_msg="time_out" + ctx)
        np.testing.assert_array_equal(s["gait_time"], fx["step_gait_time"][t], err_msg="gait_time" + ctx)
        np.testing.assert_array_equal(s["episode_length_buf"], fx["step_episode_length_buf"][t], err_msg="ep_len" + ctx)
        np.testing.assert_array_equal(s["dof_lag"], fx["step_dof_lag_timestep"][t], err_msg="dof_lag" + ctx)
        np.testing.assert_array_equal(s["imu_lag"], fx["step_imu_lag_timestep"][t], err_msg="imu_lag" + ctx)
        np.testing.assert_array_equal(s["lag"], fx["step_lag_timestep"][t], err_msg="lag" + ctx)
        assert_close("gait_start", s["gait_start"], fx["step_gait_start"][t], ctx=ctx)
        assert_close("torques", s["torques"], fx["step_torques"][t], atol=torque_atol(), ctx=ctx)
        for k in ("commands", "ref_dof_pos", "feet_air_time", "feet_height", "ext_forces",
                  "env_origins", "root_states", "episode_sums", "dof_state"):
            assert_close(k, s[k], fx["step_" + k][t], ctx=ctx)
        assert_close("kp", s["kp"], fx["step_randomized_p_gains"][t], ctx=ctx)
        assert_close("armature", s["armature"], fx["step_joint_armatures"][t], ctx=ctx)
        assert_close("obs", s["obs"], fx["step_obs"][t], ctx=ctx)
        assert_close("priv", s["priv"], fx["step_priv"][t], ctx=ctx)
        assert_close("rew", s["rew"], fx["step_rew"][t], ctx=ctx)
        if measures_heights(fx):   # int16 samples x vertical_scale: exact (a wrong cell is off by >= 0.005)
            np.testing.assert_array_equal(s["measured_heights"], fx["step_measured_heights"][t],
                                          err_msg="measured_heights" + ctx)
        if t > 0:
            assert_close("extras_episode", s["extras_episode"], fx["step_extras_episode"][t], ctx=ctx)
            assert abs(s["max_command_x"] - float(fx["step_extras_max_command_x"][t])) < 1e-6, ctx
            if str(fx["mesh_type"]) == "trimesh":   # reported whatever the curriculum setting (t1:535-536)
                assert abs(s["terrain_level"] - float(fx["step_extras_terrain_level"][t])) < 1e-5, ctx
            if fx["step_force_applied"][t]:
                assert_close("applied_force", s["applied_force"], fx["step_applied_force"][t][:, 0, :], ctx=ctx)
    if len(outs) == len(fx["step_rew"]):
        assert_close("obs_full_last", outs[-1]["full_obs"], fx["obs_full_last"])
