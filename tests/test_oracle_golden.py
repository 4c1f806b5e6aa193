"""Pin the CPU oracle (oracle/t1_oracle.py) against the reference's own outputs (tests/golden/*.npz).

Tolerance: 1e-4 relative (north_star) with a 1e-6 absolute floor for values near zero; exact for
bool / integer state.  Obs/priv are compared after clipping, as returned by step().
"""
import numpy as np
import pytest

from golden_util import (SCENARIOS, assert_close, load, measures_heights, mid_reset, push_interval_s, synth_physics,
                         terrain_curriculum, terrain_of)
from oracle import rng as R
from oracle.t1_oracle import REWARD_NAMES, T1Oracle


def run_oracle(fx):
    n = int(fx["num_envs"])
    terrain = terrain_of(fx)
    push = push_interval_s(fx)
    o = T1Oracle(n, seed=int(fx["seed"]), mesh_type=str(fx["mesh_type"]), terrain=terrain,
                 measure_heights=measures_heights(fx), push_robots=push is not None,
                 terrain_curriculum=terrain_curriculum(fx),
                 **({"push_interval_s": push} if push is not None else {}))
    phys = synth_physics(fx)
    outs = []
    o.reset(phys)
    outs.append(snapshot(o))
    if "override_episode_length_buf" in fx:
        o.episode_length_buf[:] = fx["override_episode_length_buf"]
    if "override_common_step_counter" in fx:
        o.common_step_counter = int(fx["override_common_step_counter"])
    if "override_episode_sums_tracking_lin_vel" in fx:
        o.episode_sums["tracking_lin_vel"][:] = fx["override_episode_sums_tracking_lin_vel"]
    for t in range(fx["actions"].shape[0]):
        o.step(fx["actions"][t], phys)
        outs.append(snapshot(o))
        ids = mid_reset(fx, t)
        if ids is not None:
            o.reset_idx(np.asarray(ids), between_steps=True)
    return o, outs


def snapshot(o):
    return dict(obs=o.obs_buf[:, -47:].copy(), priv=o.priv_buf.copy(), rew=o.rew_buf.copy(),
                reset=o.reset_buf.copy(), time_out=o.time_out_buf.copy(), torques=np.stack(o.torque_log),
                commands=o.commands.copy(), gait_time=o.gait_time.copy(), ref_dof_pos=o.ref_dof_pos.copy(),
                feet_air_time=o.feet_air_time.copy(), feet_height=o.feet_height.copy(),
                episode_length_buf=o.episode_length_buf.copy(), ext_forces=o.ext_forces.copy(),
                env_origins=o.env_origins.copy(), dof_state=o.dof.copy(), root_states=o.root.copy(),
                episode_sums=np.stack([o.episode_sums[k] for k in REWARD_NAMES]),
                extras_episode=np.array([o.extras["episode"]["rew_" + k] for k in REWARD_NAMES], np.float32),
                max_command_x=o.extras["episode"]["max_command_x"],
                terrain_level=o.extras["episode"].get("terrain_level"), applied_force=o.applied_force.copy(),
                full_obs=o.obs_buf.copy(), measured_heights=o.measured_heights.copy())


@pytest.mark.parametrize("name", SCENARIOS)
def test_oracle_matches_reference(name):
    fx = load(name)
    o, outs = run_oracle(fx)
    assert_close("env_frictions", o.friction, fx["init_env_frictions"][:, 0])
    assert_close("body_mass", o.body_mass, fx["init_body_mass"][:, 0])
    if "init_terrain_levels" in fx:
        np.testing.assert_array_equal(o.env_origins.shape, fx["init_env_origins"].shape)
    for t, s in enumerate(outs):
        ctx = f" [{name} step {t}]"
        np.testing.assert_array_equal(s["reset"], fx["step_reset"][t], err_msg="reset" + ctx)
        np.testing.assert_array_equal(s["time_out"], fx["step_time_out"][t], err_msg="time_out" + ctx)
        np.testing.assert_array_equal(s["gait_time"], fx["step_gait_time"][t], err_msg="gait_time" + ctx)
        np.testing.assert_array_equal(s["episode_length_buf"], fx["step_episode_length_buf"][t],
                                      err_msg="episode_length" + ctx)
        for k in ("torques", "commands", "ref_dof_pos", "feet_air_time", "feet_height", "ext_forces",
                  "env_origins", "root_states", "episode_sums"):
            assert_close(k, s[k], fx["step_" + k][t], ctx=ctx)
        assert_close("dof_state", s["dof_state"], fx["step_dof_state"][t], ctx=ctx)
        assert_close("obs", s["obs"], fx["step_obs"][t], ctx=ctx)
        assert_close("priv", s["priv"], fx["step_priv"][t], ctx=ctx)
        assert_close("rew", s["rew"], fx["step_rew"][t], ctx=ctx)
        if measures_heights(fx):   # sample heights are int16 x vertical_scale: a wrong cell is off by >= 0.005
            np.testing.assert_array_equal(s["measured_heights"], fx["step_measured_heights"][t],
                                          err_msg="measured_heights" + ctx)
        if t > 0:
            ref_ep = fx["step_extras_episode"][t]
            assert_close("extras_episode", s["extras_episode"], ref_ep, ctx=ctx)
            assert s["max_command_x"] == pytest.approx(float(fx["step_extras_max_command_x"][t])), ctx
            if str(fx["mesh_type"]) == "trimesh":
                assert s["terrain_level"] == pytest.approx(float(fx["step_extras_terrain_level"][t])), ctx
            if fx["step_force_applied"][t]:
                assert_close("applied_force", s["applied_force"], fx["step_applied_force"][t], ctx=ctx)
    assert_close("obs_full_last", outs[-1]["full_obs"], fx["obs_full_last"])
