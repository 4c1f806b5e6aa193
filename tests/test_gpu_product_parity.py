"""Pin the PRODUCT step kernels against the oracle at BASELINE sizes -- needs the MI355X.

The product's fused step is k_dyn6 (eight role waves, t1env_dyn6.hip) at every config except config 5's fp16 histories,
where t1env picks k_dyn4 (t1_dyn_waves_default); k_dyn5 stays selectable (T1ENV_DYN_KERNEL).  Every case below runs for
each of them (the dyn_kernel fixture of conftest.py).

The golden fixtures pin post-physics through the injected-physics test hook (k_physics_injected, test_gpu_parity.py).
Every real step instead runs the step kernel, with its own PD (pd_torques_staged), its own sensor-lag capture and its
fused post-physics epilogue.  This test runs that kernel as bench.py runs it -- real dynamics on real terrain -- with the
substep log on (t1env_set_substep_log: the root / dof state after every substep and the torques of every substep),
and replays the logged states through the oracle's injected-physics step (oracle/t1_oracle.py: the CPU restatement
pinned by the golden fixtures, tests/test_oracle_golden.py).  Physics divergence cannot enter: both sides see the
same states, so what is compared is the step kernel's own arithmetic around the solver:

  * the torques of every substep (lagged action ring, randomized PD, viscous / Coulomb friction, per-substep torque
    multiplier, clip: legged_robot.py:1019-1074);
  * the lagged dof samples the kernel captured into its ring vs the oracle's dof_lag_buffer entry the observation
    reads (legged_robot.py:412-418, t1_dh_stand_env.py:378-390);
  * obs (the whole 66-frame history), priv, rew, reset, time_out and the state post-physics writes (commands,
    feet_air_time, feet_height, ref_dof_pos, episode sums, gait times, episode lengths, terrain levels, origins,
    root / dof state after resets and pushes).

Tolerance: 1e-4 relative with a 1e-6 absolute floor (golden_util.RTOL / ATOL), exact for bool / integer buffers.
Every 7th env starts near its time-out so the reset path runs inside the fused epilogue.  Cases: BASELINE configs[1]
(4096 envs, plane), configs[2] (8192 envs, trimesh curriculum + full DR) and configs[4] (32768 envs, height field,
pushes), plus a ragged 777-env trimesh run (last workgroup partly empty), also replayed over 60 steps (the kernel's
state carried through many resets, pushes and lag-ring wraps, each step compared).  Two more cases start the step counter just
before an external-force window (`counter % 400 <= duration`, t1_dh_stand_env.py:205-215): at 400 (duration 0: the
forces are drawn, enter the critic frame and are never applied) and at 96,400 (duration index 1 = 0.05 s: drawn at
96,400, applied to the base of standing envs from 96,401 to 96,405, t1_dh_stand_env.py:233-247,
t1_dh_stand_config.py:197-204), so the kernel's fused draw, its critic-frame terms and `applied_force` are compared.
"""
import numpy as np
import pytest
import torch

from golden_util import assert_close, torque_atol
from oracle.t1_oracle import DECIMATION, REWARD_NAMES, T1Oracle

pytestmark = pytest.mark.gpu

PUSH_INTERVAL_S = 0.02   # push every other step (config 5 pushes; DHT1StandCfg's 6 s would never fire in a test)


def _push_hook(cfg):
    cfg.domain_rand.push_robots = True
    cfg.domain_rand.push_interval_s = PUSH_INTERVAL_S


def oracle_for(env, push):
    terrain = None
    if env.mesh_type in ("heightfield", "trimesh"):
        tc = env.cfg.terrain
        terrain = {"terrain_origins": env._terrain.env_origins, "height_samples": env._terrain.heightsamples,
                   "horizontal_scale": tc.horizontal_scale, "vertical_scale": tc.vertical_scale,
                   "border_size": tc.border_size, "num_envs_total": env.num_envs_total,
                   "env_length": tc.terrain_length, "platform": getattr(tc, "platform", 3.0),
                   "max_init_terrain_level": tc.max_init_terrain_level}
    kw = {"push_robots": True, "push_interval_s": PUSH_INTERVAL_S} if push else {}
    return T1Oracle(env.num_envs, seed=int(env.cfg.seed), mesh_type=env.mesh_type, terrain=terrain, **kw)


class Replay:
    """physics(g, torques, state) for the oracle: the step kernel's substep log of the step just run."""

    def __init__(self, env):
        lg = env.substep_log
        self.root = lg["root"].cpu().numpy()
        self.dof = lg["dof"].cpu().numpy()
        self.torque = lg["torque"].cpu().numpy()
        self.rigid = env.rigid_state.cpu().numpy()
        self.contact = env.contact_forces.cpu().numpy()
        self.s = 0

    def __call__(self, g, torques, state):
        s = self.s
        self.s += 1
        return self.root[s].copy(), self.dof[s].copy(), self.rigid.copy(), self.contact.copy()


def np_(t):
    return t.detach().cpu().numpy()


def compare(env, o, rp, step):
    ctx = f" [step {step}]"
    assert rp.s == DECIMATION
    assert_close("torques", np.stack(o.torque_log), rp.torque, atol=torque_atol(), ctx=ctx)
    np.testing.assert_array_equal(np_(env.reset_buf), o.reset_buf, err_msg="reset" + ctx)
    np.testing.assert_array_equal(np_(env.time_out_buf), o.time_out_buf, err_msg="time_out" + ctx)
    np.testing.assert_array_equal(np_(env.episode_length_buf), o.episode_length_buf, err_msg="episode_length" + ctx)
    np.testing.assert_array_equal(np_(env.gait_time), o.gait_time, err_msg="gait_time" + ctx)
    np.testing.assert_array_equal(np_(env.dof_lag_timestep), o.dof_lag_timestep, err_msg="dof_lag" + ctx)
    if o.curriculum:
        np.testing.assert_array_equal(np_(env.terrain_levels), o.terrain_levels, err_msg="terrain_levels" + ctx)
    assert_close("rew", np_(env.rew_buf), o.rew_buf, ctx=ctx)
    assert_close("obs", np_(env.obs_buf), o.obs_buf, ctx=ctx)
    assert_close("priv", np_(env.privileged_obs_buf), o.priv_buf, ctx=ctx)
    for name, a, b in (("commands", env.commands, o.commands), ("feet_air_time", env.feet_air_time, o.feet_air_time),
                       ("feet_height", env.feet_height, o.feet_height), ("ref_dof_pos", env.ref_dof_pos, o.ref_dof_pos),
                       ("env_origins", env.env_origins, o.env_origins), ("root_states", env.root_states, o.root),
                       ("dof_state", env.dof_state.view(-1, 12, 2), o.dof),
                       ("last_root_vel", env.last_root_vel, o.last_root_vel)):
        assert_close(name, np_(a), b, ctx=ctx)
    assert_close("episode_sums", np.stack([np_(env.episode_sums[k]) for k in REWARD_NAMES]),
                 np.stack([o.episode_sums[k] for k in REWARD_NAMES]), ctx=ctx)
    # the external-force draw (_add_ext_force) and the base force the next step's first substep applies
    assert_close("ext_forces", np_(env.ext_forces), o.ext_forces, ctx=ctx)
    assert_close("ext_torques", np_(env.ext_torques), o.ext_torques, ctx=ctx)
    # (the library writes the force for the next simulate every step, zeros outside a window; the oracle keeps its
    # last _add_ext_force value, consumed by the next step's first substep: force_pending)
    af = o.applied_force[:, 0, :] if o.force_pending else np.zeros((env.num_envs, 3), np.float32)
    assert_close("applied_force", np_(env.applied_force), af, ctx=ctx)
    # the lag sample the step kernel captured (ring slot of step ctr - lag // 10) vs the dof_lag_buffer entry the observation
    # reads (index dof_lag_timestep): (q, qd) of substep 9 - lag % 10
    ctr = env.common_step_counter - 1
    lag = o.dof_lag_timestep
    slot = (ctr - lag // 10) & 3
    got = np_(env._dof_hist)[np.arange(env.num_envs), slot]
    ref = o.dof_lag_buffer[np.arange(env.num_envs), :, lag]
    assert_close("dof_lag_sample", got, ref, ctx=ctx)


@pytest.mark.parametrize("n,mesh,push,steps,counter0", [
    (4096, "plane", False, 6, None), (8192, "trimesh", False, 6, None), (32768, "heightfield", True, 4, None),
    (777, "trimesh", True, 5, None), (4096, "trimesh", False, 5, 397), (8192, "trimesh", False, 10, 96397),
    (777, "trimesh", True, 60, None)],
    ids=["config2_4096_plane", "config3_8192_trimesh", "config5_32768_hf_push", "ragged777_trimesh_push",
         "extforce_window_400", "extforce_window_96400_applied", "ragged777_trimesh_push_long60"])
def test_product_kernel_matches_oracle(n, mesh, push, steps, counter0, dyn_solver):
    from ti5_isaacgym_amd import make_t1_env
    env = make_t1_env(num_envs=n, mesh_type=mesh, seed=3, device="cuda:0", cfg_hook=_push_hook if push else None)
    o = oracle_for(env, push)
    # creation-time state (k_init vs legged_robot.py:692-730, 786-824, 1477-1512 as the oracle restates it)
    assert_close("env_frictions", np_(env.env_frictions)[:, 0], o.friction)
    assert_close("body_mass", np_(env.body_mass)[:, 0], o.body_mass)
    assert_close("link_mass_scale", np_(env.link_mass_scale), o.link_mass_scale)
    assert_close("com_displacements", np_(env.com_displacements), o.com_disp)
    assert_close("restitution", np_(env.restitution_coeffs)[:, 0], o.restitution)
    assert_close("env_origins_init", np_(env.env_origins), o.env_origins)
    env.set_substep_log(True)
    env.reset()
    torch.cuda.synchronize()
    rp = Replay(env)
    o.reset(rp)
    compare(env, o, rp, 0)
    # every 7th env times out within a few steps: reset_idx runs in the fused epilogue
    el = np_(env.episode_length_buf).copy()
    el[::7] = int(env.max_episode_length) - 3 - np.arange(0, n, 7) % 4
    env.episode_length_buf = torch.from_numpy(el)
    o.episode_length_buf[:] = el
    if counter0 is not None:   # jump to just before an external-force window (both sides: is_first_add_force stays True)
        # the library's action / sensor-lag rings are indexed by the step counter (slot = counter & 3), so the jump
        # keeps the counter's residue mod 4: the rings then hold what the oracle's shift registers hold
        assert env.is_first_add_force and o.is_first_add_force
        assert (counter0 - env.common_step_counter) % 4 == 0
        env.common_step_counter = o.common_step_counter = counter0
    g = torch.Generator(device="cuda:0").manual_seed(0)
    resets = pushes = applied = drawn = 0
    for t in range(steps):
        a = torch.randn(n, 12, device="cuda:0", generator=g)
        env.step(a)
        torch.cuda.synchronize()
        rp = Replay(env)
        o.step(np_(a), rp)
        compare(env, o, rp, t + 1)
        resets += int(o.reset_buf.sum())
        pushes += int(push and env.common_step_counter % env.push_interval == 0)
        drawn += int(np.abs(o.ext_forces).max() > 0)
        applied += int(o.force_pending and np.abs(o.applied_force).max() > 0)
    env.set_substep_log(False)
    assert resets > 0, "no env reset: the fused epilogue's reset path was not exercised"
    assert pushes > 0 or not push
    if counter0 is not None:
        assert drawn > 0, "the external-force window was not reached"
        assert (applied > 0) == (counter0 >= 96000), (applied, counter0)
