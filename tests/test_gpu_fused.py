"""The fused step (t1env_step as one launch: dynamics + history shift + post-physics epilogue; for both
dynamics kernels, k_dyn4 with its LDS-staged epilogue and the 2-wave k_dynamics) gives the same buffers as
the split kernel sequence (k_dynamics, k_post_a, k_post_b -- the path pinned by the golden
fixtures through the injected-physics hook).

Two envs with the same seed and config run the same actions, one fused and one split.  Before every step the
split env's whole state is copied into the fused one, so each step starts from identical buffers (the two
kernels are separate instantiations of the dynamics code, and FMA contraction may differ by an ulp between
them; over many steps that would grow into different trajectories).  Every 7th env starts near its
time-out, so reset_idx, the any-reset command resample and the reset-row zeroing handoff between the shift
workgroups and the dynamics workgroups are exercised.  Discrete buffers (resets, time-outs, episode
lengths, contacts) must be identical; float buffers agree to 1e-5 relative / 1e-6 absolute; the history
must be the exactly shifted previous history with zeroed reset rows in both.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

EXACT = ["reset_buf", "time_out_buf", "episode_length_buf", "phase_length_buf", "last_contacts", "gait_time",
         "terrain_levels"]
# the fused epilogue splits post-physics over two waves (rewards | state + observations): the reward-owned
# buffers (episode sums, feet state) and the state-owned ones are both compared
CLOSE = ["obs_buf", "privileged_obs_buf", "rew_buf", "root_states", "dof_state", "rigid_state", "contact_forces",
         "commands", "last_actions", "feet_air_time", "feet_height", "last_feet_z", "feet_euler_xyz",
         "_episode_sums", "base_lin_vel", "ref_dof_pos", "env_origins"]


def _sync(dst, src):
    for k, t in src._keepalive.items():
        dst._keepalive[k].copy_(t)
    for k in range(2):
        dst._obs[k].copy_(src._obs[k])
        dst._priv[k].copy_(src._priv[k])


def _env(n, mesh, fused):
    from ti5_isaacgym_amd import make_t1_env
    env = make_t1_env(num_envs=n, mesh_type=mesh, seed=11, device="cuda:0")
    env.set_fused(fused)
    env.reset()
    env.episode_length_buf[::7] = int(env.max_episode_length) - 2 - torch.arange(0, n, 7, device="cuda:0") % 6
    return env


# 16384 envs: k_dyn4 fills every CU, so the history shift runs as its own launch ahead of the fused kernel and
# the epilogue zeroes the reset rows directly (t1_shift_prelaunch)
# 1 env: one workgroup with 63 shadow lanes; 65 envs: a second workgroup holding one live env; 13001: the
# prelaunched shift with a ragged last workgroup
@pytest.mark.parametrize("n,mesh", [(8192, "trimesh"), (777, "plane"), (16384, "plane"), (1, "plane"),
                                    (65, "trimesh"), (13001, "plane")],
                         ids=["8192_trimesh", "ragged777_plane", "16384_plane_prelaunched_shift", "single_env",
                              "65_trimesh", "ragged13001_prelaunched_shift"])
def test_fused_step_equals_split_sequence(n, mesh, dyn_kernel):
    fused, split = _env(n, mesh, True), _env(n, mesh, False)
    g = torch.Generator(device="cuda:0").manual_seed(1)
    resets = 0
    for t in range(30):
        a = torch.randn(n, 12, device="cuda:0", generator=g)
        _sync(fused, split)
        fused.step(a)
        split.step(a)
        resets += int(fused.reset_buf.sum())
        for f in EXACT:
            x, y = getattr(fused, f), getattr(split, f)
            assert torch.equal(x, y), f"step {t}: {f} differs"
        for f in CLOSE:
            torch.testing.assert_close(getattr(fused, f), getattr(split, f), rtol=1e-5, atol=1e-6,
                                       msg=lambda m, f=f, t=t: f"step {t}: {f}: {m}")
        r = split.reset_buf.bool()
        for env in (fused, split):  # reset rows: zeroed history (the handoff path in the fused kernel)
            assert not env.obs_buf[r, :-47].any() and not env.privileged_obs_buf[r, :-73].any()
        ef, es = fused.extras["episode"], split.extras["episode"]
        for k in ef:
            torch.testing.assert_close(torch.as_tensor(ef[k]), torch.as_tensor(es[k]), rtol=1e-5, atol=1e-7)
    assert resets > 0

