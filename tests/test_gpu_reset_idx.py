"""env.reset_idx(env_ids) between steps on the real-physics path (t1env_reset_idx), 8192 envs on trimesh: the
masked envs restart (episode length 0, reset flag, zeroed history in the buffer the next step shifts from, DR
redrawn), the others are untouched, and after the next step the masked envs' 65 older obs frames / 2 older
critic frames are zero while the other envs' history is the shifted previous one.  The golden scenario
resetidx16 (test_gpu_parity.py) pins the values against the reference's own reset_idx."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_reset_idx_between_steps():
    from ti5_isaacgym_amd import make_t1_env
    n = 8192
    env = make_t1_env(num_envs=n, mesh_type="trimesh", seed=9, device="cuda:0")
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(4)
    for _ in range(5):
        env.step(0.3 * torch.randn(n, 12, device="cuda:0", generator=g))
    ids = torch.arange(3, n, 97, device="cuda:0")
    mask = torch.zeros(n, dtype=torch.bool, device="cuda:0")
    mask[ids] = True
    kp_before = env.randomized_p_gains.clone()
    el_before = env.episode_length_buf.clone()
    obs_prev = env.obs_buf.clone()
    env.reset_idx(ids)
    torch.cuda.synchronize()
    assert (env.episode_length_buf[mask] == 0).all()
    assert torch.equal(env.episode_length_buf[~mask], el_before[~mask])
    assert env.reset_buf[mask].all()
    assert not env.obs_buf[mask].any() and not env.privileged_obs_buf[mask].any()
    assert torch.equal(env.obs_buf[~mask], obs_prev[~mask])
    assert not torch.equal(env.randomized_p_gains[mask], kp_before[mask])
    assert torch.equal(env.randomized_p_gains[~mask], kp_before[~mask])
    ep = env.extras["episode"]
    assert all(torch.isfinite(torch.as_tensor(v)).all() for v in ep.values())
    prev = env.obs_buf.clone()
    env.step(0.3 * torch.randn(n, 12, device="cuda:0", generator=g))
    r = env.reset_buf.bool() | mask
    assert not env.obs_buf[mask, :-47].any() and not env.privileged_obs_buf[mask, :-73].any()
    keep = ~r
    torch.testing.assert_close(env.obs_buf[keep, :-47], prev[keep, 47:], rtol=0, atol=0)
    assert (env.episode_length_buf[mask & ~env.reset_buf.bool()] == 1).all()
    assert torch.isfinite(env.obs_buf).all() and torch.isfinite(env.root_states).all()


def test_reset_idx_after_in_step_reset_draws_fresh_values():
    """An env that terminated inside step c and is passed to reset_idx before step c + 1 must redraw its DR (the
    reference's generator advances): the between-step reset keys on counter | BETWEEN_STEP_SALT, the in-step reset
    of step c on the plain counter."""
    from ti5_isaacgym_amd import make_t1_env
    n = 256
    env = make_t1_env(num_envs=n, mesh_type="plane", seed=9, device="cuda:0")
    env.reset()
    env.episode_length_buf[::5] = int(env.max_episode_length)   # these envs time out in the next step
    env.step(torch.zeros(n, 12, device="cuda:0"))
    r = env.reset_buf.bool()
    assert r[::5].all()
    kp, lag, gs = env.randomized_p_gains.clone(), env.lag_timestep.clone(), env.gait_time.clone()
    ids = torch.nonzero(r).flatten()
    env.reset_idx(ids)
    torch.cuda.synchronize()
    assert (env.randomized_p_gains[r] != kp[r]).all(dim=1).all(), "reset_idx reused the in-step reset's draws"
    assert not torch.equal(env.lag_timestep[r], lag[r]) or not torch.equal(env.gait_time[r], gs[r])
    assert torch.equal(env.randomized_p_gains[~r], kp[~r])


def test_reset_after_stepping_draws_fresh_values():
    """env.reset() on an env that has stepped (reset_idx of every env between steps): the envs the last step reset
    must not redraw that step's values -- t1env_reset_all keys on counter | BETWEEN_STEP_SALT once counter > 0, like
    the oracle's reset()."""
    from ti5_isaacgym_amd import make_t1_env
    n = 256
    env = make_t1_env(num_envs=n, mesh_type="plane", seed=9, device="cuda:0")
    env.reset()
    env.episode_length_buf[::5] = int(env.max_episode_length)   # these envs time out in the next step
    env.step(torch.zeros(n, 12, device="cuda:0"))
    r = env.reset_buf.bool()
    assert r[::5].all()
    kp = env.randomized_p_gains.clone()
    env.reset_idx_all()
    torch.cuda.synchronize()
    assert (env.randomized_p_gains[r] != kp[r]).all(dim=1).all(), "reset() reused the in-step reset's draws"
