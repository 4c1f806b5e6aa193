"""Height scan (terrain.measure_heights = True; inactive in DHT1StandCfg) on the MI355X.

The golden scenario heights16 (test_gpu_parity.py) pins it against the reference's own outputs.  Here:
  * k_measure_heights against the oracle's restatement of _get_heights (legged_robot.py:1551-1587) on random
    base poses over the whole field and past its edges (the clip to [0, rows-2] x [0, cols-2]), exact: the
    samples are int16 x vertical_scale, so a wrong cell is off by >= 0.005;
  * the full (real dynamics) step at 8192 envs: the critic history with heights, (N, 3 x 260), is the 73-wide
    critic history interleaved with the heights frames, the newest heights frame is
    clip(root_z - 0.5 - measured, -1, 1) x 5, and the older frames are the previous step's shifted frames,
    zero for envs reset this step (t1_dh_stand_env.py:466-468, 548-558).
"""
import numpy as np
import pytest
import torch

from oracle.t1_oracle import get_heights, height_points

pytestmark = pytest.mark.gpu


def _hook(cfg):
    cfg.terrain.measure_heights = True


def _env(n, mesh="trimesh"):
    from ti5_isaacgym_amd import make_t1_env
    return make_t1_env(num_envs=n, mesh_type=mesh, seed=3, device="cuda:0", cfg_hook=_hook)


def test_measure_heights_matches_oracle_on_random_poses():
    from ti5_isaacgym_amd import _lib
    n = 4096
    env = _env(n)
    tc = env.cfg.terrain
    hs = env.height_samples.cpu().numpy()
    assert np.unique(hs).size > 10
    rng = np.random.default_rng(7)
    ext_x = hs.shape[0] * tc.horizontal_scale - tc.border_size
    ext_y = hs.shape[1] * tc.horizontal_scale - tc.border_size
    root = np.zeros((n, 13), np.float32)
    root[:, 0] = rng.uniform(-tc.border_size - 3, ext_x + 3, n)
    root[:, 1] = rng.uniform(-tc.border_size - 3, ext_y + 3, n)
    root[:, 2] = rng.uniform(0.5, 1.5, n)
    q = rng.standard_normal((n, 4)).astype(np.float32)
    q /= np.linalg.norm(q, axis=1, keepdims=True)
    q[:64, :2] = 0.0          # pure yaw
    q[64:96, 2:4] = 0.0       # no yaw component: the clamped 1e-9 norm path
    root[:, 3:7] = q
    env.root_states.copy_(torch.from_numpy(root))
    out = torch.full((n, env.num_height_points), float("nan"), device="cuda:0")
    _lib.check(env._lib.t1env_measure_heights(env._handle, env._height_pts.data_ptr(), env.num_height_points,
                                              out.data_ptr(), env._stream()), "t1env_measure_heights")
    torch.cuda.synchronize()
    ref = get_heights(root[:, :3], root[:, 3:7], height_points(), hs, tc.horizontal_scale, tc.vertical_scale,
                      tc.border_size)
    got = out.cpu().numpy()
    np.testing.assert_array_equal(got[96:], ref[96:])
    # zero quaternion components: the reference divides 0 by the 1e-9 clamp -> q = 0, points unrotated but
    # collapsed (q_w = 0): same formula on both sides
    np.testing.assert_array_equal(got[64:96], ref[64:96])
    np.testing.assert_array_equal(got[:64], ref[:64])


def test_plane_measures_zero():
    env = _env(256, "plane")
    env.reset()
    assert env.privileged_obs_buf.shape == (256, 3 * (73 + 187))
    torch.testing.assert_close(env.measured_heights, torch.zeros_like(env.measured_heights))
    new = env.privileged_obs_buf.view(256, 3, 260)[:, 2, 73:]
    ref = torch.clamp(env.root_states[:, 2:3] - 0.5, -1, 1) * 5.0
    torch.testing.assert_close(new, ref.expand_as(new), rtol=0, atol=0)


def test_step_critic_history_with_heights():
    n = 8192
    env = _env(n)
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(2)
    env.episode_length_buf[::5] = int(env.max_episode_length) - 1 - torch.arange(0, n, 5, device="cuda:0") % 4
    resets = 0
    prev = env.privileged_obs_buf.view(n, 3, 260).clone()
    for t in range(12):
        env.step(0.3 * torch.randn(n, 12, device="cuda:0", generator=g))
        ext = env.privileged_obs_buf.view(n, 3, 260)
        base = env._priv[env._slot ^ 1].view(n, 3, 73)
        torch.testing.assert_close(ext[:, :, :73], base, rtol=0, atol=0)
        newest = torch.clamp(env.root_states[:, 2:3] - 0.5 - env.measured_heights, -1, 1) * 5.0
        torch.testing.assert_close(ext[:, 2, 73:], newest, rtol=0, atol=1e-6)
        r = env.reset_buf.bool()
        resets += int(r.sum())
        assert not ext[r, :2, 73:].any()
        torch.testing.assert_close(ext[~r, :2, 73:], prev[~r, 1:, 73:], rtol=0, atol=0)
        assert torch.isfinite(ext).all()
        prev = ext.clone()
    assert resets > 0
    # the heights vary over the curriculum terrain (the scan is not sampling a constant)
    assert env.measured_heights.std() > 0
