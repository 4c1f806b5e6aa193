"""Full HIP step path (k_dynamics + its history-shift workgroups, k_post_a, k_post_b) at BASELINE sizes.

The golden fixtures pin post-physics on injected states at small N (test_gpu_parity.py).  Here the product
path runs as bench.py runs it -- real dynamics, the history shift fused into the dynamics launch -- at the
BASELINE configs, checked through properties that hold at any size:

  * history: for envs not reset this step, the 66-frame obs and 3-frame critic histories are the previous
    step's shifted by one frame (bit-exact); for reset envs the older frames are zero (t1_dh_stand_env.py
    reset_idx clears the deques before compute_observations appends the newest frame);
  * (every 7th env is started near its time-out so reset rows occur)
  * every buffer stays finite and obs / critic obs stay within clip_observations.

Cases: configs[2] (8192 envs, trimesh curriculum + DR), a ragged 777-env plane run (last workgroup partly
empty, history length not a multiple of the 16-B chunk), and configs[4]'s 32768 envs with pushes on a
height field (state kept in fp32 here).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _push_hook(cfg):
    cfg.domain_rand.push_robots = True
    cfg.domain_rand.push_interval_s = 0.05


@pytest.mark.parametrize("n,mesh,hook", [(8192, "trimesh", None), (777, "plane", None),
                                         (32768, "heightfield", _push_hook)],
                         ids=["config3_8192_trimesh", "ragged777_plane", "config5_fp32_32768_hf_push"])
def test_step_history_shift_and_invariants(n, mesh, hook):
    from ti5_isaacgym_amd import make_t1_env
    env = make_t1_env(num_envs=n, mesh_type=mesh, seed=3, device="cuda:0", cfg_hook=hook)
    F, Fp = env.cfg.env.num_single_obs, env.cfg.env.single_num_privileged_obs
    clip = env.cfg.normalization.clip_observations
    env.reset()
    # every 7th env times out within a few steps, so reset rows occur on the product path
    env.episode_length_buf[::7] = int(env.max_episode_length) - 3 - torch.arange(0, n, 7, device="cuda:0") % 5
    g = torch.Generator(device="cuda:0").manual_seed(0)
    prev_o, prev_p = env.obs_buf.clone(), env.privileged_obs_buf.clone()
    resets = 0
    for _ in range(60):
        obs, priv, rew, reset, _ = env.step(torch.randn(n, 12, device="cuda:0", generator=g))
        r = reset.bool()
        k = ~r
        resets += int(r.sum())
        assert torch.equal(obs[k, :-F], prev_o[k, F:])
        assert torch.equal(priv[k, :-Fp], prev_p[k, Fp:])
        assert not obs[r, :-F].any() and not priv[r, :-Fp].any()
        assert torch.isfinite(obs).all() and torch.isfinite(priv).all() and torch.isfinite(rew).all()
        assert obs.abs().max() <= clip and priv.abs().max() <= clip
        prev_o, prev_p = obs.clone(), priv.clone()
    assert torch.isfinite(env.root_states).all() and torch.isfinite(env.dof_pos).all()
    assert resets > 0, "no env reset in 60 random-action steps: the reset rows were not exercised"
