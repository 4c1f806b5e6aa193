"""BASELINE config 5's fp16 state storage (cfg.env.state_dtype = "fp16", t1env_config.obs_half) -- needs the MI355X.

With fp16 histories the env computes every observation / critic value in fp32 exactly as with fp32 histories and
rounds it once to fp16 (round to nearest even) when it stores the newest frame; the shift then moves halves.  The
histories do not feed back into the physics or the rewards, so an fp16 env and an fp32 env started from the same
seed and stepped with the same actions must agree:

  * obs / critic histories: fp16 == the fp32 env's values rounded to fp16, bit for bit (every frame, so also the
    shifted and the reset-zeroed ones);  |fp16 - fp32| <= 2**-11 |fp32| follows (half an fp16 ulp, relative);
  * rewards, resets, root / dof state and every other buffer: bit-identical (same kernels, same inputs).

Run at configs[4]'s size (32768 envs, height field, pushes; the history shift is its own launch there) and on a
ragged 777-env trimesh run (fused shift workgroups, partial last unit), each for 12 steps with resets.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _make(n, mesh, dtype):
    from ti5_isaacgym_amd import make_t1_env

    def hook(cfg):
        cfg.env.state_dtype = dtype
        cfg.domain_rand.push_robots = True
        cfg.domain_rand.push_interval_s = 0.03
    return make_t1_env(num_envs=n, mesh_type=mesh, seed=4, device="cuda:0", cfg_hook=hook)


@pytest.mark.parametrize("kernel", ["6", "4"])
@pytest.mark.parametrize("n,mesh", [(32768, "heightfield"), (777, "trimesh")], ids=["config5_32768_hf", "ragged777"])
def test_fp16_histories_equal_rounded_fp32(n, mesh, kernel, monkeypatch):
    # one step kernel for both envs (the default takes k_dyn4 for fp16 histories above one workgroup round, k_dyn6
    # for fp32: different fp32 summation orders, t1_dyn_waves_default)
    monkeypatch.setenv("T1ENV_DYN_KERNEL", kernel)
    e32, e16 = _make(n, mesh, "fp32"), _make(n, mesh, "fp16")
    assert e16.obs_buf.dtype == torch.float16 and e32.obs_buf.dtype == torch.float32
    for e in (e32, e16):
        e.reset()
        e.episode_length_buf[::5] = int(e.max_episode_length) - 4 - torch.arange(0, n, 5, device="cuda:0") % 6
    g = torch.Generator(device="cuda:0").manual_seed(2)
    resets = 0
    for t in range(12):
        a = torch.randn(n, 12, device="cuda:0", generator=g)
        o32, p32, r32, d32, _ = e32.step(a)
        o16, p16, r16, d16, _ = e16.step(a)
        assert torch.equal(o16, o32.half()), f"obs step {t}"
        assert torch.equal(p16, p32.half()), f"priv step {t}"
        assert torch.equal(r16, r32) and torch.equal(d16, d32), f"rew/reset step {t}"
        assert torch.equal(e16.root_states, e32.root_states) and torch.equal(e16.dof_state, e32.dof_state)
        err = (o16.float() - o32).abs()
        assert (err <= o32.abs() * 2.0 ** -11 + 2.0 ** -25).all()
        resets += int(d32.sum())
    assert resets > 0
