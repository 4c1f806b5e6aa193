"""T1DHStandEnv exposes the env contract the reference's runner uses: every attribute the reference's
DHOnPolicyRunner touched when tests/golden/gen_runner_golden.py drove it (the fixture's env_attrs), the nested config
fields its constructor reads (dh_on_policy_runner.py:42-58), and what learn() does with them -- reset / observation
shapes, step()'s five outputs with extras["episode"] / extras["time_outs"], a writable episode_length_buf
(init_at_random_ep_len) -- on the HIP env."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "runner_learn2.npz")


def test_hip_env_exposes_the_reference_runner_contract():
    from ti5_isaacgym_amd import make_t1_env
    attrs = [str(a) for a in np.load(FIX)["env_attrs"]]
    n = 64
    env = make_t1_env(num_envs=n, mesh_type="plane", device="cuda:0")
    for a in attrs + ["episode_length_buf", "max_episode_length"]:
        assert hasattr(env, a), a
    c = env.cfg
    for path in ("terrain.measure_heights", "terrain.num_height", "env.c_frame_stack", "env.single_num_privileged_obs"):
        obj = c
        for part in path.split("."):
            obj = getattr(obj, part)
    obs, priv = env.reset()
    assert obs.shape == (n, env.num_obs) and priv.shape == (n, env.num_privileged_obs)
    assert env.get_observations().shape == (n, env.num_obs)
    assert env.get_privileged_observations().shape == (n, env.num_privileged_obs)
    assert env.num_short_obs == 5 * env.num_single_obs and env.num_actions == 12
    # init_at_random_ep_len: the runner assigns a random episode_length_buf
    env.episode_length_buf = torch.randint_like(env.episode_length_buf, high=int(env.max_episode_length))
    out = env.step(torch.zeros(n, env.num_actions, device="cuda:0"))
    assert len(out) == 5
    o, p, r, d, infos = out
    assert o.shape == obs.shape and p.shape == priv.shape and r.shape == (n,) and d.shape == (n,)
    assert "episode" in infos and infos["time_outs"].shape == (n,)
    # learn()'s bookkeeping: rewards add, dones index
    cur = torch.zeros(n, device="cuda:0") + r
    new_ids = (d > 0).nonzero(as_tuple=False)
    assert cur[new_ids].shape[0] == int((d > 0).sum())
