"""Frame-history rollout storage (algo/rollout.py, history=(frame, frames)) rebuilds the same observation rows, bit for
bit, as the full storage -- through resets at every position of the rollout.

The rollout is produced the way the T1 env produces its actor observations (t1_dh_stand_env.py:368-481, 548-558): the
history shifts by one frame per step, a reset env's history is zeroed before the new frame is appended."""
import numpy as np
import torch

from ti5_isaacgym_amd.algo.rollout import RolloutStorage

FRAME, FRAMES, T, N = 5, 7, 12, 9


def _rollout(seed):
    g = torch.Generator().manual_seed(seed)
    hist = torch.randn(N, FRAMES, FRAME, generator=g)          # the history before the rollout
    hist[::4, :3] = 0.0                                         # some envs reset shortly before the rollout
    steps = []
    for k in range(T):
        done = torch.rand(N, generator=g) < 0.25
        steps.append((hist.reshape(N, -1).clone(), done))
        new = torch.randn(N, FRAME, generator=g)
        hist = torch.cat([hist[:, 1:], new[:, None]], 1)
        hist[done, :-1] = 0.0                                   # reset: zeroed history, then the new frame
    return steps


def _fill(storage, steps):
    t = RolloutStorage.Transition()
    for obs, done in steps:
        t.observations, t.critic_observations = obs, obs[:, :3]
        t.actions = torch.zeros(N, 2)
        t.rewards, t.dones = torch.zeros(N), done
        t.values, t.actions_log_prob = torch.zeros(N, 1), torch.zeros(N)
        t.action_mean, t.action_sigma = torch.zeros(N, 2), torch.ones(N, 2)
        storage.add_transitions(t)


def test_history_storage_rebuilds_every_row():
    steps = _rollout(0)
    full = RolloutStorage(N, T, [FRAME * FRAMES], [3], [2])
    comp = RolloutStorage(N, T, [FRAME * FRAMES], [3], [2], history=(FRAME, FRAMES))
    _fill(full, steps)
    _fill(comp, steps)
    assert sum(int(d.sum()) for _, d in steps) > 5
    for dtype in (None, torch.bfloat16):
        torch.manual_seed(3)
        a = list(full.mini_batch_generator(3, 2, obs_dtype=dtype))
        torch.manual_seed(3)
        b = list(comp.mini_batch_generator(3, 2, obs_dtype=dtype))
        assert len(a) == len(b) == 6
        for x, y in zip(a, b):
            assert x[0].dtype == y[0].dtype
            assert torch.equal(x[0], y[0]), (x[0] - y[0]).abs().max()
            for u, v in zip(x[1:9], y[1:9]):
                assert torch.equal(u, v)


def test_history_storage_size():
    comp = RolloutStorage(8192, 24, [47 * 66], [219], [12], history=(47, 66))
    assert comp.observations is None
    nbytes = comp.obs0.numel() * 4 + comp.frames.numel() * 4
    assert nbytes < 140e6 and 24 * 8192 * 3102 * 4 > 2.4e9
