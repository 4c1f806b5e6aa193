"""Data-parallel PPO update on 2 gloo ranks == the single-process update on all envs.

Each rank holds half of a deterministic rollout (keyed by global env id).  With full-batch epochs the
bucketed gradient all-reduce, the all-reduced advantage statistics and the all-reduced KL mean (adaptive
learning rate) must reproduce the single-process update of the concatenated rollout, and both ranks must
end with identical weights.  The same code runs over RCCL on MI355X (backend "nccl").
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ti5_isaacgym_amd.algo import DHPPO
from ti5_isaacgym_amd.envs.configs import DHT1StandCfgPPO
from ti5_isaacgym_amd.utils.helpers import class_to_dict
from test_ppo import t1_policy

N_TOTAL, T, WORLD = 16, 6, 2


def _alg(env_ids):
    torch.manual_seed(5)
    cfg = class_to_dict(DHT1StandCfgPPO())["algorithm"]
    cfg.update(num_mini_batches=1, num_learning_epochs=2, schedule="adaptive", learning_rate=1e-3)
    alg = DHPPO(t1_policy(), device="cpu", **cfg)
    n = len(env_ids)
    alg.init_storage(n, T, [66 * 47], [219], [12])
    s = alg.storage
    e = torch.as_tensor(env_ids, dtype=torch.float32)
    for t in range(T):
        k = torch.arange(66 * 47, dtype=torch.float32)
        s.observations[t] = torch.sin(0.01 * k[None] * (1 + 0.1 * e[:, None]) + 0.5 * t) * 0.5
        s.privileged_observations[t] = torch.cos(0.03 * torch.arange(219.0)[None] + e[:, None] + t) * 0.5
        s.actions[t] = torch.sin(e[:, None] + torch.arange(12.0)[None] + t)
        s.rewards[t, :, 0] = torch.cos(0.7 * e + t)
        s.values[t, :, 0] = 0.3 * torch.sin(0.2 * e - t)
        s.dones[t, :, 0] = torch.from_numpy(((env_ids + t) % 4 == 0).astype(np.uint8))
        s.actions_log_prob[t, :, 0] = -12.0 + 0.1 * torch.sin(e + t)
        s.mu[t] = 0.2 * torch.cos(e[:, None] + torch.arange(12.0)[None] - t)
        s.sigma[t] = 1.0
    s.step = T
    alg.storage.compute_returns(0.1 * torch.cos(e)[:, None], alg.gamma, alg.lam)
    return alg


def _flat(alg):
    return torch.cat([p.detach().reshape(-1) for p in alg.actor_critic.parameters()]).numpy()


def _worker(rank, port, out):
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    ids = np.arange(N_TOTAL // WORLD) + rank * (N_TOTAL // WORLD)
    alg = _alg(ids)
    losses = alg.update()
    np.save(os.path.join(out, f"params{rank}.npy"), _flat(alg))
    np.save(os.path.join(out, f"meta{rank}.npy"), np.array([alg.learning_rate, *losses]))
    dist.barrier()
    dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_update_equals_single_process(tmp_path):
    mp.spawn(_worker, args=(_port(), str(tmp_path)), nprocs=WORLD, join=True)
    p0, p1 = np.load(tmp_path / "params0.npy"), np.load(tmp_path / "params1.npy")
    np.testing.assert_array_equal(p0, p1)  # ranks stay in lock-step
    single = _alg(np.arange(N_TOTAL))
    before = _flat(single)
    single.update()
    ref = _flat(single)
    assert np.abs(ref - before).max() > 1e-5, "the update did not move the weights"
    np.testing.assert_allclose(p0, ref, rtol=0, atol=2e-6)
    m0 = np.load(tmp_path / "meta0.npy")
    assert m0[0] == single.learning_rate  # same adaptive learning-rate decisions
