"""The data-parallel PPO update on the device, graphed -- needs the MI355X.

Under data parallelism DHPPO replays the minibatch step as two captured graphs -- A: forward, losses, this rank's KL
mean, backward into the gradient bucket; B: the adaptive learning-rate decision, clipping, Adam -- with the gradient
and KL all-reduce between them (dh_ppo.py:139-151, 180-182).  Two `gloo` ranks on cuda:0, each with half of a
deterministic rollout (keyed by global env id, as tests/test_ppo_distributed.py on the CPU):

  * the two ranks end bit-identical (weights, Adam state, learning rate);
  * the graphed DP update equals the eager DP update bit for bit (the same kernels, replayed);
  * both equal the single-process graphed update of the concatenated rollout within fp32 summation order.

The same code runs over RCCL on an 8-GPU node (backend "nccl"), which this pool does not give a test process.
"""
import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N_TOTAL, T, WORLD, ITERS = 64, 6, 2, 2


def _alg(env_ids, graphed, amp=None):
    from ti5_isaacgym_amd.algo import DHPPO
    from ti5_isaacgym_amd.envs.configs import DHT1StandCfgPPO
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    from test_ppo import t1_policy
    torch.manual_seed(5)
    cfg = class_to_dict(DHT1StandCfgPPO())["algorithm"]
    # full-batch epochs: the minibatch is the whole (local) rollout, so the ranks' and the single process's batches
    # hold the same transitions; 4 epochs = 2 eager warm-up steps, the capture and a replay
    cfg.update(num_mini_batches=1, num_learning_epochs=4, schedule="adaptive", learning_rate=1e-3)
    alg = DHPPO(t1_policy().to("cuda:0"), device="cuda:0", amp_dtype=amp, **cfg)
    alg.graph_update = graphed
    alg.init_storage(len(env_ids), T, [66 * 47], [219], [12])
    return alg


def _fill(alg, env_ids, it):
    s = alg.storage
    e = torch.as_tensor(env_ids, dtype=torch.float32, device="cuda:0")
    k = torch.arange(66 * 47, dtype=torch.float32, device="cuda:0")
    j = torch.arange(12.0, device="cuda:0")
    for t in range(T):
        u = t + 3 * it
        s.observations[t] = torch.sin(0.01 * k[None] * (1 + 0.1 * e[:, None]) + 0.5 * u) * 0.5
        s.privileged_observations[t] = torch.cos(0.03 * torch.arange(219.0, device="cuda:0")[None] + e[:, None] + u) * 0.5
        s.actions[t] = torch.sin(e[:, None] + j[None] + u)
        s.rewards[t, :, 0] = torch.cos(0.7 * e + u)
        s.values[t, :, 0] = 0.3 * torch.sin(0.2 * e - u)
        s.dones[t, :, 0] = ((e.long() + u) % 4 == 0).to(torch.uint8)
        s.actions_log_prob[t, :, 0] = -12.0 + 0.1 * torch.sin(e + u)
        s.mu[t] = 0.2 * torch.cos(e[:, None] + j[None] - u)
        s.sigma[t] = 1.0
    s.step = T
    s.compute_returns(0.1 * torch.cos(e)[:, None], alg.gamma, alg.lam)


def _snapshot(alg):
    w = torch.cat([p.detach().reshape(-1) for p in alg.actor_critic.parameters()]).cpu().numpy()
    st = [torch.cat([v[k].reshape(-1).float() for v in alg.optimizer.state.values()]).cpu().numpy()
          for k in ("exp_avg", "exp_avg_sq")]
    return w, st[0], st[1], alg.learning_rate


def _run(ids, graphed, amp=None):
    alg = _alg(ids, graphed, amp)
    losses = []
    for it in range(ITERS):
        _fill(alg, ids, it)
        alg.actor_critic.train()
        losses.append(alg.update())
    if graphed:
        assert alg._upd is not None, "the minibatch steps were not replayed"
    return _snapshot(alg), losses


def _worker(rank, port, out, amp_name):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        ids = np.arange(N_TOTAL // WORLD) + rank * (N_TOTAL // WORLD)
        for graphed in (True, False):
            (w, m, v, lr), losses = _run(ids, graphed, AMPS[amp_name])
            np.savez(os.path.join(out, f"r{rank}_g{int(graphed)}.npz"), w=w, m=m, v=v, lr=lr,
                     losses=np.array(losses))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


AMPS = {"fp32": None, "bf16": torch.bfloat16}


@pytest.mark.parametrize("amp_name", sorted(AMPS))
def test_graphed_dp_update_on_device(tmp_path, amp_name):
    """fp32 (the reference's dtype) and the opt-in bf16 update (under bf16 graph A also holds the parameters'
    bf16 shadows, the wgrad kernel adding into the bucket views, the field gather and the fold backward): the ranks stay
    bit-identical and graphed == eager DP bit for bit in both; against the single process fp32 agrees within fp32
    summation order, bf16 within 5% of the update's own size (a summation-order difference of a weight can flip its bf16
    rounding in the next minibatch's forward)."""
    import torch.multiprocessing as mp
    amp = AMPS[amp_name]
    mp.spawn(_worker, args=(_port(), str(tmp_path), amp_name), nprocs=WORLD, join=True)
    r = {(k, g): np.load(tmp_path / f"r{k}_g{g}.npz") for k in range(WORLD) for g in (0, 1)}
    for g in (0, 1):   # the ranks stay in lock-step (the logged losses are each rank's own means, as the reference's)
        for f in ("w", "m", "v", "lr"):
            np.testing.assert_array_equal(r[(0, g)][f], r[(1, g)][f], err_msg=f"rank 0 vs 1, graphed={g}: {f}")
    for k in range(WORLD):
        for f in ("w", "m", "v", "lr", "losses"):   # graphed == eager, bit for bit
            np.testing.assert_array_equal(r[(k, 1)][f], r[(k, 0)][f], err_msg=f"rank {k} graphed vs eager DP: {f}")
    (w, m, v, lr), losses = _run(np.arange(N_TOTAL), True, amp)   # the single process, the concatenated rollout
    w0 = torch.cat([p.detach().reshape(-1) for p in _alg(np.arange(N_TOTAL), False).actor_critic.parameters()])
    moved = np.abs(w - w0.cpu().numpy()).max()
    assert moved > 1e-5, "the updates did not move the weights"
    # equal shards: the mean of the ranks' mean losses is the single process's mean loss
    ml = 0.5 * (r[(0, 1)]["losses"] + r[(1, 1)]["losses"])
    if amp is None:
        np.testing.assert_allclose(r[(0, 1)]["w"], w, rtol=0, atol=5e-6)
        np.testing.assert_allclose(ml, np.array(losses), rtol=1e-5, atol=1e-6)
        assert float(r[(0, 1)]["lr"]) == lr   # the same adaptive learning-rate decisions
    else:
        gap = np.abs(r[(0, 1)]["w"] - w).max()
        print(f"bf16 DP vs single process: max weight gap {gap:.3g} against an update of {moved:.3g}")
        assert gap <= 0.05 * moved, (gap, moved)
        np.testing.assert_allclose(ml, np.array(losses), rtol=2e-2, atol=1e-4)
