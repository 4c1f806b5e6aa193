"""f1: the build's PPO (ti5_isaacgym_amd/algo: DHPPO, RolloutStorage, ActorCriticDH) vs the reference's own update.

tests/golden/ppo_update.npz was produced by the reference's DHPPO / RolloutStorage / ActorCriticDH
(humanoid/algo/ppo/dh_ppo.py:112-205, rollout_storage.py:97-173, actor_critic_dh.py) on a seeded policy and a seeded
synthetic rollout (tests/golden/gen_ppo_golden.py, which this test shares the input generator with).  Replayed
through the build with the reference's recorded actions and minibatch permutation:

  * act(): values, log-probs, action mean / sigma of the recorded actions (1e-5 relative);
  * process_env_step(): the time-out bootstrapped rewards (1e-6);
  * compute_returns(): GAE returns and normalised advantages (1e-5);
  * update(): the learning rate of every minibatch (adaptive KL schedule: equal), the three mean losses it returns
    (1e-4 relative), and per parameter tensor the change of the weights (sum and abs-sum of new - old within 1 % of
    the abs-sum; 8 probed elements within 2 % of the largest probe).  Adam's first steps move each weight by about
    +-lr whatever the gradient's size, so a gradient element that is zero up to rounding may take either sign:
    hence the abs-sum-relative bounds rather than elementwise equality.

CPU here (the reference's device): measured, the updated weights come out bit-identical to the reference's and the
losses within 2e-7 (the build sums them on the device).  The same replay runs on the MI355X (the HIP fp32 update
kernels: three-part bf16 split weight gradients, the packed conv, hipBLASLt or the HIP GEMM) in the gpu test, with the
same bounds (measured: losses within 2.5e-5, weight-delta abs-sums within 1.1e-6).
"""
import numpy as np
import pytest
import torch

from gen_ppo_golden import ALGO, N, POLICY, POLICY_SEED, T, probe_index, synthetic_rollout
from golden_util import GOLDEN


def load():
    d = np.load(f"{GOLDEN}/ppo_update.npz")
    return {k: d[k] for k in d.files}


def close(name, got, ref, rtol, atol=0.0):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, (name, got.shape, ref.shape)
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=atol, err_msg=name)


def replay(device, monkeypatch):
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH
    from ti5_isaacgym_amd.algo.dh_update import DHPPO
    fx = load()
    torch.manual_seed(POLICY_SEED)
    ac = ActorCriticDH(235, 47, 219, 12, **POLICY)
    alg = DHPPO(ac, device=device, **ALGO)
    alg.graph_act = False
    alg.init_storage(N, T, [66 * 47], [219], [12])
    obs, cobs, rew, dones, tout = synthetic_rollout()
    close("obs_digest", [obs.double().sum().item(), obs.double().abs().sum().item()], fx["obs_digest"], 1e-12)
    dev = torch.device(device)
    obs, cobs, rew, dones, tout = (x.to(dev) for x in (obs, cobs, rew, dones, tout))
    tol = 1e-5 if dev.type == "cpu" else 2e-4
    with torch.no_grad():
        for t in range(T):
            tr = alg.transition
            a = torch.from_numpy(fx["actions"][t]).to(dev)
            ac.act(obs[t])
            tr.actions = a
            tr.values = ac.evaluate(cobs[t])
            tr.actions_log_prob = ac.get_actions_log_prob(a)
            tr.action_mean, tr.action_sigma = ac.action_mean, ac.action_std
            tr.observations, tr.critic_observations = obs[t], cobs[t]
            close(f"values[{t}]", tr.values.cpu(), fx["values"][t], tol, 1e-6)
            close(f"log_prob[{t}]", tr.actions_log_prob.cpu(), fx["log_prob"][t], tol, 1e-5)
            close(f"mu[{t}]", tr.action_mean.cpu(), fx["mu"][t], tol, 1e-6)
            close(f"sigma[{t}]", tr.action_sigma.cpu(), fx["sigma"][t], 1e-7)
            alg.process_env_step(rew[t], dones[t], {"time_outs": tout[t]})
            close(f"stored_rewards[{t}]", alg.storage.rewards[t].cpu(), fx["stored_rewards"][t], 1e-6, 1e-7)
        alg.compute_returns(cobs[T])
    close("returns", alg.storage.returns.cpu(), fx["returns"], tol, 1e-6)
    close("advantages", alg.storage.advantages.cpu(), fx["advantages"], 10 * tol, 1e-5)
    perm = torch.from_numpy(fx["perm"])
    monkeypatch.setattr(torch, "randperm", lambda n, **kw: perm.to(kw.get("device", "cpu")))
    before = {k: v.detach().clone().double().cpu() for k, v in ac.state_dict().items()}
    lrs = []
    orig_step = alg.optimizer.step

    def step_and_record(*a, **k):
        lr = alg.optimizer.param_groups[0]["lr"]
        lrs.append(float(lr))   # the device keeps it as a tensor (read here: a sync, test only)
        return orig_step(*a, **k)
    alg.optimizer.step = step_and_record
    alg.graph_update = False   # every minibatch through the Python step (a captured graph replays without it)
    losses = alg.update()
    return fx, ac, before, lrs, losses


def check_update(fx, ac, before, lrs, losses, loss_rtol, lr_rtol=0.0):
    # the host keeps the reference's float64 learning rate; the device an fp32 tensor (DHPPO._lr_t)
    np.testing.assert_allclose(np.array(lrs), fx["lrs"], rtol=lr_rtol, atol=0)
    rel = np.abs(np.asarray(losses, np.float64) - fx["losses"]) / np.abs(fx["losses"])
    print("losses relative error vs the reference:", rel)
    close("losses", losses, fx["losses"], loss_rtol)
    names = [str(n) for n in fx["names"]]
    sd = ac.state_dict()
    worst = 0.0
    assert names == list(sd.keys())
    for i, k in enumerate(names):
        d = (sd[k].detach().double().cpu() - before[k]).reshape(-1)
        s, a, _ = fx["delta_stats"][i]
        assert a > 0 or k == "std", k
        worst = max(worst, abs(d.abs().sum().item() - a) / a if a > 0 else 0.0)
        assert abs(d.abs().sum().item() - a) <= 0.01 * a + 1e-12, (k, d.abs().sum().item(), a)
        assert abs(d.sum().item() - s) <= 0.01 * a + 1e-12, (k, d.sum().item(), s, a)
        p = d[torch.from_numpy(probe_index(d.numel()))].numpy()
        ref = fx["delta_probes"][i]
        assert np.abs(p - ref).max() <= 0.02 * np.abs(ref).max() + 1e-12, (k, p, ref)
    print(f"weight deltas: worst abs-sum relative gap {worst:.2e}")


def test_update_matches_reference_cpu(monkeypatch):
    check_update(*replay("cpu", monkeypatch), loss_rtol=1e-4)


@pytest.mark.gpu
def test_update_matches_reference_gpu(monkeypatch):
    # the CPU's loss bound: the fp32 update's weight gradients are fp32-class on the device too (three-part bf16 split
    # on the matrix cores; measured within 2.5e-5 relative of the reference's losses, profiles/r06e_update_tests.txt)
    check_update(*replay("cuda:0", monkeypatch), loss_rtol=1e-4, lr_rtol=1e-6)
