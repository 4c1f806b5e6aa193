"""Phase timing of one DH-PPO minibatch step on the MI355X (where the update's time goes): the minibatch gather,
the forward passes (history CNN, state estimator, actor, critic), the losses, backward, gradient clipping and Adam.
CUDA events around each phase, averaged over the update's 8 minibatches after a warm-up update.

    python tools/prof_ppo_update.py [--num-envs 8192]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd import task_registry  # noqa: E402
from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH  # noqa: E402
from ti5_isaacgym_amd.algo.dh_update import DHPPO  # noqa: E402
from ti5_isaacgym_amd.utils.helpers import class_to_dict  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--num-envs", type=int, default=8192)
p.add_argument("--steps", type=int, default=24)
a = p.parse_args()
dev = torch.device("cuda:0")
_, tc = task_registry.get_cfgs("t1_dh_stand")
cfg = class_to_dict(tc)
torch.manual_seed(0)
ac = ActorCriticDH(235, 47, 219, 12, **cfg["policy"]).to(dev)
alg = DHPPO(ac, device=str(dev), **cfg["algorithm"])
N, T = a.num_envs, a.steps
alg.init_storage(N, T, [3102], [219], [12])
st = alg.storage
g = torch.Generator(device=dev).manual_seed(1)
st.observations.normal_(generator=g)
st.privileged_observations.normal_(generator=g)
st.actions.normal_(generator=g)
st.values.normal_(generator=g)
st.returns.normal_(generator=g)
st.advantages.normal_(generator=g)
st.actions_log_prob.normal_(generator=g)
st.mu.normal_(generator=g)
st.sigma.fill_(1.0)

names = ["gather", "history_cnn", "state_est+actor", "critic", "losses", "backward", "clip", "adam"]
acc = {k: 0.0 for k in names}
count = 0


def run(record):
    global count
    gen = st.mini_batch_generator(alg.num_mini_batches, alg.num_learning_epochs)
    mse = nn.MSELoss()
    it = iter(gen)
    while True:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
        ev[0].record()
        try:
            obs_b, critic_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b, old_sigma_b, _, _ = next(it)
        except StopIteration:
            return
        ev[1].record()
        short = obs_b[..., -ac.num_short_obs:]
        code = ac.long_history(obs_b.view(-1, ac.in_channels, ac.num_proprio_obs))
        ev[2].record()
        est = ac.state_estimator(short)
        ac.update_distribution(torch.cat((short, est, code), dim=-1))
        logp = ac.get_actions_log_prob(actions_b)
        ev[3].record()
        value = ac.evaluate(critic_b)
        ev[4].record()
        ratio = torch.exp(logp - torch.squeeze(old_logp_b))
        adv = torch.squeeze(adv_b)
        surr = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 0.8, 1.2)).mean()
        v_clip = target_values_b + (value - target_values_b).clamp(-0.2, 0.2)
        vloss = torch.max((value - returns_b).pow(2), (v_clip - returns_b).pow(2)).mean()
        se = mse(ac.state_estimator(short), critic_b[:, alg.lin_vel_idx:alg.lin_vel_idx + 3])
        loss = surr + vloss - alg.entropy_coef * ac.entropy.mean() + se
        ev[5].record()
        alg.optimizer.zero_grad(set_to_none=False)
        loss.backward()
        ev[6].record()
        nn.utils.clip_grad_norm_(ac.parameters(), alg.max_grad_norm)
        ev[7].record()
        alg.optimizer.step()
        ev[8].record()
        if record:
            torch.cuda.synchronize()
            for i, k in enumerate(names):
                acc[k] += ev[i].elapsed_time(ev[i + 1])
            count += 1


run(False)
torch.cuda.synchronize()
run(True)
mb = N * T // alg.num_mini_batches
out = {"num_envs": N, "minibatch": mb, "minibatches": count,
       "ms_per_minibatch": {k: round(v / count, 3) for k, v in acc.items()},
       "ms_per_update": round(sum(acc.values()) / count * alg.num_mini_batches * alg.num_learning_epochs, 2)}
print(json.dumps(out))
