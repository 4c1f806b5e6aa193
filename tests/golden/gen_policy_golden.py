"""Generate tests/golden/policy_dh.npz from the reference's own ActorCriticDH (run here, where /root/reference
exists; the fixture travels, the reference does not).

The reference module (humanoid/algo/ppo/actor_critic_dh.py) is pure torch and is loaded by file path.  Recorded
for a fixed seed with the t1 policy config (t1_dh_stand_config.py:434-445): per-parameter (sum, |sum|, first
element) of the initial weights, and on fixed inputs act_inference, evaluate, log_prob of fixed actions and
the entropy.  tests/test_ppo.py checks the build's ActorCriticDH against it.

    python tests/golden/gen_policy_golden.py [/root/reference]
"""
import importlib.util
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SEED = 11
POLICY = dict(init_noise_std=1.0, actor_hidden_dims=[512, 256, 128], critic_hidden_dims=[768, 256, 128],
              state_estimator_hidden_dims=[256, 128, 64], kernel_size=[6, 4], filter_size=[32, 16],
              stride_size=[3, 2], lh_output_dim=64, in_channels=66)


def main():
    path = os.path.join(REF, "humanoid", "algo", "ppo", "actor_critic_dh.py")
    spec = importlib.util.spec_from_file_location("ref_actor_critic_dh", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    torch.manual_seed(SEED)
    m = mod.ActorCriticDH(235, 47, 219, 12, **POLICY)
    sd = m.state_dict()
    names = list(sd.keys())
    stats = np.array([[v.double().sum().item(), v.double().abs().sum().item(), v.reshape(-1)[0].double().item()]
                      for v in sd.values()])
    g = torch.Generator().manual_seed(7)
    obs = torch.randn(4, 66 * 47, generator=g)
    cobs = torch.randn(4, 219, generator=g)
    actions = torch.randn(4, 12, generator=g)
    with torch.no_grad():
        act_inf = m.act_inference(obs)
        value = m.evaluate(cobs)
        m.act(obs)  # sets the distribution
        logp = m.get_actions_log_prob(actions)
        ent = m.entropy
    np.savez(os.path.join(HERE, "policy_dh.npz"), seed=SEED, names=np.array(names), stats=stats,
             obs=obs.numpy(), critic_obs=cobs.numpy(), actions=actions.numpy(), act_inference=act_inf.numpy(),
             value=value.numpy(), log_prob=logp.numpy(), entropy=ent.numpy())
    print("wrote", os.path.join(HERE, "policy_dh.npz"), len(names), "tensors")


if __name__ == "__main__":
    main()
