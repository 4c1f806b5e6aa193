"""Dev probe: the opt-in bf16 PPO update (DHPPO.amp_dtype) against the fp32 update on the same rollout.

    python tools/ppo_amp_check.py [--num-envs 8192] [--iters 3]

For each of --iters iterations: one rollout of the fp32 policy on the MI355X env (24 steps x N envs), then DHPPO.update()
twice from the same weights, optimizer state, storage and minibatch permutation (reseeded) -- in fp32 and in bf16.
Reported per iteration: the three mean losses of each, the relative L2 difference of the weight updates
|dW_bf16 - dW_fp32| / |dW_fp32| over all parameters, and the per-minibatch update time of each (CUDA events).  The
fp32 update's weights are kept, so the iterations follow the fp32 training trajectory.
"""
import argparse
import copy
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd import make_t1_env, task_registry  # noqa: E402
from ti5_isaacgym_amd.algo import DHOnPolicyRunner  # noqa: E402
from ti5_isaacgym_amd.utils.helpers import class_to_dict  # noqa: E402


def snapshot_storage(st):
    return {k: v.clone() for k, v in vars(st).items() if torch.is_tensor(v)}


def restore_storage(st, snap):
    with torch.inference_mode():   # the rollout wrote some storage rows as inference tensors
        for k, v in snap.items():
            getattr(st, k).copy_(v)


def timed_update(alg, dtype, seed):
    alg.amp_dtype = dtype
    torch.manual_seed(seed)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    losses = alg.update()
    e1.record()
    torch.cuda.synchronize()
    return losses, e0.elapsed_time(e1)


def compare_updates(r, seed):
    """bf16 then fp32 DHPPO.update() from the same weights, optimizer state, storage and minibatch seed; the fp32
    result is kept.  Returns (losses_fp32, losses_bf16, relative L2 difference of the weight updates, ms fp32,
    ms bf16)."""
    alg = r.alg
    snap = snapshot_storage(alg.storage)
    w0 = [q.detach().clone() for q in alg.actor_critic.parameters()]
    opt0 = copy.deepcopy(alg.optimizer.state_dict())
    lr0 = alg.learning_rate
    ls_bf16, ms_bf16 = timed_update(alg, torch.bfloat16, seed)
    w_bf16 = [q.detach().clone() for q in alg.actor_critic.parameters()]
    # back to the start of the iteration, then the fp32 update (kept)
    with torch.no_grad():
        for q, q0 in zip(alg.actor_critic.parameters(), w0):
            q.copy_(q0)
    alg.optimizer.load_state_dict(copy.deepcopy(opt0))   # adopted as is, then changed in place
    alg.learning_rate = lr0
    for g in alg.optimizer.param_groups:
        g["lr"] = lr0
    restore_storage(alg.storage, snap)
    alg.storage.step = r.num_steps_per_env
    ls_fp32, ms_fp32 = timed_update(alg, None, seed)
    w_fp32 = [q.detach() for q in alg.actor_critic.parameters()]
    num = sum(((wb - wf) ** 2).sum() for wb, wf in zip(w_bf16, w_fp32)) ** 0.5
    den = sum(((wf - w) ** 2).sum() for wf, w in zip(w_fp32, w0)) ** 0.5
    return ls_fp32, ls_bf16, float(num / den), ms_fp32, ms_bf16


def compare_cast_once(r, seed):
    """The bf16 update with the actor observations cast per minibatch by autocast (cast_obs_once off) and then
    cast once per update (on, the default), from the same weights, optimizer state, storage and minibatch seed;
    the second result is kept.  Returns (losses off, losses on, max |dW| difference, ms off, ms on)."""
    alg = r.alg
    snap = snapshot_storage(alg.storage)
    w0 = [q.detach().clone() for q in alg.actor_critic.parameters()]
    opt0 = copy.deepcopy(alg.optimizer.state_dict())
    lr0 = alg.learning_rate
    alg.cast_obs_once = False
    ls_off, ms_off = timed_update(alg, torch.bfloat16, seed)
    w_off = [q.detach().clone() for q in alg.actor_critic.parameters()]
    with torch.no_grad():
        for q, q0 in zip(alg.actor_critic.parameters(), w0):
            q.copy_(q0)
    alg.optimizer.load_state_dict(copy.deepcopy(opt0))   # adopted as is, then changed in place
    alg.learning_rate = lr0
    for g in alg.optimizer.param_groups:
        g["lr"] = lr0
    restore_storage(alg.storage, snap)
    alg.storage.step = r.num_steps_per_env
    alg.cast_obs_once = True
    ls_on, ms_on = timed_update(alg, torch.bfloat16, seed)
    alg.amp_dtype = None
    diff = max(float((a - b.detach()).abs().max()) for a, b in zip(w_off, alg.actor_critic.parameters()))
    return ls_off, ls_on, diff, ms_off, ms_on


def rollout(r, obs, critic):
    alg = r.alg
    with torch.inference_mode():
        for _ in range(r.num_steps_per_env):
            actions = alg.act(obs, critic)
            obs, priv, rew, dones, infos = r.env.step(actions)
            critic = priv if priv is not None else obs
            alg.process_env_step(rew, dones, infos)
        alg.compute_returns(critic)
    return obs, critic


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--num-envs", type=int, default=8192)
    p.add_argument("--iters", type=int, default=3)
    p.add_argument("--cast-ab", action="store_true",
                   help="bf16 update: actor observations cast per minibatch (autocast) vs once per update")
    a = p.parse_args()
    dev = torch.device("cuda:0")
    env = make_t1_env(num_envs=a.num_envs, mesh_type="trimesh", seed=5, device=str(dev))
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    r = DHOnPolicyRunner(env, class_to_dict(tc), None, device=str(dev))
    alg = r.alg
    alg.actor_critic.train()
    obs, priv = env.reset()
    critic = priv if priv is not None else obs
    out = []
    for it in range(a.iters + 1):   # iteration 0 warms the libraries up (not reported)
        obs, critic = rollout(r, obs, critic)
        if a.cast_ab:
            ls_off, ls_on, diff, ms_off, ms_on = compare_cast_once(r, 1000 + it)
            if it > 0:
                out.append({"iter": it, "losses_cast_per_minibatch": ls_off, "losses_cast_once": ls_on,
                            "max_abs_weight_diff": diff, "update_ms_cast_per_minibatch": round(ms_off, 2),
                            "update_ms_cast_once": round(ms_on, 2)})
            continue
        ls_fp32, ls_bf16, rel, ms_fp32, ms_bf16 = compare_updates(r, 1000 + it)
        if it > 0:
            out.append({"iter": it, "losses_fp32": [round(x, 6) for x in ls_fp32],
                        "losses_bf16": [round(x, 6) for x in ls_bf16],
                        "rel_weight_update_diff": round(rel, 5),
                        "update_ms_fp32": round(ms_fp32, 2), "update_ms_bf16": round(ms_bf16, 2)})
    print(json.dumps({"num_envs": a.num_envs, "minibatches": alg.num_mini_batches, "epochs": alg.num_learning_epochs,
                      "iters": out}))


if __name__ == "__main__":
    main()
