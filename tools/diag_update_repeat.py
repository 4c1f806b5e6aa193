"""Dev probe: the same DHPPO.update() twice from one snapshot (weights, optimizer state, storage, seed) -- must give
identical losses; with the graphed and the eager minibatch step, fp32 and bf16."""
import importlib.util
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd import make_t1_env, task_registry  # noqa: E402
from ti5_isaacgym_amd.algo import DHOnPolicyRunner  # noqa: E402
from ti5_isaacgym_amd.utils.helpers import class_to_dict  # noqa: E402

spec = importlib.util.spec_from_file_location("chk", os.path.join(os.path.dirname(os.path.abspath(__file__)), "ppo_amp_check.py"))
chk = importlib.util.module_from_spec(spec)
spec.loader.exec_module(chk)
import copy  # noqa: E402

env = make_t1_env(num_envs=1024, mesh_type="plane", seed=5, device="cuda:0")
_, train_cfg = task_registry.get_cfgs("t1_dh_stand")
torch.manual_seed(0)
r = DHOnPolicyRunner(env, class_to_dict(train_cfg), None, device="cuda:0")
r.alg.actor_critic.train()
obs, priv = env.reset()
obs, critic = chk.rollout(r, obs, priv if priv is not None else obs)
alg = r.alg
snap = chk.snapshot_storage(alg.storage)
w0 = [q.detach().clone() for q in alg.actor_critic.parameters()]
opt0 = copy.deepcopy(alg.optimizer.state_dict())
lr0 = alg.learning_rate
for graphed in (True, False):
    for dt in (None, torch.bfloat16):
        for rep in range(3):
            with torch.no_grad():
                for q, q0 in zip(alg.actor_critic.parameters(), w0):
                    q.copy_(q0)
            alg.optimizer.load_state_dict(copy.deepcopy(opt0))   # adopted as is, then changed in place
            alg.learning_rate = lr0
            for g in alg.optimizer.param_groups:
                g["lr"] = lr0
            chk.restore_storage(alg.storage, snap)
            alg.storage.step = r.num_steps_per_env
            alg.graph_update = graphed
            alg.amp_dtype = dt
            torch.manual_seed(5)
            ls = alg.update()
            print("graphed", graphed, "dtype", dt, "rep", rep, ls, "lr", alg.learning_rate, flush=True)
