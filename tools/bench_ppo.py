"""PPO iteration timing on one GPU: rollout collection (policy inference + env.step) and the update.

    python tools/bench_ppo.py [--num-envs 8192] [--iters 3]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd import make_t1_env, task_registry  # noqa: E402
from ti5_isaacgym_amd.algo import DHOnPolicyRunner  # noqa: E402
from ti5_isaacgym_amd.utils.helpers import class_to_dict  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--num-envs", type=int, default=8192)
p.add_argument("--iters", type=int, default=3)
p.add_argument("--no-graph", action="store_true", help="eager act() in the rollout (DHPPO.graph_act off)")
p.add_argument("--conv-search", action="store_true", help="torch.backends.cudnn.benchmark (MIOpen find) for the conv")
a = p.parse_args()
torch.backends.cudnn.benchmark = a.conv_search
env = make_t1_env(num_envs=a.num_envs, mesh_type="trimesh", seed=5, device="cuda:0")
_, tc = task_registry.get_cfgs("t1_dh_stand")
cfg = class_to_dict(tc)
torch.manual_seed(0)
r = DHOnPolicyRunner(env, cfg, None, device="cuda:0")
r.alg.graph_act = not a.no_graph
r.learn(1)  # warm-up (allocations, kernels)
torch.cuda.synchronize()
t0 = time.perf_counter()
r.learn(a.iters)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
steps = a.iters * cfg["runner"]["num_steps_per_env"] * a.num_envs

# phase breakdown: rollout (policy inference + env.step + storage) vs the PPO update
alg, T = r.alg, r.num_steps_per_env
obs, cobs = env.get_observations(), env.get_privileged_observations()
t_roll = t_env = t_upd = 0.0
for _ in range(a.iters):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with torch.inference_mode():
        for i in range(T):
            act = alg.act(obs, cobs)
            torch.cuda.synchronize()
            te = time.perf_counter()
            obs, cobs, rew, dones, infos = env.step(act)
            torch.cuda.synchronize()
            t_env += time.perf_counter() - te
            alg.process_env_step(rew, dones, infos)
        alg.compute_returns(cobs)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    alg.update()
    torch.cuda.synchronize()
    t_upd += time.perf_counter() - t1
    t_roll += t1 - t0
print(json.dumps({"num_envs": a.num_envs, "iters": a.iters, "graph_act": r.alg.graph_act, "env_steps_per_s_incl_update": round(steps / dt, 1),
                  "s_per_iter": round(dt / a.iters, 4),
                  "phases_s_per_iter": {"rollout": round(t_roll / a.iters, 4), "env_step_in_rollout": round(t_env / a.iters, 4),
                                        "update": round(t_upd / a.iters, 4)}}))
