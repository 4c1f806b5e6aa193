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
a = p.parse_args()
env = make_t1_env(num_envs=a.num_envs, mesh_type="trimesh", seed=5, device="cuda:0")
_, tc = task_registry.get_cfgs("t1_dh_stand")
cfg = class_to_dict(tc)
torch.manual_seed(0)
r = DHOnPolicyRunner(env, cfg, None, device="cuda:0")
r.learn(1)  # warm-up (allocations, kernels)
torch.cuda.synchronize()
t0 = time.perf_counter()
r.learn(a.iters)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
steps = a.iters * cfg["runner"]["num_steps_per_env"] * a.num_envs
print(json.dumps({"num_envs": a.num_envs, "iters": a.iters, "env_steps_per_s_incl_update": round(steps / dt, 1),
                  "s_per_iter": round(dt / a.iters, 4)}))
