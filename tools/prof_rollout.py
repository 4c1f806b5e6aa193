"""Dev probe: where the PPO rollout's time goes at 8192 envs (DHOnPolicyRunner's inner loop: act, env.step,
process_env_step), without a sync between the phases.

    python tools/prof_rollout.py [--num-envs 8192] [--bf16]

Prints one JSON line of wall times per rollout step (24 steps, one sync at the end): the whole loop, act() alone,
env.step() alone, process_env_step() alone (on replayed inputs), then a torch.profiler table of one rollout.
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


def wall(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    return (t1 - t0) / n * 1e3, (time.perf_counter() - t0) / n * 1e3


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--num-envs", type=int, default=8192)
    a = p.parse_args()
    dev = torch.device("cuda:0")
    env = make_t1_env(num_envs=a.num_envs, mesh_type="trimesh", seed=5, device=str(dev))
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    r = DHOnPolicyRunner(env, class_to_dict(tc), None, device=str(dev))
    r.learn(1)   # warm-up: allocations, graph capture
    alg, T = r.alg, r.num_steps_per_env
    obs, cobs = env.get_observations(), env.get_privileged_observations()
    out = {"num_envs": a.num_envs}

    def rollout():
        nonlocal obs, cobs
        with torch.inference_mode():
            for _ in range(T):
                act = alg.act(obs, cobs)
                obs, cobs, rew, dones, infos = env.step(act)
                alg.process_env_step(rew, dones, infos)
        alg.storage.clear()

    enq, tot = wall(rollout, 3)
    out["rollout_ms_per_step"] = {"enqueue": round(enq / T, 4), "wall": round(tot / T, 4)}
    with torch.inference_mode():
        act = alg.act(obs, cobs)
        enq, tot = wall(lambda: alg.act(obs, cobs), 48)
        out["act_ms"] = {"enqueue": round(enq, 4), "wall": round(tot, 4)}
        enq, tot = wall(lambda: env.step(act), 48)
        out["env_step_ms"] = {"enqueue": round(enq, 4), "wall": round(tot, 4)}
        obs, cobs, rew, dones, infos = env.step(act)

        def pes():
            alg.act(obs, cobs)
            alg.process_env_step(rew, dones, infos)
            if alg.storage.step >= T:
                alg.storage.clear()
        enq, tot = wall(pes, 48)
        out["act_plus_process_env_step_ms"] = {"enqueue": round(enq, 4), "wall": round(tot, 4)}
    alg.storage.clear()
    print(json.dumps(out), flush=True)
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        rollout()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25, max_name_column_width=60))
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=20, max_name_column_width=60))


if __name__ == "__main__":
    main()
