"""Dev probe: host-side (CPU) and device time of one DHPPO.update() in fp32 or under the opt-in bf16 autocast.

    python tools/ppo_update_profile.py [--bf16] [--num-envs 8192] [--rows 25]

Runs two warm-up iterations (rollout + update), then one rollout and one update under torch.profiler (CPU + device
activities) and prints the wall time of that update and the top --rows ops by self CPU time and by device time.
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd import make_t1_env, task_registry  # noqa: E402
from ti5_isaacgym_amd.algo import DHOnPolicyRunner  # noqa: E402
from ti5_isaacgym_amd.utils.helpers import class_to_dict  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--num-envs", type=int, default=8192)
    p.add_argument("--bf16", action="store_true")
    p.add_argument("--rows", type=int, default=25)
    p.add_argument("--eager", action="store_true", help="the eager minibatch step (DHPPO.graph_update off): the same "
                   "kernels, each visible to the profiler")
    a = p.parse_args()
    dev = torch.device("cuda:0")
    env = make_t1_env(num_envs=a.num_envs, mesh_type="trimesh", seed=5, device=str(dev))
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    r = DHOnPolicyRunner(env, class_to_dict(tc), None, device=str(dev))
    alg = r.alg
    alg.amp_dtype = torch.bfloat16 if a.bf16 else None
    alg.graph_update = not a.eager
    alg.actor_critic.train()
    obs, priv = env.reset()
    critic = priv if priv is not None else obs

    def rollout():
        nonlocal obs, critic
        with torch.inference_mode():
            for _ in range(r.num_steps_per_env):
                actions = alg.act(obs, critic)
                obs, priv_, rew, dones, infos = env.step(actions)
                critic = priv_ if priv_ is not None else obs
                alg.process_env_step(rew, dones, infos)
            alg.compute_returns(critic)

    for _ in range(2):
        rollout()
        alg.update()
    rollout()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        t0 = time.perf_counter()
        alg.update()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(f"update wall {dt * 1e3:.1f} ms ({'bf16' if a.bf16 else 'fp32'}, {'eager' if a.eager else 'graphed'})")
    ka = prof.key_averages()
    print(ka.table(sort_by="self_cpu_time_total", row_limit=a.rows, max_name_column_width=60))
    print(ka.table(sort_by="self_device_time_total", row_limit=a.rows, max_name_column_width=60))
    rows = [e for e in prof.key_averages(group_by_input_shape=True) if e.key.startswith("aten::")
            and e.self_device_time_total > 0]
    rows.sort(key=lambda e: -e.self_device_time_total)
    for e in rows[:60]:   # the device time by op and input shapes: where the casts, sums and GEMMs come from
        print(f"{e.key:22s} calls {e.count:4d} device {e.self_device_time_total / 1e3:8.3f} ms total "
              f"{e.self_device_time_total / max(e.count, 1):8.1f} us/call  {e.input_shapes}")


if __name__ == "__main__":
    main()
