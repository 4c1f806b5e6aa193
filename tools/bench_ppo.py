"""PPO iteration timing (BASELINE config 4's training loop): rollout collection (policy inference + env.step) and the
DH-PPO update, on one GPU or data-parallel over N GPUs of one node.

    python tools/bench_ppo.py [--num-envs 8192] [--iters 3]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \\
        tools/bench_ppo.py --num-envs 8192 --iters 3

One process per GPU (RCCL = torch.distributed "nccl"): rank r steps global envs [r*N, (r+1)*N) and the update
all-reduces the flat policy gradient once per minibatch (8 per iteration, ti5_isaacgym_amd/algo/distributed.py) --
the exchange config 4 names.  Timed: --iters whole learn() iterations after one warm-up iteration, bracketed by a
barrier + synchronize, max over ranks; then a phase breakdown (the rollout as learn() runs it, compute_returns, the
rollout again with a sync around every env.step for the env share, the update) and the mean
gradient all-reduce time (CUDA events around every all-reduce of the timed iterations).  Rank 0 prints one JSON line.
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
p.add_argument("--num-envs", type=int, default=8192, help="envs per GPU")
p.add_argument("--iters", type=int, default=3)
p.add_argument("--mesh", default="trimesh")
p.add_argument("--no-graph", action="store_true", help="eager act() in the rollout (DHPPO.graph_act off)")
p.add_argument("--conv-search", action="store_true", help="torch.backends.cudnn.benchmark (MIOpen find) for the conv")
p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
               help="gloo + --one-gpu: rehearse the data-parallel path with every rank on cuda:0 (one-GPU box)")
p.add_argument("--one-gpu", action="store_true", help="all ranks on cuda:0 (rehearsal only; not a scaling number)")
p.add_argument("--bf16", action="store_true", help="opt-in bf16 PPO update (DHPPO.amp_dtype; tools/ppo_amp_check.py)")
a = p.parse_args()
world = int(os.environ.get("WORLD_SIZE", "1"))
rank = int(os.environ.get("RANK", "0"))
local = 0 if a.one_gpu else int(os.environ.get("LOCAL_RANK", "0"))
dev = torch.device(f"cuda:{local}")
torch.cuda.set_device(dev)
if world > 1:
    if a.backend == "nccl":
        torch.distributed.init_process_group("nccl", device_id=dev)
    else:
        torch.distributed.init_process_group("gloo")
torch.backends.cudnn.benchmark = a.conv_search
N = a.num_envs
env = make_t1_env(num_envs=N, mesh_type=a.mesh, seed=5, device=str(dev), env_offset=rank * N, num_envs_total=world * N)
_, tc = task_registry.get_cfgs("t1_dh_stand")
cfg = class_to_dict(tc)
torch.manual_seed(rank)
r = DHOnPolicyRunner(env, cfg, None, device=str(dev))
r.alg.graph_act = not a.no_graph
r.alg.amp_dtype = torch.bfloat16 if a.bf16 else None


def barrier():
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize(dev)


def max_over_ranks(x):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev if a.backend == "nccl" else "cpu")
    torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t.item())


r.learn(1)  # warm-up (allocations, kernels, graph capture)
barrier()
r.alg.grads.timing = []
t0 = time.perf_counter()
r.learn(a.iters)
barrier()
dt = max_over_ranks(time.perf_counter() - t0)
ar_ms = r.alg.grads.all_reduce_ms()
r.alg.grads.timing = None
T = r.num_steps_per_env
steps = a.iters * T * N * world

# phase breakdown: rollout (policy inference + env.step + storage) vs the PPO update
alg = r.alg
obs, cobs = env.get_observations(), env.get_privileged_observations()
t_roll = t_env = t_upd = t_free = t_ret = 0.0
for _ in range(a.iters):
    # the rollout as learn() runs it (no sync inside): act + env.step + process_env_step, then compute_returns
    barrier()
    t0 = time.perf_counter()
    with torch.inference_mode():
        for i in range(T):
            act = alg.act(obs, cobs)
            obs, cobs, rew, dones, infos = env.step(act)
            alg.process_env_step(rew, dones, infos)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        alg.compute_returns(cobs)
    barrier()
    t_free += t1 - t0
    t_ret += time.perf_counter() - t1
    alg.storage.clear()
    # the same with a sync around every env.step: the env's share (the syncs add their own idle time)
    barrier()
    t0 = time.perf_counter()
    with torch.inference_mode():
        for i in range(T):
            act = alg.act(obs, cobs)
            torch.cuda.synchronize(dev)
            te = time.perf_counter()
            obs, cobs, rew, dones, infos = env.step(act)
            torch.cuda.synchronize(dev)
            t_env += time.perf_counter() - te
            alg.process_env_step(rew, dones, infos)
        alg.compute_returns(cobs)
    barrier()
    t1 = time.perf_counter()
    alg.update()
    barrier()
    t_upd += time.perf_counter() - t1
    t_roll += t1 - t0
t_roll, t_env, t_upd, t_free, t_ret = (max_over_ranks(x) for x in (t_roll, t_env, t_upd, t_free, t_ret))
line = {"bench": "ppo_iteration", "n_gpus": 1 if a.one_gpu else world, "ranks": world, "num_envs_per_gpu": N,
        "global_envs": N * world, "mesh": a.mesh, "iters": a.iters, "graph_act": r.alg.graph_act,
        "update_dtype": "bf16" if a.bf16 else "fp32", "env_steps_per_s_incl_update": round(steps / dt, 1),
        "env_steps_per_s_per_gpu": round(steps / dt / world, 1), "s_per_iter": round(dt / a.iters, 4),
        "phases_s_per_iter": {"rollout": round(t_free / a.iters, 4), "compute_returns": round(t_ret / a.iters, 4),
                              "rollout_synced": round(t_roll / a.iters, 4),
                              "env_step_in_rollout_synced": round(t_env / a.iters, 4),
                              "update": round(t_upd / a.iters, 4)},
        "grad_allreduce": {"bytes": r.alg.grads.flat.numel() * 4, "per_iter": cfg["algorithm"]["num_learning_epochs"]
                           * cfg["algorithm"]["num_mini_batches"],
                           "mean_us": round(ar_ms * 1e3, 1) if ar_ms is not None else None,
                           "backend": torch.distributed.get_backend() if world > 1 else None}}
if rank == 0:
    print(json.dumps(line), flush=True)
if world > 1:
    torch.distributed.destroy_process_group()
