"""Train t1_dh_stand with DH-PPO on the HIP env (reference humanoid/scripts/train.py).

    python -m ti5_isaacgym_amd.scripts.train --task t1_dh_stand --num_envs 8192 --max_iterations 30000
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m ti5_isaacgym_amd.scripts.train --num_envs 8192          # 8 x 8192 envs, RCCL gradient all-reduce

One process per GPU: rank r steps global envs [r*N, (r+1)*N) on cuda:LOCAL_RANK; the PPO update all-reduces
the policy gradient over RCCL (ti5_isaacgym_amd/algo/distributed.py); rank 0 logs and checkpoints.
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from ti5_isaacgym_amd import get_args, task_registry  # noqa: E402


def train(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.distributed.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        args.sim_device = args.rl_device = f"cuda:{local}"
    torch.cuda.set_device(torch.device(args.sim_device))
    env_cfg, train_cfg = task_registry.get_cfgs(args.task)
    n = args.num_envs or env_cfg.env.num_envs
    env, env_cfg = task_registry.make_env(name=args.task, args=args, env_offset=rank * n, num_envs_total=world * n)
    torch.manual_seed((args.seed if args.seed is not None else train_cfg.seed) + rank)  # per-rank action sampling
    # resume (--resume / train_cfg.runner.resume, --load_run, --checkpoint) is make_alg_runner's, as in the
    # reference (task_registry.py:136-143): every rank loads the same checkpoint, rank 0 alone logs
    runner, train_cfg, log_dir = task_registry.make_alg_runner(env=env, name=args.task, args=args,
                                                                log_to_dir=rank == 0)
    runner.learn(num_learning_iterations=train_cfg.runner.max_iterations, init_at_random_ep_len=False)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    train(get_args(sys.argv[1:]))
