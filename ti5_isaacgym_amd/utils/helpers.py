"""Host helpers mirroring humanoid/utils/helpers.py's public functions used around the env path.

class_to_dict walks ``dir()`` (alphabetical), which is what fixes the reward summation order
(reference helpers.py:14-29).  get_args() parses the reference's CLI flags with argparse (Isaac Gym's
gymutil parser is not available); --sim_device / --rl_device / --num_envs / --seed keep their meaning.
"""
import argparse
import os
import random

import numpy as np
import torch


def class_to_dict(obj) -> dict:
    if not hasattr(obj, "__dict__"):
        return obj
    out = {}
    for key in dir(obj):
        if key.startswith("_"):
            continue
        val = getattr(obj, key)
        out[key] = [class_to_dict(v) for v in val] if isinstance(val, list) else class_to_dict(val)
    return out


def update_class_from_dict(obj, d):
    for key, val in d.items():
        attr = getattr(obj, key, None)
        if isinstance(attr, type):
            update_class_from_dict(attr, val)
        else:
            setattr(obj, key, val)


def set_seed(seed):
    if seed == -1:
        seed = np.random.randint(0, 10000)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    os.environ["PYTHONHASHSEED"] = str(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    return seed


def get_load_path(root, load_run=-1, checkpoint=-1):
    """Checkpoint path of a run (reference humanoid/utils/helpers.py:94-125): the last run under root (sorted names,
    "exported" skipped) unless load_run names one, and in it model_<checkpoint>.pt or the last model file."""
    try:
        runs = sorted(os.listdir(root))
        if "exported" in runs:
            runs.remove("exported")
        last_run = os.path.join(root, runs[-1])
    except Exception:
        raise ValueError("No runs in this directory: " + str(root))
    load_run = last_run if load_run == -1 else os.path.join(root, load_run)
    if checkpoint == -1:
        models = sorted((f for f in os.listdir(load_run) if "model" in f), key=lambda m: "{0:0>15}".format(m))
        model = models[-1]
    else:
        model = "model_{}.pt".format(checkpoint)
    return os.path.join(load_run, model)


def update_cfg_from_args(env_cfg, cfg_train, args):
    if env_cfg is not None and getattr(args, "num_envs", None) is not None:
        env_cfg.env.num_envs = args.num_envs
    if cfg_train is not None:
        for k in ("seed",):
            if getattr(args, k, None) is not None:
                setattr(cfg_train, k, getattr(args, k))
        for k in ("max_iterations", "experiment_name", "run_name", "load_run", "checkpoint"):
            if getattr(args, k, None) is not None:
                setattr(cfg_train.runner, k, getattr(args, k))
        if getattr(args, "resume", False):
            cfg_train.runner.resume = True
    return env_cfg, cfg_train


def get_args(argv=None):
    p = argparse.ArgumentParser(description="RL Policy")
    p.add_argument("--task", type=str, default="t1_dh_stand")
    p.add_argument("--resume", action="store_true", default=False)
    p.add_argument("--experiment_name", type=str)
    p.add_argument("--run_name", type=str, default="ti5")
    p.add_argument("--load_run", type=str)
    p.add_argument("--checkpoint", type=int)
    p.add_argument("--headless", action="store_true", default=False)
    p.add_argument("--horovod", action="store_true", default=False)
    p.add_argument("--rl_device", type=str, default="cuda:0")
    p.add_argument("--sim_device", type=str, default="cuda:0")
    p.add_argument("--num_envs", type=int)
    p.add_argument("--seed", type=int)
    p.add_argument("--max_iterations", type=int)
    args = p.parse_args(argv if argv is not None else [])
    args.physics_engine = "hip"
    return args
