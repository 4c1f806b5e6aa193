"""TEST-ONLY: import the reference's own env code behind the isaacgym stand-in and construct it.

Requires /root/reference (this container only; it never exists on the GPU box).
"""
import os
import sys
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("T1_REFERENCE_ROOT", "/root/reference")


def setup_paths():
    for p in (os.path.join(HERE, "harness"), REPO, REF):
        if p not in sys.path:
            sys.path.insert(0, p)
    if "torch.utils.tensorboard" not in sys.modules:
        tb = types.ModuleType("torch.utils.tensorboard")

        class SummaryWriter:  # placeholder: the runner is not exercised by the harness
            def __init__(self, *a, **k):
                pass
        tb.SummaryWriter = SummaryWriter
        sys.modules["torch.utils.tensorboard"] = tb


def make_env(num_envs=16, mesh_type="plane", cfg_hook=None, seed=5):
    setup_paths()
    import numpy as np
    import torch
    import draws
    import fake_gym
    from isaacgym import gymapi
    draws.install()
    fake_gym.FakeGym.reset_instance()
    import humanoid.envs  # noqa: F401  (registers t1_dh_stand)
    from humanoid.utils.task_registry import task_registry
    from humanoid.utils.helpers import class_to_dict, set_seed
    env_cfg, train_cfg = task_registry.get_cfgs("t1_dh_stand")
    import copy
    env_cfg = copy.deepcopy(env_cfg)
    env_cfg.env.num_envs = num_envs
    env_cfg.terrain.mesh_type = mesh_type
    if cfg_hook is not None:
        cfg_hook(env_cfg)
    set_seed(seed)
    draws.SEED = env_cfg.seed
    sim_params = gymapi.SimParams()
    sim_params.dt = env_cfg.sim.dt
    sim_params.substeps = env_cfg.sim.substeps
    env_cls = task_registry.get_task_class("t1_dh_stand")
    env = env_cls(cfg=env_cfg, sim_params=sim_params, physics_engine=gymapi.SIM_PHYSX,
                  sim_device="cpu", headless=True)
    return env, env_cfg, fake_gym.FakeGym.instance()
