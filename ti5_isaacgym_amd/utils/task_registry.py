"""Task registry with the reference's API (humanoid/utils/task_registry.py:16-148).

``task_registry.make_env("t1_dh_stand", args)`` builds the HIP env; ``make_alg_runner`` instantiates the
runner class named by ``train_cfg.runner_class_name`` from ``task_registry.runner_classes`` (register the
reference's DHOnPolicyRunner there, or use ti5_isaacgym_amd.algo's) -- the runner itself is unchanged.
"""
import copy
import os
from datetime import datetime

from .helpers import class_to_dict, get_args, get_load_path, set_seed, update_cfg_from_args


class TaskRegistry:
    def __init__(self):
        self.task_classes, self.env_cfgs, self.train_cfgs = {}, {}, {}
        self.runner_classes = {}

    def register(self, name, task_class, env_cfg, train_cfg):
        self.task_classes[name] = task_class
        self.env_cfgs[name] = env_cfg
        self.train_cfgs[name] = train_cfg

    def register_runner(self, name, cls):
        self.runner_classes[name] = cls

    def get_task_class(self, name):
        return self.task_classes[name]

    def get_cfgs(self, name):
        env_cfg, train_cfg = self.env_cfgs[name], self.train_cfgs[name]
        env_cfg.seed = train_cfg.seed
        return env_cfg, train_cfg

    def make_env(self, name, args=None, env_cfg=None, env_offset=0, num_envs_total=None):
        if args is None:
            args = get_args()
        if name not in self.task_classes:
            raise ValueError(f"Task with name: {name} was not registered")
        task_class = self.task_classes[name]
        if env_cfg is None:
            env_cfg, _ = self.get_cfgs(name)
            env_cfg = copy.deepcopy(env_cfg)
        env_cfg, _ = update_cfg_from_args(env_cfg, None, args)
        set_seed(env_cfg.seed)
        env = task_class(cfg=env_cfg, sim_params=None, physics_engine=getattr(args, "physics_engine", None),
                         sim_device=getattr(args, "sim_device", "cuda:0"), headless=getattr(args, "headless", True),
                         env_offset=env_offset, num_envs_total=num_envs_total)
        self.env_cfg_for_wandb = env_cfg
        return env, env_cfg

    def make_alg_runner(self, env, name=None, args=None, train_cfg=None, log_root="default", log_to_dir=True):
        if args is None:
            args = get_args()
        if train_cfg is None:
            if name is None:
                raise ValueError("Either 'name' or 'train_cfg' must be not None")
            _, train_cfg = self.get_cfgs(name)
        _, train_cfg = update_cfg_from_args(None, train_cfg, args)
        stamp = datetime.now().strftime("%Y-%m-%d_%H-%M-%S")
        if log_root == "default":
            log_root = os.path.join("logs", train_cfg.runner.experiment_name, "exported_data")
        log_dir = None if log_root is None else os.path.join(log_root, stamp + train_cfg.runner.run_name)
        if not log_to_dir:   # data-parallel ranks other than 0 resolve the resume path but write nothing
            log_dir = None
        all_cfg = {**class_to_dict(train_cfg), **class_to_dict(self.env_cfg_for_wandb)}
        cls = self.runner_classes.get(train_cfg.runner_class_name)
        if cls is None:
            raise ValueError(f"runner class {train_cfg.runner_class_name!r} not registered "
                             "(task_registry.register_runner(name, cls))")
        runner = cls(env, all_cfg, log_dir, device=getattr(args, "rl_device", "cuda:0"))
        if train_cfg.runner.resume:   # task_registry.py:136-143: weights only, the optimizer starts fresh
            resume_path = get_load_path(log_root, load_run=train_cfg.runner.load_run,
                                        checkpoint=train_cfg.runner.checkpoint)
            print(f"Loading model from: {resume_path}")
            runner.load(resume_path, load_optimizer=False)
        return runner, train_cfg, log_dir


task_registry = TaskRegistry()
