"""ti5_isaacgym_amd: MI355X-native T1 humanoid env hot path (LeggedRobot.step) behind the reference API.

    from ti5_isaacgym_amd import task_registry, get_args
    env, env_cfg = task_registry.make_env("t1_dh_stand", get_args(["--num_envs", "8192"]))

The HIP library (ti5_isaacgym_amd/_lib/libt1env_hip.so) is loaded when an env is constructed; there is
no CPU fallback.
"""
import copy

from .envs.configs import BaseConfig, DHT1StandCfg, DHT1StandCfgPPO, LeggedRobotCfg, LeggedRobotCfgPPO
from .algo import ActorCriticDH, DHOnPolicyRunner, DHPPO, RolloutStorage
from .envs.t1_env import T1DHStandEnv
from .utils.helpers import class_to_dict, get_args, set_seed, update_class_from_dict
from .utils.task_registry import task_registry

task_registry.register("t1_dh_stand", T1DHStandEnv, DHT1StandCfg(), DHT1StandCfgPPO())
task_registry.register_runner("DHOnPolicyRunner", DHOnPolicyRunner)


def make_t1_env(num_envs=4096, mesh_type=None, seed=5, device="cuda:0", env_offset=0, num_envs_total=None,
                cfg_hook=None):
    """Convenience constructor: DHT1StandCfg defaults with num_envs / terrain / seed overrides."""
    env_cfg, _ = task_registry.get_cfgs("t1_dh_stand")
    env_cfg = copy.deepcopy(env_cfg)
    env_cfg.env.num_envs = num_envs
    env_cfg.seed = seed
    if mesh_type is not None:
        env_cfg.terrain.mesh_type = mesh_type
    if cfg_hook is not None:
        cfg_hook(env_cfg)
    set_seed(seed)
    return T1DHStandEnv(env_cfg, sim_device=device, env_offset=env_offset, num_envs_total=num_envs_total)
