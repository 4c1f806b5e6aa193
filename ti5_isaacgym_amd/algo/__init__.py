"""PPO over the HIP env: the reference's DH-PPO stack (humanoid/algo) restated for one process per GPU.

    VecEnv            vec_env.py      -- the env interface the runner consumes
    ActorCriticDH     dh_policy.py    -- policy / value / state-estimator / long-history networks
    RolloutStorage    rollout.py      -- on-device rollout buffer + GAE
    DHPPO             dh_update.py    -- PPO update (+ bucketed RCCL gradient all-reduce when distributed)
    DHOnPolicyRunner  runner.py       -- rollout / update / log / checkpoint loop
"""
from .dh_policy import ActorCriticDH
from .dh_update import DHPPO
from .rollout import RolloutStorage
from .runner import DHOnPolicyRunner
from .vec_env import VecEnv

__all__ = ["ActorCriticDH", "DHPPO", "RolloutStorage", "DHOnPolicyRunner", "VecEnv"]
