"""DH-PPO runner over the HIP env on the GPU: rollout -> GAE -> update for a few iterations."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_runner_over_hip_env(tmp_path):
    from ti5_isaacgym_amd import make_t1_env, task_registry
    from ti5_isaacgym_amd.algo import DHOnPolicyRunner
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    env = make_t1_env(num_envs=256, mesh_type="plane", seed=5, device="cuda:0")
    _, train_cfg = task_registry.get_cfgs("t1_dh_stand")
    cfg = class_to_dict(train_cfg)
    cfg["runner"]["num_steps_per_env"] = 8
    cfg["runner"]["save_interval"] = 100
    torch.manual_seed(0)
    runner = DHOnPolicyRunner(env, cfg, str(tmp_path), device="cuda:0")
    runner.learn(2)
    assert runner.current_learning_iteration == 2
    for p in runner.alg.actor_critic.parameters():
        assert torch.isfinite(p).all()
    s = runner.alg.storage
    assert torch.isfinite(s.returns).all() and torch.isfinite(s.advantages).all()
    pol = runner.get_inference_policy()
    with torch.no_grad():
        a = pol(env.get_observations())
    assert a.shape == (256, 12) and torch.isfinite(a).all()
