"""Generate tests/golden/runner_learn2.npz from the reference's own DHOnPolicyRunner (this container only: /root/reference
is read here; the fixture travels, the reference does not).  VERDICT r3 #7: pins the claim that the reference's runner
loop drops in over the build's env contract.

The reference's humanoid/algo/ppo/dh_on_policy_runner.py is imported by file path as the package humanoid.algo.ppo
(humanoid/__init__.py, which pulls in Isaac Gym, is not executed), with two placeholders in sys.modules: wandb (unused,
tests/golden/harness/wandb.py) and torch.utils.tensorboard (absent from this image; its SummaryWriter here records every
add_scalar call -- the runner's log output).  Its learn(2) runs on the CPU over tests/fake_vec_env.py (16 envs) with
the t1_dh_stand train config (the build's config classes, whose values restate t1_dh_stand_config.py:425-480), every
env access recorded through a proxy.  Recorded:

  scalars   every logged scalar of both iterations except wall-clock ones (Perf/*, */time): losses, learning rate,
            action noise std, mean reward / episode length, the episode infos
  weights   per parameter tensor of the final policy: float64 sum, abs-sum and 8 probed values
  env_attrs the env attributes the reference runner read or wrote (the contract T1DHStandEnv must expose)

tests/test_runner_golden.py replays the same seeds through the build's DHOnPolicyRunner and compares; a GPU test checks
T1DHStandEnv against env_attrs.

    python tests/golden/gen_runner_golden.py [/root/reference]
"""
import importlib
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
TESTS = os.path.dirname(HERE)
REPO = os.path.dirname(TESTS)
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
N_ENVS, ITERS, INIT_SEED, LEARN_SEED, PROBE = 16, 2, 21, 22, 8
SKIP = ("Perf/", "/time")


def train_cfg():
    """The t1_dh_stand train config as the runner receives it (class_to_dict of the config classes)."""
    sys.path.insert(0, REPO)
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    return class_to_dict(tc)


class EnvRecorder:
    """Forwards to the wrapped env and records every attribute name the runner reads or writes."""

    def __init__(self, env):
        object.__setattr__(self, "_env", env)
        object.__setattr__(self, "_seen", set())

    def __getattr__(self, k):
        self._seen.add(k)
        return getattr(self._env, k)

    def __setattr__(self, k, v):
        self._seen.add(k)
        setattr(self._env, k, v)


def probe_index(numel):
    return (np.arange(PROBE, dtype=np.int64) * 7919 + 13) % numel


def weight_summary(module):
    out = {}
    for name, p in module.named_parameters():
        w = p.detach().double().flatten()
        out[f"w_sum/{name}"] = np.array(w.sum().item())
        out[f"w_abs/{name}"] = np.array(w.abs().sum().item())
        out[f"w_probe/{name}"] = w[torch.from_numpy(probe_index(w.numel()))].numpy()
    return out


def load_reference_runner():
    sys.modules["wandb"] = importlib.import_module("harness.wandb")
    scalars = []

    class SummaryWriter:  # torch.utils.tensorboard placeholder recording the runner's scalars
        def __init__(self, log_dir=None, flush_secs=10):
            self.log_dir = log_dir

        def add_scalar(self, tag, value, step):
            scalars.append((tag, float(value), int(step)))

    tb = types.ModuleType("torch.utils.tensorboard")
    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb
    for name, sub in (("humanoid", ""), ("humanoid.algo", "algo"), ("humanoid.algo.ppo", "algo/ppo")):
        pkg = types.ModuleType(name)
        pkg.__path__ = [os.path.join(REF, "humanoid", sub)]
        sys.modules[name] = pkg
    return importlib.import_module("humanoid.algo.ppo.dh_on_policy_runner"), scalars


def main():
    sys.path.insert(0, HERE)
    sys.path.insert(0, TESTS)
    from fake_vec_env import FakeVecEnv
    cfg = train_cfg()
    mod, scalars = load_reference_runner()
    env = EnvRecorder(FakeVecEnv(N_ENVS))
    with tempfile.TemporaryDirectory() as log_dir:
        torch.manual_seed(INIT_SEED)
        runner = mod.DHOnPolicyRunner(env, cfg, log_dir=log_dir, device="cpu")
        torch.manual_seed(LEARN_SEED)
        runner.learn(ITERS)
    out = {}
    tags = sorted({t for t, _, _ in scalars if not any(s in t for s in SKIP)})
    for tag in tags:
        rows = [(s, v) for t, v, s in scalars if t == tag]
        out[f"scalar/{tag}"] = np.array(rows, np.float64)
    out.update(weight_summary(runner.alg.actor_critic))
    out["env_attrs"] = np.array(sorted(env._seen))
    out["meta"] = np.array([N_ENVS, ITERS, INIT_SEED, LEARN_SEED], np.int64)
    dst = os.path.join(HERE, "runner_learn2.npz")
    np.savez_compressed(dst, **out)
    print("wrote", dst, len(tags), "scalar tags;", "env attrs:", sorted(env._seen))


if __name__ == "__main__":
    main()
