"""Deterministic CPU VecEnv for the PPO tests (the HIP env needs a GPU).

Observations, rewards and terminations are smooth functions of (global env id, step, actions), so a run is
reproducible and a sharded run sees exactly the data of the unsharded one.  Implements what the runner reads
from the reference's env.
"""
from types import SimpleNamespace

import torch


class FakeVecEnv:
    def __init__(self, num_envs, env_offset=0, device="cpu", episode_len=7):
        self.num_envs, self.env_offset, self.device = num_envs, env_offset, torch.device(device)
        self.num_single_obs, self.num_short_obs, self.num_obs = 47, 235, 66 * 47
        self.num_privileged_obs, self.num_actions = 219, 12
        self.max_episode_length = 2400.0
        self.cfg = SimpleNamespace(terrain=SimpleNamespace(measure_heights=False, num_height=187),
                                   env=SimpleNamespace(c_frame_stack=3, single_num_privileged_obs=73))
        self.episode_len = episode_len
        self.ids = torch.arange(num_envs, device=self.device, dtype=torch.float32) + env_offset
        self.episode_length_buf = torch.zeros(num_envs, dtype=torch.long, device=self.device)
        self.t = 0
        self._fill(torch.zeros(num_envs, 12, device=self.device))

    def _fill(self, actions):
        e = self.ids[:, None]
        k = torch.arange(self.num_obs, device=self.device, dtype=torch.float32)[None]
        kp = torch.arange(self.num_privileged_obs, device=self.device, dtype=torch.float32)[None]
        a = actions.sum(-1, keepdim=True).clamp(-5, 5)
        self.obs_buf = torch.sin(0.013 * k * (1 + 0.1 * e) + 0.3 * self.t) * 0.5 + 0.05 * a
        self.privileged_obs_buf = torch.cos(0.021 * kp + 0.7 * e + 0.2 * self.t) * 0.5 + 0.05 * a
        self.rew_buf = (torch.sin(0.5 * self.ids + 0.9 * self.t) - 0.1 * actions.pow(2).mean(-1)).float()

    def reset(self):
        return self.obs_buf, self.privileged_obs_buf

    def get_observations(self):
        return self.obs_buf

    def get_privileged_observations(self):
        return self.privileged_obs_buf

    def step(self, actions):
        self.t += 1
        self.episode_length_buf += 1
        self._fill(actions)
        done = ((self.ids.long() + self.t) % self.episode_len) == 0
        time_out = done & (self.ids.long() % 2 == 0)
        self.episode_length_buf[done] = 0
        infos = {"episode": {"rew_tracking": torch.tensor(0.1 * self.t), "max_command_x": 0.5},
                 "time_outs": time_out}
        return self.obs_buf, self.privileged_obs_buf, self.rew_buf, done, infos
