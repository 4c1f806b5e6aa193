"""DHPPO: PPO with the state-estimator auxiliary loss (reference humanoid/algo/ppo/dh_ppo.py:13-205).

Same constructor arguments, API (``init_storage``, ``act``, ``process_env_step``, ``compute_returns``,
``update``) and losses as the reference:
  loss = clipped surrogate + value_loss_coef * clipped value loss - entropy_coef * entropy
         + MSE(state_estimator(short history), privileged base linear velocity [lin_vel_idx : +3]).
Additions for data-parallel training over RCCL (distributed.py): one bucketed gradient all-reduce between
backward() and clip_grad_norm_, the KL mean all-reduced before the adaptive learning-rate decision, and
rank-0 weights broadcast at start.  Losses are accumulated on the device and read once per update.
On a HIP device the rollout's act() (policy sample, value, log-prob) replays a captured HIP graph, one per
pair of observation buffers the env hands out (its ping-pong buffers): the same kernels as the eager call,
without the per-kernel launch cost that dominates at one call per env step.
"""
import contextlib
import math
import warnings

import torch
import torch.nn as nn
import torch.optim as optim
from torch.distributions import Normal

from . import distributed as dist_util
from .dh_policy import ActorCriticDH
from .rollout import RolloutStorage


class DHPPO:
    actor_critic: ActorCriticDH

    def __init__(self, actor_critic, num_learning_epochs=1, num_mini_batches=1, clip_param=0.2, gamma=0.998,
                 lam=0.95, value_loss_coef=1.0, entropy_coef=0.0, learning_rate=1e-3, max_grad_norm=1.0,
                 lin_vel_idx=45, use_clipped_value_loss=True, schedule="fixed", desired_kl=0.01, device="cpu",
                 amp_dtype=None):
        self.device = device
        # opt-in mixed precision of the update (not in the reference): torch.bfloat16 runs the update's forward and
        # backward GEMMs in bf16 (fp32 accumulation, fp32 weights, optimizer and losses); None = fp32 as the reference
        self.amp_dtype = amp_dtype
        self.cast_obs_once = True
        self.desired_kl, self.schedule, self.learning_rate = desired_kl, schedule, learning_rate
        self.actor_critic = actor_critic
        self.actor_critic.to(self.device)
        self.storage = None
        self.optimizer = optim.Adam(self.actor_critic.parameters(), lr=learning_rate)
        # created (and checkpointed) like the reference's; its separate step is disabled there as well
        self.state_estimator_optimizer = optim.Adam(self.actor_critic.state_estimator.parameters(), lr=learning_rate)
        self.transition = RolloutStorage.Transition()
        self.clip_param, self.num_learning_epochs, self.num_mini_batches = clip_param, num_learning_epochs, num_mini_batches
        self.value_loss_coef, self.entropy_coef = value_loss_coef, entropy_coef
        self.gamma, self.lam, self.max_grad_norm = gamma, lam, max_grad_norm
        self.use_clipped_value_loss = use_clipped_value_loss
        self.num_short_obs = self.actor_critic.num_short_obs
        self.lin_vel_idx = lin_vel_idx
        # .grad of every parameter is a view into one flat bucket: the DP gradient all-reduce is one collective
        self.grads = dist_util.GradientBucket(self.actor_critic.parameters())
        self.grads.broadcast_params_()
        # graphed rollout act(): {(obs ptr, critic obs ptr, shapes): (graph, static outputs)}; None = eager
        self.graph_act = torch.device(device).type == "cuda"
        self._act_graphs = {}

    def init_storage(self, num_envs, num_transitions_per_env, actor_obs_shape, critic_obs_shape, action_shape,
                     history=None):
        """history=(frame, frames): the actor observations are a frame history the env shifts every step (the T1
        env's, T1DHStandEnv.obs_frame_history): stored as frames (RolloutStorage)."""
        self.storage = RolloutStorage(num_envs, num_transitions_per_env, actor_obs_shape, critic_obs_shape,
                                      action_shape, None, self.device, history=history)

    def test_mode(self):
        self.actor_critic.test()

    def train_mode(self):
        self.actor_critic.train()

    def _act_body(self, obs, critic_obs):
        """act() as one fixed kernel sequence (ActorCriticDH.act / evaluate / get_actions_log_prob).  Two host
        checks cannot run inside a graph: the distribution's argument validation (built without it) and
        torch.normal's std >= 0 test (the sample is drawn as mean + std * N(0, 1), the same distribution)."""
        ac = self.actor_critic
        obs, critic_obs = obs.float(), critic_obs.float()   # fp16 env histories (state_dtype="fp16"): no-op for fp32
        mean = ac.actor(ac.actor_input(obs))
        std = mean * 0.0 + ac.std
        dist = Normal(mean, std, validate_args=False)
        actions = mean + std * torch.randn_like(mean)
        return actions, ac.critic(critic_obs), dist.log_prob(actions).sum(dim=-1), mean, std

    def _graphed_act(self, obs, critic_obs):
        key = (obs.data_ptr(), critic_obs.data_ptr(), tuple(obs.shape), tuple(critic_obs.shape))
        entry = self._act_graphs.get(key)
        if entry is None:
            if len(self._act_graphs) >= 4:  # not the env's fixed buffers: stay eager
                return None
            side = torch.cuda.Stream(device=obs.device)
            side.wait_stream(torch.cuda.current_stream(obs.device))
            with torch.cuda.stream(side):  # warm-up outside the capture (allocator, library handles)
                for _ in range(2):
                    self._act_body(obs, critic_obs)
            torch.cuda.current_stream(obs.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(graph):
                    outs = self._act_body(obs, critic_obs)
            except RuntimeError as e:  # a library call that cannot be captured: the eager act() from now on
                warnings.warn(f"DHPPO: act() graph capture failed, running eager: {e}")
                self.graph_act = False
                return None
            entry = self._act_graphs[key] = (graph, outs)
        entry[0].replay()
        return entry[1]

    def act(self, obs, critic_obs):
        ac, t = self.actor_critic, self.transition
        outs = self._graphed_act(obs, critic_obs) if self.graph_act and obs.is_cuda else None
        if outs is not None:
            t.actions, t.values, t.actions_log_prob, t.action_mean, t.action_sigma = outs
            t.observations = obs
            t.critic_observations = critic_obs
            return t.actions
        t.actions = ac.act(obs.float()).detach()
        t.values = ac.evaluate(critic_obs.float()).detach()
        t.actions_log_prob = ac.get_actions_log_prob(t.actions).detach()
        t.action_mean = ac.action_mean.detach()
        t.action_sigma = ac.action_std.detach()
        t.observations = obs  # recorded before env.step(); the env's obs buffer of this step stays valid
        t.critic_observations = critic_obs
        return t.actions

    def process_env_step(self, rewards, dones, infos):
        t = self.transition
        t.rewards = rewards.clone()
        t.dones = dones
        if "time_outs" in infos:  # bootstrap on time-outs
            t.rewards += self.gamma * torch.squeeze(t.values * infos["time_outs"].unsqueeze(1).to(self.device), 1)
        self.storage.add_transitions(t)
        t.clear()
        self.actor_critic.reset(dones)

    def compute_returns(self, last_critic_obs):
        last_values = self.actor_critic.evaluate(last_critic_obs).detach()
        self.storage.compute_returns(last_values, self.gamma, self.lam)

    def _adapt_lr(self, mu, sigma, old_mu, old_sigma):
        with torch.inference_mode():
            kl = torch.sum(torch.log(sigma / old_sigma + 1.0e-5)
                           + (torch.square(old_sigma) + torch.square(old_mu - mu)) / (2.0 * torch.square(sigma)) - 0.5,
                           axis=-1)
            kl_mean = dist_util.all_reduce_mean_(torch.mean(kl).reshape(1))[0]
            kl_mean = float(kl_mean)
        if kl_mean > self.desired_kl * 2.0:
            self.learning_rate = max(1e-5, self.learning_rate / 1.5)
        elif 0.0 < kl_mean < self.desired_kl / 2.0:
            self.learning_rate = min(1e-2, self.learning_rate * 1.5)
        for g in self.optimizer.param_groups:
            g["lr"] = self.learning_rate

    def update(self):
        ac = self.actor_critic
        sums = torch.zeros(3, device=self.device)  # value, surrogate, state-estimator losses
        mse = nn.MSELoss()
        use_amp = self.amp_dtype is not None and torch.device(self.device).type == "cuda"
        amp = torch.autocast(device_type="cuda", dtype=self.amp_dtype) if use_amp else contextlib.nullcontext()
        # under the bf16 update every consumer of the actor observations is a bf16 GEMM: cast them once per update
        # (same values as autocast's per-minibatch casts) unless cast_obs_once is switched off (A/B)
        gen = self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs,
                                                obs_dtype=self.amp_dtype if use_amp and self.cast_obs_once else None)
        # the distribution's argument checks are host syncs (three per minibatch) on the device: off for the update,
        # replaced by one finiteness check of the losses below (the reference would raise at the first non-finite mean)
        validate = ac.validate_args
        if torch.device(self.device).type == "cuda":
            ac.validate_args = False
        try:
            for (obs_b, critic_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b, old_sigma_b,
                 hid_b, masks_b) in gen:
                with amp:
                    loss, value_loss, surrogate_loss, se_loss = self._losses(
                        ac, obs_b, critic_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b,
                        old_sigma_b, hid_b, masks_b, mse)
                self.optimizer.zero_grad(set_to_none=False)   # keep the .grad views into the all-reduce bucket
                loss.backward()
                self.grads.all_reduce_()
                nn.utils.clip_grad_norm_(ac.parameters(), self.max_grad_norm)
                self.optimizer.step()
                sums += torch.stack([value_loss.detach(), surrogate_loss.detach(), se_loss.detach()])
        finally:
            ac.validate_args = validate
        n = self.num_learning_epochs * self.num_mini_batches
        self.storage.clear()
        mv, ms, mse_ = (sums / n).tolist()
        if not all(map(math.isfinite, (mv, ms, mse_))):
            raise ValueError(f"DHPPO.update: non-finite losses (value {mv}, surrogate {ms}, state estimator {mse_})")
        return mv, ms, mse_

    def _losses(self, ac, obs_b, critic_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b,
                old_sigma_b, hid_b, masks_b, mse):
        """The reference's minibatch losses (dh_ppo.py:130-178); the distribution terms in fp32 under autocast."""
        ac.act(obs_b, masks=masks_b, hidden_states=hid_b[0])
        est_lin_vel = ac.state_estimator(obs_b[:, -self.num_short_obs:])
        ref_lin_vel = critic_b[:, self.lin_vel_idx:self.lin_vel_idx + 3].clone()
        logp_b = ac.get_actions_log_prob(actions_b)
        value_b = ac.evaluate(critic_b, masks=masks_b, hidden_states=hid_b[1])
        mu_b, sigma_b, entropy_b = ac.action_mean, ac.action_std, ac.entropy
        if self.desired_kl is not None and self.schedule == "adaptive":
            self._adapt_lr(mu_b, sigma_b, old_mu_b, old_sigma_b)
        # clipped surrogate
        ratio = torch.exp(logp_b - torch.squeeze(old_logp_b))
        adv = torch.squeeze(adv_b)
        surrogate_loss = torch.max(-adv * ratio,
                                   -adv * torch.clamp(ratio, 1.0 - self.clip_param, 1.0 + self.clip_param)).mean()
        # value loss
        if self.use_clipped_value_loss:
            v_clip = target_values_b + (value_b - target_values_b).clamp(-self.clip_param, self.clip_param)
            value_loss = torch.max((value_b - returns_b).pow(2), (v_clip - returns_b).pow(2)).mean()
        else:
            value_loss = (returns_b - value_b).pow(2).mean()
        se_loss = mse(est_lin_vel.float(), ref_lin_vel)
        loss = surrogate_loss + self.value_loss_coef * value_loss - self.entropy_coef * entropy_b.mean() + se_loss
        return loss, value_loss, surrogate_loss, se_loss
