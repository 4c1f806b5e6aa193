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
without the per-kernel launch cost that dominates at one call per env step.  The update's minibatch step (gather,
forward, losses, backward, clipping, the adaptive learning rate, Adam) replays a captured graph as well: Adam keeps
its step count and learning rate on the device (capturable, a tensor lr), the adaptive schedule's decision
(dh_ppo.py:141-151) is taken on the device, and the losses are summed there, so an update has no host sync until its
mean losses are read.  The first update's first minibatches run eagerly (the warm-up the capture needs), the rest
replay the graph; eager and graphed steps run the same kernels (bit-identical, tests/test_gpu_ppo.py).
"""
import contextlib
import math
import os
import warnings

import torch
import torch.nn as nn
import torch.optim as optim
from torch.distributions import Normal

from . import dh_policy
from . import distributed as dist_util
from .dh_policy import ActorCriticDH, heads_forward, refresh_packed_weights
from .rollout import RolloutStorage

# the update's gradient clipping over the flat gradient bucket on the device (T1_FLAT_CLIP=0: torch's
# clip_grad_norm_, A/B)
FLAT_CLIP = os.environ.get("T1_FLAT_CLIP", "1") != "0"
# the rollout's act() through the fused HIP heads (t1policy_heads_forward; T1_FUSED_ACT=0: the torch layers, A/B)
FUSED_ACT = os.environ.get("T1_FUSED_ACT", "1") != "0"


_GRAPH_RNG_ANCHOR = {}


def _init_graph_rng(device):
    """Let the device generator create its graph-capture state (seed / offset tensors) outside inference mode, and
    keep it: the generator allocates that state when the first live graph registers with it and drops it when the
    last one is gone.  The rollout's act() is captured under torch.inference_mode, where it would otherwise be made
    as inference tensors, which a later capture outside inference mode (the update's) may not update in place.  A
    one-node graph held for the process anchors it."""
    device = torch.device(device)
    if device in _GRAPH_RNG_ANCHOR or torch.is_inference_mode_enabled():
        return
    x = torch.empty(1, device=device)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        x.normal_()
    _GRAPH_RNG_ANCHOR[device] = (graph, x)


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
        self.desired_kl, self.schedule = desired_kl, schedule
        self._lr = float(learning_rate)
        self.actor_critic = actor_critic
        self.actor_critic.to(self.device)
        self.storage = None
        cuda = torch.device(device).type == "cuda"
        # the device learning rate (a 0-d tensor Adam reads) on a HIP device; None on the host (the reference's floats).
        # The adaptive schedule runs on _lr64, an fp64 device copy (the reference's Python float: lr / 1.5 and lr * 1.5
        # round as it does), and _lr_t, the fp32 value Adam reads, is refreshed from it
        self._lr_t = torch.tensor(float(learning_rate), device=device) if cuda else None
        self._lr64 = torch.tensor(float(learning_rate), dtype=torch.float64, device=device) if cuda else None
        self._c15 = torch.tensor(1.5, dtype=torch.float64, device=device) if cuda else None
        if cuda:
            # fused: one kernel per step (the capturable foreach Adam ran ~0.75 ms per step, r03x)
            self.optimizer = optim.Adam(self.actor_critic.parameters(), lr=self._lr_t, capturable=True, fused=True)
        else:
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
        self.graph_act = cuda
        self._act_graphs = {}
        # graphed update minibatch step: (key, graph) once captured; under data parallelism (key, (graph A, graph B))
        # with the gradient / KL all-reduce eager between them
        self.graph_update = cuda
        # graphed process_env_step: {(storage slot, every input's address): graph}, one per rollout slot and env
        # buffer parity (the env's observation buffers alternate between two addresses); False = eager
        self.graph_store = cuda
        self._store_graphs = {}
        if cuda:
            _init_graph_rng(device)
        self._upd = None
        self._upd_warm = 0
        self._idx = None
        self._sums = torch.zeros(3, device=device)
        self._kl = torch.zeros(1, device=device)   # this rank's KL mean, then the all-reduced one (DP graphed step)
        self._kl_deferred = False

    @property
    def learning_rate(self):
        """The current learning rate (the adaptive schedule's; on a HIP device read from the device)."""
        return float(self._lr64) if self._lr64 is not None else self._lr

    @learning_rate.setter
    def learning_rate(self, v):
        self._lr = float(v)
        if self._lr_t is not None:
            self._lr64.fill_(float(v))
            self._lr_t.fill_(float(v))

    def after_optimizer_load(self):
        """After optimizer.load_state_dict (a checkpoint resume): load_state_dict replaces every param-group
        hyperparameter with the saved one, so a state written by the reference (or by an older build) comes back with
        capturable=False / fused=None, under which the device-tensor learning rate is rejected.  Restore the flags this
        optimizer was built with and move the step counters to the parameters' device as fp32 (capturable Adam keeps
        them there).

        The learning rate follows the reference's runner.load (dh_on_policy_runner.py:311-318, dh_ppo.py:36, 141-151),
        which loads the optimizer state but leaves DHPPO.learning_rate at this process's value (the constructor's after
        a fresh start): under the adaptive schedule the first KL step overwrites the loaded lr with that value / 1.5,
        * 1.5 or itself, so the device lr continues from learning_rate, not from the checkpoint; under
        the fixed schedule the reference never writes the param groups' lr, so Adam keeps the checkpoint's lr while
        learning_rate (what the runner logs) stays this process's value.  The host path (a plain Adam) does both by
        itself."""
        if self._lr_t is None:
            return
        loaded = float(self.optimizer.param_groups[0]["lr"])
        for g in self.optimizer.param_groups:
            g["capturable"] = True
            g["fused"] = True
            g["foreach"] = None
            g["lr"] = self._lr_t
            for p in g["params"]:
                st = self.optimizer.state.get(p)
                if st and "step" in st:
                    st["step"] = torch.as_tensor(st["step"], dtype=torch.float32, device=p.device).reshape(())
        if self.desired_kl is not None and self.schedule == "adaptive":
            self._lr_t.copy_(self._lr64)
        else:
            self._lr_t.fill_(loaded)

    def _bind_lr(self):
        """Keep every param group's lr the device tensor (a caller may have put a float or another tensor there
        without after_optimizer_load: its value is taken over)."""
        for g in self.optimizer.param_groups:
            if g["lr"] is not self._lr_t:
                self._lr64.fill_(float(g["lr"]))
                self._lr_t.fill_(float(g["lr"]))
                g["lr"] = self._lr_t

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

    def _act_body(self, obs, critic_obs, eps=None):
        """act() as one fixed kernel sequence (ActorCriticDH.act / evaluate / get_actions_log_prob).  Two host
        checks cannot run inside a graph: the distribution's argument validation (built without it) and
        torch.normal's std >= 0 test (the sample is drawn as mean + std * N(0, 1), the same distribution).
        eps: the N(0, 1) draw of the mean's shape, made by the caller (the graphed act() draws it before each replay,
        so its graph holds no RNG kernel); None: drawn here."""
        ac = self.actor_critic
        obs, critic_obs = obs.float(), critic_obs.float()   # fp16 env histories (state_dtype="fp16"): no-op for fp32
        if obs.is_cuda and FUSED_ACT:
            # the fused HIP heads (t1policy_heads_forward): the same draw (randn of the mean's shape), one kernel for
            # every layer after the first conv plus the sample and its log-prob
            if eps is None:
                eps = torch.randn(obs.shape[0], ac.std.numel(), device=obs.device)
            out = heads_forward(ac, obs, critic_obs, eps)
            if out is not None:
                mean, actions, sigma, logp, value = out
                return actions, value, logp, mean, sigma
        mean = ac.actor(ac.actor_input(obs))
        std = mean * 0.0 + ac.std
        dist = Normal(mean, std, validate_args=False)
        # a refused fused call (no compiled instance for this model / shape) keeps its draw: one draw per act() either
        # way, so the RNG stream does not depend on the path
        actions = mean + std * (eps if eps is not None else torch.randn_like(mean))
        return actions, ac.critic(critic_obs), dist.log_prob(actions).sum(dim=-1), mean, std

    def _graphed_act(self, obs, critic_obs):
        key = (obs.data_ptr(), critic_obs.data_ptr(), tuple(obs.shape), tuple(critic_obs.shape))
        entry = self._act_graphs.get(key)
        if entry is None:
            if len(self._act_graphs) >= 4:  # not the env's fixed buffers: stay eager
                return None
            # the sample's N(0, 1) draw lives outside the graph (eps.normal_() before each replay, the values
            # torch.randn would draw): a graph with an RNG kernel makes every replay first refill the generator's seed
            # and offset tensors (two fill launches, ~9 us per act at 8192 envs, profiles/r07e)
            eps = torch.empty(obs.shape[0], self.actor_critic.std.numel(), device=obs.device)
            side = torch.cuda.Stream(device=obs.device)
            side.wait_stream(torch.cuda.current_stream(obs.device))
            with torch.cuda.stream(side):  # warm-up outside the capture (allocator, library handles)
                for _ in range(2):
                    self._act_body(obs, critic_obs, eps.normal_())
            torch.cuda.current_stream(obs.device).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(graph):
                    outs = self._act_body(obs, critic_obs, eps)
            except RuntimeError as e:  # a library call that cannot be captured: the eager act() from now on
                warnings.warn(f"DHPPO: act() graph capture failed, running eager: {e}")
                self.graph_act = False
                return None
            entry = self._act_graphs[key] = (graph, outs, eps)
        refresh_packed_weights(self.actor_critic)  # the conv's packed weights after a PPO update (in place)
        entry[2].normal_()
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

    def _store_body(self, rewards, dones, time_outs, k):
        """process_env_step's device work for rollout slot k: the time-out bootstrap and the transition's copies."""
        t = self.transition
        t.rewards = rewards.clone()
        t.dones = dones
        if time_outs is not None:  # bootstrap on time-outs
            t.rewards += self.gamma * torch.squeeze(t.values * time_outs.unsqueeze(1).to(self.device), 1)
        self.storage.write_transition(t, k)

    def _graphed_store(self, rewards, dones, time_outs):
        """The slot's store as a captured graph (a dozen small copies and element-wise kernels a step: their launch
        gaps, not their bytes, set the eager time).  Keyed by the slot and every input's address, so a replay reads
        the tensors it was captured on; anything else stays eager."""
        t, k = self.transition, self.storage.step
        ins = (rewards, dones, time_outs, t.observations, t.critic_observations, t.actions, t.values,
               t.actions_log_prob, t.action_mean, t.action_sigma)
        if any(x is not None and not x.is_cuda for x in ins) or t.next_proprio_obs is not None:
            return False
        # the slot and every input's address, shape and dtype (a replay reads exactly the tensors it was captured on)
        key = (k,) + tuple((x.data_ptr(), tuple(x.shape), x.dtype) if x is not None else 0 for x in ins)
        g = self._store_graphs.get(key)
        if g is None:
            if len(self._store_graphs) >= 4 * self.storage.num_transitions_per_env:
                return False   # not the rollout's fixed buffers
            self._store_body(rewards, dones, time_outs, k)   # this step eagerly; capture for the next time
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g):
                    self._store_body(rewards, dones, time_outs, k)
            except RuntimeError as e:
                warnings.warn(f"DHPPO: process_env_step graph capture failed, running eager: {e}")
                self.graph_store = False
                return True
            self._store_graphs[key] = g
            return True
        g.replay()
        return True

    def process_env_step(self, rewards, dones, infos):
        t = self.transition
        time_outs = infos.get("time_outs")
        if not (self.graph_store and rewards.is_cuda and self._graphed_store(rewards, dones, time_outs)):
            self._store_body(rewards, dones, time_outs, self.storage.step)
        self.storage.step += 1
        t.clear()
        self.actor_critic.reset(dones)

    def compute_returns(self, last_critic_obs):
        last_values = self.actor_critic.evaluate(last_critic_obs).detach()
        self.storage.compute_returns(last_values, self.gamma, self.lam)

    def _adapt_lr(self, mu, sigma, old_mu, old_sigma):
        with torch.no_grad():
            kl = torch.sum(torch.log(sigma / old_sigma + 1.0e-5)
                           + (torch.square(old_sigma) + torch.square(old_mu - mu)) / (2.0 * torch.square(sigma)) - 0.5,
                           axis=-1)
            if self._kl_deferred:
                # the data-parallel graphed step (_dp_part_a): this rank's KL mean, all-reduced between the two graphs
                # and decided on in _dp_part_b (the lr only matters at the optimizer step: the same decision)
                self._kl.copy_(torch.mean(kl).reshape(1))
                return
            kl_mean = dist_util.all_reduce_mean_(torch.mean(kl).reshape(1))[0]
            if self._lr_t is not None:
                self._lr_decide(kl_mean)
                return
            kl_mean = float(kl_mean)
        if kl_mean > self.desired_kl * 2.0:
            self.learning_rate = max(1e-5, self.learning_rate / 1.5)
        elif 0.0 < kl_mean < self.desired_kl / 2.0:
            self.learning_rate = min(1e-2, self.learning_rate * 1.5)
        for g in self.optimizer.param_groups:
            g["lr"] = self.learning_rate

    def _lr_decide(self, kl_mean):
        """The adaptive decision on the device (no host sync; capturable): lr / 1.5 floored at 1e-5 above twice the
        target KL, lr * 1.5 capped at 1e-2 below half of it (a KL of exactly 0 keeps lr); the KL compared in fp32 as
        the reference's tensor comparisons, the lr stepped in fp64 as its Python float."""
        lr = self._lr64
        # a tensor divisor: torch divides by a host scalar as a multiply by its reciprocal (one more rounding than the
        # reference's Python lr / 1.5)
        down = torch.clamp(lr / self._c15, min=1e-5)
        up = torch.clamp(lr * 1.5, max=1e-2)
        low = (kl_mean > 0.0) & (kl_mean < self.desired_kl / 2.0)
        lr.copy_(torch.where(kl_mean > self.desired_kl * 2.0, down, torch.where(low, up, lr)))
        self._lr_t.copy_(lr)

    # ---- the data-parallel minibatch step on the device, in two parts around the exchange (dh_ppo.py:139-151,
    # 180-182): part A forward, losses, this rank's KL mean and backward into the gradient bucket; the exchange all-reduces
    # the bucket and the KL mean (RCCL on MI355X; it cannot sit inside a captured graph with gloo, and stays outside
    # with RCCL too); part B the adaptive lr decision, clipping and Adam.  Graphed, A and B are two captured graphs.
    def _dp_part_a(self, batch, amp, mse):
        ac = self.actor_critic
        (obs_b, critic_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b, old_sigma_b, hid_b,
         masks_b) = batch
        self._kl_deferred = True
        try:
            with amp:
                loss, value_loss, surrogate_loss, se_loss = self._losses(
                    ac, obs_b, critic_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b,
                    old_sigma_b, hid_b, masks_b, mse)
        finally:
            self._kl_deferred = False
        self.optimizer.zero_grad(set_to_none=False)   # keep the .grad views into the all-reduce bucket
        with dh_policy.direct_grad_accumulation():   # a plain backward into every .grad: the wgrad kernel may add there
            loss.backward()
        self._sums += torch.stack([value_loss.detach(), surrogate_loss.detach(), se_loss.detach()])

    def _dp_exchange(self):
        self.grads.all_reduce_()
        if self._adaptive():
            dist_util.all_reduce_mean_(self._kl)

    def _dp_part_b(self):
        if self._adaptive():
            with torch.no_grad():
                self._lr_decide(self._kl[0])
        self._clip_grads()
        self.optimizer.step()

    def _clip_grads(self):
        """clip_grad_norm_ (dh_ppo.py:181).  On the device the 2-norm is taken over the flat bucket every .grad views
        (one reduction and one scale instead of torch's per-tensor norms, a norm of the norms and a scale per tensor:
        ~110 us per minibatch); the same clip, the squares summed in another order (fp32).  On the host torch's."""
        g = self.grads
        if FLAT_CLIP and g.flat.is_cuda:
            g.bind_()   # every .grad is its bucket view (no-op unless something replaced one)
            coef = torch.clamp(self.max_grad_norm / (torch.linalg.vector_norm(g.flat) + 1e-6), max=1.0)
            g.flat.mul_(coef)
        else:
            nn.utils.clip_grad_norm_(self.actor_critic.parameters(), self.max_grad_norm)

    def _adaptive(self):
        return self.desired_kl is not None and self.schedule == "adaptive"

    def _minibatch_step(self, batch, amp, mse):
        """One minibatch of the update: losses, backward, gradient all-reduce, clipping, Adam; the losses summed into
        self._sums on the device."""
        ac = self.actor_critic
        (obs_b, critic_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b, old_sigma_b, hid_b,
         masks_b) = batch
        with amp:
            loss, value_loss, surrogate_loss, se_loss = self._losses(
                ac, obs_b, critic_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b, old_sigma_b,
                hid_b, masks_b, mse)
        self.optimizer.zero_grad(set_to_none=False)   # keep the .grad views into the all-reduce bucket
        with dh_policy.direct_grad_accumulation():   # a plain backward into every .grad: the wgrad kernel may add there
            loss.backward()
        self.grads.all_reduce_()
        self._clip_grads()
        self.optimizer.step()
        self._sums += torch.stack([value_loss.detach(), surrogate_loss.detach(), se_loss.detach()])

    def _step_eager(self, batch, amp, mse):
        """One eager minibatch step: the single-process / host step, or on the device under data parallelism the two
        parts of the graphed step around the exchange (the same kernels as its graph replays)."""
        if self._lr_t is not None and dist_util.active():
            self._dp_part_a(batch, amp, mse)
            self._dp_exchange()
            self._dp_part_b()
        else:
            self._minibatch_step(batch, amp, mse)

    def update(self):
        ac = self.actor_critic
        mse = nn.MSELoss()
        cuda = torch.device(self.device).type == "cuda"
        use_amp = self.amp_dtype is not None and cuda
        # cache_enabled=False: a captured graph must not depend on autocast's weight-cast cache (same values)
        amp = torch.autocast(device_type="cuda", dtype=self.amp_dtype, cache_enabled=False) if use_amp \
            else contextlib.nullcontext()
        # under the bf16 update every consumer of the actor observations is a bf16 GEMM: cast them once per update
        # (same values as autocast's per-minibatch casts) unless cast_obs_once is switched off (A/B)
        obs_dtype = self.amp_dtype if use_amp and self.cast_obs_once else None
        self._sums.zero_()
        if self._lr_t is not None:
            self._bind_lr()
        # the distribution's argument checks are host syncs (three per minibatch) on the device: off for the update,
        # replaced by one finiteness check of the losses below (the reference would raise at the first non-finite mean)
        validate = ac.validate_args
        if cuda:
            ac.validate_args = False
        try:
            if cuda and self.graph_update:
                self._update_graphed(amp, mse, obs_dtype)
            else:
                for batch in self.storage.mini_batch_generator(self.num_mini_batches, self.num_learning_epochs,
                                                               obs_dtype=obs_dtype):
                    self._step_eager(batch, amp, mse)
        finally:
            ac.validate_args = validate
        if cuda:  # the optimizer steps were graph replays (no version bump): repack the conv's fragments now
            refresh_packed_weights(ac, force=True)
        n = self.num_learning_epochs * self.num_mini_batches
        self.storage.clear()
        mv, ms, mse_ = (self._sums / n).tolist()
        if not all(map(math.isfinite, (mv, ms, mse_))):
            raise ValueError(f"DHPPO.update: non-finite losses (value {mv}, surrogate {ms}, state estimator {mse_})")
        return mv, ms, mse_

    WARMUP_STEPS = 2   # eager minibatch steps (on a side stream) before the capture

    def _update_graphed(self, amp, mse, obs_dtype):
        """The minibatches of mini_batch_generator, each as (copy its indices into a static buffer, replay); under data
        parallelism each as (copy, replay part A, exchange, replay part B)."""
        st = self.storage
        dp = dist_util.active()
        mb = st.num_envs * st.num_transitions_per_env // self.num_mini_batches
        perm = torch.randperm(self.num_mini_batches * mb, requires_grad=False, device=self.device)
        take = st.minibatch_source(obs_dtype)
        key = self._graph_key(mb, take)
        if self._upd is None or self._upd[0] != key:
            # (re)capture after WARMUP_STEPS eager steps, which also create any missing Adam state: a state tensor
            # created inside the capture would be re-initialised by every replay
            self._upd, self._upd_warm = None, 0
        if self._idx is None or self._idx.numel() != mb:
            self._idx = torch.empty(mb, dtype=torch.int64, device=self.device)
        cur = torch.cuda.current_stream(self._idx.device)
        for _ in range(self.num_learning_epochs):
            for i in range(self.num_mini_batches):
                self._idx.copy_(perm[i * mb:(i + 1) * mb])
                if not self.graph_update:   # a capture failed earlier in this update: the rest runs eagerly
                    self._step_eager(take(self._idx), amp, mse)
                elif self._upd is not None:
                    if dp:
                        self._upd[1][0].replay()
                        self._dp_exchange()
                        self._upd[1][1].replay()
                    else:
                        self._upd[1].replay()
                elif self._upd_warm < self.WARMUP_STEPS or any(len(self.optimizer.state.get(p, {})) == 0
                                                               for p in self.grads.params):
                    side = torch.cuda.Stream(device=self._idx.device)
                    side.wait_stream(cur)
                    with torch.cuda.stream(side):
                        self._step_eager(take(self._idx), amp, mse)
                    cur.wait_stream(side)
                    self._upd_warm += 1
                elif dp:
                    # every rank captures part A, then they agree on its success before the first exchange: a rank
                    # whose capture failed must not leave the others waiting in the bucket all-reduce.  On a
                    # failure every rank runs this minibatch and the rest of the update eagerly.
                    ga, gb = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
                    err = self._try_capture(ga, lambda: self._dp_part_a(take(self._idx), amp, mse))
                    if not self._all_ranks_ok(err is None):
                        self._capture_failed(err)
                        self._step_eager(take(self._idx), amp, mse)
                        continue
                    ga.replay()
                    self._dp_exchange()
                    err = self._try_capture(gb, self._dp_part_b)
                    if not self._all_ranks_ok(err is None):
                        # the exchange already ran: finish this minibatch eagerly (part B alone), the rest eager too
                        self._capture_failed(err)
                        self._dp_part_b()
                        continue
                    gb.replay()
                    self._upd = (self._graph_key(mb, take), (ga, gb))
                else:
                    graph = torch.cuda.CUDAGraph()
                    err = self._try_capture(graph, lambda: self._minibatch_step(take(self._idx), amp, mse))
                    if err is not None:
                        self._capture_failed(err)
                        self._step_eager(take(self._idx), amp, mse)
                        continue
                    self._upd = (self._graph_key(mb, take), graph)
                    graph.replay()

    @staticmethod
    def _try_capture(graph, body):
        """Capture body() into graph; the RuntimeError of a failed capture, else None."""
        try:
            with torch.cuda.graph(graph):
                body()
        except RuntimeError as e:
            return e
        return None

    @staticmethod
    def _all_ranks_ok(ok):
        """Every rank's capture succeeded (a MIN all-reduce of the flags under data parallelism)."""
        if not dist_util.active():
            return ok
        import torch.distributed as dist
        f = torch.tensor([1 if ok else 0], dtype=torch.int32,
                         device=torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl"
                         else "cpu")
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        return bool(f.item())

    def _capture_failed(self, err):
        warnings.warn(f"DHPPO: update graph capture failed ({err if err is not None else 'on another rank'}); "
                      "the update runs eagerly")
        self.graph_update = False
        self._upd = None

    def _graph_key(self, mb, take):
        """Everything a captured minibatch step holds as a constant: the buffers' addresses (storage sources, Adam's
        state -- replaced by optimizer.load_state_dict, created lazily by the first step --, the learning rate), the
        update dtype and the loss hyperparameters."""
        opt = []
        for g in self.optimizer.param_groups:
            opt.append(g["lr"].data_ptr() if torch.is_tensor(g["lr"]) else g["lr"])
            for p in g["params"]:
                st = self.optimizer.state.get(p, {})
                opt.extend(st[k].data_ptr() if k in st else None for k in ("step", "exp_avg", "exp_avg_sq"))
        return (mb, take.key, tuple(opt), str(self.amp_dtype), self.schedule, self.desired_kl, self.clip_param,
                self.value_loss_coef, self.entropy_coef, self.max_grad_norm, self.use_clipped_value_loss,
                self.lin_vel_idx, dist_util.active())

    def _losses(self, ac, *args):
        """The reference's minibatch losses (dh_ppo.py:130-178); the distribution terms in fp32 under autocast.  Under
        the device autocast the parameters' low-precision copies are made by one multi-tensor cast first
        (dh_policy.param_shadows: the same values as the per-layer casts)."""
        if args[0].is_cuda and torch.is_autocast_enabled("cuda") and dh_policy.PARAM_SHADOWS:
            with dh_policy.param_shadows(ac, torch.get_autocast_dtype("cuda")):
                return self._losses_body(ac, *args)
        return self._losses_body(ac, *args)

    def _losses_body(self, ac, obs_b, critic_b, actions_b, target_values_b, adv_b, returns_b, old_logp_b, old_mu_b,
                     old_sigma_b, hid_b, masks_b, mse):
        # the reference calls ac.act() here for its distribution and drops the sample.  On the device the distribution
        # alone (a sample's std >= 0 check is a host sync, which no graph capture allows; the losses do not use it); on
        # the CPU the sample is drawn and dropped like the reference's, so the global RNG stream -- the next rollout's
        # action samples -- stays the reference's (tests/test_runner_golden.py)
        if obs_b.is_cuda:
            # one state-estimator pass feeds both the actor input and the estimator loss (the reference evaluates the
            # same network on the same rows twice, dh_ppo.py:123-126: the same values; the two uses' gradients are
            # summed at its output instead of in its parameters) -- its forward and backward once per minibatch
            est_lin_vel = ac.state_estimator(obs_b[:, -self.num_short_obs:])
            ac.update_distribution(ac.actor_input(obs_b, est_lin_vel))
        else:
            ac.update_distribution(ac.actor_input(obs_b))
            ac.distribution.sample()
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
