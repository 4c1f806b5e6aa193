"""RolloutStorage: on-device PPO rollout buffer + GAE (reference humanoid/algo/ppo/rollout_storage.py:3-173).

Same API (``Transition``, ``add_transitions``, ``compute_returns``, ``mini_batch_generator``,
``get_statistics``, ``clear``) and the same arithmetic.  Everything stays resident in HBM.  With data-parallel
training the advantage normalisation uses the mean / std over all ranks, which equals the
single-GPU statistics of the concatenated rollout.

Frame-history storage (``history=(frame, frames)``): the actor observation of the T1 env is a stack of
`frames` frames of `frame` features, oldest first, which the env shifts by one frame per step and clears (zeros)
when an env resets (t1_dh_stand_env.py:368-481, 548-558).  Storing all 24 x 8192 x 3102 fp32 (2.4 GB) costs a
101 MB copy per rollout step; with `history` the storage keeps the first step's full history plus each later step's
newest frame (137 MB in all), and the minibatch generator rebuilds every sampled history from them and the stored
dones -- the same bits as the full rows.  Callers whose observations are not such a history keep the full storage.
"""
import os

import warnings

import torch

from . import distributed as dist_util


# the minibatch's per-transition fields gathered by one HIP launch on the device (t1policy_gather_rows; T1_GATHER_ROWS=0:
# torch's index per field, A/B)
GATHER_ROWS = os.environ.get("T1_GATHER_ROWS", "1") != "0"


class _FieldGather:
    """fields[k][idx] for every field by one launch (t1policy_gather_rows): 2-D, contiguous, 32-bit device tensors of
    the same row count; anything else is indexed by torch.  Output buffers are fresh per call (graph-pool memory
    inside a captured update)."""

    def __init__(self, fields):
        self.fields = fields
        self.ok = (all(f.is_cuda and f.dim() == 2 and f.is_contiguous() and f.element_size() == 4 for f in fields)
                   and len({f.shape[0] for f in fields}) == 1 and len(fields) <= 12)

    def __call__(self, idx):
        if not self.ok:
            return [f[idx] for f in self.fields]
        import ctypes as C
        from .. import _lib
        lib = _lib.load()
        idx = idx.contiguous()
        rows = idx.shape[0]
        outs = [torch.empty(rows, f.shape[1], device=f.device, dtype=f.dtype) for f in self.fields]
        n = len(self.fields)
        srcs = (C.c_uint64 * n)(*[f.data_ptr() for f in self.fields])
        dsts = (C.c_uint64 * n)(*[o.data_ptr() for o in outs])
        widths = (C.c_int * n)(*[f.shape[1] for f in self.fields])
        rc = lib.t1policy_gather_rows(srcs, dsts, widths, n, idx.data_ptr(), rows,
                                      torch.cuda.current_stream(idx.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"t1policy_gather_rows failed (rc={rc})")
        return outs


class RolloutStorage:
    class Transition:
        __slots__ = ("observations", "critic_observations", "actions", "rewards", "dones", "values",
                     "actions_log_prob", "action_mean", "action_sigma", "hidden_states", "next_proprio_obs")

        def __init__(self):
            self.clear()

        def clear(self):
            for k in self.__slots__:
                setattr(self, k, None)

    def __init__(self, num_envs, num_transitions_per_env, obs_shape, privileged_obs_shape, actions_shape,
                 num_single_obs=None, device="cpu", history=None):
        T, N, d = num_transitions_per_env, num_envs, device
        self.device = device
        self.obs_shape, self.privileged_obs_shape, self.actions_shape = obs_shape, privileged_obs_shape, actions_shape
        self.num_transitions_per_env, self.num_envs, self.num_single_obs = T, N, num_single_obs

        def buf(*shape, dtype=torch.float32):
            return torch.zeros(T, N, *shape, device=d, dtype=dtype)

        self.history = None
        if history is not None:
            frame, frames = (int(x) for x in history)
            if tuple(obs_shape) != (frame * frames,):
                raise ValueError(f"history {history} does not match obs_shape {tuple(obs_shape)}")
            self.history = (frame, frames)
            self.obs0 = torch.zeros(N, frame * frames, device=d)   # the first step's whole history
            self.frames = buf(frame)                                # each step's newest frame
            self.observations = None
        else:
            self.observations = buf(*obs_shape)
        self.privileged_observations = buf(*privileged_obs_shape) if privileged_obs_shape[0] is not None else None
        self.rewards = buf(1)
        self.actions = buf(*actions_shape)
        self.dones = buf(1, dtype=torch.uint8)
        self.actions_log_prob = buf(1)
        self.values = buf(1)
        self.returns = buf(1)
        self.advantages = buf(1)
        self.mu = buf(*actions_shape)
        self.sigma = buf(*actions_shape)
        self.next_proprio_obs = buf(num_single_obs) if num_single_obs is not None else None
        self.saved_hidden_states_a = None
        self.saved_hidden_states_c = None
        self.step = 0
        self.graph_gae = True   # compute_returns' backward pass as a captured graph on a HIP device
        self._gae_graph = None
        self._gae_lv = None
        self._rows = None       # the frame-history rows source (_HistoryRows), rebuilt in place every update
        self._obs_cast = None   # the full storage's observations cast to the update's dtype, in place every update

    def add_transitions(self, t):
        self.write_transition(t, self.step)
        self.step += 1

    def write_transition(self, t, k):
        """The transition's copies into slot k (add_transitions without the step count: DHPPO's graphed store)."""
        if k >= self.num_transitions_per_env:
            raise AssertionError("Rollout buffer overflow")
        if self.history is not None:
            if k == 0:
                self.obs0.copy_(t.observations)
            self.frames[k].copy_(t.observations[:, -self.history[0]:])
        else:
            self.observations[k].copy_(t.observations)
        if self.privileged_observations is not None:
            self.privileged_observations[k].copy_(t.critic_observations)
        self.actions[k].copy_(t.actions)
        self.rewards[k].copy_(t.rewards.view(-1, 1))
        self.dones[k].copy_(t.dones.view(-1, 1))
        self.values[k].copy_(t.values)
        self.actions_log_prob[k].copy_(t.actions_log_prob.view(-1, 1))
        self.mu[k].copy_(t.action_mean)
        self.sigma[k].copy_(t.action_sigma)
        if self.next_proprio_obs is not None:
            self.next_proprio_obs[k].copy_(t.next_proprio_obs)

    def clear(self):
        self.step = 0

    def _gae(self, last_values, gamma, lam):
        adv = torch.zeros_like(last_values)
        next_values = last_values
        for k in range(self.num_transitions_per_env - 1, -1, -1):
            not_done = 1.0 - self.dones[k].float()
            delta = self.rewards[k] + not_done * gamma * next_values - self.values[k]
            adv = delta + not_done * gamma * lam * adv
            self.returns[k] = adv + self.values[k]
            next_values = self.values[k]
        # in place: the minibatch sources keep their addresses across updates (a captured update graph reads them)
        torch.sub(self.returns, self.values, out=self.advantages)

    def compute_returns(self, last_values, gamma, lam):
        """Generalised advantage estimation, backwards over the rollout (rollout_storage.py:91-116).  On a HIP device
        the backward pass (about 200 small element-wise kernels) replays a captured graph over the storage's own
        buffers and a static copy of last_values: the same kernels, without their launch gaps."""
        if last_values.is_cuda and self.graph_gae:
            key = (tuple(last_values.shape), last_values.dtype, float(gamma), float(lam))
            if self._gae_graph is None or self._gae_graph[0] != key:
                self._gae_lv = last_values.clone()
                self._gae(self._gae_lv, gamma, lam)   # this call eagerly; captured for the next ones
                g = torch.cuda.CUDAGraph()
                try:
                    with torch.cuda.graph(g):
                        self._gae(self._gae_lv, gamma, lam)
                    self._gae_graph = (key, g)
                except RuntimeError as e:   # as DHPPO's graphed store: fall back to the eager pass
                    warnings.warn(f"RolloutStorage: GAE graph capture failed, running eager: {e}")
                    # nothing runs during a capture: the eager pass above already produced this call's results
                    self.graph_gae, self._gae_graph = False, None
            else:
                self._gae_lv.copy_(last_values)
                self._gae_graph[1].replay()
        else:
            self._gae(last_values, gamma, lam)
        mean, std = dist_util.global_mean_std(self.advantages)
        self.advantages.sub_(mean).div_(std + 1e-8)

    def get_statistics(self):
        done = self.dones
        done[-1] = 1
        flat = done.permute(1, 0, 2).reshape(-1, 1)
        idx = torch.cat((flat.new_tensor([-1], dtype=torch.int64), flat.nonzero(as_tuple=False)[:, 0]))
        return (idx[1:] - idx[:-1]).float().mean(), self.rewards.mean()

    def minibatch_source(self, obs_dtype=None):  # noqa: C901
        """take(idx) -> the reference generator's minibatch tuple (rollout_storage.py:153-173) for the flattened rows
        idx.  Every source is one of this storage's own buffers (the frame-history rows and the obs cast are rebuilt
        in place), so take() reads the same addresses every update and can sit inside a captured HIP graph;
        take.key names those addresses.  obs_dtype (not in the reference): the actor observations are cast once per
        update to that dtype (the opt-in bf16 update, DHPPO.amp_dtype, whose GEMMs cast every obs-fed operand to bf16
        anyway), so each minibatch gathers, unfolds and saves half the bytes."""
        flat = lambda x: x.flatten(0, 1)  # noqa: E731
        if self.history is not None:
            dt = obs_dtype if obs_dtype is not None else self.obs0.dtype
            if self._rows is None or self._rows.seq.dtype != dt:
                self._rows = _HistoryRows(self, dt)
            self._rows.refresh(self)
            obs, okey = self._rows, self._rows.seq.data_ptr()
        else:
            obs = flat(self.observations)
            if obs_dtype is not None and obs.dtype != obs_dtype:
                if self._obs_cast is None or self._obs_cast.dtype != obs_dtype:
                    self._obs_cast = torch.empty(obs.shape, dtype=obs_dtype, device=obs.device)
                obs = self._obs_cast.copy_(obs)
            okey = obs.data_ptr()
        critic = flat(self.privileged_observations) if self.privileged_observations is not None else obs
        cols = [flat(self.actions), flat(self.values), flat(self.advantages), flat(self.returns),
                flat(self.actions_log_prob), flat(self.mu), flat(self.sigma)]
        extra = None
        if self.next_proprio_obs is not None:
            extra = (flat(self.next_proprio_obs), flat(self.rewards))

        gather = _FieldGather([critic] + cols) if (GATHER_ROWS and critic is not obs) else None

        def take(idx):
            if gather is not None and idx.is_cuda:
                critic_b, actions, values, advantages, returns, logp, mu, sigma = gather(idx)
            else:
                critic_b = critic[idx]
                actions, values, advantages, returns, logp, mu, sigma = (c[idx] for c in cols)
            if extra is not None:
                return (extra[0][idx], extra[1][idx], obs[idx], critic_b, actions, values, advantages, returns,
                        logp, mu, sigma, (None, None), None)
            return obs[idx], critic_b, actions, values, advantages, returns, logp, mu, sigma, (None, None), None

        take.key = (okey, obs_dtype, critic.data_ptr(), *(c.data_ptr() for c in cols))
        return take

    def mini_batch_generator(self, num_mini_batches, num_epochs=8, obs_dtype=None):
        """The reference's generator (rollout_storage.py:153-173) over minibatch_source(obs_dtype)."""
        batch = self.num_envs * self.num_transitions_per_env
        mb = batch // num_mini_batches
        perm = torch.randperm(num_mini_batches * mb, requires_grad=False, device=self.device)
        take = self.minibatch_source(obs_dtype)
        for _ in range(num_epochs):
            for i in range(num_mini_batches):
                yield take(perm[i * mb:(i + 1) * mb])


class _HistoryRows:
    """Rows [idx] of the flattened (T * N, frame * frames) observations, rebuilt from the frame-history storage.

    Per env the frames form one sequence: the first step's history (frames oldest..newest = times -frames+1..0), then
    the newest frame of steps 1..T-1 (times 1..T-1).  Step k's history is the window of times k-frames+1..k, with the
    frames older than the env's latest reset at or before step k zeroed: obs k is post-reset when dones[k-1] is set
    (the env zeroes the history and appends the new frame), and the zeros stay until the frames shift out."""

    def __init__(self, st, dtype):
        frame, frames = st.history
        T, N = st.num_transitions_per_env, st.num_envs
        dev = st.obs0.device
        self.frame, self.frames, self.N, self.T = frame, frames, N, T
        self.seq = torch.empty(N, frames + T - 1, frame, device=dev, dtype=dtype)
        self.first = torch.empty(T, N, dtype=torch.int64, device=dev)
        self.win = torch.arange(frames, device=dev)
        self._steps = torch.arange(T, device=dev).view(T, 1).expand(T, N)

    def refresh(self, st):
        """Rebuild the sequences and reset marks from the storage, in place."""
        N, T, frames = self.N, self.T, self.frames
        self.seq[:, :frames] = st.obs0.view(N, frames, self.frame)
        if T > 1:
            self.seq[:, frames:] = st.frames[1:].transpose(0, 1)
        # first time step whose frame is valid for step k's history (frames of earlier times are zero)
        dn = st.dones.view(T, N) > 0
        reset_at = torch.where(torch.cat([torch.zeros(1, N, dtype=torch.bool, device=dn.device), dn[:-1]]),
                               self._steps, torch.full_like(self._steps, -(frames + T)))
        self.first.copy_(torch.cummax(reset_at, 0).values)

    def __getitem__(self, idx):
        if self.seq.is_cuda:   # one HIP gather (include/t1policy.h t1policy_history_rows): the same rows, bit for bit
            from .. import _lib
            out = torch.empty(idx.numel(), self.frames * self.frame, dtype=self.seq.dtype, device=self.seq.device)
            idx = idx.contiguous()
            rc = _lib.load().t1policy_history_rows(self.seq.data_ptr(), self.first.data_ptr(), idx.data_ptr(),
                                                   out.data_ptr(), idx.numel(), self.N, self.T, self.frames, self.frame,
                                                   self.seq.element_size(),
                                                   torch.cuda.current_stream(self.seq.device).cuda_stream)
            if rc != 0:
                raise RuntimeError(f"t1policy_history_rows failed (rc={rc})")
            return out
        k, n = idx // self.N, idx % self.N
        pos = k.unsqueeze(1) + self.win.unsqueeze(0)                     # seq index = time + frames - 1
        rows = self.seq[n.unsqueeze(1), pos]                              # (M, frames, frame)
        old = (pos - (self.frames - 1)) < self.first[k, n].unsqueeze(1)   # frame time before the latest reset
        return rows.masked_fill_(old.unsqueeze(2), 0).reshape(idx.numel(), self.frames * self.frame)
