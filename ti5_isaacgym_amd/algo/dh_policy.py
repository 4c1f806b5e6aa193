"""ActorCriticDH: the t1_dh_stand policy and value networks (reference humanoid/algo/ppo/actor_critic_dh.py:8-188).

Same architecture, parameter names and initialisation as the reference, so its checkpoints load with
``torch.load(..., weights_only=True)`` and its runner calls (``act``, ``act_inference``, ``evaluate``,
``get_actions_log_prob``, ``action_mean``/``action_std``/``entropy``) behave identically:

  long_history  Conv1d over the 66-frame history (channels = frames, length = 47 features):
                32@k6/s3 -> ReLU -> 16@k4/s2 -> ReLU -> flatten (16 x 6) -> 128 -> ELU -> 64
  state_estimator  the newest 5 frames (235) -> 256 -> 128 -> 64 -> 3 (base linear velocity), ELU
  actor         [5 frames (235) | estimated velocity (3) | history code (64)] = 302 -> 512 -> 256 -> 128 -> 12
  critic        privileged 3 x 73 = 219 -> 768 -> 256 -> 128 -> 1
  std           12 learned action standard deviations (Normal policy)

856,972 parameters with the t1 config.  On MI355X the dense layers run as hipBLASLt GEMMs
through PyTorch-ROCm; the per-step inference batch is every env on the rank.
"""
import torch
import torch.nn as nn
from torch.distributions import Normal


def _mlp(sizes, act):
    """Linear layers between consecutive sizes, `act` after every hidden layer (not after the output)."""
    layers = []
    for i, (a, b) in enumerate(zip(sizes[:-1], sizes[1:])):
        layers.append(nn.Linear(a, b))
        if i < len(sizes) - 2:
            layers.append(act)
    return nn.Sequential(*layers)


def _history_encoder(frames, features, filters, kernels, strides, code_dim):
    layers, ch, length = [], frames, features
    for out_ch, k, s in zip(filters, kernels, strides):
        layers += [nn.Conv1d(ch, out_ch, kernel_size=k, stride=s), nn.ReLU()]
        length = (length - k + s) // s  # the reference's length bookkeeping (equals floor((L - k) / s) + 1)
        ch = out_ch
    layers += [nn.Flatten(), nn.Linear(length * ch, 128), nn.ELU(), nn.Linear(128, code_dim)]
    return nn.Sequential(*layers)


class ActorCriticDH(nn.Module):
    is_recurrent = False

    def __init__(self, num_short_obs, num_proprio_obs, num_critic_obs, num_actions,
                 actor_hidden_dims=(256, 256, 256), critic_hidden_dims=(256, 256, 256),
                 state_estimator_hidden_dims=(256, 128, 64), in_channels=66, kernel_size=(6, 4),
                 filter_size=(32, 16), stride_size=(3, 2), lh_output_dim=64, init_noise_std=1.0,
                 activation=None, **kwargs):
        if kwargs:
            print("ActorCriticDH.__init__ got unexpected arguments, which will be ignored: " + str(list(kwargs)))
        super().__init__()
        act = activation if activation is not None else nn.ELU()
        self.num_short_obs = num_short_obs
        self.num_proprio_obs = num_proprio_obs
        self.in_channels = in_channels
        self.actor = _mlp([num_short_obs + 3 + lh_output_dim, *actor_hidden_dims, num_actions], act)
        self.critic = _mlp([num_critic_obs, *critic_hidden_dims, 1], act)
        self.std = nn.Parameter(init_noise_std * torch.ones(num_actions))
        self.distribution = None
        Normal.set_default_validate_args = False
        self.long_history = _history_encoder(in_channels, num_proprio_obs, filter_size, kernel_size, stride_size,
                                             lh_output_dim)
        self.state_estimator = _mlp([num_short_obs, *state_estimator_hidden_dims, 3], act)

    # ------------------------------------------------------------------ reference API
    def reset(self, dones=None):
        pass

    def forward(self):
        raise NotImplementedError

    @property
    def action_mean(self):
        return self.distribution.mean

    @property
    def action_std(self):
        return self.distribution.stddev

    @property
    def entropy(self):
        return self.distribution.entropy().sum(dim=-1)

    def actor_input(self, observations):
        """[short history | estimated base velocity | long-history code] (302 features)."""
        short = observations[..., -self.num_short_obs:]
        code = self.long_history(observations.view(-1, self.in_channels, self.num_proprio_obs))
        return torch.cat((short, self.state_estimator(short), code), dim=-1)

    def update_distribution(self, actor_obs):
        mean = self.actor(actor_obs)
        self.distribution = Normal(mean, mean * 0.0 + self.std)

    def act(self, observations, **kwargs):
        self.update_distribution(self.actor_input(observations))
        return self.distribution.sample()

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)

    def act_inference(self, observations):
        return self.actor(self.actor_input(observations))

    def evaluate(self, critic_observations, **kwargs):
        return self.critic(critic_observations)
