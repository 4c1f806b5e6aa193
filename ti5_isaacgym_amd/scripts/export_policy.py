"""Export a trained ActorCriticDH as TorchScript (reference humanoid/scripts/export_policy_dh.py:14-36).

    python -m ti5_isaacgym_amd.scripts.export_policy <checkpoint.pt> <out.jit>

The exported module maps the 66-frame observation history (N, 3102) to (action mean (N, 12), estimated base
linear velocity (N, 3)) -- the deployment interface of the reference's policy_dh.jit.  Checkpoints are read
with weights_only=True.
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

from ti5_isaacgym_amd.algo import ActorCriticDH  # noqa: E402
from ti5_isaacgym_amd.algo.dh_policy import plain_copy  # noqa: E402
from ti5_isaacgym_amd.envs.configs import DHT1StandCfgPPO  # noqa: E402
from ti5_isaacgym_amd.utils.helpers import class_to_dict  # noqa: E402


class ExportedDH(torch.nn.Module):
    def __init__(self, ac: ActorCriticDH):
        super().__init__()
        # plain torch layers (the device-path Linear / HistoryEncoder subclasses are not scriptable)
        self.actor = plain_copy(ac.actor).cpu()
        self.long_history = plain_copy(ac.long_history).cpu()
        self.state_estimator = plain_copy(ac.state_estimator).cpu()
        self.num_short_obs = ac.num_short_obs
        self.in_channels = ac.in_channels
        self.num_proprio_obs = ac.num_proprio_obs

    def forward(self, observations):
        short = observations[..., -self.num_short_obs:]
        est_vel = self.state_estimator(short)
        code = self.long_history(observations.view(-1, self.in_channels, self.num_proprio_obs))
        return self.actor(torch.cat((short, est_vel, code), dim=-1)), est_vel


def load_policy(checkpoint, policy_cfg=None):
    cfg = policy_cfg or class_to_dict(DHT1StandCfgPPO())["policy"]
    ac = ActorCriticDH(235, 47, 219, 12, **cfg)
    state = torch.load(checkpoint, map_location="cpu", weights_only=True)
    ac.load_state_dict(state["model_state_dict"])
    return ac.eval()


def export(checkpoint, out_path):
    module = torch.jit.script(ExportedDH(load_policy(checkpoint)))
    module.save(out_path)
    return out_path


if __name__ == "__main__":
    print(export(sys.argv[1], sys.argv[2]))
