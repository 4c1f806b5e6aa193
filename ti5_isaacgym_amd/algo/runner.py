"""DHOnPolicyRunner: rollout + PPO update loop over the HIP env (reference humanoid/algo/ppo/dh_on_policy_runner.py:19-337).

Same constructor, ``learn``, ``log``, ``save``, ``load``, ``get_inference_policy`` / ``get_inference_critic``
and checkpoint layout as the reference.  Differences, all outside the arithmetic:
  * episode bookkeeping (reward / length buffers for logging) is recorded on the device with masks and read
    once per iteration instead of a nonzero() host sync every env step; the buffers receive the same values
    in the same order;
  * data-parallel runs (one process per GPU, torchrun): every rank rolls out its own env shard, DHPPO
    all-reduces gradients / KL / advantage statistics (so losses, learning rate and weights are the same on every
    rank), rank 0 logs and saves.  The episode statistics rank 0 logs (mean reward / length, extras["episode"])
    are those of its own env shard, not reduced over ranks; fps and total timesteps count all ranks;
  * TensorBoard is optional (not in this image): scalars then go to ``<log_dir>/scalars.jsonl``.
"""
import json
import os
import statistics
import time
from collections import deque

import torch

from . import distributed as dist_util
from .dh_policy import ActorCriticDH
from .dh_update import DHPPO

POLICY_CLASSES = {"ActorCriticDH": ActorCriticDH}
ALGORITHM_CLASSES = {"DHPPO": DHPPO}


class ScalarWriter:
    """Minimal SummaryWriter stand-in: one JSON object per add_scalar call."""

    def __init__(self, log_dir, flush_secs=10):
        os.makedirs(log_dir, exist_ok=True)
        self.f = open(os.path.join(log_dir, "scalars.jsonl"), "a")
        self.flush_secs, self.t = flush_secs, time.time()

    def add_scalar(self, tag, value, step):
        self.f.write(json.dumps({"tag": tag, "value": float(value), "step": int(step)}) + "\n")
        if time.time() - self.t > self.flush_secs:
            self.f.flush()
            self.t = time.time()

    def close(self):
        self.f.close()


def _make_writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir=log_dir, flush_secs=10)
    except ImportError:
        return ScalarWriter(log_dir)


class DHOnPolicyRunner:
    def __init__(self, env, train_cfg, log_dir=None, device="cpu"):
        self.cfg, self.alg_cfg, self.policy_cfg = train_cfg["runner"], train_cfg["algorithm"], train_cfg["policy"]
        self.all_cfg = train_cfg
        self.device = device
        self.env = env
        self.rank0 = not dist_util.active() or torch.distributed.get_rank() == 0
        num_critic_obs = env.num_privileged_obs if env.num_privileged_obs is not None else env.num_obs
        if env.cfg.terrain.measure_heights:
            num_critic_obs = env.cfg.env.c_frame_stack * (env.cfg.env.single_num_privileged_obs
                                                         + env.cfg.terrain.num_height)
        policy_cls = POLICY_CLASSES[self.cfg["policy_class_name"]]
        actor_critic = policy_cls(env.num_short_obs, env.num_single_obs, num_critic_obs, env.num_actions,
                                  **self.policy_cfg).to(self.device)
        alg_cls = ALGORITHM_CLASSES[self.cfg["algorithm_class_name"]]
        self.alg = alg_cls(actor_critic, device=self.device, **self.alg_cfg)
        self.num_steps_per_env = self.cfg["num_steps_per_env"]
        self.save_interval = self.cfg["save_interval"]
        # an env whose actor observations are a shifted frame history (T1DHStandEnv.obs_frame_history) lets the
        # storage keep frames instead of whole histories (rollout.py)
        self.alg.init_storage(env.num_envs, self.num_steps_per_env, [env.num_obs], [num_critic_obs], [env.num_actions],
                              history=getattr(env, "obs_frame_history", None))
        self.log_dir = log_dir if self.rank0 else None
        self.writer = None
        self.current_learning_iteration = 0
        self.tot_timesteps = 0
        self.tot_time = 0.0
        self.it = 0
        _, _ = self.env.reset()

    def learn(self, num_learning_iterations, init_at_random_ep_len=False):
        if self.log_dir is not None and self.writer is None:
            self.writer = _make_writer(self.log_dir)
        env, T, N = self.env, self.num_steps_per_env, self.env.num_envs
        if init_at_random_ep_len:
            env.episode_length_buf = torch.randint_like(env.episode_length_buf, high=int(env.max_episode_length))
        obs = env.get_observations()
        privileged_obs = env.get_privileged_observations()
        critic_obs = privileged_obs if privileged_obs is not None else obs
        obs, critic_obs = obs.to(self.device), critic_obs.to(self.device)
        self.alg.actor_critic.train()
        ep_infos = []
        rewbuffer, lenbuffer = deque(maxlen=100), deque(maxlen=100)
        cur_reward_sum = torch.zeros(N, dtype=torch.float, device=self.device)
        cur_episode_length = torch.zeros(N, dtype=torch.float, device=self.device)
        ended_rew = torch.zeros(T, N, device=self.device)
        ended_len = torch.zeros(T, N, device=self.device)
        ended = torch.zeros(T, N, dtype=torch.bool, device=self.device)
        tot_iter = self.current_learning_iteration + num_learning_iterations
        for it in range(self.current_learning_iteration, tot_iter):
            self.it = it
            start = time.time()
            with torch.inference_mode():
                for i in range(T):
                    actions = self.alg.act(obs, critic_obs)
                    obs, privileged_obs, rewards, dones, infos = env.step(actions)
                    critic_obs = privileged_obs if privileged_obs is not None else obs
                    obs, critic_obs, rewards, dones = (obs.to(self.device), critic_obs.to(self.device),
                                                       rewards.to(self.device), dones.to(self.device))
                    self.alg.process_env_step(rewards, dones, infos)
                    if self.log_dir is not None:
                        if "episode" in infos:
                            ep_infos.append(infos["episode"])
                        cur_reward_sum += rewards
                        cur_episode_length += 1
                        d = dones > 0
                        ended_rew[i] = cur_reward_sum
                        ended_len[i] = cur_episode_length
                        ended[i] = d
                        keep = (~d).float()
                        cur_reward_sum *= keep
                        cur_episode_length *= keep
                if self.log_dir is not None:  # completed episodes, step-major / env-ascending like the reference
                    idx = ended.nonzero(as_tuple=True)
                    rewbuffer.extend(ended_rew[idx].cpu().tolist())
                    lenbuffer.extend(ended_len[idx].cpu().tolist())
                stop = time.time()
                collection_time = stop - start
                start = stop
                self.alg.compute_returns(critic_obs)
            mean_value_loss, mean_surrogate_loss, mean_state_estimator_loss = self.alg.update()
            stop = time.time()
            learn_time = stop - start
            if self.log_dir is not None:
                self.log(locals())
                if it % self.save_interval == 0:
                    self.save(os.path.join(self.log_dir, "model_{}.pt".format(it)))
            ep_infos.clear()
        self.current_learning_iteration += num_learning_iterations
        if self.log_dir is not None:
            self.save(os.path.join(self.log_dir, "model_{}.pt".format(self.current_learning_iteration)))

    def log(self, locs, width=80, pad=35):
        self.tot_timesteps += self.num_steps_per_env * self.env.num_envs * dist_util.world()
        iteration_time = locs["collection_time"] + locs["learn_time"]
        self.tot_time += iteration_time
        ep_string = ""
        if locs["ep_infos"]:
            for key in locs["ep_infos"][0]:
                vals = []
                for info in locs["ep_infos"]:
                    v = info[key]
                    v = v if isinstance(v, torch.Tensor) else torch.tensor([float(v)])
                    vals.append(v.reshape(-1).float().to(self.device))
                value = torch.mean(torch.cat(vals))
                self.writer.add_scalar("Episode/" + key, value, locs["it"])
                ep_string += f"""{f'Mean episode {key}:':>{pad}} {value:.4f}\n"""
        mean_std = self.alg.actor_critic.std.mean()
        fps = int(self.num_steps_per_env * self.env.num_envs * dist_util.world() / iteration_time)
        w, it = self.writer, locs["it"]
        w.add_scalar("Loss/value_function", locs["mean_value_loss"], it)
        w.add_scalar("Loss/surrogate", locs["mean_surrogate_loss"], it)
        w.add_scalar("Loss/state_estimator", locs["mean_state_estimator_loss"], it)
        w.add_scalar("Loss/learning_rate", self.alg.learning_rate, it)
        w.add_scalar("Policy/mean_noise_std", mean_std.item(), it)
        w.add_scalar("Perf/total_fps", fps, it)
        w.add_scalar("Perf/collection time", locs["collection_time"], it)
        w.add_scalar("Perf/learning_time", locs["learn_time"], it)
        head = f" \033[1m Learning iteration {it}/{self.current_learning_iteration + locs['num_learning_iterations']} \033[0m "
        s = (f"""{'#' * width}\n{head.center(width, ' ')}\n\n"""
             f"""{'Computation:':>{pad}} {fps:.0f} steps/s (collection: {locs['collection_time']:.3f}s, """
             f"""learning {locs['learn_time']:.3f}s)\n"""
             f"""{'Value function loss:':>{pad}} {locs['mean_value_loss']:.4f}\n"""
             f"""{'Surrogate loss:':>{pad}} {locs['mean_surrogate_loss']:.4f}\n""")
        if len(locs["rewbuffer"]) > 0:
            mr, ml = statistics.mean(locs["rewbuffer"]), statistics.mean(locs["lenbuffer"])
            w.add_scalar("Train/mean_reward", mr, it)
            w.add_scalar("Train/mean_episode_length", ml, it)
            w.add_scalar("Train/mean_reward/time", mr, self.tot_time)
            w.add_scalar("Train/mean_episode_length/time", ml, self.tot_time)
            s += (f"""{'State estimator loss:':>{pad}} {locs['mean_state_estimator_loss']:.4f}\n"""
                  f"""{'Mean action noise std:':>{pad}} {mean_std.item():.2f}\n"""
                  f"""{'Mean reward:':>{pad}} {mr:.2f}\n"""
                  f"""{'Mean episode length:':>{pad}} {ml:.2f}\n""")
        else:
            s += f"""{'Mean action noise std:':>{pad}} {mean_std.item():.2f}\n"""
        s += ep_string
        eta = self.tot_time / (it + 1) * (locs["num_learning_iterations"] - it)
        s += (f"""{'-' * width}\n{'Total timesteps:':>{pad}} {self.tot_timesteps}\n"""
              f"""{'Iteration time:':>{pad}} {iteration_time:.2f}s\n{'Total time:':>{pad}} {self.tot_time:.2f}s\n"""
              f"""{'ETA:':>{pad}} {eta:.1f}s\n""")
        print(s)

    def save(self, path, infos=None):
        torch.save({"model_state_dict": self.alg.actor_critic.state_dict(),
                    "optimizer_state_dict": self.alg.optimizer.state_dict(),
                    "es_optimizer_state_dict": self.alg.state_estimator_optimizer.state_dict(),
                    "iter": self.it, "infos": infos}, path)

    def load(self, path, load_optimizer=True):
        d = torch.load(path, map_location=self.device, weights_only=True)
        self.alg.actor_critic.load_state_dict(d["model_state_dict"])
        if load_optimizer:
            self.alg.optimizer.load_state_dict(d["optimizer_state_dict"])
            self.alg.state_estimator_optimizer.load_state_dict(d["es_optimizer_state_dict"])
            self.alg.after_optimizer_load()  # capturable / fused flags and the device lr after a foreign state
        self.current_learning_iteration = d["iter"]
        return d["infos"]

    def get_inference_policy(self, device=None):
        self.alg.actor_critic.eval()
        if device is not None:
            self.alg.actor_critic.to(device)
        return self.alg.actor_critic.act_inference

    def get_inference_critic(self, device=None):
        self.alg.actor_critic.eval()
        if device is not None:
            self.alg.actor_critic.to(device)
        return self.alg.actor_critic.evaluate
