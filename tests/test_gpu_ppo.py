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
    # the rollout's act() ran as replayed HIP graphs, one per env observation buffer pair
    assert runner.alg.graph_act and 1 <= len(runner.alg._act_graphs) <= 2


def test_graphed_act_matches_eager():
    """The graphed act() (DHPPO._graphed_act) against the eager ActorCriticDH calls on the same buffers:
    mean, std, value exactly (same kernels), the log-prob of the sampled actions exactly, samples distinct
    across replays, and the graph follows in-place weight updates."""
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH
    from ti5_isaacgym_amd.algo.dh_update import DHPPO
    from torch.distributions import Normal
    env_cfg, train_cfg = task_registry.get_cfgs("t1_dh_stand")
    pc = train_cfg.policy
    torch.manual_seed(0)
    ac = ActorCriticDH(235, 47, 219, 12, actor_hidden_dims=pc.actor_hidden_dims, critic_hidden_dims=pc.critic_hidden_dims,
                       state_estimator_hidden_dims=pc.state_estimator_hidden_dims, in_channels=66, kernel_size=pc.kernel_size,
                       filter_size=pc.filter_size, stride_size=pc.stride_size, lh_output_dim=pc.lh_output_dim,
                       init_noise_std=pc.init_noise_std)
    alg = DHPPO(ac, device="cuda:0")
    n = 1024
    obs = torch.randn(n, 66 * 47, device="cuda:0")
    cobs = torch.randn(n, 219, device="cuda:0")
    # the graphed act() runs the fused HIP heads (split-fp16 matrix cores, fp32-class: tests/test_gpu_policy_heads.py)
    # against torch's fp32 layers here; FUSED_ACT=0 would run the same torch kernels
    tol = dict(rtol=1e-5, atol=1e-5)
    with torch.inference_mode():
        a1, v1, lp1, m1, s1 = [t.clone() for t in alg._graphed_act(obs, cobs)]
        a2 = alg._graphed_act(obs, cobs)[0].clone()
        mean = ac.actor(ac.actor_input(obs))
        torch.testing.assert_close(m1, mean, **tol)
        torch.testing.assert_close(s1, (mean * 0.0 + ac.std).expand_as(s1), **tol)
        torch.testing.assert_close(v1, ac.critic(cobs), **tol)
        lp = Normal(m1, s1, validate_args=False).log_prob(a1).sum(-1)
        torch.testing.assert_close(lp1, lp, rtol=1e-6, atol=1e-5)
        assert not torch.equal(a1, a2)
    with torch.no_grad():
        for p in ac.parameters():   # in-place update (what the optimizer step does)
            p.add_(0.01)
    with torch.inference_mode():
        m3 = alg._graphed_act(obs, cobs)[3]
        torch.testing.assert_close(m3, ac.actor(ac.actor_input(obs)), **tol)
    assert len(alg._act_graphs) == 1


def test_bf16_update_tracks_fp32():
    """The opt-in bf16 update (DHPPO.amp_dtype) against the fp32 update from the same weights, optimizer state,
    rollout and minibatch permutation (tools/ppo_amp_check.py): the three mean losses within 5 % (+1e-4) and the
    weight updates within 5 % relative L2 (measured 0.8-1.0 % at 8192 envs, profiles/r02ap_ppo_bf16.md)."""
    import importlib.util
    import os
    from ti5_isaacgym_amd import make_t1_env, task_registry
    from ti5_isaacgym_amd.algo import DHOnPolicyRunner
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "ppo_amp_check.py")
    spec = importlib.util.spec_from_file_location("ppo_amp_check", path)
    chk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(chk)
    env = make_t1_env(num_envs=1024, mesh_type="plane", seed=5, device="cuda:0")
    _, train_cfg = task_registry.get_cfgs("t1_dh_stand")
    torch.manual_seed(0)
    r = DHOnPolicyRunner(env, class_to_dict(train_cfg), None, device="cuda:0")
    r.alg.actor_critic.train()
    obs, priv = env.reset()
    critic = priv if priv is not None else obs
    for it in range(2):
        obs, critic = chk.rollout(r, obs, critic)
        ls32, ls16, rel, _, _ = chk.compare_updates(r, 1000 + it)
        for a, b in zip(ls16, ls32):
            assert abs(a - b) <= 0.05 * abs(b) + 1e-4, (ls16, ls32)
        assert rel < 0.05, rel
    assert r.alg.amp_dtype is None   # compare_updates leaves the fp32 update in place


def test_bf16_update_obs_cast_once_is_exact():
    """The bf16 update's actor observations cast to bf16 once per update (RolloutStorage.mini_batch_generator
    obs_dtype) against autocast's per-minibatch casts: the same bf16 operands reach the same GEMMs, so the losses and
    weights agree to the bit (a GEMM library picking another solution for the other layout would show here)."""
    import importlib.util
    import os
    from ti5_isaacgym_amd import make_t1_env, task_registry
    from ti5_isaacgym_amd.algo import DHOnPolicyRunner
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "ppo_amp_check.py")
    spec = importlib.util.spec_from_file_location("ppo_amp_check", path)
    chk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(chk)
    env = make_t1_env(num_envs=1024, mesh_type="plane", seed=5, device="cuda:0")
    _, train_cfg = task_registry.get_cfgs("t1_dh_stand")
    torch.manual_seed(0)
    r = DHOnPolicyRunner(env, class_to_dict(train_cfg), None, device="cuda:0")
    r.alg.actor_critic.train()
    obs, priv = env.reset()
    critic = priv if priv is not None else obs
    obs, critic = chk.rollout(r, obs, critic)
    ls_off, ls_on, diff, _, _ = chk.compare_cast_once(r, 77)
    assert list(ls_off) == list(ls_on), (ls_off, ls_on)
    assert diff == 0.0, diff


@pytest.mark.parametrize("amp", [None, torch.bfloat16], ids=["fp32", "bf16"])
def test_graphed_update_matches_eager(amp):
    """DHPPO.update with its minibatch step replayed as a captured HIP graph (the default on the device) against the
    eager step: the same storage, permutation and initial weights, three updates with the adaptive learning rate --
    weights, Adam state, learning rate and losses bit-identical (the same kernels run), and the graph is captured
    once and follows the storage's in-place refills."""
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH
    from ti5_isaacgym_amd.algo.dh_update import DHPPO
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    cfg = class_to_dict(tc)
    N, T, dev = 1024, 24, torch.device("cuda:0")
    algs = []
    for graphed in (False, True):
        torch.manual_seed(0)
        ac = ActorCriticDH(235, 47, 219, 12, **cfg["policy"]).to(dev)
        alg = DHPPO(ac, device=str(dev), amp_dtype=amp, **cfg["algorithm"])
        alg.graph_update = graphed
        alg.init_storage(N, T, [3102], [219], [12], history=(47, 66))
        algs.append(alg)
    assert algs[0].schedule == "adaptive"
    g = torch.Generator(device=dev)
    lrs = []
    for it in range(3):
        losses = []
        for alg in algs:
            st = alg.storage
            g.manual_seed(10 + it)
            for t in (st.obs0, st.frames, st.privileged_observations, st.actions, st.values, st.returns,
                      st.actions_log_prob, st.mu):
                t.normal_(generator=g)
            st.sigma.uniform_(0.5, 1.5, generator=g)
            st.dones.copy_((torch.rand(st.dones.shape, generator=g, device=dev) < 0.05).to(torch.uint8))
            st.rewards.normal_(generator=g)
            st.step = T
            alg.compute_returns(torch.randn(N, 219, device=dev, generator=g))
            alg.actor_critic.train()
            torch.manual_seed(100 + it)
            losses.append(alg.update())
        assert losses[0] == losses[1], (it, losses)
        lrs.append((algs[0].learning_rate, algs[1].learning_rate))
        assert lrs[-1][0] == lrs[-1][1]
        for p0, p1 in zip(algs[0].actor_critic.parameters(), algs[1].actor_critic.parameters()):
            assert torch.equal(p0, p1)
        for s0, s1 in zip(algs[0].optimizer.state.values(), algs[1].optimizer.state.values()):
            assert all(torch.equal(s0[k], s1[k]) for k in ("exp_avg", "exp_avg_sq", "step"))
    assert algs[1]._upd is not None and algs[0]._upd is None
    print("learning rates", lrs)


def test_graphed_update_follows_optimizer_reload():
    """The same update twice from one snapshot (weights, optimizer.load_state_dict of the saved state, storage, seed),
    as tools/ppo_amp_check.py and a checkpoint resume do: the loaded Adam state replaces the tensors a captured graph
    held, so the graph is recaptured and both runs give the same losses and weights."""
    import copy
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH
    from ti5_isaacgym_amd.algo.dh_update import DHPPO
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    cfg = class_to_dict(tc)
    N, T, dev = 512, 24, torch.device("cuda:0")
    torch.manual_seed(0)
    ac = ActorCriticDH(235, 47, 219, 12, **cfg["policy"]).to(dev)
    alg = DHPPO(ac, device=str(dev), **cfg["algorithm"])
    alg.init_storage(N, T, [3102], [219], [12], history=(47, 66))
    st = alg.storage
    g = torch.Generator(device=dev).manual_seed(3)
    for t in (st.obs0, st.frames, st.privileged_observations, st.actions, st.values, st.returns, st.actions_log_prob,
              st.mu, st.rewards):
        t.normal_(generator=g)
    st.sigma.uniform_(0.5, 1.5, generator=g)
    alg.compute_returns(torch.randn(N, 219, device=dev, generator=g))
    for first in (True, False):   # the second snapshot has Adam state (the first has none yet)
        snap = {k: v.clone() for k, v in vars(st).items() if torch.is_tensor(v)}
        w0 = [p.detach().clone() for p in ac.parameters()]
        opt0 = copy.deepcopy(alg.optimizer.state_dict())
        lr0 = alg.learning_rate
        runs = []
        for rep in range(3):
            with torch.no_grad():
                for p, p0 in zip(ac.parameters(), w0):
                    p.copy_(p0)
            # a copy: load_state_dict adopts device tensors as they are, and the update then changes them in place
            alg.optimizer.load_state_dict(copy.deepcopy(opt0))
            alg.learning_rate = lr0
            for k, v in snap.items():
                getattr(st, k).copy_(v)
            st.step = T
            torch.manual_seed(9)
            runs.append((alg.update(), [p.detach().clone() for p in ac.parameters()]))
        for ls, w in runs[1:]:
            assert ls == runs[0][0], (first, [r[0] for r in runs])
            assert all(torch.equal(a, b) for a, b in zip(w, runs[0][1]))


def _fill_storage(alg, N, T, dev, seed):
    st = alg.storage
    g = torch.Generator(device=dev).manual_seed(seed)
    for t in (st.obs0, st.frames, st.privileged_observations, st.actions, st.values, st.returns, st.actions_log_prob,
              st.mu, st.rewards):
        t.normal_(generator=g)
    st.sigma.uniform_(0.5, 1.5, generator=g)
    st.step = T
    alg.compute_returns(torch.randn(N, 219, device=dev, generator=g))


def test_graphed_act_follows_graphed_updates():
    """the graphed update's Adam steps are graph replays, which do not bump the weights' version
    counter, so a conv-fragment cache keyed on it went stale from the second update on.  After three graphed updates
    the graphed act() mean must equal the autograd path's (conv as an unfolded GEMM, no packed fragments)."""
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH
    from ti5_isaacgym_amd.algo.dh_update import DHPPO
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    cfg = class_to_dict(tc)
    N, T, dev = 512, 24, torch.device("cuda:0")
    torch.manual_seed(0)
    ac = ActorCriticDH(235, 47, 219, 12, **cfg["policy"]).to(dev)
    alg = DHPPO(ac, device=str(dev), **cfg["algorithm"])
    assert alg.graph_update and alg.graph_act
    alg.init_storage(N, T, [3102], [219], [12], history=(47, 66))
    obs = torch.randn(N, 66 * 47, device=dev)
    cobs = torch.randn(N, 219, device=dev)
    for it in range(3):
        with torch.inference_mode():
            alg._graphed_act(obs, cobs)
        _fill_storage(alg, N, T, dev, 20 + it)
        ac.train()
        alg.update()
    assert alg._upd is not None  # the minibatch steps were replays
    with torch.inference_mode():
        m = alg._graphed_act(obs, cobs)[3].clone()
    with torch.enable_grad():
        ref = ac.actor(ac.actor_input(obs)).detach()
    torch.testing.assert_close(m, ref, rtol=1e-5, atol=2e-5)


def test_update_after_loading_plain_adam_state():
    """a checkpoint's optimizer state written by a plain (non-capturable) torch Adam -- the
    reference's, or an older build's -- replaces the param groups' flags on load; after_optimizer_load restores the
    capturable fused Adam with the device learning rate, so the next update runs.  The learning rate follows the
    reference's runner.load: DHPPO.learning_rate keeps this process's value; under the adaptive schedule Adam
    continues from it, under the fixed schedule Adam keeps the checkpoint's lr (the reference never writes it)."""
    from torch import optim
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH
    from ti5_isaacgym_amd.algo.dh_update import DHPPO
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    cfg = class_to_dict(tc)
    N, T, dev = 256, 24, torch.device("cuda:0")
    torch.manual_seed(0)
    ac = ActorCriticDH(235, 47, 219, 12, **cfg["policy"]).to(dev)
    plain = optim.Adam(ac.parameters(), lr=3e-4)
    for p in ac.parameters():
        p.grad = torch.zeros_like(p)
    plain.step()
    sd = plain.state_dict()
    assert sd["param_groups"][0]["capturable"] is False
    alg = DHPPO(ac, device=str(dev), **cfg["algorithm"])
    lr0 = float(cfg["algorithm"]["learning_rate"])
    assert alg.schedule == "adaptive" and abs(lr0 - 3e-4) > 1e-6
    alg.init_storage(N, T, [3102], [219], [12], history=(47, 66))
    alg.optimizer.load_state_dict(sd)
    alg.after_optimizer_load()
    assert abs(alg.learning_rate - lr0) < 1e-12 and abs(float(alg._lr_t) - lr0) < 1e-9  # not the checkpoint's 3e-4
    fixed = DHPPO(ActorCriticDH(235, 47, 219, 12, **cfg["policy"]).to(dev), device=str(dev),
                  **dict(cfg["algorithm"], schedule="fixed"))
    fixed.optimizer.load_state_dict(sd)
    fixed.after_optimizer_load()
    assert abs(fixed.learning_rate - lr0) < 1e-12 and abs(float(fixed._lr_t) - 3e-4) < 1e-10
    assert fixed.optimizer.param_groups[0]["lr"] is fixed._lr_t
    _fill_storage(alg, N, T, dev, 5)
    ac.train()
    losses = alg.update()
    assert all(map(lambda x: x == x, losses))
    g = alg.optimizer.param_groups[0]
    assert g["capturable"] and g["fused"] and g["lr"] is alg._lr_t
    alg.learning_rate = 1e-4   # an assignment after the load wins
    _fill_storage(alg, N, T, dev, 6)
    alg.schedule = "fixed"
    alg.update()
    assert abs(alg.learning_rate - 1e-4) < 1e-10


def test_device_lr_schedule_matches_python_floats():
    """the adaptive schedule on the device steps the learning rate in fp64 like the reference's Python
    float (dh_ppo.py:120-135), so 40 down / up steps land on exactly the reference's value; Adam reads its fp32 copy."""
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH
    from ti5_isaacgym_amd.algo.dh_update import DHPPO
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    cfg = class_to_dict(tc)
    dev = torch.device("cuda:0")
    ac = ActorCriticDH(235, 47, 219, 12, **cfg["policy"]).to(dev)
    alg = DHPPO(ac, device=str(dev), **cfg["algorithm"])
    ref = alg.learning_rate
    mu = torch.zeros(8, 12, device=dev)
    sig = torch.ones(8, 12, device=dev)
    g = torch.Generator().manual_seed(3)
    for _ in range(40):
        big = bool(torch.rand(1, generator=g) < 0.5)
        old_mu = mu + (0.5 if big else 1e-4)   # KL far above 2 x desired, or far below half of it
        kl = float(torch.sum((torch.square(old_mu - mu)) / 2.0, -1).mean())
        if kl > alg.desired_kl * 2.0:
            ref = max(1e-5, ref / 1.5)
        elif 0.0 < kl < alg.desired_kl / 2.0:
            ref = min(1e-2, ref * 1.5)
        alg._adapt_lr(mu, sig, old_mu, sig)
        assert alg.learning_rate == ref
    assert float(alg._lr_t) == torch.tensor(ref, dtype=torch.float32).item()
    assert alg.optimizer.param_groups[0]["lr"] is alg._lr_t


def test_update_capture_failure_runs_eagerly(monkeypatch):
    """a failed capture of the minibatch step (here forced) warns, switches the update to eager for the rest
    of that update and after it, and gives the eager update's bits; a failed GAE capture falls back the same way."""
    import warnings
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH
    from ti5_isaacgym_amd.algo.dh_update import DHPPO
    from ti5_isaacgym_amd.algo.rollout import RolloutStorage
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    cfg = class_to_dict(tc)
    N, T, dev = 512, 24, torch.device("cuda:0")
    algs = []
    for graphed in (False, True):
        torch.manual_seed(0)
        ac = ActorCriticDH(235, 47, 219, 12, **cfg["policy"]).to(dev)
        alg = DHPPO(ac, device=str(dev), **cfg["algorithm"])
        alg.graph_update = graphed
        alg.init_storage(N, T, [3102], [219], [12], history=(47, 66))
        algs.append(alg)
    monkeypatch.setattr(DHPPO, "_try_capture", staticmethod(lambda graph, body: RuntimeError("forced")))
    real_graph = torch.cuda.graph

    def failing_graph(*a, **k):   # the GAE capture fails too
        raise RuntimeError("forced GAE capture failure")
    for it in range(2):
        out = []
        for alg in algs:
            monkeypatch.setattr(torch.cuda, "graph", failing_graph if alg is algs[1] else real_graph)
            with warnings.catch_warnings(record=True) as w:
                warnings.simplefilter("always")
                _fill_storage(alg, N, T, dev, 20 + it)
                torch.manual_seed(50 + it)
                out.append(alg.update())
            if alg is algs[1] and it == 0:
                msgs = " ".join(str(x.message) for x in w)
                assert "capture failed" in msgs, msgs
            monkeypatch.setattr(torch.cuda, "graph", real_graph)
        assert out[0] == out[1], (it, out)
        for p0, p1 in zip(algs[0].actor_critic.parameters(), algs[1].actor_critic.parameters()):
            assert torch.equal(p0, p1)
    assert algs[1].graph_update is False and algs[1]._upd is None
    assert algs[1].storage.graph_gae is False
    assert isinstance(algs[1].storage, RolloutStorage)
