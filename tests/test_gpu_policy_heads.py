"""The fused policy heads (t1policy_heads_forward, ti5_isaacgym_amd/csrc/t1policy_heads.hip) against an fp64 forward of
the same ActorCriticDH (the reference's layers, actor_critic_dh.py:45-111,163-188, evaluated in torch fp64): action
mean, value, the sample mean + std eps, sigma and the sample's log-prob.  Needs the MI355X.

Tolerance: the kernel multiplies split fp16 operands (hi + lo / 2^11) on the matrix cores with fp32 accumulation,
~2^-22 of each product; torch's own fp32 forward is held to the same bound beside it, so the test also shows the
fused kernel is as close to fp64 as the fp32 layers it replaces."""
import pytest
import torch

pytestmark = pytest.mark.gpu
TOL = dict(rtol=2e-5, atol=2e-5)


def _model(seed=0, scale=1.0):
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    torch.manual_seed(seed)
    ac = ActorCriticDH(235, 47, 219, 12, **class_to_dict(tc)["policy"])
    with torch.no_grad():
        for p in ac.parameters():   # trained-policy-like magnitudes on top of the default init
            p.mul_(scale)
        ac.std.copy_(torch.linspace(0.2, 1.3, 12))
    return ac


def _ref64(ac, obs, cobs, eps):
    from torch.distributions import Normal
    a64 = _copy(ac).double()
    with torch.no_grad():
        o, c, e = obs.double(), cobs.double(), eps.double()
        mean = a64.actor(a64.actor_input(o))
        value = a64.critic(c)
        std = a64.std.expand_as(mean)
        act = mean + std * e
        logp = Normal(mean, std).log_prob(act).sum(-1)
    return mean, act, std, logp, value


def _copy(ac):
    import copy
    m = copy.deepcopy(ac).cpu()
    return m


# 3000: the batch of round 5's reverted side-stream split, whose first test faulted -- the shipped
# one-launch kernel at that ragged batch (93 full 32-env workgroups and a 24-env tail)
@pytest.mark.parametrize("n,scale", [(1000, 1.0), (4096, 1.5), (33, 1.0), (3000, 1.0)])
def test_fused_heads_match_fp64(n, scale):
    from ti5_isaacgym_amd.algo.dh_policy import heads_forward
    ac = _model(scale=scale)
    dev = torch.device("cuda:0")
    acd = _copy(ac).to(dev)
    g = torch.Generator().manual_seed(n)
    obs = (torch.randn(n, 66 * 47, generator=g) * 2.0).clamp(-18, 18)
    cobs = torch.randn(n, 219, generator=g) * 2.0
    eps = torch.randn(n, 12, generator=g)
    with torch.inference_mode():
        out = heads_forward(acd, obs.to(dev), cobs.to(dev), eps.to(dev))
        assert out is not None, "the fused heads have no instance for the t1 policy"
        mean, act, sigma, logp, value = [t.cpu().double() for t in out]
        # torch's own fp32 layers on the device, for the same bound
        m32 = acd.actor(acd.actor_input(obs.to(dev))).cpu().double()
        v32 = acd.critic(cobs.to(dev)).cpu().double()
    rm, ra, rs, rl, rv = _ref64(ac, obs, cobs, eps)
    torch.testing.assert_close(m32, rm, **TOL)
    torch.testing.assert_close(v32, rv, **TOL)
    torch.testing.assert_close(mean, rm, **TOL)
    torch.testing.assert_close(value, rv, **TOL)
    torch.testing.assert_close(act, ra, **TOL)
    torch.testing.assert_close(sigma, rs, rtol=0, atol=0)
    torch.testing.assert_close(logp, rl, rtol=2e-5, atol=1e-4)
    # the error budget in ulps of fp32: the fused kernel within 4x of torch's fp32 layers (+ 1e-6)
    assert (mean - rm).abs().max() <= 4 * (m32 - rm).abs().max() + 1e-6
    assert (value - rv).abs().max() <= 4 * (v32 - rv).abs().max() + 1e-6


@pytest.mark.parametrize("n", [3000, 8192, 33])
def test_heads64_equals_heads32(n, monkeypatch):
    """k_heads64 (64 envs per workgroup, the 512- / 768-wide layers in halves / thirds feeding the next layer's
    accumulators) against the 32-env k_heads (T1POLICY_HEADS64=0): the same fragments, the same k order into the same
    fp32 accumulators per env column, so every output is bit-identical."""
    from ti5_isaacgym_amd.algo.dh_policy import heads_forward
    ac = _model(scale=1.5)
    dev = torch.device("cuda:0")
    acd = _copy(ac).to(dev)
    g = torch.Generator().manual_seed(n + 1)
    obs = ((torch.randn(n, 66 * 47, generator=g) * 2.0).clamp(-18, 18)).to(dev)
    cobs = (torch.randn(n, 219, generator=g) * 2.0).to(dev)
    eps = torch.randn(n, 12, generator=g).to(dev)
    with torch.inference_mode():
        monkeypatch.setenv("T1POLICY_HEADS64", "1")
        o64 = [t.clone() for t in heads_forward(acd, obs, cobs, eps)]
        monkeypatch.setenv("T1POLICY_HEADS64", "0")
        o32 = [t.clone() for t in heads_forward(acd, obs, cobs, eps)]
    for name, a, b in zip(("mean", "actions", "sigma", "logp", "value"), o64, o32):
        assert torch.equal(a, b), (name, (a - b).abs().max().item())


def test_fused_heads_propagate_nan_like_torch():
    """A NaN in one env's inputs reaches that env's outputs as NaN (torch's ELU keeps NaN; the kernel's expm1 for ELU's
    negative branch must not clamp it to -1), and no other env is touched."""
    from ti5_isaacgym_amd.algo.dh_policy import heads_forward
    ac = _model()
    dev = torch.device("cuda:0")
    acd = _copy(ac).to(dev)
    n = 96
    g = torch.Generator().manual_seed(7)
    obs = (torch.randn(n, 66 * 47, generator=g) * 2.0).clamp(-18, 18)
    cobs = torch.randn(n, 219, generator=g) * 2.0
    eps = torch.randn(n, 12, generator=g)
    obs[5, -3] = float("nan")     # the short history: the estimator and the actor
    cobs[40, 7] = float("nan")    # the critic
    with torch.inference_mode():
        mean, act, sigma, logp, value = [t.cpu() for t in heads_forward(acd, obs.to(dev), cobs.to(dev), eps.to(dev))]
        m32 = acd.actor(acd.actor_input(obs.to(dev))).cpu()
        v32 = acd.critic(cobs.to(dev)).cpu()
    assert torch.isnan(m32[5]).all() and torch.isnan(v32[40]).all()   # torch's own layers
    assert torch.isnan(mean[5]).all() and torch.isnan(logp[5])
    assert torch.isnan(value[40]).all()
    keep = torch.ones(n, dtype=torch.bool)
    keep[5] = False
    assert torch.isfinite(mean[keep]).all() and torch.isfinite(logp[keep]).all()
    keep = torch.ones(n, dtype=torch.bool)
    keep[40] = False
    assert torch.isfinite(value[keep]).all()


def test_fused_heads_follow_weight_updates():
    """heads_forward repacks the weights when a parameter changed: an in-place parameter change shows up in the next
    call."""
    from ti5_isaacgym_amd.algo.dh_policy import heads_forward
    dev = torch.device("cuda:0")
    ac = _model(seed=3).to(dev)
    obs = torch.randn(256, 66 * 47, device=dev)
    cobs = torch.randn(256, 219, device=dev)
    eps = torch.zeros(256, 12, device=dev)
    with torch.inference_mode():
        m0 = heads_forward(ac, obs, cobs, eps)[0].clone()
        with torch.no_grad():
            for p in ac.actor.parameters():
                p.add_(0.01)
        m1 = heads_forward(ac, obs, cobs, eps)[0]
        ref = ac.actor(ac.actor_input(obs))
    assert not torch.allclose(m0, m1)
    torch.testing.assert_close(m1, ref, **TOL)


def test_fused_heads_refuse_other_shapes():
    """A policy the kernel has no instance for (other hidden sizes) returns None: the caller keeps torch's layers."""
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH, heads_forward
    dev = torch.device("cuda:0")
    ac = ActorCriticDH(235, 47, 219, 12, actor_hidden_dims=[256, 256, 128], critic_hidden_dims=[768, 256, 128],
                       state_estimator_hidden_dims=[256, 128, 64], kernel_size=[6, 4], filter_size=[32, 16],
                       stride_size=[3, 2], lh_output_dim=64).to(dev)
    obs = torch.randn(64, 66 * 47, device=dev)
    with torch.inference_mode():
        assert heads_forward(ac, obs, torch.randn(64, 219, device=dev), torch.zeros(64, 12, device=dev)) is None


def test_fused_heads_pack_only_when_weights_move(monkeypatch):
    """the heads' weight fragments are packed once and reused while no parameter moved; an in-place
    change repacks on the next call, and refresh_packed_weights(force=True) (after a graphed update) repacks."""
    from ti5_isaacgym_amd import _lib
    from ti5_isaacgym_amd.algo.dh_policy import heads_forward, refresh_packed_weights
    dev = torch.device("cuda:0")
    ac = _model(seed=4).to(dev)
    obs = torch.randn(128, 66 * 47, device=dev)
    cobs = torch.randn(128, 219, device=dev)
    eps = torch.zeros(128, 12, device=dev)
    lib = _lib.load()
    real = lib.t1policy_heads_pack
    calls = []
    monkeypatch.setattr(lib, "t1policy_heads_pack", lambda *a: (calls.append(1), real(*a))[1])
    with torch.inference_mode():
        m0 = heads_forward(ac, obs, cobs, eps)[0].clone()
        assert len(calls) == 1
        m1 = heads_forward(ac, obs, cobs, eps)[0].clone()
        assert len(calls) == 1 and torch.equal(m0, m1)
        with torch.no_grad():
            ac.critic[0].bias.add_(0.5)
        heads_forward(ac, obs, cobs, eps)
        assert len(calls) == 2
        refresh_packed_weights(ac)
        assert len(calls) == 2
        refresh_packed_weights(ac, force=True)
        assert len(calls) == 3
