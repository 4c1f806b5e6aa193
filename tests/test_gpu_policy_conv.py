"""The HIP direct conv of the policy's history encoder (include/t1policy.h) against torch's Conv1d, fp32."""
import pytest
import torch
import torch.nn as nn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("batch", [1, 777, 8192])
def test_conv1d_direct_matches_torch(batch):
    from ti5_isaacgym_amd.algo.dh_policy import conv1d_direct
    torch.manual_seed(batch)
    conv = nn.Conv1d(66, 32, kernel_size=6, stride=3).to("cuda:0")
    x = torch.randn(batch, 66, 47, device="cuda:0")
    with torch.no_grad():
        ref = nn.functional.conv1d(x.double(), conv.weight.double(), conv.bias.double(), stride=3)  # (B, O, Lout)
        y = conv1d_direct(x, conv)
    torch.cuda.synchronize()
    assert y.shape == (batch, 14, 32)
    # fp32 sum of 396 products against fp64: |err| <= 1e-5 * (1 + |ref|)
    err = (y.double() - ref.transpose(1, 2)).abs()
    assert float((err / (1 + ref.transpose(1, 2).abs())).max()) < 1e-5


@pytest.mark.parametrize("batch", [1, 2, 777, 8192])
def test_packed_and_tap_major_entries_match_torch(batch):
    """Both C-ABI forms: the packed-fragment kernel (one wave per SIMD, fragments in registers; odd samples start 8 B
    past a 16-byte boundary) and the tap-major one (the fallback for unaligned inputs)."""
    from ti5_isaacgym_amd import _lib
    lib = _lib.load()
    torch.manual_seed(100 + batch)
    conv = nn.Conv1d(66, 32, kernel_size=6, stride=3).to("cuda:0")
    x = torch.randn(batch, 66, 47, device="cuda:0")
    w = conv.weight.detach().contiguous()
    b = conv.bias.detach().contiguous()
    sp = torch.cuda.current_stream().cuda_stream
    frag = torch.empty(lib.t1policy_conv1d_frag_bytes(), device="cuda:0", dtype=torch.uint8)
    y1 = torch.full((batch, 14, 32), float("nan"), device="cuda:0")
    y2 = torch.full((batch, 14, 32), float("nan"), device="cuda:0")
    assert lib.t1policy_conv1d_pack_weights(w.data_ptr(), frag.data_ptr(), 66, 32, 6, sp) == 0
    assert lib.t1policy_conv1d_forward_packed(x.data_ptr(), frag.data_ptr(), b.data_ptr(), y1.data_ptr(), batch, 66, 47,
                                              32, 6, 3, sp) == 0
    wt = w.permute(1, 2, 0).contiguous()
    assert lib.t1policy_conv1d_forward(x.data_ptr(), wt.data_ptr(), b.data_ptr(), y2.data_ptr(), batch, 66, 47, 32, 6,
                                       3, sp) == 0
    # unsupported shapes and misaligned inputs are refused, not computed
    assert lib.t1policy_conv1d_forward_packed(x.data_ptr() + 4, frag.data_ptr(), b.data_ptr(), y1.data_ptr(), batch,
                                              66, 47, 32, 6, 3, sp) == -1
    assert lib.t1policy_conv1d_forward_packed(x.data_ptr(), frag.data_ptr(), b.data_ptr(), y1.data_ptr(), batch, 66,
                                              47, 32, 5, 3, sp) == 1
    torch.cuda.synchronize()
    with torch.no_grad():
        ref = nn.functional.conv1d(x.double(), w.double(), b.double(), stride=3).transpose(1, 2)
    for y in (y1, y2):
        assert bool(torch.isfinite(y).all())
        assert float(((y.double() - ref).abs() / (1 + ref.abs())).max()) < 1e-5


def test_history_encoder_inference_uses_direct_conv_and_matches():
    """ActorCriticDH.actor_input without autograd (the rollout's act) runs the direct conv; its output equals the
    autograd path's (unfold + GEMM) within fp32 summation-order tolerance."""
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.algo import dh_policy
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH
    _, train_cfg = task_registry.get_cfgs("t1_dh_stand")
    pc = train_cfg.policy
    torch.manual_seed(0)
    ac = ActorCriticDH(235, 47, 219, 12, actor_hidden_dims=pc.actor_hidden_dims, critic_hidden_dims=pc.critic_hidden_dims,
                       state_estimator_hidden_dims=pc.state_estimator_hidden_dims, in_channels=66, kernel_size=pc.kernel_size,
                       filter_size=pc.filter_size, stride_size=pc.stride_size, lh_output_dim=pc.lh_output_dim,
                       init_noise_std=pc.init_noise_std).to("cuda:0")
    obs = torch.randn(4096, 66 * 47, device="cuda:0")
    calls = []
    orig = dh_policy.conv1d_direct
    dh_policy.conv1d_direct = lambda x, m: calls.append(1) or orig(x, m)
    try:
        with torch.inference_mode():
            a = ac.actor_input(obs)
        b = ac.actor_input(obs).detach()   # grad enabled: unfold + GEMM
    finally:
        dh_policy.conv1d_direct = orig
    assert calls == [1]
    torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
