"""The device path of the long-history CNN (algo/dh_policy.py HistoryEncoder: Conv1d as unfold + GEMM, channels-last
activations) vs the reference layer stack run as plain nn.Sequential (nn.Conv1d), forward and backward, in fp64 on
the host so only the formulation is compared (the device's fp32 summation order is bounded by test_ppo_golden.py)."""
import torch
import torch.nn as nn

from ti5_isaacgym_amd.algo.dh_policy import _history_encoder, conv1d_as_gemm


def device_path(enc, x):
    last = False
    for m in enc:
        if isinstance(m, nn.Conv1d):
            x = conv1d_as_gemm(x, m, channels_last=last)
            last = True
        elif isinstance(m, nn.Flatten) and last:
            x = x.transpose(1, 2).reshape(x.shape[0], -1)
            last = False
        else:
            x = m(x)
    return x


def test_conv_gemm_equals_conv1d_forward_and_backward():
    torch.manual_seed(0)
    enc = _history_encoder(66, 47, [32, 16], [6, 4], [3, 2], 64).double()
    x = torch.randn(37, 66, 47, dtype=torch.float64, requires_grad=True)
    ref = nn.Sequential(*enc)(x)
    gy = torch.randn_like(ref)
    gref = torch.autograd.grad(ref, [x, *enc.parameters()], gy)
    out = device_path(enc, x)
    gout = torch.autograd.grad(out, [x, *enc.parameters()], gy)
    assert out.shape == ref.shape == (37, 64)
    torch.testing.assert_close(out, ref, rtol=1e-12, atol=1e-12)
    for a, b in zip(gout, gref):
        torch.testing.assert_close(a, b, rtol=1e-11, atol=1e-11)


def test_state_dict_keys_unchanged():
    enc = _history_encoder(66, 47, [32, 16], [6, 4], [3, 2], 64)
    assert list(enc.state_dict()) == list(nn.Sequential(*enc).state_dict())


def test_splitk_linear_gradients():
    """The split-K weight gradient (dh_policy.wgrad_splitk / _LinearSplitK) == autograd of addmm, incl. a ragged K."""
    from ti5_isaacgym_amd.algo import dh_policy as P
    torch.manual_seed(1)
    for K in (5 * P.SPLITK_ROWS + 37, 3 * P.SPLITK_ROWS, 100):
        x = torch.randn(K, 19, dtype=torch.float64, requires_grad=True)
        w = torch.randn(7, 19, dtype=torch.float64, requires_grad=True)
        b = torch.randn(7, dtype=torch.float64, requires_grad=True)
        gy = torch.randn(K, 7, dtype=torch.float64)
        ref = torch.autograd.grad(torch.addmm(b, x, w.t()), [x, w, b], gy)
        got = torch.autograd.grad(P._LinearSplitK.apply(x, w, b), [x, w, b], gy)
        for a, r in zip(got, ref):
            torch.testing.assert_close(a, r, rtol=1e-11, atol=1e-10)
