"""The update's first history conv under the bf16 update as HIP kernels (t1policy_conv1_*_bf16,
ti5_isaacgym_amd/csrc/t1policy_train.hip) against fp64 torch on the same bf16 operands -- needs the MI355X.

forward: y = bf16(sum of the bf16 products + bf16(bias)) -- autocast's addmm arithmetic -- within one bf16 rounding of
the fp64 value; weight / bias gradients: fp32 sums over every (sample, position) within 1e-3 relative of fp64, the
same bits on a second run (the partials are summed in a fixed order, which the graphed == eager update relies on)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _conv():
    torch.manual_seed(0)
    return torch.nn.Conv1d(66, 32, kernel_size=6, stride=3).to(DEV)


def _ref_forward(x, conv):
    w = conv.weight.detach().to(torch.bfloat16).double()
    b = conv.bias.detach().to(torch.bfloat16).double()
    return torch.nn.functional.conv1d(x.double(), w, b, stride=3).transpose(1, 2)  # (B, 14, 32)


@pytest.mark.parametrize("n", [1, 777, 8192])
def test_conv1_bf16_forward_matches_fp64(n):
    from ti5_isaacgym_amd.algo.dh_policy import conv1d_train_bf16
    conv = _conv()
    g = torch.Generator(device=DEV).manual_seed(n)
    x = (torch.randn(n, 66, 47, device=DEV, generator=g) * 2.0).to(torch.bfloat16)
    with torch.no_grad():
        y = conv1d_train_bf16(x, conv)
    assert y is not None and y.dtype == torch.bfloat16 and y.shape == (n, 14, 32)
    ref = _ref_forward(x, conv)
    # one bf16 rounding (2^-8 relative) of the fp32-accumulated value, plus the fp32 summation order
    err = (y.double() - ref).abs()
    assert (err <= ref.abs() * 2.0 ** -8 + 1e-4).all(), float((err - ref.abs() * 2.0 ** -8).max())


@pytest.mark.parametrize("n", [777, 49152])
def test_conv1_bf16_weight_gradient_matches_fp64(n):
    from ti5_isaacgym_amd.algo.dh_policy import conv1d_train_bf16
    conv = _conv()
    g = torch.Generator(device=DEV).manual_seed(n + 1)
    x = (torch.randn(n, 66, 47, device=DEV, generator=g) * 2.0).to(torch.bfloat16)
    gy = torch.randn(n, 14, 32, device=DEV, generator=g).to(torch.bfloat16)
    y = conv1d_train_bf16(x, conv)
    y.backward(gy)
    gw, gb = conv.weight.grad.clone(), conv.bias.grad.clone()
    # fp64 reference on the same bf16 operands: gW[o, c, t] = sum_{b,l} gy[b,l,o] x[b,c,3l+t]
    win = x.double().unfold(2, 6, 3)                       # (B, 66, 14, 6)
    ref_w = torch.einsum("blo,bclt->oct", gy.double(), win)
    ref_b = gy.double().sum((0, 1))
    torch.testing.assert_close(gw.double(), ref_w, rtol=1e-3, atol=1e-3 * ref_w.abs().max().item() * 1e-2)
    torch.testing.assert_close(gb.double(), ref_b, rtol=1e-3, atol=1e-2)
    # deterministic: a second backward gives the same bits
    conv.weight.grad = None
    conv.bias.grad = None
    conv1d_train_bf16(x, conv).backward(gy)
    assert torch.equal(conv.weight.grad, gw) and torch.equal(conv.bias.grad, gb)


def test_conv1_bf16_refuses_other_shapes():
    from ti5_isaacgym_amd.algo.dh_policy import conv1d_train_bf16
    conv = torch.nn.Conv1d(66, 16, kernel_size=6, stride=3).to(DEV)
    x = torch.randn(4, 66, 47, device=DEV).to(torch.bfloat16)
    assert conv1d_train_bf16(x, conv) is None
    assert conv1d_train_bf16(x.float(), _conv()) is None


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("rows,cols", [(49152, 256), (49152, 3), (777, 768)])
def test_bias_colsum_matches_fp64(rows, cols, dtype, monkeypatch):
    """The update's Linear bias gradients (dh_policy.bias_grad, t1policy_colsum): fp32 sums in a fixed order, within
    fp32 summation error of an fp64 sum, the same bits on a second call."""
    from ti5_isaacgym_amd.algo import dh_policy
    from ti5_isaacgym_amd.algo.dh_policy import bias_grad
    monkeypatch.setattr(dh_policy, "BIAS_COLSUM", True)   # the opt-in kernel (torch's sum is the default)
    g = torch.Generator(device=DEV).manual_seed(rows + cols)
    gy = torch.randn(rows, cols, device=DEV, generator=g).to(dtype)
    out = bias_grad(gy)
    assert out.dtype == torch.float32 and out.shape == (cols,)
    ref = gy.double().sum(0)
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-3)
    assert torch.equal(bias_grad(gy), out)


@pytest.mark.parametrize("slices,shape", [(24, (512, 302)), (24, (3, 64)), (5, (7, 13)), (1, (768, 219)), (9, (128, 96))])
def test_splitk_slice_sum_is_the_ordered_fp32_sum(slices, shape):
    """The split-K weight gradient's reduction (dh_policy.slice_sum, t1policy_slice_sum): bit-identical to the fp32 sum
    of the slices taken s = 0, 1, ... in order (float4 path for sizes divisible by 4, scalar path otherwise)."""
    from ti5_isaacgym_amd.algo.dh_policy import slice_sum
    g = torch.Generator(device=DEV).manual_seed(slices * 1000 + shape[0])
    part = torch.randn(slices, *shape, device=DEV, generator=g) * 10.0
    out = slice_sum(part)
    ref = part[0].clone()
    for s in range(1, slices):
        ref += part[s]
    assert out.shape == shape and out.dtype == torch.float32
    assert torch.equal(out, ref)


def test_wgrad_splitk_uses_slice_sum_and_matches_fp64():
    """wgrad_splitk on the device (bf16 operands, fp32 partials, HIP slice sum) against fp64, at whole slices (the
    update's 49,152 rows are 24 of them; a ragged tail's bf16 GEMM output is rounded to bf16 before the widening)."""
    from ti5_isaacgym_amd.algo import dh_policy
    g = torch.Generator(device=DEV).manual_seed(7)
    K = 3 * dh_policy.SPLITK_ROWS
    gy = torch.randn(K, 96, device=DEV, generator=g).to(torch.bfloat16)
    x = torch.randn(K, 130, device=DEV, generator=g).to(torch.bfloat16)
    gw = dh_policy.wgrad_splitk(gy, x)
    ref = gy.double().t() @ x.double()
    assert gw.dtype == torch.float32
    torch.testing.assert_close(gw.double(), ref, rtol=1e-4, atol=1e-2)


# ---- the fp32 update (the reference's precision): the fp32-accurate packed forward and the three-part-split weight
# gradient (t1policy_conv1_wgrad_f32), both against fp64 on the fp32 operands at fp32-class bounds
@pytest.mark.parametrize("n", [1, 777, 8192])
def test_conv1_f32_forward_matches_fp64(n):
    from ti5_isaacgym_amd.algo.dh_policy import conv1d_train_f32
    conv = _conv()
    g = torch.Generator(device=DEV).manual_seed(n + 7)
    x = torch.randn(n, 66, 47, device=DEV, generator=g) * 2.0
    y = conv1d_train_f32(x, conv)
    assert y is not None and y.dtype == torch.float32 and y.shape == (n, 14, 32)
    ref = torch.nn.functional.conv1d(x.double(), conv.weight.detach().double(), conv.bias.detach().double(),
                                     stride=3).transpose(1, 2)
    mag = torch.nn.functional.conv1d(x.double().abs(), conv.weight.detach().double().abs(),
                                     conv.bias.detach().double().abs(), stride=3).transpose(1, 2)
    err = (y.double() - ref).abs()
    assert (err <= 2e-6 * mag + 1e-30).all(), float((err / mag).max())


@pytest.mark.parametrize("n", [777, 49152])
def test_conv1_f32_weight_gradient_matches_fp64(n):
    """fp32-class: every gW / gb element within 2e-6 of sum |gy| |x| of the fp64 sum (fp32's unit roundoff is 6e-8;
    a few dozen roundings along the fixed-order sum), the same bits on a second backward."""
    from ti5_isaacgym_amd.algo.dh_policy import conv1d_train_f32
    conv = _conv()
    g = torch.Generator(device=DEV).manual_seed(n + 3)
    x = torch.randn(n, 66, 47, device=DEV, generator=g) * 2.0
    gy = torch.randn(n, 14, 32, device=DEV, generator=g) * 1e-3
    y = conv1d_train_f32(x, conv)
    y.backward(gy)
    gw, gb = conv.weight.grad.clone(), conv.bias.grad.clone()
    win = x.double().unfold(2, 6, 3)                       # (B, 66, 14, 6)
    ref_w = torch.einsum("blo,bclt->oct", gy.double(), win)
    mag_w = torch.einsum("blo,bclt->oct", gy.double().abs(), win.abs())
    ref_b, mag_b = gy.double().sum((0, 1)), gy.double().abs().sum((0, 1))
    ew = (gw.double() - ref_w).abs()
    eb = (gb.double() - ref_b).abs()
    print(f"n={n}: max |gW err| / (|gy|^T|x|) = {float((ew / mag_w).max()):.2e}, bias {float((eb / mag_b).max()):.2e}")
    assert (ew <= 2e-6 * mag_w).all() and (eb <= 2e-6 * mag_b).all()
    conv.weight.grad = None
    conv.bias.grad = None
    conv1d_train_f32(x, conv).backward(gy)
    assert torch.equal(conv.weight.grad, gw) and torch.equal(conv.bias.grad, gb)


def test_history_encoder_fp32_update_uses_the_hip_conv(monkeypatch):
    """Under autograd in fp32 the history encoder's first conv takes conv1d_train_f32 (no unfold), and the encoder's
    output and weight gradients match the unfold + GEMM path (T1_CONV1_TRAIN off) within fp32 summation order."""
    from ti5_isaacgym_amd.algo import dh_policy
    torch.manual_seed(1)
    enc = dh_policy._history_encoder(66, 47, [32, 16], [6, 4], [3, 2], 16).to(DEV)
    x = torch.randn(512, 66, 47, device=DEV)
    calls = []
    real = dh_policy.conv1d_train_f32
    monkeypatch.setattr(dh_policy, "conv1d_train_f32", lambda *a: (calls.append(1), real(*a))[1])
    out = enc(x)
    out.square().sum().backward()
    g1 = [p.grad.clone() for p in enc.parameters()]
    assert calls, "the fp32 HIP conv was not used"
    enc.zero_grad()
    monkeypatch.setattr(dh_policy, "CONV1_TRAIN", False)
    out2 = enc(x)
    out2.square().sum().backward()
    torch.testing.assert_close(out, out2, rtol=1e-5, atol=1e-6)
    for a, b in zip(g1, [p.grad for p in enc.parameters()]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6 * b.abs().max().item())
