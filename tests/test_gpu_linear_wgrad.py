"""The bf16 update's Linear weight + bias gradients as one HIP MFMA kernel (t1policy_linear_wgrad_bf16,
ti5_isaacgym_amd/csrc/t1policy_wgrad.hip; dh_policy._LinearSplitK.backward) against fp64 torch on the same bf16
operands -- needs the MI355X.

Bound: the kernel sums exact bf16 products in fp32 (MFMA accumulation over a slice's rows, then the slices in order),
so each output is within a few hundred fp32 roundings of |gy|^T |x|: the test holds it to 1e-5 of that magnitude sum
(about 170 ulps), element by element.  Determinism: a second call gives the same bits (the graphed == eager update
relies on it)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

# (rows, M = outputs, N = inputs): the update's layers at the 49,152-row minibatch (the odd widths take the 16-bit
# load path: the state estimator's 235 inputs, the critic's 219, the estimator head's 3 outputs, the value head's 1),
# the second conv as a GEMM (294,912 rows), and ragged / tiny shapes
SHAPES = [(49152, 768, 219), (49152, 256, 235), (49152, 512, 302), (49152, 3, 64), (49152, 1, 128),
          (294912, 16, 128), (49152, 256, 768), (1000, 12, 128), (31, 5, 7), (4097, 130, 97), (64, 300, 2),
          (777, 219, 235), (3001, 1, 3)]


def _operands(rows, M, N, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    gy = (torch.randn(rows, M, device=DEV, generator=g) * 0.1).to(torch.bfloat16)
    x = torch.randn(rows, N, device=DEV, generator=g).to(torch.bfloat16)
    return gy, x


def _check(gw, gb, gy, x):
    gyd, xd = gy.double(), x.double()
    ref_w = gyd.t() @ xd
    mag_w = gyd.abs().t() @ xd.abs()
    err = (gw.double() - ref_w).abs()
    assert (err <= 1e-5 * mag_w + 1e-30).all(), float((err / (mag_w + 1e-30)).max())
    if gb is not None:
        ref_b = gyd.sum(0)
        mag_b = gyd.abs().sum(0)
        errb = (gb.double() - ref_b).abs()
        assert (errb <= 1e-5 * mag_b + 1e-30).all(), float((errb / (mag_b + 1e-30)).max())


@pytest.mark.parametrize("rows,M,N", SHAPES)
def test_linear_wgrad_matches_fp64(rows, M, N):
    from ti5_isaacgym_amd.algo.dh_policy import linear_wgrad_bf16
    gy, x = _operands(rows, M, N, rows + 7 * M + N)
    gw, gb = linear_wgrad_bf16(gy, x)
    assert gw.shape == (M, N) and gw.dtype == torch.float32 and gb.shape == (M,) and gb.dtype == torch.float32
    _check(gw, gb, gy, x)
    gw2, gb2 = linear_wgrad_bf16(gy, x)
    assert torch.equal(gw, gw2) and torch.equal(gb, gb2)
    gw3, gb3 = linear_wgrad_bf16(gy, x, need_bias=False)   # no bias: the same weight gradient
    assert gb3 is None and torch.equal(gw3, gw)


def test_linear_wgrad_rounds_fp32_inputs_to_bf16():
    """An fp32 saved input is rounded to bf16 first, as autocast's GEMM would round it."""
    from ti5_isaacgym_amd.algo.dh_policy import linear_wgrad_bf16
    gy, _ = _operands(5000, 64, 1, 3)
    x = torch.randn(5000, 235, device=DEV)
    gw, _ = linear_wgrad_bf16(gy, x)
    gw16, _ = linear_wgrad_bf16(gy, x.to(torch.bfloat16))
    assert torch.equal(gw, gw16)


def test_linear_backward_uses_the_kernel_under_bf16_autocast(monkeypatch):
    """A Linear of the policy under the bf16 update's autocast: the kernel's gradients (fp32, within the fp64 bound of
    the bf16 operands autograd saved) and the split-K path's agree to bf16-GEMM precision."""
    from ti5_isaacgym_amd.algo import dh_policy
    torch.manual_seed(0)
    lin = dh_policy.Linear(302, 512).to(DEV)
    x = torch.randn(49152, 302, device=DEV).to(torch.bfloat16)
    g = torch.randn(49152, 512, device=DEV).to(torch.bfloat16) * 0.01

    def grads(flag):
        monkeypatch.setattr(dh_policy, "LINEAR_WGRAD", flag)
        lin.weight.grad = lin.bias.grad = None
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
            y = lin(x)
        y.backward(g)
        return lin.weight.grad.clone(), lin.bias.grad.clone()

    gw, gb = grads(True)
    _check(gw, gb, g, x)
    gw0, gb0 = grads(False)
    torch.testing.assert_close(gw, gw0, rtol=1e-2, atol=1e-3 * gw0.abs().max().item())
    torch.testing.assert_close(gb, gb0, rtol=1e-2, atol=1e-3 * gb0.abs().max().item())


def test_linear_wgrad_rejects_bad_arguments():
    from ti5_isaacgym_amd import _lib
    lib = _lib.load()
    assert lib.t1policy_linear_wgrad_workspace_bytes(0, 4, 4) == -1
    gy, x = _operands(64, 8, 8, 1)
    ws = torch.empty(16, device=DEV, dtype=torch.uint8)
    gw = torch.empty(8, 8, device=DEV)
    # a workspace smaller than workspace_bytes is refused, not overrun
    assert lib.t1policy_linear_wgrad_bf16(gy.data_ptr(), x.data_ptr(), 64, 8, 8, ws.data_ptr(), 16, gw.data_ptr(),
                                          None, 0, torch.cuda.current_stream().cuda_stream) == -1


def test_linear_wgrad_accumulates_into_existing_grads(monkeypatch):
    """into=: the sums ADDED to existing fp32 gradients; through autograd (GRAD_DIRECT, the PPO update's bucket views) a
    preset .grad ends as the same bits as autograd's own accumulation of the returned gradient."""
    from ti5_isaacgym_amd.algo import dh_policy
    gy, x = _operands(3000, 96, 130, 11)
    base_w = torch.randn(96, 130, device=DEV)
    base_b = torch.randn(96, device=DEV)
    gw0, gb0 = dh_policy.linear_wgrad_bf16(gy, x)
    w, b = base_w.clone(), base_b.clone()
    dh_policy.linear_wgrad_bf16(gy, x, into=(w, b))
    assert torch.equal(w, base_w + gw0) and torch.equal(b, base_b + gb0)
    torch.manual_seed(1)
    lin = dh_policy.Linear(130, 96).to(DEV)

    calls = []
    real = dh_policy.linear_wgrad_bf16
    monkeypatch.setattr(dh_policy, "linear_wgrad_bf16",
                        lambda *a, **k: (calls.append(k.get("into") is not None), real(*a, **k))[1])

    def grads(flag):
        lin.weight.grad, lin.bias.grad = base_w.clone(), base_b.clone()
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
            y = lin(x)
        with dh_policy.direct_grad_accumulation(flag):
            y.backward(gy)
        return lin.weight.grad.clone(), lin.bias.grad.clone()

    (wd, bd), (wa, ba) = grads(True), grads(False)
    assert calls == [True, False]   # the direct path ran only inside the context
    assert torch.equal(wd, wa) and torch.equal(bd, ba)
    assert torch.equal(wd, base_w + gw0)


def test_autograd_grad_leaves_preset_grads_alone():
    """outside direct_grad_accumulation() the kernel's gradients go back through autograd.  torch.autograd.grad
    under bf16 autocast with preset .grad tensors returns the weight / bias gradients and leaves .grad unchanged, and
    backward(inputs=[x]) touches no parameter's .grad."""
    from ti5_isaacgym_amd.algo import dh_policy
    gy, x = _operands(2048, 64, 96, 5)
    gw0, gb0 = dh_policy.linear_wgrad_bf16(gy, x)
    torch.manual_seed(2)
    lin = dh_policy.Linear(96, 64).to(DEV)
    pw, pb = torch.randn(64, 96, device=DEV), torch.randn(64, device=DEV)
    lin.weight.grad, lin.bias.grad = pw.clone(), pb.clone()
    with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
        y = lin(x)
    gw, gb = torch.autograd.grad(y, (lin.weight, lin.bias), gy)
    assert gw is not None and gb is not None
    assert torch.equal(gw, gw0) and torch.equal(gb, gb0)
    assert torch.equal(lin.weight.grad, pw) and torch.equal(lin.bias.grad, pb)
    xi = x.float().clone().requires_grad_(True)
    with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
        y = lin(xi)
    y.backward(gy, inputs=[xi])
    assert xi.grad is not None
    assert torch.equal(lin.weight.grad, pw) and torch.equal(lin.bias.grad, pb)


# ---- the fp32 update's kernel (t1policy_linear_wgrad_f32): fp32 operands, three-part bf16 split, fp32-class sums
def _operands_f32(rows, M, N, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(rows, M, device=DEV, generator=g) * 1e-2, torch.randn(rows, N, device=DEV, generator=g)


@pytest.mark.parametrize("rows,M,N", SHAPES)
def test_linear_wgrad_f32_matches_fp64(rows, M, N):
    """Every gW / gb element within 2e-6 of |gy|^T |x| of the fp64 sum (fp32-class: the bf16 kernel's bound is 1e-5 on
    already-rounded operands; here the operands are the fp32 values themselves), the same bits on a second call."""
    from ti5_isaacgym_amd.algo.dh_policy import linear_wgrad_f32
    gy, x = _operands_f32(rows, M, N, rows + M + N)
    gw, gb = linear_wgrad_f32(gy, x)
    gyd, xd = gy.double(), x.double()
    ew = (gw.double() - gyd.t() @ xd).abs()
    mw = gyd.abs().t() @ xd.abs()
    eb = (gb.double() - gyd.sum(0)).abs()
    mb = gyd.abs().sum(0)
    assert (ew <= 2e-6 * mw + 1e-30).all(), float((ew / (mw + 1e-30)).max())
    assert (eb <= 2e-6 * mb + 1e-30).all(), float((eb / (mb + 1e-30)).max())
    gw2, gb2 = linear_wgrad_f32(gy, x)
    assert torch.equal(gw, gw2) and torch.equal(gb, gb2)


def test_linear_backward_uses_the_f32_kernel(monkeypatch):
    """In fp32 (no autocast) the Linear's weight / bias gradients come from t1policy_linear_wgrad_f32, within fp32
    summation order of torch's, and inside direct_grad_accumulation() they are added into the existing .grad."""
    from ti5_isaacgym_amd.algo import dh_policy
    calls = []
    real = dh_policy.linear_wgrad_f32
    monkeypatch.setattr(dh_policy, "linear_wgrad_f32", lambda *a, **k: (calls.append(1), real(*a, **k))[1])
    torch.manual_seed(3)
    lin = dh_policy.Linear(219, 768).to(DEV)
    x = torch.randn(4096, 219, device=DEV)
    gy = torch.randn(4096, 768, device=DEV) * 1e-2
    lin(x).backward(gy)
    assert calls
    ref_w = (gy.double().t() @ x.double()).float()
    torch.testing.assert_close(lin.weight.grad, ref_w, rtol=1e-5, atol=1e-5 * ref_w.abs().max().item())
    torch.testing.assert_close(lin.bias.grad, gy.sum(0), rtol=1e-5, atol=1e-6)
    pw, pb = lin.weight.grad.clone(), lin.bias.grad.clone()
    with dh_policy.direct_grad_accumulation():
        lin(x).backward(gy)
    torch.testing.assert_close(lin.weight.grad, 2 * pw, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(lin.bias.grad, 2 * pb, rtol=1e-6, atol=1e-7)


# ---- the fp32 update's forward / input-gradient GEMM (t1policy_gemm_nt_f32)
GEMM_SHAPES = [(49152, 768, 219), (49152, 256, 768), (49152, 512, 302), (49152, 3, 64), (49152, 1, 128),
               (294912, 16, 128), (49152, 219, 768), (777, 130, 97), (31, 5, 7), (64, 300, 2)]


@pytest.mark.parametrize("R,N,K", GEMM_SHAPES)
def test_gemm_nt_f32_matches_fp64(R, N, K):
    """a b^T + bias within 2e-6 of |a| |b|^T + |bias| of the fp64 value (fp32-class), ELU applied after the same sum
    (act=1), and the same bits on a second call."""
    from ti5_isaacgym_amd.algo.dh_policy import gemm_nt_f32
    g = torch.Generator(device=DEV).manual_seed(R + N + K)
    a = torch.randn(R, K, device=DEV, generator=g)
    b = torch.randn(N, K, device=DEV, generator=g) * 0.1
    bias = torch.randn(N, device=DEV, generator=g)
    y = gemm_nt_f32(a, b, bias)
    ref = a.double() @ b.double().t() + bias.double()
    mag = a.double().abs() @ b.double().abs().t() + bias.double().abs()
    err = (y.double() - ref).abs()
    assert (err <= 2e-6 * mag).all(), float((err / mag).max())
    assert torch.equal(y, gemm_nt_f32(a, b, bias))
    ye = gemm_nt_f32(a, b, bias, act=1)
    torch.testing.assert_close(ye, torch.nn.functional.elu(y), rtol=1e-6, atol=1e-7)
    aux = torch.randn(R, N, device=DEV, generator=g)
    yd = gemm_nt_f32(a, b, bias, act=2, aux=aux)
    assert torch.equal(yd, y * torch.where(aux > 0, torch.ones_like(aux), aux + 1.0))


@pytest.mark.parametrize("R,N,K,wide", [(49152, 256, 235, 3102), (777, 130, 97, 131), (4096, 302, 512, 600),
                                         (31, 5, 7, 9), (8192, 16, 128, 128)])
def test_gemm_f32_strided_operands_read_in_place(R, N, K, wide):
    """t1policy_gemm_f32: A a column slice of a wider matrix (lda > K), B the transpose of a contiguous weight (b_kn: the
    input gradient's W read in place) or a row-strided slice -- the same bits as the contiguous copies (the same parts,
    products and k order), and no copy made."""
    from ti5_isaacgym_amd.algo.dh_policy import gemm_nt_f32
    g = torch.Generator(device=DEV).manual_seed(R + N + K + wide)
    big = torch.randn(R, wide, device=DEV, generator=g)
    a = big[:, wide - K:]                      # (R, K), row stride `wide`
    w = torch.randn(K, N, device=DEV, generator=g) * 0.1
    bt = w.t()                                 # (N, K), strides (1, N): b_kn
    bwide = torch.randn(N, K + 3, device=DEV, generator=g)[:, :K]  # row stride K + 3
    bias = torch.randn(N, device=DEV, generator=g)
    aux = torch.randn(R, N, device=DEV, generator=g)
    for b in (bt, bwide):
        for act in (0, 1, 2):
            y = gemm_nt_f32(a, b, bias, act=act, aux=aux if act == 2 else None)
            y0 = gemm_nt_f32(a.contiguous(), b.contiguous(), bias, act=act, aux=aux if act == 2 else None)
            assert torch.equal(y, y0), (act, float((y - y0).abs().max()))
    ref = a.double() @ bt.double().t() + bias.double()
    mag = a.double().abs() @ bt.double().abs().t() + bias.double().abs()
    assert ((gemm_nt_f32(a, bt, bias).double() - ref).abs() <= 2e-6 * mag).all()


@pytest.mark.parametrize("rows,M,N,wide", [(49152, 256, 235, 3102), (777, 219, 235, 240), (3001, 1, 3, 8)])
def test_linear_wgrad_f32_strided_x_read_in_place(rows, M, N, wide):
    """t1policy_linear_wgrad_f32x: x a column slice (row stride > N) -- the same bits as on the contiguous copy."""
    from ti5_isaacgym_amd.algo.dh_policy import linear_wgrad_f32
    g = torch.Generator(device=DEV).manual_seed(rows + M + N)
    gy = torch.randn(rows, M, device=DEV, generator=g) * 0.1
    x = torch.randn(rows, wide, device=DEV, generator=g)[:, wide - N:]
    gw, gb = linear_wgrad_f32(gy, x)
    gw0, gb0 = linear_wgrad_f32(gy, x.contiguous())
    assert torch.equal(gw, gw0) and torch.equal(gb, gb0)


def test_linear_fp32_forward_and_input_gradient_use_the_gemm(monkeypatch):
    """In fp32 under autograd the Linear's forward and input gradient come from t1policy_gemm_nt_f32, within fp32
    summation order of torch's; T1 GEMM_F32 off gives torch's."""
    from ti5_isaacgym_amd.algo import dh_policy
    calls = []
    real = dh_policy.gemm_nt_f32
    monkeypatch.setattr(dh_policy, "gemm_nt_f32", lambda *a, **k: (calls.append(1), real(*a, **k))[1])
    torch.manual_seed(5)
    lin = dh_policy.Linear(302, 512).to(DEV)
    x = torch.randn(8192, 302, device=DEV, requires_grad=True)
    gy = torch.randn(8192, 512, device=DEV) * 1e-2
    y = lin(x)
    y.backward(gy)
    assert len(calls) == 2   # forward and input gradient
    ref_y = torch.addmm(lin.bias, x, lin.weight.t())
    torch.testing.assert_close(y, ref_y, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad, gy @ lin.weight, rtol=1e-5, atol=1e-6)


def test_mlp_fp32_fused_node_matches_layer_by_layer(monkeypatch):
    """The fp32 update's MLP as one autograd node (_MlpF32: ELU fused into the forward GEMMs, ELU's derivative into the
    input-gradient GEMMs) against the layer-by-layer path (T1_MLP_F32 off): outputs and every gradient within fp32
    summation order, and inside direct_grad_accumulation() the weight gradients added into the existing .grad."""
    from ti5_isaacgym_amd.algo import dh_policy
    torch.manual_seed(11)
    mlp = dh_policy._mlp([302, 512, 256, 128, 12], torch.nn.ELU()).to(DEV)
    assert isinstance(mlp, dh_policy.MLP) and mlp._fusable()
    x = torch.randn(6000, 302, device=DEV, requires_grad=True)
    go = torch.randn(6000, 12, device=DEV)

    def run(flag):
        monkeypatch.setattr(dh_policy, "MLP_F32", flag)
        mlp.zero_grad(set_to_none=True)
        x.grad = None
        y = mlp(x)
        y.backward(go)
        return y.detach().clone(), x.grad.clone(), [p.grad.clone() for p in mlp.parameters()]

    y1, gx1, g1 = run(True)
    y0, gx0, g0 = run(False)
    torch.testing.assert_close(y1, y0, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(gx1, gx0, rtol=1e-4, atol=1e-5 * gx0.abs().max().item())
    for a, b in zip(g1, g0):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5 * b.abs().max().item())
    # direct accumulation: a second backward inside the context doubles every .grad
    monkeypatch.setattr(dh_policy, "MLP_F32", True)
    for p, a in zip(mlp.parameters(), g1):
        p.grad = a.clone()
    with dh_policy.direct_grad_accumulation():
        mlp(x).backward(go)
    for a, p in zip(g1, mlp.parameters()):
        torch.testing.assert_close(p.grad, 2 * a, rtol=1e-6, atol=1e-7)
