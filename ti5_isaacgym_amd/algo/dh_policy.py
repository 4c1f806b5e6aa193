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
import contextlib
import os

import torch
import torch.nn as nn
from torch.distributions import Normal


# rows of the batch (K of the weight-gradient GEMM) per split-K slice (T1_SPLITK_ROWS: A/B)
def _splitk_rows(v):
    """T1_SPLITK_ROWS, checked at import (a bad value would otherwise fail deep inside a backward pass)."""
    try:
        r = int(v)
    except ValueError:
        r = 0
    if r <= 0:
        raise ValueError(f"T1_SPLITK_ROWS must be a positive integer, got {v!r}")
    return r


SPLITK_ROWS = _splitk_rows(os.environ.get("T1_SPLITK_ROWS", "2048"))
# bf16 split-K partial products returned in fp32 by the GEMM itself (T1_WGRAD_OUT_F32=0: the bf16 partials widened
# afterwards, the round-2 path; A/B)
WGRAD_OUT_F32 = os.environ.get("T1_WGRAD_OUT_F32", "1") != "0"


# the split-K partial products summed by the HIP slice sum (t1policy_slice_sum, slices in order) on the device;
# T1_SLICE_SUM=0: torch's part.sum(0) (A/B)
SLICE_SUM = os.environ.get("T1_SLICE_SUM", "1") != "0"


def slice_sum(part):
    """part.sum(0) of the (S, M, N) split-K partial products: on the device the HIP slice sum (fp32, s = 0, 1, ... in
    order: one HBM pass instead of torch's dim-0 reduction kernel), on the host or for other dtypes torch's."""
    if not (part.is_cuda and SLICE_SUM and part.dtype == torch.float32):
        return part.sum(0)
    from .. import _lib
    lib = _lib.load()
    part = part.contiguous()
    out = torch.empty(part.shape[1:], device=part.device, dtype=torch.float32)
    rc = lib.t1policy_slice_sum(part.data_ptr(), part.shape[0], out.numel(), out.data_ptr(),
                                torch.cuda.current_stream(part.device).cuda_stream)
    if rc != 0:
        raise RuntimeError(f"t1policy_slice_sum failed (rc={rc})")
    return out


def wgrad_splitk(gy, x):
    """dW = gy^T x for a batch of K rows (gy: K x M, x: K x N) as a batched GEMM over K-slices of SPLITK_ROWS rows plus
    a sum: the PPO update's weight gradients have K = 49,152 (688,128 for the first conv) and M x N of a few hundred
    squared, so a single GEMM has only a handful of output tiles -- a few workgroups on 256 CUs.  Slicing K gives
    every slice its own tiles (hipBLASLt strided-batched GEMM), then one reduction."""
    K, M = gy.shape
    S = K // SPLITK_ROWS
    if S < 2:
        return gy.t().mm(x)
    c = S * SPLITK_ROWS
    # the slices' partial products are summed in at least fp32 (they are bf16 under the opt-in bf16 update,
    # DHPPO.amp_dtype)
    wide = lambda t: t if t.dtype in (torch.float32, torch.float64) else t.float()  # noqa: E731
    if M < 8 and gy.dtype != wide(gy).dtype:
        # the heads (M = 1, 3, 12 outputs): hipBLASLt's bf16 batched GEMM spends ~11 ms of host time per call on a
        # 1-row output (profiles/r02ap_ppo_bf16.md), and one GEMM over all K rows has a single output tile (141 us for
        # M = 3, N = 64).  Widen (a few MB) and take the split-K batched GEMM in fp32, outside autocast (which would
        # narrow it again): 28-57 us (profiles/r02bf_small_m_wgrad.txt)
        with torch.autocast(device_type="cuda", enabled=False):
            return wgrad_splitk(wide(gy), wide(x))
    a, b = gy[:c].view(S, SPLITK_ROWS, M).transpose(1, 2), x[:c].view(S, SPLITK_ROWS, -1)
    if WGRAD_OUT_F32 and gy.is_cuda and gy.dtype in (torch.bfloat16, torch.float16):
        # bf16 operands, fp32 partial products straight from the GEMM (aten::bmm.dtype): no bf16 rounding of the
        # 2,048-row partial sums and no widening copy of them.  An fp32 saved input is rounded to the gradient's dtype
        # first, as autocast's bmm would (the once-per-update obs cast stays bit-identical to the per-minibatch one)
        gw = slice_sum(torch.bmm(a, b if b.dtype == gy.dtype else b.to(gy.dtype), out_dtype=torch.float32))
    else:
        gw = slice_sum(wide(torch.bmm(a, b)))
    if c < K:
        gw = gw + wide(gy[c:].t().mm(x[c:]))
    return gw


# the Linear bias gradients as the HIP column sum (opt-in, T1_BIAS_COLSUM=1): measured slower than torch's dim-0 sum
# in the graphed update (bf16 update 39.8 vs 38.1 ms per iteration, profiles/r04q3_*), so torch's stays the default
BIAS_COLSUM = os.environ.get("T1_BIAS_COLSUM", "0") == "1"


def bias_grad(gy):
    """gy.sum(0) of a (K, M) gradient: on the device the HIP column sum (t1policy_colsum: fp32 accumulation in a fixed
    order, an fp32 result for the fp32 bias), on the host torch's."""
    if not (gy.is_cuda and BIAS_COLSUM and gy.dim() == 2 and gy.dtype in (torch.bfloat16, torch.float32)):
        return gy.sum(0)
    from .. import _lib
    lib = _lib.load()
    gy = gy.contiguous()
    K, M = gy.shape
    ws = torch.empty(lib.t1policy_colsum_workspace_bytes(K, M), device=gy.device, dtype=torch.uint8)
    out = torch.empty(M, device=gy.device, dtype=torch.float32)
    rc = lib.t1policy_colsum(gy.data_ptr(), gy.element_size(), K, M, ws.data_ptr(), out.data_ptr(),
                             torch.cuda.current_stream(gy.device).cuda_stream)
    if rc != 0:
        raise RuntimeError(f"t1policy_colsum failed (rc={rc})")
    return out


# ... added by that kernel straight into an existing .grad of the layer's leaf parameters (T1_GRAD_DIRECT=0: returned
# to autograd, which adds them, A/B).  Only inside direct_grad_accumulation(), which DHPPO opens around its own
# loss.backward(): anywhere else (torch.autograd.grad, backward(inputs=...), a caller's own backward) the gradients go
# back through autograd, so what autograd returns and which .grad it touches are exactly torch's.
GRAD_DIRECT = os.environ.get("T1_GRAD_DIRECT", "1") != "0"
# a module flag, not a contextvar: autograd runs a CUDA node's backward on its device worker thread, which does not
# see the calling thread's context variables
_DIRECT_GRAD = [False]


@contextlib.contextmanager
def direct_grad_accumulation(enabled=True):
    """Within the block, a backward() of _LinearSplitK under the bf16 update may add its weight / bias gradients straight
    into the leaf parameters' existing fp32 .grad (returning None to autograd for them).  Valid only around a plain
    loss.backward() that accumulates into every parameter's .grad -- DHPPO's minibatch step."""
    prev = _DIRECT_GRAD[0]
    _DIRECT_GRAD[0] = bool(enabled)
    try:
        yield
    finally:
        _DIRECT_GRAD[0] = prev
# the bf16 update's Linear weight + bias gradients as one HIP MFMA kernel (t1policy_linear_wgrad_bf16); T1_LINEAR_WGRAD=0:
# the split-K batched GEMM + slice sum + torch's bias sum (A/B)
LINEAR_WGRAD = os.environ.get("T1_LINEAR_WGRAD", "1") != "0"


# the fp32 update's Linear weight + bias gradients as the HIP three-part-split kernel (t1policy_linear_wgrad_f32);
# T1_LINEAR_WGRAD_F32=0: the split-K batched GEMM + slice sum + bias sum (A/B)
LINEAR_WGRAD_F32 = os.environ.get("T1_LINEAR_WGRAD_F32", "1") != "0"


def linear_wgrad_bf16(gy, x, need_bias=True, into=None):
    """(gy^T x, gy.sum(0)) in fp32 for bf16 gy (K, M) and x (K, N) (x in fp32 is rounded to bf16 first, as autocast's
    GEMM would): the HIP wgrad kernel, fixed-order fp32 sums of the exact bf16 products.  Device tensors only.
    into = (gw, gb): existing fp32 gradients (gb may be None) the sums are ADDED to (autograd's accumulation into a
    .grad, done by the kernel's last pass); returns them."""
    gy = gy.contiguous()
    x = (x if x.dtype == torch.bfloat16 else x.to(torch.bfloat16)).contiguous()
    return _linear_wgrad("t1policy_linear_wgrad_bf16", gy, x, need_bias, into)


def linear_wgrad_f32(gy, x, need_bias=True, into=None):
    """linear_wgrad_bf16 for the fp32 update: fp32 gy and x, each value split into three bf16 parts on the matrix cores
    (six part products per product, fp32-class fixed-order sums; t1policy_linear_wgrad_f32)."""
    gy = gy.float().contiguous()
    x = x.float()
    if x.dim() == 2 and x.stride(1) == 1 and x.stride(0) > x.shape[1] and x.shape[0] > 1:  # a column slice, in place
        return _linear_wgrad("t1policy_linear_wgrad_f32x", gy, x, need_bias, into, ldx=x.stride(0))
    return _linear_wgrad("t1policy_linear_wgrad_f32", gy, x.contiguous(), need_bias, into)


# the fp32 update's Linear forward / input-gradient GEMMs as the HIP three-part-split GEMM (t1policy_gemm_nt_f32);
# T1_GEMM_F32=0: hipBLASLt's fp32 addmm / mm (A/B)
GEMM_F32 = os.environ.get("T1_GEMM_F32", "1") != "0"


def gemm_nt_f32(a, b, bias=None, act=0, aux=None):
    """a (R, K) @ b (N, K)^T (+ bias) in fp32 on the matrix cores (t1policy_gemm_nt_f32: each value in three bf16 parts,
    fp32-class sums in k order), then act=1: ELU (alpha 1); act=2: times ELU's derivative at the ELU outputs aux (R, N)
    (1 where aux > 0, else aux + 1) -- the backward of a Linear whose input came out of an ELU.  Device fp32 tensors."""
    from .. import _lib
    lib = _lib.load()
    R, K = a.shape
    N = b.shape[0]
    if b.shape[1] != K or a.dtype != torch.float32 or b.dtype != torch.float32:
        raise ValueError(f"gemm_nt_f32: {tuple(a.shape)} x {tuple(b.shape)}^T ({a.dtype}, {b.dtype})")
    # strided operands read in place (t1policy_gemm_f32): A a row-strided view (a column slice), B row-strided or the
    # transpose of a contiguous matrix (a Linear weight's .t() in the input gradient); anything else is copied
    if a.stride(1) != 1 or a.stride(0) < K or R == 1:
        a = a.contiguous()
    if b.stride(1) == 1 and b.stride(0) >= K and N > 1:
        b_kn, ldb = 0, b.stride(0)
    elif b.stride(0) == 1 and b.stride(1) >= N and K > 1:
        b_kn, ldb = 1, b.stride(1)
    else:
        b = b.contiguous()
        b_kn, ldb = 0, K
    out = torch.empty(R, N, device=a.device, dtype=torch.float32)
    bp = xp = None
    if bias is not None:
        bias = bias.contiguous()
        bp = bias.data_ptr()
    if act == 2:
        if aux is None or tuple(aux.shape) != (R, N) or aux.dtype != torch.float32:
            raise ValueError("gemm_nt_f32: act=2 needs the (R, N) fp32 ELU outputs")
        aux = aux.contiguous()
        xp = aux.data_ptr()
    st = torch.cuda.current_stream(a.device).cuda_stream
    lda = a.stride(0)
    if lda == K and ldb == K and not b_kn:
        rc = lib.t1policy_gemm_nt_f32(a.data_ptr(), b.data_ptr(), bp, xp, out.data_ptr(), R, N, K, act, st)
    else:
        rc = lib.t1policy_gemm_f32(a.data_ptr(), lda, b.data_ptr(), ldb, b_kn, bp, xp, out.data_ptr(), R, N, K, act, st)
    if rc != 0:
        raise RuntimeError(f"t1policy_gemm_f32 failed (rc={rc}; R {R}, N {N}, K {K}, lda {lda}, ldb {ldb}, b_kn {b_kn})")
    return out


def _linear_wgrad(fn, gy, x, need_bias, into, ldx=None):
    from .. import _lib
    lib = _lib.load()
    K, M = gy.shape
    N = x.shape[1]
    if x.shape[0] != K:
        raise ValueError(f"{fn}: {K} gradient rows against {x.shape[0]} input rows")
    nbytes = lib.t1policy_linear_wgrad_workspace_bytes(K, M, N)
    if nbytes <= 0:
        raise RuntimeError(f"t1policy_linear_wgrad_workspace_bytes failed ({nbytes})")
    ws = torch.empty(nbytes, device=gy.device, dtype=torch.uint8)
    if into is not None:
        gw, gb = into
        ok = lambda t, shape: (t.dtype == torch.float32 and t.is_contiguous() and tuple(t.shape) == shape  # noqa: E731
                               and t.device == gy.device)
        if not ok(gw, (M, N)) or (gb is not None and not ok(gb, (M,))):
            raise ValueError(f"{fn}: into= needs contiguous fp32 (M, N) / (M,) device gradients")
    else:
        gw = torch.empty(M, N, device=gy.device, dtype=torch.float32)
        gb = torch.empty(M, device=gy.device, dtype=torch.float32) if need_bias else None
    rows_args = (K, M, N) if ldx is None else (ldx, K, M, N)
    rc = getattr(lib, fn)(gy.data_ptr(), x.data_ptr(), *rows_args, ws.data_ptr(), nbytes, gw.data_ptr(),
                          gb.data_ptr() if gb is not None else None, int(into is not None),
                          torch.cuda.current_stream(gy.device).cuda_stream)
    if rc != 0:
        raise RuntimeError(f"{fn} failed (rc={rc})")
    return gw, gb


# the update's bf16 weight copies made by one multi-tensor cast per minibatch (param_shadows) instead of one cast
# kernel per Linear weight and bias (T1_PARAM_SHADOWS=0: the per-layer casts, A/B)
PARAM_SHADOWS = os.environ.get("T1_PARAM_SHADOWS", "1") != "0"
_ACTIVE_SHADOWS = {}


@contextlib.contextmanager
def param_shadows(module, dtype):
    """Inside the block, the device fp32 parameters of `module` have `dtype` copies made by one torch._foreach_copy_
    (persistent buffers on the module, rewritten on entry), which _LinearSplitK's forward uses instead of casting each
    weight and bias itself -- the same values as its per-layer cast.  The copies stay valid until the parameters
    change (the forward saves them for its backward; the optimizer step comes after the backward)."""
    params = [p for p in module.parameters() if p.is_cuda and p.dtype == torch.float32]
    st = getattr(module, "_t1_shadows", None)
    if (st is None or st[0] != dtype or len(st[1]) != len(params)
            or any(b.shape != p.shape or b.device != p.device for p, b in zip(params, st[1]))):
        st = module._t1_shadows = (dtype, [torch.empty_like(p, dtype=dtype) for p in params])
    if params:
        torch._foreach_copy_(st[1], [p.detach() for p in params])
    prev = dict(_ACTIVE_SHADOWS)
    _ACTIVE_SHADOWS.update({id(p): (p, b) for p, b in zip(params, st[1])})
    try:
        yield
    finally:
        _ACTIVE_SHADOWS.clear()
        _ACTIVE_SHADOWS.update(prev)


def _cast_param(t, dt):
    e = _ACTIVE_SHADOWS.get(id(t))
    if e is not None and e[0] is t and e[1].dtype == dt:
        return e[1]
    return t.to(dt)


class _LinearSplitK(torch.autograd.Function):
    # custom_fwd / custom_bwd: under torch.autocast (the opt-in bf16 update) the GEMMs run in the autocast dtype in
    # both passes; autograd casts the returned gradients to the fp32 parameters' dtype
    @staticmethod
    @torch.amp.custom_fwd(device_type="cuda")
    def forward(ctx, x, w, b):
        # the leaf parameters, for the backward's direct accumulation into their .grad (GRAD_DIRECT)
        ctx.leaves = (w if w.is_leaf else None, b if b.is_leaf else None)
        if x.is_cuda and torch.is_autocast_enabled("cuda"):
            # the operands cast once, here, and saved cast: the backward's input-gradient GEMM and weight gradient use
            # the same bf16 weight / input instead of casting the fp32 ones again (19 weight casts per minibatch; the
            # values are the casts autocast's addmm would make, so the results are the same bits)
            dt = torch.get_autocast_dtype("cuda")
            x, w, b = x.to(dt), _cast_param(w, dt), _cast_param(b, dt)
        ctx.save_for_backward(x, w)
        if (GEMM_F32 and x.is_cuda and x.dtype == torch.float32 and w.dtype == torch.float32 and x.dim() == 2
                and not torch.is_autocast_enabled("cuda")):
            return gemm_nt_f32(x, w, b)   # the fp32 update: the three-part-split HIP GEMM
        return torch.addmm(b, x, w.t())

    @staticmethod
    @torch.amp.custom_bwd(device_type="cuda")
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy = gy.contiguous()
        gx = None
        if ctx.needs_input_grad[0]:
            if GEMM_F32 and gy.is_cuda and gy.dtype == torch.float32 and w.dtype == torch.float32:
                gx = gemm_nt_f32(gy, w.t())   # gy W as gy (W^T)^T: the reduction index contiguous in both operands
            else:
                gx = gy.mm(w)
        kern = None
        if gy.is_cuda and ctx.needs_input_grad[1]:
            if LINEAR_WGRAD and gy.dtype == torch.bfloat16:
                kern = linear_wgrad_bf16
            elif LINEAR_WGRAD_F32 and gy.dtype == torch.float32 and x.dtype == torch.float32:
                kern = linear_wgrad_f32   # the fp32 update (the reference's precision)
        if kern is not None:
            wl, bl = ctx.leaves
            need_b = ctx.needs_input_grad[2]
            if (GRAD_DIRECT and _DIRECT_GRAD[0] and wl is not None and wl.grad is not None and wl.grad.dtype == torch.float32
                    and wl.grad.is_contiguous() and (not need_b or (bl is not None and bl.grad is not None
                                                                    and bl.grad.dtype == torch.float32))):
                # the weight / bias gradients added straight into the existing .grad (the PPO update's views into
                # the all-reduce bucket) by the kernel's reduction: autograd's accumulation pass per parameter
                # (one add_ kernel each, ~38 per minibatch) is not needed, so no gradient is returned for them
                kern(gy, x, into=(wl.grad, bl.grad if need_b else None))
                return gx, None, None
            gw, gb = kern(gy, x, need_bias=need_b)
            return gx, gw, gb
        gw = wgrad_splitk(gy, x) if ctx.needs_input_grad[1] else None
        gb = bias_grad(gy) if ctx.needs_input_grad[2] else None
        return gx, gw, gb


def linear(x, layer):
    """layer(x) for an nn.Linear on 2-D x; on the MI355X with split-K weight gradients (same math, fp32 summation
    order aside), on the host exactly nn.Linear (the reference's CPU path)."""
    if x.is_cuda and x.dim() == 2 and torch.is_grad_enabled():
        return _LinearSplitK.apply(x.contiguous(), layer.weight, layer.bias)
    return nn.functional.linear(x, layer.weight, layer.bias)


class Linear(nn.Linear):
    """nn.Linear (same parameters and state-dict keys) with the split-K weight gradient on the device."""

    def forward(self, x):
        return linear(x, self)


def plain_copy(module):
    """A copy of a policy sub-network built from plain torch layers only (nn.Linear for Linear, nn.Sequential for
    HistoryEncoder), same parameters: what TorchScript export scripts (scripts/export_policy.py)."""
    import copy
    if isinstance(module, Linear):
        m = nn.Linear(module.in_features, module.out_features)
        m.load_state_dict(module.state_dict())
        return m
    if isinstance(module, nn.Sequential):
        return nn.Sequential(*[plain_copy(m) for m in module])
    return copy.deepcopy(module)


# the fp32 update's MLPs (actor, critic, state estimator) as one autograd node on the fused HIP GEMMs (_MlpF32; default,
# T1_MLP_F32=0 runs them layer by layer): the ELU and ELU-backward passes (3.3 ms per update) go into the GEMM epilogues
# -- update 38.1-38.2 -> 34.5-35.6 ms (profiles/r06t_*), once the epilogue loads its ELU outputs together (its first
# form loaded them one by one behind the bounds checks and cost as much as it saved)
MLP_F32 = os.environ.get("T1_MLP_F32", "1") == "1"


class _MlpF32(torch.autograd.Function):
    """Linear, ELU, Linear, ELU, ..., Linear (actor_critic_dh.py:45-111) in the fp32 update on the matrix cores, with
    each ELU fused into a GEMM: forward, every hidden layer is gemm_nt_f32(x, W, b, ELU) (no separate ELU pass over
    the activations); backward, the input gradient of layer i + 1 comes out of its GEMM already multiplied by ELU's
    derivative at layer i's output (act=2, no separate ELU-backward pass), then layer i's weight gradient is the
    three-part-split wgrad kernel (added straight into .grad inside direct_grad_accumulation(), as _LinearSplitK).
    The same sums as the layer-by-layer path in fp32 (up to the ELU being applied to the GEMM's fp32 result in its
    epilogue instead of by torch's kernel)."""

    @staticmethod
    def forward(ctx, x, *params):
        n = len(params) // 2
        h, outs = x, []
        for i in range(n):
            h = gemm_nt_f32(h, params[2 * i], params[2 * i + 1], act=1 if i < n - 1 else 0)
            if i < n - 1:
                outs.append(h)
        ctx.n = n
        # the leaf parameters (their .grad for the direct accumulation), as _LinearSplitK
        ctx.leaves = [p if p.is_leaf else None for p in params]
        ctx.save_for_backward(x, *params, *outs)
        return h

    @staticmethod
    def backward(ctx, g):
        n = ctx.n
        saved = ctx.saved_tensors
        x, params, outs = saved[0], saved[1:1 + 2 * n], saved[1 + 2 * n:]
        grads = [None] * (2 * n)
        g = g.contiguous()
        direct = GRAD_DIRECT and _DIRECT_GRAD[0]
        gx = None
        for i in range(n - 1, -1, -1):
            w = params[2 * i]
            inp = x if i == 0 else outs[i - 1]
            need_w, need_b = ctx.needs_input_grad[1 + 2 * i], ctx.needs_input_grad[2 + 2 * i]
            wl, bl = ctx.leaves[2 * i], ctx.leaves[2 * i + 1]
            if need_w:
                if (direct and wl is not None and wl.grad is not None and wl.grad.dtype == torch.float32
                        and wl.grad.is_contiguous() and (not need_b or (bl is not None and bl.grad is not None
                                                                        and bl.grad.dtype == torch.float32))):
                    linear_wgrad_f32(g, inp, into=(wl.grad, bl.grad if need_b else None))
                else:
                    grads[2 * i], gb = linear_wgrad_f32(g, inp, need_bias=need_b)
                    grads[2 * i + 1] = gb
            elif need_b:
                grads[2 * i + 1] = g.sum(0)
            if i > 0:
                g = gemm_nt_f32(g, w.t(), act=2, aux=outs[i - 1])   # (g W) * ELU'(layer i-1's output)
            elif ctx.needs_input_grad[0]:
                gx = gemm_nt_f32(g, w.t())
        return (gx, *grads)


class MLP(nn.Sequential):
    """The reference's MLP (nn.Sequential of Linear and the shared activation, actor_critic_dh.py:45-111; the same
    parameter names).  On the host, and whenever the layers are not Linear / ELU(alpha 1) alternating, it runs as
    written; in the fp32 update on the device (autograd on, no autocast) as one _MlpF32 node."""

    def _fusable(self):
        mods = list(self)
        if len(mods) % 2 != 1:
            return False
        for i, m in enumerate(mods):
            if i % 2 == 0 and not (isinstance(m, nn.Linear) and m.bias is not None and m.weight.dtype == torch.float32):
                return False
            if i % 2 == 1 and not (isinstance(m, nn.ELU) and m.alpha == 1.0):
                return False
        return True

    def forward(self, x):
        if (MLP_F32 and GEMM_F32 and LINEAR_WGRAD_F32 and x.is_cuda and x.dtype == torch.float32 and x.dim() == 2
                and torch.is_grad_enabled() and not torch.is_autocast_enabled("cuda") and self._fusable()):
            params = []
            for m in list(self)[::2]:
                params += [m.weight, m.bias]
            return _MlpF32.apply(x.contiguous(), *params)
        return super().forward(x)


def _mlp(sizes, act):
    """Linear layers between consecutive sizes, `act` after every hidden layer (not after the output)."""
    layers = []
    for i, (a, b) in enumerate(zip(sizes[:-1], sizes[1:])):
        layers.append(Linear(a, b))
        if i < len(sizes) - 2:
            layers.append(act)
    return MLP(*layers)


def conv1d_direct(x, conv):
    """Inference forward of a (B, C, L) Conv1d as the HIP direct-conv kernel (include/t1policy.h), channels-last
    (B, Lout, O) like conv1d_as_gemm: one pass over x instead of the unfolded-row copy plus a GEMM.  Returns None for
    a shape the library has no instance of (the caller keeps the GEMM path)."""
    from .. import _lib
    lib = _lib.load()
    k, st = conv.kernel_size[0], conv.stride[0]
    x = x.contiguous()
    B, C, L = x.shape
    O = conv.out_channels
    lout = (L - k) // st + 1
    bias = conv.bias.detach().contiguous()
    y = torch.empty(B, lout, O, device=x.device, dtype=torch.float32)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    if x.data_ptr() % 16 == 0 and B * C * L * 4 < 2 ** 31:
        frag = packed_conv_weights(conv, stream)
        rc = 1 if frag is None else lib.t1policy_conv1d_forward_packed(
            x.data_ptr(), frag.data_ptr(), bias.data_ptr(), y.data_ptr(), B, C, L, O, k, st, stream)
    else:
        wt = conv.weight.detach().permute(1, 2, 0).contiguous()   # tap-major: wt[c, t, o]
        rc = lib.t1policy_conv1d_forward(x.data_ptr(), wt.data_ptr(), bias.data_ptr(), y.data_ptr(), B, C, L, O, k,
                                         st, stream)
    if rc == 1:
        return None
    if rc != 0:
        raise RuntimeError(f"t1policy_conv1d_forward failed (rc={rc})")
    return y


def packed_conv_weights(conv, stream=None, force=False):
    """The conv's weights as the packed-fragment kernel's split fp16 fragments (t1policy_conv1d_pack_weights), kept on
    the module and rebuilt when the weight changed.  An eager in-place change (a load_state_dict, an eager optimizer
    step) moves the weight's version counter; a REPLAYED optimizer step (the graphed PPO update) does not -- a graph
    replay bypasses the dispatcher -- so DHPPO.update() repacks with force=True after every update.  A
    captured act() graph reads the buffer in place.  None for a shape the library has no instance of."""
    from .. import _lib
    w = conv.weight
    key = (w._version, w.data_ptr())
    frag = getattr(conv, "_t1_frag", None)
    if not force and frag is not None and getattr(conv, "_t1_frag_key", None) == key:
        return frag
    lib = _lib.load()
    if frag is None or frag.device != w.device:
        frag = torch.empty(lib.t1policy_conv1d_frag_bytes(), device=w.device, dtype=torch.uint8)
    if stream is None:
        stream = torch.cuda.current_stream(w.device).cuda_stream
    wc = w.detach().contiguous()
    rc = lib.t1policy_conv1d_pack_weights(wc.data_ptr(), frag.data_ptr(), conv.in_channels, conv.out_channels,
                                          conv.kernel_size[0], stream)
    if rc == 1:
        return None
    if rc != 0:
        raise RuntimeError(f"t1policy_conv1d_pack_weights failed (rc={rc})")
    conv._t1_frag, conv._t1_frag_key = frag, key
    return frag


def refresh_packed_weights(module, force=False):
    """Repack every Conv1d under `module` whose packed fragments are stale (before replaying a captured act()), or
    every packed one (force: after an update whose optimizer steps were graph replays); likewise the fused heads'
    fragments of a policy that has them."""
    for m in module.modules():
        if isinstance(m, nn.Conv1d) and getattr(m, "_t1_frag", None) is not None:
            packed_conv_weights(m, force=force)
        if getattr(m, "_t1_heads_frag", None) is not None:
            packed_heads_weights(m, force=force)


def _heads_args(ac, layers):
    """The heads kernel's (pointer array, dims array, version key) of the policy's parameters, or None for a layer the
    kernel cannot read (not fp32 / not contiguous)."""
    import ctypes as C
    dims, ptrs, key = [], [], []
    for m in layers:
        w = m.weight
        if w.dtype != torch.float32 or not w.is_contiguous() or not m.bias.is_contiguous():
            return None
        dims += [w.shape[0], w[0].numel()]
        ptrs += [w.data_ptr(), m.bias.data_ptr()]
        key += [(w._version, w.data_ptr()), (m.bias._version, m.bias.data_ptr())]
    ptrs.append(ac.std.data_ptr())
    key.append((ac.std._version, ac.std.data_ptr()))
    return (C.c_uint64 * 31)(*ptrs), (C.c_int * 30)(*dims), tuple(key)


def packed_heads_weights(ac, stream=None, force=False):
    """The fused heads' weights as the kernel's split fp16 fragments (t1policy_heads_pack, 3.6 MB), kept on the policy and
    repacked only when a parameter changed -- the conv's rule (packed_conv_weights): an eager change moves a version
    counter, a graph-replayed optimizer step does not, so DHPPO.update() repacks with force=True after every update and
    DHPPO._graphed_act refreshes before each replay.  The pack ran on every act() before (5 us of 0.14 ms, VERDICT r5
    #4).  Returns (frag, ptrs, dims), or None when the model has no compiled instance."""
    from .. import _lib
    layers = _heads_layers(ac)
    if layers is None:
        return None
    args = _heads_args(ac, layers)
    if args is None:
        return None
    ptrs_c, dims_c, key = args
    dev = ac.std.device
    frag = getattr(ac, "_t1_heads_frag", None)
    if not force and frag is not None and frag.device == dev and getattr(ac, "_t1_heads_key", None) == key:
        return frag, ptrs_c, dims_c
    lib = _lib.load()
    if frag is None or frag.device != dev:
        frag = torch.empty(lib.t1policy_heads_frag_bytes(), device=dev, dtype=torch.uint8)
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    rc = lib.t1policy_heads_pack(ptrs_c, dims_c, frag.data_ptr(), stream)
    if rc == 1:
        return None
    if rc != 0:
        raise RuntimeError(f"t1policy_heads_pack failed (rc={rc})")
    ac._t1_heads_frag, ac._t1_heads_key = frag, key
    return frag, ptrs_c, dims_c


# the update's first history conv as HIP kernels under the bf16 update (T1_CONV1_TRAIN=0: unfold + GEMM, A/B)
CONV1_TRAIN = os.environ.get("T1_CONV1_TRAIN", "1") != "0"


def _conv1_train_call(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


class _HistoryConvBf16(torch.autograd.Function):
    """The history encoder's first Conv1d in the PPO update on bf16 inputs (the opt-in bf16 update): the HIP forward
    (t1policy_conv1_forward_bf16, channels-last (B, Lout, O) bf16, autocast's addmm arithmetic) and weight gradient
    (t1policy_conv1_wgrad_bf16: fp32 sums in a fixed order), no unfolded copy of the input.  The input is the
    observation history, which needs no gradient."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        from .. import _lib
        lib = _lib.load()
        B, C, L = x.shape
        O, _, K = weight.shape
        stream = torch.cuda.current_stream(x.device).cuda_stream
        frag = torch.empty(lib.t1policy_conv1_bf16_frag_bytes(), device=x.device, dtype=torch.uint8)
        _conv1_train_call(lib.t1policy_conv1_pack_bf16(weight.detach().contiguous().data_ptr(), frag.data_ptr(), C, O, K,
                                                       stream), "t1policy_conv1_pack_bf16")
        lout = (L - K) // 3 + 1
        y = torch.empty(B, lout, O, device=x.device, dtype=torch.bfloat16)
        _conv1_train_call(lib.t1policy_conv1_forward_bf16(x.data_ptr(), frag.data_ptr(),
                                                          bias.detach().contiguous().data_ptr(), y.data_ptr(), B, C, L,
                                                          O, K, 3, stream), "t1policy_conv1_forward_bf16")
        ctx.save_for_backward(x)
        ctx.shape = (C, L, O, K)
        return y

    @staticmethod
    def backward(ctx, gy):
        from .. import _lib
        lib = _lib.load()
        x, = ctx.saved_tensors
        C, L, O, K = ctx.shape
        gy = gy.to(torch.bfloat16).contiguous()
        stream = torch.cuda.current_stream(x.device).cuda_stream
        ws = torch.empty(lib.t1policy_conv1_bf16_workspace_bytes(), device=x.device, dtype=torch.uint8)
        gw = torch.empty(O, C, K, device=x.device, dtype=torch.float32)
        gb = torch.empty(O, device=x.device, dtype=torch.float32)
        _conv1_train_call(lib.t1policy_conv1_wgrad_bf16(x.data_ptr(), gy.data_ptr(), ws.data_ptr(), gw.data_ptr(),
                                                        gb.data_ptr(), x.shape[0], C, L, O, K, 3, stream),
                          "t1policy_conv1_wgrad_bf16")
        return None, gw, gb


class _HistoryConvF32(torch.autograd.Function):
    """The history encoder's first Conv1d in the fp32 PPO update (the reference's precision, dh_ppo.py:155-182): the
    forward as the fp32-accurate packed direct conv (t1policy_conv1d_forward_packed: split fp16 operands, the rollout's
    inference kernel), the weights packed on every call (inside a captured update graph the optimizer's replayed steps
    move no version counter), and the weight gradient as t1policy_conv1_wgrad_f32 (three-part bf16 split, six MFMAs:
    fp32-class, fixed-order sums) -- no unfolded (B x 14, 396) copy (667 us per minibatch) and no split-K GEMM on it.
    Channels-last (B, 14, 32) fp32 out, as conv1d_as_gemm.  The input is the observation history (no gradient)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        from .. import _lib
        lib = _lib.load()
        B, C, L = x.shape
        O, _, K = weight.shape
        stream = torch.cuda.current_stream(x.device).cuda_stream
        frag = torch.empty(lib.t1policy_conv1d_frag_bytes(), device=x.device, dtype=torch.uint8)
        _conv1_train_call(lib.t1policy_conv1d_pack_weights(weight.detach().contiguous().data_ptr(), frag.data_ptr(), C,
                                                           O, K, stream), "t1policy_conv1d_pack_weights")
        lout = (L - K) // 3 + 1
        y = torch.empty(B, lout, O, device=x.device, dtype=torch.float32)
        _conv1_train_call(lib.t1policy_conv1d_forward_packed(x.data_ptr(), frag.data_ptr(),
                                                             bias.detach().contiguous().data_ptr(), y.data_ptr(), B, C,
                                                             L, O, K, 3, stream), "t1policy_conv1d_forward_packed")
        ctx.save_for_backward(x)
        ctx.shape = (C, L, O, K)
        return y

    @staticmethod
    def backward(ctx, gy):
        from .. import _lib
        lib = _lib.load()
        x, = ctx.saved_tensors
        C, L, O, K = ctx.shape
        gy = gy.float().contiguous()
        stream = torch.cuda.current_stream(x.device).cuda_stream
        ws = torch.empty(lib.t1policy_conv1_bf16_workspace_bytes(), device=x.device, dtype=torch.uint8)
        gw = torch.empty(O, C, K, device=x.device, dtype=torch.float32)
        gb = torch.empty(O, device=x.device, dtype=torch.float32)
        _conv1_train_call(lib.t1policy_conv1_wgrad_f32(x.data_ptr(), gy.data_ptr(), ws.data_ptr(), gw.data_ptr(),
                                                       gb.data_ptr(), x.shape[0], C, L, O, K, 3, stream),
                          "t1policy_conv1_wgrad_f32")
        return None, gw, gb


def conv1d_train_f32(x, conv):
    """The first history conv of the fp32 update on an fp32 (B, 66, 47) input as the HIP kernels (channels-last (B, 14,
    32) fp32 out), or None when the conv or the input is not that shape (the caller keeps unfold + GEMM)."""
    if (conv.in_channels, conv.out_channels, conv.kernel_size[0], conv.stride[0]) != (66, 32, 6, 3) or \
            x.dim() != 3 or x.shape[1:] != (66, 47) or x.dtype != torch.float32 or conv.padding != (0,) or \
            conv.dilation != (1,) or conv.groups != 1 or conv.bias is None or conv.weight.dtype != torch.float32 or \
            torch.is_autocast_enabled("cuda"):
        return None
    x = x.contiguous()
    if x.data_ptr() % 16 != 0 or x.numel() * 4 >= 2 ** 31:
        return None
    return _HistoryConvF32.apply(x, conv.weight, conv.bias)


def _bf16_operands(x):
    """x reaches the conv's GEMM as bf16: already bf16 (the cast-once observations), or fp32 under a bf16 autocast."""
    if x.dtype == torch.bfloat16:
        return True
    return (x.dtype == torch.float32 and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16)


def conv1d_train_bf16(x, conv):
    """The first history conv of the update on a bf16 (B, 66, 47) input as the HIP kernels (channels-last (B, 14, 32)
    bf16 out), or None when the conv or the input is not that shape (the caller keeps unfold + GEMM)."""
    if (conv.in_channels, conv.out_channels, conv.kernel_size[0], conv.stride[0]) != (66, 32, 6, 3) or \
            x.dim() != 3 or x.shape[1:] != (66, 47) or x.dtype != torch.bfloat16 or conv.padding != (0,) or \
            conv.dilation != (1,) or conv.groups != 1 or conv.bias is None:
        return None
    x = x.contiguous()
    if x.data_ptr() % 4 != 0:
        return None
    return _HistoryConvBf16.apply(x, conv.weight, conv.bias)


def _heads_layers(ac):
    """The fused heads kernel's 15 layers in its parameter order (include/t1policy.h t1policy_heads_*): the history
    encoder's second conv and its two Linears, the state estimator's four, the actor's four, the critic's four.  None
    when the model is not built from those parts (ELU activations, ReLU after the convs, alpha 1)."""
    lin = lambda seq: [m for m in seq if isinstance(m, nn.Linear)]   # noqa: E731
    acts = [m for seq in (ac.actor, ac.critic, ac.state_estimator) for m in seq if not isinstance(m, nn.Linear)]
    if not all(isinstance(m, nn.ELU) and m.alpha == 1.0 for m in acts):
        return None
    lh = list(ac.long_history)
    convs = [m for m in lh if isinstance(m, nn.Conv1d)]
    if len(convs) != 2 or any(not isinstance(m, (nn.Conv1d, nn.ReLU, nn.Flatten, nn.Linear, nn.ELU)) for m in lh):
        return None
    layers = [convs[1], *lin(lh), *lin(ac.state_estimator), *lin(ac.actor), *lin(ac.critic)]
    return layers if len(layers) == 15 else None


def heads_forward(ac, obs, critic_obs, eps):
    """The rollout's act() after the first conv as the fused HIP kernel (t1policy_heads_forward): returns mean,
    actions = mean + std eps, sigma (B, 12), log-prob (B,) and value (B, 1) -- DHPPO._act_body's outputs -- or None
    when the model or inputs have no compiled instance (the caller keeps the torch path).  The weights are packed
    into the kernel's split fp16 fragments when a parameter changed (packed_heads_weights); a captured act() graph
    reads them in place and is refreshed before each replay."""
    from .. import _lib
    layers = _heads_layers(ac)
    if (layers is None or not obs.is_cuda or obs.dtype != torch.float32 or critic_obs.dtype != torch.float32
            or obs.dim() != 2 or critic_obs.dim() != 2 or eps.shape != (obs.shape[0], ac.std.numel())):
        return None
    # the kernel reads critic_obs and obs row by row up to the batch: shapes it was not built for are refused here,
    # not read out of bounds on the device
    if (critic_obs.shape[0] != obs.shape[0] or obs.shape[1] != ac.in_channels * ac.num_proprio_obs
            or critic_obs.shape[1] != layers[11].in_features):
        return None
    lib = _lib.load()
    if _heads_args(ac, layers) is None or ac.std.device != obs.device:
        return None
    dev = obs.device
    stream = torch.cuda.current_stream(dev).cuda_stream
    obs = obs.contiguous()
    B = obs.shape[0]
    y1 = conv1d_direct(obs.view(B, ac.in_channels, ac.num_proprio_obs), ac.long_history[0])
    if y1 is None:
        return None
    packed = packed_heads_weights(ac, stream)   # repacked only when a parameter changed
    if packed is None:
        return None
    frag, ptrs_c, dims_c = packed
    critic_obs, eps = critic_obs.contiguous(), eps.contiguous()
    na = ac.std.numel()
    mean = torch.empty(B, na, device=dev)
    actions, sigma = torch.empty_like(mean), torch.empty_like(mean)
    logp = torch.empty(B, device=dev)
    value = torch.empty(B, 1, device=dev)
    rc = lib.t1policy_heads_forward(ptrs_c, dims_c, frag.data_ptr(), y1.data_ptr(), obs.data_ptr(), obs.shape[1],
                                    critic_obs.data_ptr(), critic_obs.shape[1], eps.data_ptr(), mean.data_ptr(),
                                    actions.data_ptr(), sigma.data_ptr(), logp.data_ptr(), value.data_ptr(), B, stream)
    if rc == 1:
        return None
    if rc != 0:
        raise RuntimeError(f"t1policy_heads_forward failed (rc={rc})")
    return mean, actions, sigma, logp, value


# the unfolded rows' input gradient as the HIP gather (t1policy_fold_rows) instead of torch's unfold backward
# (T1_FOLD_ROWS=0: torch's, A/B)
FOLD_ROWS = os.environ.get("T1_FOLD_ROWS", "1") != "0"


class _UnfoldRows(torch.autograd.Function):
    """The (B * Lout, C * k) window rows of a channels-last (B, L, C) device tensor (x.unfold(1, k, st), copied); the
    backward is the HIP gather t1policy_fold_rows -- each input element sums its (at most k / st) window entries in
    fp32 and rounds once, bit-identical to torch's scatter-add when at most two windows meet (k = 4, st = 2 here)."""

    @staticmethod
    def forward(ctx, x, k, st):
        ctx.geom = (tuple(x.shape), k, st)
        win = x.unfold(1, k, st)
        B, Lout, C, _ = win.shape
        return win.reshape(B * Lout, C * k)

    @staticmethod
    def backward(ctx, g):
        from .. import _lib
        lib = _lib.load()
        (B, L, C), k, st = ctx.geom
        g = g.contiguous()
        gx = torch.empty(B, L, C, device=g.device, dtype=g.dtype)
        rc = lib.t1policy_fold_rows(g.data_ptr(), gx.data_ptr(), B, L, C, k, st, g.element_size(),
                                    torch.cuda.current_stream(g.device).cuda_stream)
        if rc != 0:
            raise RuntimeError(f"t1policy_fold_rows failed (rc={rc})")
        return gx, None, None


def conv1d_as_gemm(x, conv, channels_last=False):
    """nn.Conv1d (no padding / dilation / groups) as one GEMM over unfolded windows.  x: (B, C, L), or (B, L, C) with
    channels_last; returns (B, Lout, O) (channels last).  The windows x[b, :, s*l : s*l + k] become rows of a
    (B*Lout, C*k) matrix (c-major, then tap: the layout of conv.weight.view(O, C*k)), so the product is one
    hipBLASLt GEMM + bias, and autograd's unfold backward (a strided scatter-add) gives the input gradient."""
    k, st = conv.kernel_size[0], conv.stride[0]
    if (channels_last and FOLD_ROWS and x.is_cuda and torch.is_grad_enabled() and x.requires_grad
            and x.dtype in (torch.bfloat16, torch.float32)):
        rows = _UnfoldRows.apply(x, k, st)               # (B * Lout, C * k), the HIP gather as its backward
        B, Lout = x.shape[0], (x.shape[1] - k) // st + 1
        return _LinearSplitK.apply(rows, conv.weight.reshape(conv.out_channels, -1), conv.bias).view(B, Lout, -1)
    if channels_last:
        win = x.unfold(1, k, st)                      # (B, Lout, C, k)
    else:
        win = x.unfold(2, k, st).permute(0, 2, 1, 3)  # (B, C, Lout, k) -> (B, Lout, C, k)
    B, Lout, C, _ = win.shape
    rows = win.reshape(B * Lout, C * k)
    w = conv.weight.reshape(conv.out_channels, C * k)
    if torch.is_grad_enabled():   # split-K weight gradient (K = B * Lout rows)
        y = _LinearSplitK.apply(rows, w, conv.bias)
    else:
        y = torch.addmm(conv.bias, rows, w.t())
    return y.view(B, Lout, conv.out_channels)


class HistoryEncoder(nn.Sequential):
    """The reference's long-history CNN (actor_critic_dh.py:75-96): the same nn.Sequential layers and parameter
    names (so checkpoints load either way).  On the host the layers run as written (nn.Conv1d, bit-identical to the
    reference's CPU path); on the MI355X the two Conv1d run as unfold + GEMM (conv1d_as_gemm) with the activations
    kept channels-last: MIOpen's Conv1d kernels for this shape (66-channel, length-47 input, batch 49,152 in the PPO
    update) were the update's dominant cost.  Without autograd (the rollout's act()) the first conv is the HIP
    direct-conv kernel (conv1d_direct).  Same arithmetic up to fp32 summation order."""

    def forward(self, x):
        if not x.is_cuda:
            return super().forward(x)
        last = False   # x is (B, C, L) until the first conv; channels-last after it
        for m in self:
            if isinstance(m, nn.Conv1d):
                y = None
                if not last and not torch.is_grad_enabled() and x.dtype == torch.float32 and m.weight.dtype == x.dtype:
                    y = conv1d_direct(x, m)   # inference (the rollout's act()): the HIP direct conv
                elif not last and torch.is_grad_enabled() and CONV1_TRAIN and _bf16_operands(x):
                    # the bf16 update: the HIP forward + weight gradient on the bf16 operands autocast would make
                    y = conv1d_train_bf16(x.to(torch.bfloat16), m)
                elif not last and torch.is_grad_enabled() and CONV1_TRAIN and x.dtype == torch.float32:
                    # the fp32 update: the fp32-accurate HIP forward + three-part-split weight gradient
                    y = conv1d_train_f32(x, m)
                x = y if y is not None else conv1d_as_gemm(x, m, channels_last=last)
                last = True
            elif isinstance(m, nn.Flatten) and last:
                x = x.transpose(1, 2).reshape(x.shape[0], -1)   # (B, O, Lout) order, as nn.Flatten of NCL
                last = False
            else:
                x = m(x)
        return x


def _history_encoder(frames, features, filters, kernels, strides, code_dim):
    layers, ch, length = [], frames, features
    for out_ch, k, s in zip(filters, kernels, strides):
        layers += [nn.Conv1d(ch, out_ch, kernel_size=k, stride=s), nn.ReLU()]
        length = (length - k + s) // s  # the reference's length bookkeeping (equals floor((L - k) / s) + 1)
        ch = out_ch
    layers += [nn.Flatten(), Linear(length * ch, 128), nn.ELU(), Linear(128, code_dim)]
    return HistoryEncoder(*layers)


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
        self.validate_args = None
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

    def actor_input(self, observations, es_vel=None):
        """[short history | estimated base velocity | long-history code] (302 features); es_vel: the state estimator's
        output on this short history when the caller already has it."""
        short = observations[..., -self.num_short_obs:]
        code = self.long_history(observations.view(-1, self.in_channels, self.num_proprio_obs))
        return torch.cat((short, self.state_estimator(short) if es_vel is None else es_vel, code), dim=-1)

    def update_distribution(self, actor_obs):
        mean = self.actor(actor_obs).float()   # fp32 distribution under the opt-in bf16 update (no-op in fp32)
        # validate_args None = torch's default, as the reference; DHPPO.update turns it off on the device, where each
        # argument check is a host sync (it checks the losses' finiteness once per update instead)
        self.distribution = Normal(mean, mean * 0.0 + self.std, validate_args=self.validate_args)

    def act(self, observations, **kwargs):
        self.update_distribution(self.actor_input(observations))
        return self.distribution.sample()

    def get_actions_log_prob(self, actions):
        return self.distribution.log_prob(actions).sum(dim=-1)

    def act_inference(self, observations):
        return self.actor(self.actor_input(observations))

    def evaluate(self, critic_observations, **kwargs):
        return self.critic(critic_observations).float()
