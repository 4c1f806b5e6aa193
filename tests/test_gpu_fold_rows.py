"""The history encoder's second conv in the update: the unfolded rows' input gradient as the HIP gather
(t1policy_fold_rows, dh_policy._UnfoldRows) against torch's unfold backward -- needs the MI355X.  At kernel 4 /
stride 2 at most two windows meet at an input element, so the fp32 sum rounded once is bit-identical to torch's
zero-filled scatter-add, in bf16 and fp32."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32], ids=["bf16", "fp32"])
@pytest.mark.parametrize("batch,length,ch,k,st", [(1, 14, 32, 4, 2), (4099, 14, 32, 4, 2), (9000, 14, 32, 4, 2),
                                                   (37, 15, 24, 4, 2), (37, 14, 5, 2, 2)])
def test_fold_rows_is_torchs_unfold_backward(dtype, batch, length, ch, k, st):
    """The compiled kernel-4 / stride-2 instance (channels dividing 256, batch past the 8192-workgroup grid) and the
    generic one (24 channels; kernel 2)."""
    from ti5_isaacgym_amd.algo.dh_policy import _UnfoldRows
    g = torch.Generator(device=DEV).manual_seed(batch)
    x = torch.randn(batch, length, ch, device=DEV, generator=g).to(dtype)
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    rows = _UnfoldRows.apply(x1, k, st)
    lout = (length - k) // st + 1
    ref = x2.unfold(1, k, st).reshape(batch * lout, ch * k)
    assert torch.equal(rows, ref)
    gr = torch.randn(rows.shape, device=DEV, generator=g).to(dtype)
    rows.backward(gr)
    ref.backward(gr)
    assert x1.grad.dtype == dtype and torch.equal(x1.grad, x2.grad)


def test_history_encoder_grads_unchanged_by_the_gather(monkeypatch):
    """The whole history encoder under the bf16 update's autocast: every parameter gradient is the same bits with the
    gather and with torch's unfold backward."""
    from ti5_isaacgym_amd.algo import dh_policy
    torch.manual_seed(0)
    ac = dh_policy.ActorCriticDH(235, 47, 219, 12).to(DEV)
    obs = torch.randn(2048, 66, 47, device=DEV).to(torch.bfloat16)

    def grads(flag):
        monkeypatch.setattr(dh_policy, "FOLD_ROWS", flag)
        ac.zero_grad(set_to_none=True)
        with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
            code = ac.long_history(obs)
        code.float().square().sum().backward()
        return [p.grad.clone() for p in ac.long_history.parameters()]

    a, b = grads(True), grads(False)
    assert all(torch.equal(u, v) for u, v in zip(a, b))
