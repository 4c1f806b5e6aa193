"""The HIP gather of the PPO minibatch rows from the frame-history rollout storage (include/t1policy.h
t1policy_history_rows) against the torch restatement of the same rows (algo/rollout.py _HistoryRows on the host),
bit for bit, in fp32 and bf16, with resets inside the rollout and indices covering every step."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("frames", [66, 3])   # even row length (32-bit word copy), odd (one element per lane)
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16], ids=["fp32", "bf16"])
def test_history_rows_kernel_matches_torch(dtype, frames):
    from ti5_isaacgym_amd.algo.rollout import RolloutStorage
    N, T, frame = 333, 24, 47
    g = torch.Generator().manual_seed(4)
    stores = {}
    for dev in ("cpu", "cuda:0"):
        st = RolloutStorage(N, T, [frame * frames], [219], [12], device=dev, history=(frame, frames))
        stores[dev] = st
    obs0 = torch.randn(N, frame * frames, generator=g)
    fr = torch.randn(T, N, frame, generator=g)
    dones = (torch.rand(T, N, 1, generator=g) < 0.07).to(torch.uint8)
    for dev, st in stores.items():
        st.obs0.copy_(obs0)
        st.frames.copy_(fr)
        st.dones.copy_(dones)
        st.step = T
    src = {dev: st.minibatch_source(dtype if dtype != torch.float32 else None) for dev, st in stores.items()}
    idx = torch.cat([torch.randperm(N * T, generator=g), torch.tensor([0, N * T - 1, N - 1, N])])
    ref = src["cpu"](idx)[0]
    got = src["cuda:0"](idx.to("cuda:0"))[0].cpu()
    assert got.dtype == ref.dtype == dtype
    assert torch.equal(got, ref)
    assert bool((dones[:-1] > 0).any())   # resets inside the rollout are exercised


def test_field_gather_is_torch_indexing():
    """The minibatch's per-transition fields by one launch (t1policy_gather_rows, rollout._FieldGather) == torch's
    index of each field, bit for bit; a field it cannot take (fp16) keeps torch's path."""
    from ti5_isaacgym_amd.algo.rollout import _FieldGather
    g = torch.Generator(device="cuda:0").manual_seed(3)
    rows = 24 * 333
    fields = [torch.randn(rows, w, device="cuda:0", generator=g) for w in (219, 12, 1, 1, 1, 1, 12, 12)]
    idx = torch.randperm(rows, device="cuda:0", generator=g)[:4097]
    got = _FieldGather(fields)(idx)
    assert all(torch.equal(a, f[idx]) for a, f in zip(got, fields))
    half = _FieldGather([fields[0].half(), fields[1]])
    assert not half.ok and all(torch.equal(a, f[idx]) for a, f in zip(half(idx), [fields[0].half(), fields[1]]))
