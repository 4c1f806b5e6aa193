"""Time the policy history conv kernels (include/t1policy.h) at the rollout's batch: the tap-major k_conv1d_mfma
(t1policy_conv1d_forward) against the packed-fragment k_conv1d_regs (t1policy_conv1d_pack_weights +
t1policy_conv1d_forward_packed), HIP events around each launch on one stream, and each against torch's fp64 conv.

    python tools/conv_bench.py [--batch 8192] [--iters 200] [--out gpurun_out/conv.json]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd import _lib  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--batch", type=int, default=8192)
p.add_argument("--iters", type=int, default=200)
p.add_argument("--out", default=None)
a = p.parse_args()

lib = _lib.load()
dev = torch.device("cuda:0")
torch.manual_seed(0)
conv = nn.Conv1d(66, 32, kernel_size=6, stride=3).to(dev)
B = a.batch
x = torch.randn(B, 66, 47, device=dev)
w = conv.weight.detach().contiguous()
wt = w.permute(1, 2, 0).contiguous()
bias = conv.bias.detach().contiguous()
frag = torch.empty(lib.t1policy_conv1d_frag_bytes(), device=dev, dtype=torch.uint8)
s = torch.cuda.current_stream(dev)
sp = s.cuda_stream
y_old = torch.empty(B, 14, 32, device=dev)
y_new = torch.empty(B, 14, 32, device=dev)


def old():
    assert lib.t1policy_conv1d_forward(x.data_ptr(), wt.data_ptr(), bias.data_ptr(), y_old.data_ptr(), B, 66, 47, 32,
                                       6, 3, sp) == 0


def pack():
    assert lib.t1policy_conv1d_pack_weights(w.data_ptr(), frag.data_ptr(), 66, 32, 6, sp) == 0


def new():
    assert lib.t1policy_conv1d_forward_packed(x.data_ptr(), frag.data_ptr(), bias.data_ptr(), y_new.data_ptr(), B, 66,
                                              47, 32, 6, 3, sp) == 0


def timed(fn, iters):
    for _ in range(10):
        fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for e0, e1 in ev:
        e0.record(s)
        fn()
        e1.record(s)
    torch.cuda.synchronize()
    t = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in ev)
    return {"median_us": t[len(t) // 2], "min_us": t[0], "mean_us": sum(t) / len(t)}


pack()
old()
new()
torch.cuda.synchronize()
with torch.no_grad():
    ref = nn.functional.conv1d(x.double(), w.double(), bias.double(), stride=3).transpose(1, 2)
res = {"batch": B, "bytes_in": B * 66 * 47 * 4, "bytes_out": B * 14 * 32 * 4}
for name, y in (("old", y_old), ("packed", y_new)):
    err = ((y.double() - ref).abs() / (1 + ref.abs())).max().item()
    res[name + "_max_rel_err"] = err
res["old"] = timed(old, a.iters)
res["pack"] = timed(pack, a.iters)
res["packed"] = timed(new, a.iters)   # k_conv1d_pair (default)
os.environ["T1POLICY_CONV"] = "regs"
new()
torch.cuda.synchronize()
res["packed_regs_max_rel_err"] = ((y_new.double() - ref).abs() / (1 + ref.abs())).max().item()
res["packed_regs"] = timed(new, a.iters)
del os.environ["T1POLICY_CONV"]
for k in ("old", "packed", "packed_regs"):
    res[k]["GBs"] = (res["bytes_in"] + res["bytes_out"]) / (res[k]["median_us"] * 1e-6) / 1e9
print(json.dumps(res))
if a.out:
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
