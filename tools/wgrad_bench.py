"""Per-layer timing of the bf16 update's Linear weight + bias gradients: the HIP kernel (t1policy_linear_wgrad_bf16)
against the split-K batched GEMM + slice sum + torch's bias sum it replaces, on the update's layer shapes at the
49,152-row minibatch.  Prints one JSON line.

    python tools/wgrad_bench.py [--reps 20] [--f32]

--f32: the fp32 update's kernel (t1policy_linear_wgrad_f32, three-part bf16 split) against the fp32 split-K path.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd.algo import dh_policy  # noqa: E402

# (rows, outputs M, inputs N) of every Linear in one minibatch's backward (actor_critic_dh.py:45-111), the second
# history conv as its GEMM
LAYERS = [(294912, 16, 128), (49152, 128, 96), (49152, 64, 128),
          (49152, 256, 235), (49152, 128, 256), (49152, 64, 128), (49152, 3, 64),
          (49152, 512, 302), (49152, 256, 512), (49152, 128, 256), (49152, 12, 128),
          (49152, 768, 219), (49152, 256, 768), (49152, 128, 256), (49152, 1, 128)]


def timed(fn, reps):
    for _ in range(3):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3   # us


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--f32", action="store_true")
    a = p.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    rows_out, tot_new, tot_old = [], 0.0, 0.0
    for rows, M, N in LAYERS:
        dt = torch.float32 if a.f32 else torch.bfloat16
        gy = (torch.randn(rows, M, device=dev, generator=g) * 0.1).to(dt)
        x = torch.randn(rows, N, device=dev, generator=g).to(dt)
        kern = dh_policy.linear_wgrad_f32 if a.f32 else dh_policy.linear_wgrad_bf16
        t_new = timed(lambda: kern(gy, x), a.reps)
        t_old = timed(lambda: (dh_policy.wgrad_splitk(gy, x), dh_policy.bias_grad(gy)), a.reps)
        flops = 2.0 * rows * M * N
        row = {"rows": rows, "M": M, "N": N, "us_kernel": round(t_new, 2), "us_splitk": round(t_old, 2),
               "tflops_kernel": round(flops / t_new * 1e-6, 1)}
        if a.f32:   # the same layer's forward (x W^T + b) and input gradient (gy W): the HIP GEMM against torch's
            w = torch.randn(M, N, device=dev, generator=g) * 0.05
            b = torch.randn(M, device=dev, generator=g)
            row["us_fwd_gemm"] = round(timed(lambda: dh_policy.gemm_nt_f32(x, w, b), a.reps), 2)
            row["us_fwd_addmm"] = round(timed(lambda: torch.addmm(b, x, w.t()), a.reps), 2)
            row["us_dgrad_gemm"] = round(timed(lambda: dh_policy.gemm_nt_f32(gy, w.t()), a.reps), 2)
            row["us_dgrad_mm"] = round(timed(lambda: gy.mm(w), a.reps), 2)
        rows_out.append(row)
        tot_new += t_new
        tot_old += t_old
    print(json.dumps({"bench": "linear_wgrad_f32" if a.f32 else "linear_wgrad_bf16",
                      "wg_per_cu": os.environ.get("T1_WGRAD_WG_PER_CU", "2"), "layers": rows_out, "us_per_minibatch_kernel": round(tot_new, 1),
                      "us_per_minibatch_splitk": round(tot_old, 1)}))


if __name__ == "__main__":
    main()
