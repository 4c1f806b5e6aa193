"""Dev probe: host and device time of the split-K weight-gradient GEMM (dh_policy.wgrad_splitk's shape: K = 49,152
batch rows in slices of 2048, M x N = 512 x 256) in fp32 and bf16 through the BLAS routes PyTorch offers on ROCm.

    python tools/bf16_wgrad_probe.py [--small-m]

--small-m: the heads' weight gradients (M = 1, 3, 12 outputs, N = 64 / 128 inputs, K = 49,152 rows), which
wgrad_splitk routes through one fp32 GEMM under the bf16 update: that GEMM against split-K variants.

Per variant: wall time of 50 back-to-back calls with a sync only at the end (host-bound if the per-call host time
exceeds the device time) and the host time of the enqueue loop alone.
"""
import time

import torch


def run(name, fn, n=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name:44s} enqueue {(t1 - t0) / n * 1e6:8.1f} us/call   wall {(t2 - t0) / n * 1e6:8.1f} us/call", flush=True)


def small_m():
    K = 49152
    for M, N in ((3, 64), (1, 128), (12, 128)):
        for dt in (torch.float32, torch.bfloat16):
            gy = torch.randn(K, M, device="cuda", dtype=dt)
            x = torch.randn(K, N, device="cuda", dtype=dt)
            gw, xw = gy.float(), x.float()
            tag = f"M={M:2d} N={N:3d} {str(dt).split('.')[-1]}"
            run(f"{tag} widen + mm", lambda: gw.t().mm(xw) if dt == torch.float32 else gy.float().t().mm(x.float()))
            for R in (2048, 8192):
                S = K // R
                run(f"{tag} widen + bmm R={R} + sum",
                    lambda: torch.bmm(gy.float().view(S, R, M).transpose(1, 2), x.float().view(S, R, N)).sum(0))
            run(f"{tag} widen + x^T gy (N x M) ^T", lambda: x.float().t().mm(gy.float()).t())
            if M <= 3:
                run(f"{tag} broadcast-multiply + sum",
                    lambda: (gy.float().unsqueeze(2) * x.float().unsqueeze(1)).sum(0))


def main():
    import sys
    if "--small-m" in sys.argv:
        return small_m()
    K, M, N, R = 49152, 512, 256, 2048
    S = K // R
    for dt in (torch.float32, torch.bfloat16):
        gy = torch.randn(K, M, device="cuda", dtype=dt)
        x = torch.randn(K, N, device="cuda", dtype=dt)
        a, b = gy.view(S, R, M).transpose(1, 2), x.view(S, R, N)
        tag = str(dt).split(".")[-1]
        for lib in ("cublaslt", "cublas"):
            torch.backends.cuda.preferred_blas_library(lib)
            run(f"{tag} {lib} bmm+sum", lambda: torch.bmm(a, b).float().sum(0))
            run(f"{tag} {lib} mm", lambda: gy.t().mm(x))
            if dt == torch.bfloat16:
                run(f"{tag} {lib} bmm out fp32 +sum", lambda: torch.bmm(a, b, out_dtype=torch.float32).sum(0))
                run(f"{tag} {lib} mm out fp32", lambda: torch.mm(gy.t(), x, out_dtype=torch.float32))
                ac = a.contiguous()
                run(f"{tag} {lib} bmm contig-A +sum", lambda: torch.bmm(ac, b).float().sum(0))
    torch.backends.cuda.preferred_blas_library("cublaslt")


if __name__ == "__main__":
    main()
