"""Dev check: a numpy emulation of t1policy_heads.hip's fragment algebra (pack order, natural / permuted k-steps,
the v_mfma_f32_32x32x16_f16 lane maps of the CDNA guide, accumulator tiles as the next layer's B operand), in fp64
without the fp16 split, against the torch fp64 forward of the same ActorCriticDH.  Finds index bugs on the CPU.

    python tools/heads_emulate.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (n, k, ks, act, segs[(s0, steps, col0, len, perm)]) -- PH_L of t1policy_heads.hip
L = [
    (96, 128, 28, "relu", [(0, 28, 0, 448, 0)]),
    (128, 96, 6, "elu", [(0, 6, 0, 96, 1)]),
    (64, 128, 8, None, [(0, 8, 0, 128, 1)]),
    (256, 235, 15, "elu", [(0, 15, 0, 235, 0)]),
    (128, 256, 16, "elu", [(0, 16, 0, 256, 1)]),
    (64, 128, 8, "elu", [(0, 8, 0, 128, 1)]),
    (3, 64, 4, None, [(0, 4, 0, 64, 1)]),
    (512, 302, 20, "elu", [(0, 15, 0, 235, 0), (15, 1, 235, 3, 1), (16, 4, 238, 64, 1)]),
    (256, 512, 32, "elu", [(0, 32, 0, 512, 1)]),
    (128, 256, 16, "elu", [(0, 16, 0, 256, 1)]),
    (12, 128, 8, None, [(0, 8, 0, 128, 1)]),
    (768, 219, 14, "elu", [(0, 14, 0, 219, 0)]),
    (256, 768, 48, "elu", [(0, 48, 0, 768, 1)]),
    (128, 256, 16, "elu", [(0, 16, 0, 256, 1)]),
    (1, 128, 8, None, [(0, 8, 0, 128, 1)]),
]


def col(l, s, h, j):
    for s0, steps, c0, ln, perm in L[l][4]:
        if s0 <= s < s0 + steps:
            r = 16 * (s - s0) + (8 * (j >> 2) + 4 * h + (j & 3) if perm else 8 * h + j)
            return c0 + r if r < ln else -1
    return -1


def weight(W, l, o, c):
    if l == 0:
        oc, lp, p, ch = o // 6, o % 6, c >> 5, c & 31
        t = p - 2 * lp
        return W[oc, ch, t] if 0 <= t < 4 else 0.0
    return W[o, c]


def pack(l, W):
    """A fragments [nt][s][lane][j] of layer l."""
    n, _, ks = L[l][:3]
    nt_ = (n + 31) // 32
    A = np.zeros((nt_, ks, 64, 8))
    for nt in range(nt_):
        for s in range(ks):
            for lane in range(64):
                o, h = 32 * nt + (lane & 31), lane >> 5
                for j in range(8):
                    c = col(l, s, h, j)
                    if o < n and c >= 0:
                        A[nt, s, lane, j] = weight(W, l, o, c)
    return A


def mfma(a, b, acc):
    """v_mfma_f32_32x32x16: a, b [64 lanes][8]; A[i][8h + j] = a[lane (i, h)][j], B[8h + j][c] = b[lane (c, h)][j];
    acc [64][16] in the C/D map row = (r & 3) + 8 (r >> 2) + 4 h, col = lane & 31."""
    Am = np.zeros((32, 16))
    Bm = np.zeros((16, 32))
    for lane in range(64):
        i, h = lane & 31, lane >> 5
        Am[i, 8 * h:8 * h + 8] = a[lane]
        Bm[8 * h:8 * h + 8, i] = b[lane]
    D = Am @ Bm
    out = acc.copy()
    for lane in range(64):
        h = lane >> 5
        for r in range(16):
            out[lane, r] += D[(r & 3) + 8 * (r >> 2) + 4 * h, lane & 31]
    return out


def stage(x, steps, col0, ln, relu=False):
    """natural B fragments [s][lane][j] from rows x [32][*]."""
    F = np.zeros((steps, 64, 8))
    for s in range(steps):
        for lane in range(64):
            r, h = lane & 31, lane >> 5
            for j in range(8):
                c = 16 * s + 8 * h + j
                if c < ln:
                    v = x[r, col0 + c]
                    F[s, lane, j] = max(v, 0.0) if relu else v
    return F


def act(v, a):
    if a == "relu":
        return np.maximum(v, 0.0)
    if a == "elu":
        return np.where(v > 0, v, np.expm1(v))
    return v


def layer(l, A, bias, inp, out, out0, half=False):
    n, _, ks, a, _ = L[l]
    nt_ = (n + 31) // 32
    res = []
    for nt in range(nt_):
        acc = np.zeros((64, 16))
        for s in range(ks):
            acc = mfma(A[nt, s], inp[s], acc)
        v = np.zeros((64, 16))
        for lane in range(64):
            h = lane >> 5
            for r in range(16):
                row = 32 * nt + (r & 3) + 8 * (r >> 2) + 4 * h
                v[lane, r] = act(acc[lane, r] + (bias[row // 6 if l == 0 else row] if row < n else 0.0), a)
        if out is not None:
            for s in range(1 if half else 2):
                out[out0 + 2 * nt + s] = v[:, 8 * s:8 * s + 8]
        res.append(v)
    return res


def emulate_errors(seed=0):
    """Max |emulated - torch fp64| of the action mean and the value for 32 random envs."""
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH, _heads_layers
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    torch.manual_seed(seed)
    ac = ActorCriticDH(235, 47, 219, 12, **class_to_dict(tc)["policy"]).double()
    layers = _heads_layers(ac)
    Ws = [m.weight.detach().numpy() for m in layers]
    bs = [m.bias.detach().numpy() for m in layers]
    As = [pack(l, Ws[l]) for l in range(15)]
    g = torch.Generator().manual_seed(1)
    obs = torch.randn(32, 66 * 47, generator=g, dtype=torch.float64)
    cobs = torch.randn(32, 219, generator=g, dtype=torch.float64)
    with torch.no_grad():
        y1 = ac.long_history[0](obs.view(32, 66, 47)).permute(0, 2, 1).reshape(32, 448).numpy()  # channels-last
        mean_ref = ac.actor(ac.actor_input(obs)).numpy()
        val_ref = ac.critic(cobs).numpy()
    on = obs.numpy()
    X = np.zeros((20, 64, 8))
    P = np.zeros((48, 64, 8))
    Q = np.zeros((16, 64, 8))
    P[:28] = stage(y1, 28, 0, 448, relu=True)
    X[:15] = stage(on, 15, 3102 - 235, 235)
    layer(0, As[0], bs[0], P, Q, 0)
    layer(1, As[1], bs[1], Q, P, 0)
    layer(2, As[2], bs[2], P, X, 16)
    layer(3, As[3], bs[3], X, Q, 0)
    layer(4, As[4], bs[4], Q, P, 0)
    layer(5, As[5], bs[5], P, Q, 0)
    layer(6, As[6], bs[6], Q, X, 15, half=True)
    layer(7, As[7], bs[7], X, P, 0)
    layer(8, As[8], bs[8], P, Q, 0)
    layer(9, As[9], bs[9], Q, P, 0)
    v = layer(10, As[10], bs[10], P, None, 0)[0]
    mean = np.zeros((32, 12))
    for lane in range(64):
        h = lane >> 5
        for r in range(16):
            row = (r & 3) + 8 * (r >> 2) + 4 * h
            if row < 12:
                mean[lane & 31, row] = v[lane, r]
    Q2 = np.zeros((16, 64, 8))
    P2 = np.zeros((48, 64, 8))
    Q2[:14] = stage(cobs.numpy(), 14, 0, 219)
    layer(11, As[11], bs[11], Q2, P2, 0)
    layer(12, As[12], bs[12], P2, Q2, 0)
    layer(13, As[13], bs[13], Q2, P2, 0)
    vv = layer(14, As[14], bs[14], P2, None, 0)[0]
    value = vv[:32, 0]
    return np.abs(mean - mean_ref).max(), np.abs(value - val_ref[:, 0]).max()


if __name__ == "__main__":
    em, ev = emulate_errors()
    print("mean max err", em, "value max err", ev)
