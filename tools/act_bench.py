"""Dev probe: the rollout's act() (DHPPO.act: policy sample, value, log-prob as one replayed HIP graph) at N envs on
random observations, fused HIP heads vs torch's layers (T1_FUSED_ACT is read at import; --torch flips it here).

    python tools/act_bench.py [--num-envs 8192] [--iters 200] [--torch]

Prints one JSON line: wall ms per act() (graph replays back to back, one sync at the end), and the heads kernel's own
duration from HIP events around the fused call when it runs eagerly.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--num-envs", type=int, default=8192)
    p.add_argument("--iters", type=int, default=200)
    p.add_argument("--torch", action="store_true")
    a = p.parse_args()
    from ti5_isaacgym_amd import task_registry
    from ti5_isaacgym_amd.algo import dh_update
    from ti5_isaacgym_amd.algo.dh_policy import ActorCriticDH
    from ti5_isaacgym_amd.utils.helpers import class_to_dict
    dh_update.FUSED_ACT = not a.torch
    _, tc = task_registry.get_cfgs("t1_dh_stand")
    cfg = class_to_dict(tc)
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    ac = ActorCriticDH(235, 47, 219, 12, **cfg["policy"]).to(dev)
    alg = dh_update.DHPPO(ac, device=str(dev), **cfg["algorithm"])
    n = a.num_envs
    obs = torch.randn(n, 66 * 47, device=dev).clamp(-18, 18)
    cobs = torch.randn(n, 219, device=dev)
    out = {"num_envs": n, "path": "torch" if a.torch else "fused"}
    with torch.inference_mode():
        for _ in range(5):
            alg.act(obs, cobs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.iters):
            alg.act(obs, cobs)
        torch.cuda.synchronize()
        out["act_ms"] = round((time.perf_counter() - t0) / a.iters * 1e3, 4)
        out["graphed"] = bool(alg._act_graphs)
        # the eager body, bracketed by events (conv + pack + heads + randn for the fused path)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            alg._act_body(obs, cobs)
        e1.record()
        torch.cuda.synchronize()
        out["act_body_eager_ms"] = round(e0.elapsed_time(e1) / 50, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
