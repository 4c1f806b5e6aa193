"""Dev probe: per-launch HIP-event times of the step's parts, with the history shift as its own launch
(T1ENV_SHIFT_BLOCKS=-1 is set here): fused (dynamics + post-physics epilogue in one launch) and split (dynamics
launch, then k_post_a / k_post_b).  fused - split dynamics = what the in-launch epilogue adds.

    python tools/split_timing.py [--num-envs 8192] [--mesh trimesh] [--steps 200]
"""
import argparse
import json
import os
import sys

os.environ.setdefault("T1ENV_SHIFT_BLOCKS", "-1")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--num-envs", type=int, default=8192)
    p.add_argument("--mesh", default="trimesh")
    p.add_argument("--steps", type=int, default=200)
    a = p.parse_args()
    import torch
    from ti5_isaacgym_amd import make_t1_env
    env = make_t1_env(num_envs=a.num_envs, mesh_type=a.mesh, seed=5, device="cuda:0")
    env.reset()
    g = torch.Generator(device="cuda:0").manual_seed(0)
    acts = [torch.randn(a.num_envs, 12, device="cuda:0", generator=g) for _ in range(8)]
    out = {"num_envs": a.num_envs, "mesh": a.mesh, "lib": os.environ.get("T1ENV_LIB", "product")}
    for mode in ("fused", "split"):
        env.set_fused(mode == "fused")
        for i in range(30):
            env.step(acts[i % 8])
        torch.cuda.synchronize()
        env.set_timing(True)
        for i in range(a.steps):
            env.step(acts[i % 8])
        torch.cuda.synchronize()
        t = env.get_timing()
        env.set_timing(False)
        out[mode] = {k: round(v["ms"] / v["launches"] * 1e3, 2) for k, v in t.items() if v["launches"]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
