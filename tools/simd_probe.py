"""Dev probe: the hardware SIMD of each k_dyn6 wave (a -DT1_PROBE_SIMD build records HW_ID per wave), and the step time.

    T1ENV_LIB=ti5_isaacgym_amd/_lib/var/libd6_simd.so python tools/simd_probe.py

Prints the step time over 200 steps and how the eight waves of each workgroup are dealt over its CU's four SIMDs.
"""
import collections
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ti5_isaacgym_amd import make_t1_env  # noqa: E402


def main():
    env = make_t1_env(num_envs=8192, mesh_type="trimesh", seed=5, device="cuda:0")
    env.reset()
    acts = torch.randn(8, 8192, 12, device="cuda:0")
    for i in range(30):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(200):
        env.step(acts[i % 8])
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 200 * 1e3
    lib = ctypes.CDLL(os.environ["T1ENV_LIB"])
    out = np.zeros((256, 8), np.uint32)
    rc = lib.t1env_debug_simd6(out.ctypes.data_as(ctypes.c_void_p), 256)
    simd = (out >> 4) & 3
    patterns = collections.Counter(tuple(int(x) for x in row) for row in simd)
    pair_w0 = collections.Counter(tuple(w for w in range(1, 8) if simd[b, w] == simd[b, 0]) for b in range(256))
    print(json.dumps({"ms_per_step": round(ms, 4), "rc": rc, "simd_patterns": {str(k): v for k, v in patterns.most_common(6)},
                      "waves_sharing_w0_simd": {str(k): v for k, v in pair_w0.most_common(6)},
                      "hw_id_block0": [hex(int(x)) for x in out[0]]}))


if __name__ == "__main__":
    main()
