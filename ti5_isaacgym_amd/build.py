"""Build libt1env_hip.so for gfx950 in-tree (the .so travels to the GPU box with the repo snapshot).

    python -m ti5_isaacgym_amd.build [--debug]
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# translation unit -> optimisation level.  k_dynamics is built at -O1: at -O2/-O3 the optimiser produced wrong
# dynamics for it (caught by tests/test_gpu_dynamics.py) and -O1 is also the fastest build of it.
UNITS = [("t1env.hip", "-O3"), ("t1env_dynamics.hip", "-O1")]
OUT = os.path.join(HERE, "_lib", "libt1env_hip.so")
DEPS = [os.path.join(CSRC, f) for f in ("t1env.hip", "t1env_dynamics.hip", "t1_dynamics.h", "t1_common.h", "t1env_post.h",
                                       "t1_model_conv.h", "t1env_device.h", "t1env_internal.h")] + \
    [os.path.join(os.path.dirname(HERE), "include", "t1env.h")]
ARCH = os.environ.get("T1ENV_ARCH", "gfx950")


def build(force=False, extra=(), out=None):
    out = out or OUT
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in DEPS):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    # -fno-slp-vectorize: the SLP pass packs scalar pairs of the dynamics into v_pk_* ops, which forces aligned
    # register pairs and piles up v_mov shuffles; in k_dynamics that alone turned ~40 scratch ops into ~470.
    common = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wno-unused-result", "-fno-slp-vectorize", *extra]
    objs = []
    for src, opt in UNITS:
        obj = os.path.join(os.path.dirname(out), os.path.splitext(src)[0] + ".o")
        subprocess.run([hipcc, opt, *common, "-c", "-o", obj, os.path.join(CSRC, src)], check=True)
        objs.append(obj)
    subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp", *objs], check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force=True, extra=[a for a in sys.argv[1:] if a.startswith("-")]))
