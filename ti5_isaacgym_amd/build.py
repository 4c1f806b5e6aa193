"""Build libt1env_hip.so for gfx950 in-tree (the .so travels to the GPU box with the repo snapshot).

    python -m ti5_isaacgym_amd.build [--out=PATH] [--dyn-opt=-O3] [extra hipcc flags]
"""
import glob
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# translation unit -> optimisation level.  The dynamics unit is built at -O1 (round 1's fastest level; on the round-2
# kernel -O1/-O2/-O3 measure the same, profiles/r02bc_opt_levels.json).  Round 1's -O2/-O3 wrong dynamics bisected to the load/store vectorizer over the __restrict__
# model-pointer loads; the -O3 guard build (OUT_O3) keeps every level under the fp64 check.
UNITS = [("t1env.hip", "-O3"), ("t1env_dynamics.hip", "-O1"), ("t1env_dyn5.hip", "-O1"), ("t1env_dyn6.hip", "-O1"),
         ("t1policy.hip", "-O3"),
         ("t1policy_heads.hip", "-O3"), ("t1policy_train.hip", "-O3"),
         ("t1policy_wgrad.hip", "-O3"), ("t1policy_gemm.hip", "-O3")]
OUT = os.path.join(HERE, "_lib", "libt1env_hip.so")
# guard build: the dynamics unit at -O3 (tests/test_gpu_opt_levels.py keeps it under the fp64 dynamics check)
OUT_O3 = os.path.join(HERE, "_lib", "var", "libt1env_hip_dyn_o3.so")
# every source and header the units include (a hand-kept list missed t1env_postphys.h)
DEPS = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.h")) +
              glob.glob(os.path.join(os.path.dirname(HERE), "include", "*.h")))
ARCH = os.environ.get("T1ENV_ARCH", "gfx950")


def source_stamp():
    """A hash of every source and header the library is built from (DEPS), compiled into t1env_version() so that
    _lib.load() refuses a library built from other sources (a stale guard library failed with an undefined
    symbol instead of a clear message)."""
    import hashlib
    h = hashlib.sha256()
    for d in DEPS:
        h.update(os.path.basename(d).encode() + b"\0")
        with open(d, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


def build(force=False, extra=(), out=None, dyn_opt=None):
    """dyn_opt: optimisation level of the dynamics unit for A/B and guard variants (default -O1)."""
    out = out or OUT
    if not force and os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in DEPS):
        return out
    os.makedirs(os.path.dirname(out), exist_ok=True)
    hipcc = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")
    # -fno-slp-vectorize: the SLP pass packs scalar pairs of the dynamics into v_pk_* ops, which forces aligned
    # register pairs and piles up v_mov shuffles; in k_dynamics that alone turned ~40 scratch ops into ~470.
    common = [f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-Wno-unused-result", "-fno-slp-vectorize",
              f'-DT1_SOURCE_STAMP="{source_stamp()}"', *extra]
    objs, procs = [], []
    for src, opt in UNITS:  # the units compile concurrently
        if dyn_opt and src in ("t1env_dynamics.hip", "t1env_dyn5.hip", "t1env_dyn6.hip"):
            opt = dyn_opt
        obj = os.path.join(os.path.dirname(out), os.path.splitext(src)[0] + ".o")
        procs.append(subprocess.Popen([hipcc, opt, *common, "-c", "-o", obj, os.path.join(CSRC, src)]))
        objs.append(obj)
    failed = [pr for pr in procs if pr.wait() != 0]   # wait for every unit before reporting a failure
    if failed:
        raise subprocess.CalledProcessError(failed[0].returncode, failed[0].args)
    subprocess.run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp", *objs], check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    args = sys.argv[1:]
    out = next((a.split("=", 1)[1] for a in args if a.startswith("--out=")), None)
    dyn_opt = next((a.split("=", 1)[1] for a in args if a.startswith("--dyn-opt=")), None)
    print(build(force=True, out=out, dyn_opt=dyn_opt,
                extra=[a for a in args if a.startswith("-") and not a.startswith(("--out=", "--dyn-opt="))]))
