"""Optimisation-level guard for the dynamics unit ("Compiler note").

The product library builds t1env_dynamics.hip at -O1 (fastest).  In round 1 the -O2/-O3 builds of the then
k_dynamics gave wrong dynamics; bisected with -opt-bisect-limit, the first wrong build is the one where the
AMDGPU load/store vectorizer runs on k_dynamics<plane>, and the same source at -O3 is correct with that pass off
or without `__restrict__` on the model pointer (profiles/r02k_opt_bisect.txt).  The current kernels are
correct at every level; this test keeps it that way: the -O3 guard build (__graft_entry__.build,
ti5_isaacgym_amd/_lib/var/libt1env_hip_dyn_o3.so) must pass the same one-step check against the fp64 host
replica (tests/test_gpu_dynamics.py) and the product-kernel replay through the oracle
(tests/test_gpu_product_parity.py, config 2 case).  The library is chosen at import time, so the checks run in
a child pytest process.
"""
import os
import subprocess
import sys

import pytest

from ti5_isaacgym_amd import build as _build

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_dynamics_o3_build_matches_fp64_host():
    lib = _build.OUT_O3
    assert os.path.exists(lib), f"-O3 guard build missing: {lib} (run __graft_entry__.build())"
    env = dict(os.environ, T1ENV_LIB=lib)
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
           "tests/test_gpu_dynamics.py", "tests/test_gpu_product_parity.py", "-k", "test_dynamics_one_step or config2"]
    r = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    print(r.stdout[-2000:])
    assert r.returncode == 0, f"-O3 dynamics build fails the dynamics checks:\n{r.stdout[-4000:]}\n{r.stderr[-2000:]}"
    assert " passed" in r.stdout and "failed" not in r.stdout
