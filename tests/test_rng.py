"""The counter RNG: the kernels' copy (ti5_isaacgym_amd/csrc/t1_common.h, compiled here for the host with g++) vs the
oracle's (oracle/rng.py), which the golden harness routes the reference's own draw sites through.

Every draw of the step (DR, lags, commands, pushes, observation noise, torque multipliers) is one of hash4 /
uniform01 / rand_float / rand_int, keyed directly or through rng_key + hash_k; all must agree bit for bit, including
the between-step key domain (BETWEEN_STEP_SALT) and counters past 2**31.
"""
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

from oracle import rng as R

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ti5_isaacgym_amd", "csrc")
PROG = r"""
#include <stdio.h>
#include "t1_common.h"
using namespace t1;
int main() {
  unsigned seed, env, ctr, slot; float lo, hi; int ilo, ihi;
  while (scanf("%u %u %u %u %f %f %d %d", &seed, &env, &ctr, &slot, &lo, &hi, &ilo, &ihi) == 8) {
    const RngKey K = rng_key(seed, env, ctr);
    printf("%u %u %a %a %a %d %d\n", hash4(seed, env, ctr, slot), hash_k(K, slot), uniform01(seed, env, ctr, slot),
           rand_float(lo, hi, seed, env, ctr, slot), rand_float(lo, hi, K, slot), rand_int(ilo, ihi, seed, env, ctr, slot),
           rand_int(ilo, ihi, K, slot));
  }
  return 0;
}
"""


@pytest.fixture(scope="module")
def host_rng():
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    d = tempfile.mkdtemp()
    src, exe = os.path.join(d, "rng.cpp"), os.path.join(d, "rng")
    open(src, "w").write(PROG)
    subprocess.run([gxx, "-O2", "-std=c++17", "-ffp-contract=off", "-I", CSRC, src, "-o", exe], check=True)
    yield exe
    shutil.rmtree(d, ignore_errors=True)


def test_device_rng_equals_oracle(host_rng):
    rng = np.random.default_rng(3)
    n = 4000
    seed = rng.integers(0, 2**32, n, dtype=np.uint64)
    seed[:100] = 5
    env = rng.integers(0, 1 << 20, n, dtype=np.uint64)
    ctr = rng.integers(0, 1 << 32, n, dtype=np.uint64)
    ctr[:500] = rng.integers(0, 200000, 500)
    ctr[500:1000] = ctr[:500] | R.BETWEEN_STEP_SALT
    slot = rng.choice([1000, 1011, 2000, 3100, 3102, 4000, 4046, 5000, 5400, 5900, 5910, 6000, 6050], n).astype(np.uint64)
    lo = rng.uniform(-3, 0, n).astype(np.float32)
    hi = (lo + rng.uniform(0.01, 3, n)).astype(np.float32)
    ilo = rng.integers(-5, 5, n)
    ihi = ilo + rng.integers(1, 300, n)
    lines = "\n".join(f"{a} {b} {c} {d} {e!r} {f!r} {g} {h}"
                      for a, b, c, d, e, f, g, h in zip(seed, env, ctr, slot, lo.tolist(), hi.tolist(), ilo, ihi))
    out = subprocess.run([host_rng], input=lines, capture_output=True, text=True, check=True).stdout.split("\n")
    rows = [ln.split() for ln in out if ln]
    assert len(rows) == n
    h4 = np.array([int(r[0]) for r in rows], np.uint64)
    hk = np.array([int(r[1]) for r in rows], np.uint64)
    u = np.array([float.fromhex(r[2]) for r in rows], np.float32)
    rf = np.array([float.fromhex(r[3]) for r in rows], np.float32)
    rfk = np.array([float.fromhex(r[4]) for r in rows], np.float32)
    ri = np.array([int(r[5]) for r in rows], np.int64)
    rik = np.array([int(r[6]) for r in rows], np.int64)
    ref_h = np.array([int(R.hash4(*a)) for a in zip(seed, env, ctr, slot)], np.uint64)
    np.testing.assert_array_equal(h4, ref_h)
    np.testing.assert_array_equal(hk, ref_h)        # rng_key + hash_k == hash4 by construction
    ref_u = np.array([R.uniform(*a) for a in zip(seed, env, ctr, slot)], np.float32).reshape(-1)
    np.testing.assert_array_equal(u, ref_u)
    ref_rf = np.array([R.rand_float(l, h, *a) for l, h, *a in zip(lo, hi, seed, env, ctr, slot)], np.float32).reshape(-1)
    np.testing.assert_array_equal(rf, ref_rf)
    np.testing.assert_array_equal(rfk, ref_rf)
    ref_ri = np.array([R.randint(l, h, *a) for l, h, *a in zip(ilo, ihi, seed, env, ctr, slot)], np.int64).reshape(-1)
    np.testing.assert_array_equal(ri, ref_ri)
    np.testing.assert_array_equal(rik, ref_ri)
    assert ((ri >= ilo) & (ri < ihi)).all()
    # the salted (between-step) domain draws something else than the in-step one
    assert (h4[500:1000] != h4[:500]).mean() > 0.99
