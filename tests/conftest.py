import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def pytest_sessionfinish(session, exitstatus):
    """$T1_PARITY_REPORT=path: write the worst per-field parity error of this session (golden_util.WORST)."""
    path = os.environ.get("T1_PARITY_REPORT")
    mod = sys.modules.get("golden_util")
    if not path or mod is None or not mod.WORST:
        return
    import json
    rep = {k: {"atol_needed_at_rtol_1e-4": v[0], "max_abs_err": v[1], "max_abs_ref": v[2]}
           for k, v in sorted(mod.WORST.items())}
    with open(path, "w") as f:
        json.dump({"rtol": mod.RTOL, "atol": mod.ATOL, "fields": rep}, f, indent=1)


# the step's dynamics kernels (T1ENV_DYN_KERNEL / T1ENV_D5_SHIFT, read when an env is created): k_dyn6 (the default),
# k_dyn5 with its in-workgroup history shift, k_dyn5 beside the concurrent k_shift5 launch, and k_dyn4
DYN_KERNELS = {"dyn6": {"T1ENV_DYN_KERNEL": "6"},
               "dyn5": {"T1ENV_DYN_KERNEL": "5", "T1ENV_D5_SHIFT": "0"},
               "dyn5_concshift": {"T1ENV_DYN_KERNEL": "5", "T1ENV_D5_SHIFT": "1"},
               "dyn4": {"T1ENV_DYN_KERNEL": "4"}}


@pytest.fixture(params=sorted(DYN_KERNELS))
def dyn_kernel(request, monkeypatch):
    for k, v in DYN_KERNELS[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param


@pytest.fixture(params=["dyn6", "dyn5", "dyn4"])
def dyn_solver(request, monkeypatch):
    """The dynamics kernels (the shift mode does not touch the solver)."""
    for k, v in DYN_KERNELS[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param
