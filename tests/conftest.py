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
