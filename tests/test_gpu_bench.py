"""bench.py keeps the driver's contract on the GPU: one JSON line with the metric / config of BASELINE.json, a
roofline object for the dominant kernel and (N = 1) a cpu_baseline object."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_line():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "10", "--warmup", "3",
                        "--time-every", "2", "--cpu-seconds", "1", "--cpu-envs", "16"],
                       capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert d["metric"] == base["metric"] and d["unit"] == "env-steps/s" and d["higher_is_better"] is True
    assert d["n_gpus"] == 1 and d["steps"] == 10 and d["warmup"] == 3 and d["scaling"] == "weak"
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["config"]["num_envs_per_gpu"] == 8192
    rf = d["roofline"]
    # bound: the roofline the kernel sits closest to (bench.py derives it: HBM, or the dynamics waves' VALU issue);
    # achieved / peak / frac are the HBM roofline's in either case
    assert rf["bound"] in ("hbm", "valu_issue") and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    if rf["bound"] == "valu_issue":
        assert rf["issue"]["frac"] > rf["frac"]
    assert 0 < rf["frac"] < 1 and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert rf["kernels"][rf["kernel"]]["timed_launches"] > 0
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("port", "reference")
