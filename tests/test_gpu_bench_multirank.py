"""bench.py's N > 1 path: the driver's SCALE run launches bench.py under torch.distributed.run with one
rank per GPU over RCCL.  RCCL refuses two ranks on one GPU, so this test runs the same path with the process group's
backend overridden to gloo (T1_BENCH_BACKEND=gloo) and both ranks on cuda:0, and checks what the SCALE line relies on:

- env_offset sharding: rank r owns global envs [r N, (r + 1) N);
- the timed region's barrier + max-over-ranks timing: the line's time is the slowest rank's;
- one JSON line, from rank 0 only, with the backend and world size the process group saw.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_on_one_gpu():
    N, steps, world = 1024, 12, 2
    env = dict(os.environ, T1_BENCH_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", str(world), "--steps", str(steps), "--warmup", "3", "--num-envs", str(N), "--time-every", "4"]
    pr = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=300)
    assert pr.returncode == 0, pr.stderr[-3000:]
    lines = [ln for ln in pr.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, pr.stdout   # rank 0 only
    line = json.loads(lines[0])
    d = line["dist"]
    assert d["backend"] == "gloo" and d["world_size"] == world
    assert d["env_offsets"] == [r * N for r in range(world)] and d["envs_per_rank"] == [N] * world
    assert line["n_gpus"] == world and line["config"]["global_envs"] == N * world
    assert line["config"]["parallelism"] == f"dp{world}" and line["scaling"] == "weak"
    assert line["finite"] is True
    # the line's time is the max over the ranks' own elapsed times (each bracketed by barrier + synchronize)
    t = max(d["rank_elapsed_s"])
    assert line["ms_per_step"] == pytest.approx(t / steps * 1e3, rel=1e-3, abs=1e-4)
    assert line["value"] == pytest.approx(N * world * steps / t, rel=1e-3)
    assert "cpu_baseline" not in line   # rank 0 at N = 1 only
