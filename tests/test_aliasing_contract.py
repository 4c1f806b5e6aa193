"""The aliasing contract of INTEGRATION.md §1: how long a tensor the env returns keeps its step's
values is set by ring depths in include/t1env.h; the env, the ctypes binding and the document must agree with them.
CPU-only: parses the header and inspects the binding, no GPU call."""
import ctypes
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header():
    with open(os.path.join(REPO, "include", "t1env.h")) as f:
        return f.read()


def test_extras_ring_depth_matches_header():
    from ti5_isaacgym_amd.envs import t1_env
    m = re.search(r"#define\s+T1ENV_EXTRAS_RING\s+(\d+)", _header())
    assert m, "T1ENV_EXTRAS_RING not found in include/t1env.h"
    assert t1_env.EXTRAS_RING == int(m.group(1)) == 64


def test_observation_ping_pong_depth_matches_header():
    hdr = _header()
    for name in ("obs_buf", "priv_buf"):
        m = re.search(r"float\*\s+%s\[(\d+)\]" % name, hdr)
        assert m and int(m.group(1)) == 2, name
    from ti5_isaacgym_amd import _lib
    fields = dict(_lib.BUFFER_FIELDS)
    for name in ("obs_buf", "priv_buf"):
        t = fields[name]
        assert issubclass(t, ctypes.Array) and t._length_ == 2, name


def test_integration_doc_states_the_depths():
    with open(os.path.join(REPO, "INTEGRATION.md")) as f:
        doc = f.read()
    assert "step *t* + 2" in doc and "step *t* + 64" in doc and "T1ENV_EXTRAS_RING` = 64" in doc
