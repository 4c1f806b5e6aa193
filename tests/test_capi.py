"""C-ABI checks that need no GPU: the library loads, exports every function include/t1env.h declares, and
the ctypes mirrors have the same struct layout as the C header (compiled with gcc here)."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "t1env.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(t1env_\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    from ti5_isaacgym_amd import _lib
    from ti5_isaacgym_amd import build as b
    b.build()
    return _lib.load()


def test_exports_every_declared_symbol(lib):
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), n
    from ti5_isaacgym_amd import _lib
    assert sorted(_lib.EXPORTS) == names


def test_version_and_errors(lib):
    assert b"gfx950" in lib.t1env_version()
    from ti5_isaacgym_amd import _lib
    rc = lib.t1env_create(None, None, None, None)
    assert rc == -1 and b"null" in lib.t1env_last_error()


def test_library_carries_this_trees_source_stamp(lib, monkeypatch):
    """the library's version names the hash of the sources it was built from, and load() refuses one
    built from other sources with a clear message (not a missing symbol later)."""
    from ti5_isaacgym_amd import _lib, build
    assert lib.t1env_version().decode().endswith("src:" + build.source_stamp())
    monkeypatch.setattr(build, "source_stamp", lambda: "0" * 16)
    with pytest.raises(RuntimeError, match="stale"):
        _lib.check_stamp(lib, "libt1env_hip.so")


def test_struct_layout_matches_header():
    from ti5_isaacgym_amd import _lib
    prog = r'''
#include <stdio.h>
#include <stddef.h>
#include "t1env.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu\n", sizeof(t1env_model), sizeof(t1env_config), sizeof(t1env_buffers),
         sizeof(t1env_step_args), sizeof(t1env_injected));
  printf("%zu %zu %zu %zu %zu %zu\n", offsetof(t1env_config, reset_xy_range), offsetof(t1env_buffers, ep_accum),
         offsetof(t1env_model, base_init_state), offsetof(t1env_buffers, contact_vimp), offsetof(t1env_model, self_capsule),
         offsetof(t1env_model, bounce_threshold));
  return 0;
}
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "sz.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "sz")
        subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    sizes = list(map(int, out))
    assert sizes[:5] == [ctypes.sizeof(_lib.Model), ctypes.sizeof(_lib.Config), ctypes.sizeof(_lib.Buffers),
                         ctypes.sizeof(_lib.StepArgs), ctypes.sizeof(_lib.Injected)]
    assert sizes[5] == _lib.Config.reset_xy_range.offset
    assert sizes[6] == _lib.Buffers.ep_accum.offset
    assert sizes[7] == _lib.Model.base_init_state.offset
    assert sizes[8:] == [_lib.Buffers.contact_vimp.offset, _lib.Model.self_capsule.offset, _lib.Model.bounce_threshold.offset]


def test_env_refuses_cpu_device():
    import ti5_isaacgym_amd as t
    with pytest.raises(RuntimeError):
        t.make_t1_env(num_envs=4, mesh_type="plane", device="cpu")


def test_policy_header_exports(lib):
    """include/t1policy.h's entry points are exported by the same library, and _lib binds them."""
    src = open(os.path.join(REPO, "include", "t1policy.h")).read()
    names = sorted(set(re.findall(r"^\s*(?:int|long long)\s+(t1policy_\w+)\s*\(", src, re.M)))
    from ti5_isaacgym_amd import _lib
    assert names == sorted(_lib.POLICY_EXPORTS) and names
    for n in names:
        assert hasattr(lib, n), n
    # argument errors are reported without touching the GPU
    assert lib.t1policy_conv1d_forward(None, None, None, None, 1, 66, 47, 32, 6, 3, None) == -1
    assert lib.t1policy_conv1d_forward_packed(None, None, None, None, 1, 66, 47, 32, 6, 3, None) == -1
    assert lib.t1policy_conv1d_pack_weights(None, None, 66, 32, 6, None) == -1
    assert lib.t1policy_conv1d_frag_bytes() == 17 * 2 * 2 * 64 * 16
    assert lib.t1policy_linear_wgrad_workspace_bytes(0, 4, 4) == -1
    assert lib.t1policy_linear_wgrad_bf16(None, None, 8, 4, 4, None, 0, None, None, 0, None) == -1
    # fused heads: 1,768 step-tiles (32 outputs x 16 inputs) of hi + lo fragments, 90 output tiles of bias
    assert lib.t1policy_heads_frag_bytes() == 1768 * 2 * 64 * 16 + 90 * 4 * 64 * 16   # + the bias fragments
    assert lib.t1policy_heads_pack(None, None, None, None) == -1
    dims = (ctypes.c_int * 30)(*([1] * 30))
    ptrs = (ctypes.c_uint64 * 31)(*([1] * 31))
    frag = ctypes.c_void_p(16)
    assert lib.t1policy_heads_pack(ptrs, dims, frag, None) == 1   # shapes without a compiled instance


def test_env_refuses_external_torques():
    """ext_torque_max != 0 would draw torques into the critic frame that the HIP dynamics never applies: it raises
    (the reference applies them, t1_dh_stand_env.py:243-247; DHT1StandCfg uses 0, t1_dh_stand_config.py:201)."""
    import ti5_isaacgym_amd as t

    def hook(cfg):
        cfg.domain_rand.ext_torque_max = 2.0
    with pytest.raises(NotImplementedError, match="ext_torque_max"):
        t.make_t1_env(num_envs=4, mesh_type="plane", device="cpu", cfg_hook=hook)
