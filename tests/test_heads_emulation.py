"""The fused policy heads' fragment algebra on the CPU (tools/heads_emulate.py): the pack order, the natural and
permuted k-steps, the conv2 Toeplitz layer with its per-channel bias and the CDNA4 v_mfma_f32_32x32x16 lane maps,
emulated in fp64, reproduce the torch fp64 forward of ActorCriticDH (actor_critic_dh.py:45-111,163-188) to rounding.
The GPU test (test_gpu_policy_heads.py) then only has the hardware and the fp16 split left to check."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def test_heads_fragment_algebra_matches_fp64_forward():
    from heads_emulate import emulate_errors
    em, ev = emulate_errors(seed=0)
    assert em < 1e-12 and ev < 1e-12, (em, ev)
