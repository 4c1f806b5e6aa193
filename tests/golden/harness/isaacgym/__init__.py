"""TEST-ONLY stand-in for NVIDIA Isaac Gym Preview 4 (proprietary binary, absent from this image).

Used exclusively by tests/golden/gen_golden.py to import and drive the reference's own env code
(/root/reference/humanoid/envs/**) with injected physics states.  Nothing here is shipped or imported
by the product package.  torch_utils / terrain_utils arithmetic are restatements of the published
Isaac Gym Preview 4 helpers and are *parity unpinned* (no reference test or vector exists for them).
"""
