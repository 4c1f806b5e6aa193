"""Helpers shared by the parity tests: load a golden fixture and drive an env through the same inputs."""
import os

import numpy as np

import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SCENARIOS = ["plane16", "events16", "config1_64", "trimesh16", "heights16", "resetidx16", "push16", "trimesh_nocurr16"]


def load(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"))
    return {k: d[k] for k in d.files}


def terrain_of(fx):
    if str(fx["mesh_type"]) in ("trimesh", "heightfield"):
        t = {"terrain_origins": fx["init_terrain_origins"], "height_samples": fx["init_height_samples"]}
        if "init_terrain_scales" in fx:   # the height-scan scenario: the scan needs the field's geometry
            hs, vs, border = (float(x) for x in fx["init_terrain_scales"])
            t.update(horizontal_scale=hs, vertical_scale=vs, border_size=border)
        return t
    return None


def mid_reset(fx, t):
    """env ids the reference's reset_idx was called on between step t and t + 1 (scenario resetidx16), or None"""
    if "mid_reset_step" in fx and int(fx["mid_reset_step"]) == t:
        return fx["mid_reset_ids"]
    return None


def push_interval_s(fx):
    """push_robots scenario (push16): the scenario's push_interval_s, else None (push_robots off, the default)"""
    return float(fx["cfg_push_interval_s"]) if "cfg_push_interval_s" in fx else None


def terrain_curriculum(fx):
    """cfg.terrain.curriculum of the scenario (on unless the fixture says otherwise: trimesh_nocurr16)"""
    return bool(int(fx["cfg_terrain_curriculum"])) if "cfg_terrain_curriculum" in fx else True


def measures_heights(fx):
    return "step_measured_heights" in fx


def synth_physics(fx):
    seed = int(fx["synth_seed"])
    n = int(fx["num_envs"])

    def physics(g, torques, env):
        root, dof, rigid, contact = synth.state(seed, n, g, np.asarray(env.env_origins))
        return root, dof, rigid, contact
    return physics


def assert_close(name, got, ref, rtol=1e-4, atol=1e-4, ctx=""):
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, f"{name}{ctx}: shape {got.shape} vs {ref.shape}"
    bad = ~np.isclose(got, ref, rtol=rtol, atol=atol)
    if bad.any():
        idx = np.argwhere(bad)[:5]
        msg = ", ".join(f"{tuple(i)}: {got[tuple(i)]:.7g} vs {ref[tuple(i)]:.7g}" for i in idx)
        raise AssertionError(f"{name}{ctx}: {bad.sum()} mismatches: {msg}")
