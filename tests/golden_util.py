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


# Parity tolerance (north_star: 1e-4 relative, fp32).  The absolute floor is 1e-6: the smallest per-term reward
# values (episode sums of dof_vel / torques, median ~1e-4) are then checked to ~1%, and a term that a bug zeroed
# fails.  Measured worst floors needed at rtol 1e-4: oracle vs reference 3.8e-7 (one obs element); HIP vs reference /
# oracle are recorded per field by WORST below (tests write them to $T1_PARITY_REPORT).
RTOL, ATOL = 1e-4, 1e-6
# field -> [worst |got - ref| - rtol |ref| (the absolute floor the field needed), worst |got - ref|, max |ref|]
WORST = {}


def _record(name, got, ref, rtol):
    if got.size == 0:
        return
    err = np.abs(got - ref)
    fin = np.isfinite(err)
    if not fin.any():
        return
    need = float(np.max((err - rtol * np.abs(ref))[fin]))
    w = WORST.setdefault(name, [-np.inf, 0.0, 0.0])
    w[0] = max(w[0], need)
    w[1] = max(w[1], float(err[fin].max()))
    w[2] = max(w[2], float(np.abs(ref[np.isfinite(ref)]).max(initial=0.0)))


# T1 torque limits x 0.85, left then right leg
TORQUE_MAX = np.array([86.7, 86.7, 226.95, 226.95, 68.0, 34.0, 86.7, 86.7, 226.95, 226.95, 68.0, 34.17])


def torque_atol():
    """Per-joint absolute floor for torques: tau = Kp (a_lag + q0 - q + off) - Kd qd - visc qd - coul sign(qd), times the
    multiplier, is a difference of terms up to the joint's torque limit, so a torque near zero carries the fp32 rounding of
    those terms (the HIP kernel contracts them into FMAs, numpy rounds every product): 2e-7 x the limit (~3.4 ulp of
    the limit; measured need 3.3e-6 on a 68 N m joint, r03a)."""
    return 2e-7 * TORQUE_MAX


def assert_close(name, got, ref, rtol=RTOL, atol=ATOL, ctx=""):
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape, f"{name}{ctx}: shape {got.shape} vs {ref.shape}"
    _record(name, got, ref, rtol)
    bad = ~np.isclose(got, ref, rtol=rtol, atol=atol)
    if bad.any():
        idx = np.argwhere(bad)[:5]
        msg = ", ".join(f"{tuple(i)}: {got[tuple(i)]:.7g} vs {ref[tuple(i)]:.7g}" for i in idx)
        raise AssertionError(f"{name}{ctx}: {bad.sum()} mismatches: {msg}")
