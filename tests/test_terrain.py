"""Terrain generator (utils/terrain.py) vs the reference's own terrain (humanoid/utils/terrain.py:9-191).

The golden fixtures trimesh16 / heights16 hold the reference's height field (init_height_samples), its terrain
origins and the env -> (level, type) assignment, generated behind the isaacgym stand-in after the reference's own
set_seed(5).  The build's generator draws from numpy's global generator in the reference's call order, so under the
same seed it must reproduce the field sample for sample (int16, exact) and the origins (fp32).  The Isaac Gym
terrain_utils helper arithmetic it restates is third party; these two fixtures pin the paths they exercise (flat,
rough-flat at the default proportions; sloped / rough-sloped in heights16).  Levels and types come from the counter
RNG (oracle/rng.py) and the terrain_types formula (legged_robot.py:1477-1512).
"""
import numpy as np
import pytest

from golden_util import load, terrain_of
from oracle.t1_oracle import T1Oracle


def _cfg(heights):
    from ti5_isaacgym_amd.utils.task_registry import task_registry
    import copy
    cfg, _ = task_registry.get_cfgs("t1_dh_stand")
    cfg = copy.deepcopy(cfg)
    cfg.terrain.mesh_type = "trimesh"
    cfg.terrain.num_rows, cfg.terrain.num_cols, cfg.terrain.border_size = 6, 4, 5   # gen_golden.trimesh_hook
    if heights:   # gen_golden.heights_hook
        cfg.terrain.measure_heights = True
        cfg.terrain.terrain_proportions = [0.0, 0.25, 0.25, 0.25, 0.25, 0.0, 0.0, 0.0, 0.0, 0.0]
    return cfg


@pytest.mark.parametrize("name", ["trimesh16", "heights16"])
def test_terrain_matches_reference(name):
    from ti5_isaacgym_amd.utils.helpers import set_seed
    from ti5_isaacgym_amd.utils.terrain import Terrain
    fx = load(name)
    cfg = _cfg(name == "heights16")
    set_seed(int(fx["seed"]))
    t = Terrain(cfg.terrain, int(fx["num_envs"]))
    ref = fx["init_height_samples"]
    assert t.heightsamples.shape == ref.shape
    np.testing.assert_array_equal(t.heightsamples.astype(np.int16), ref)
    np.testing.assert_allclose(t.env_origins, fx["init_terrain_origins"], rtol=0, atol=1e-6)
    if name == "heights16":   # the sloped sub-terrains are not flat: the test is not vacuous
        assert np.ptp(ref) > 20


@pytest.mark.parametrize("name", ["trimesh16", "heights16", "resetidx16"])
def test_terrain_levels_and_types(name):
    fx = load(name)
    o = T1Oracle(int(fx["num_envs"]), seed=int(fx["seed"]), mesh_type="trimesh", terrain=terrain_of(fx))
    np.testing.assert_array_equal(o.terrain_levels, fx["init_terrain_levels"])
    np.testing.assert_array_equal(o.terrain_types, fx["init_terrain_types"])
    np.testing.assert_allclose(o.env_origins, fx["init_env_origins"], rtol=0, atol=1e-6)


@pytest.mark.parametrize("name", ["plane16", "trimesh16", "config1_64"])
def test_creation_dr_matches_reference(name):
    """Creation-time DR (legged_robot.py:692-730 randomize_rigid_body_props, 786-824 _process_rigid_shape_props) as
    the oracle restates it (and k_init computes it: tests/test_gpu_product_parity.py compares the two) vs the
    reference's link masses, COM displacements, payloads, frictions and restitutions."""
    fx = load(name)
    o = T1Oracle(int(fx["num_envs"]), seed=int(fx["seed"]), mesh_type=str(fx["mesh_type"]), terrain=terrain_of(fx))
    np.testing.assert_allclose(o.payload, fx["init_payload_masses"].reshape(-1), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(o.com_disp, fx["init_com_displacements"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(o.restitution, fx["init_restitution"].reshape(-1), rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(o.friction, fx["init_env_frictions"].reshape(-1), rtol=1e-6, atol=1e-7)
    lm = fx["init_link_masses"]
    assert lm.shape[-1] == 12, lm.shape
    np.testing.assert_allclose(o.link_mass_scale, lm.reshape(o.link_mass_scale.shape), rtol=1e-6, atol=1e-7)
