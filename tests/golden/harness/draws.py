"""Draw hook: routes the reference's random draw sites through the shared counter RNG (oracle/rng.py).

Each call is identified by (calling function, source line) in the reference snapshot and mapped to a
slot of oracle.rng; the env ids come from the caller's ``env_ids`` / ``envs`` local (or all envs), the
step counter from ``self.common_step_counter``.  Unknown call sites raise, so a reference edit cannot
silently fall back to torch's generator.
"""
import sys

import numpy as np
import torch

from oracle import rng as R

SEED = 5
CTR_SALT = 0      # R.BETWEEN_STEP_SALT while the driver calls reset_idx between steps (gen_golden.run mid_reset)
LOG = []          # (func, line, shape) of every draw, for debugging / site discovery
DISCOVER = False  # when True, unknown sites fall back to torch.rand and are only logged

_orig_randint = torch.randint
_orig_rand_like = torch.rand_like
_orig_randint_like = torch.randint_like

# (function name, line) -> (kind, slot base, column mode)
#   column mode: "col" -> slot = base + column; "i" -> slot = base + caller local i; "one" -> slot = base
SITES = {
    ("randomize_rigid_body_props", 699): ("float", R.SLOT_PAYLOAD, "col"),
    ("randomize_rigid_body_props", 703): ("float", R.SLOT_LINK_MASS, "col"),
    ("randomize_rigid_body_props", 707): ("float", R.SLOT_COM + 0, "col"),
    ("randomize_rigid_body_props", 708): ("float", R.SLOT_COM + 1, "col"),
    ("randomize_rigid_body_props", 709): ("float", R.SLOT_COM + 2, "col"),
    ("randomize_dof_props", 737): ("float", R.SLOT_DR_TORQUE, "col"),
    ("randomize_dof_props", 741): ("float", R.SLOT_DR_OFFSET, "col"),
    ("randomize_dof_props", 746): ("float", R.SLOT_DR_KP, "col"),
    ("randomize_dof_props", 747): ("float", R.SLOT_DR_KD, "col"),
    ("randomize_dof_props", 752): ("float", R.SLOT_DR_COULOMB, "col"),
    ("randomize_dof_props", 753): ("float", R.SLOT_DR_VISCOUS, "col"),
    ("randomize_dof_props", 780): ("float", R.SLOT_DR_ARMATURE, "i"),
    ("_create_envs", 1382): ("start_xy", R.SLOT_START_XY, "col"),
    ("_process_rigid_shape_props", 807): ("int", R.SLOT_FRICTION_BUCKET, "one"),
    ("_process_rigid_shape_props", 809): ("bucket", R.SLOT_FRICTION_VALUE, "one"),
    ("_process_rigid_shape_props", 811): ("bucket", R.SLOT_RESTITUTION_VALUE, "one"),
    ("_reset_dofs", 1084): ("float", R.SLOT_RESET_DOF, "col"),
    ("_reset_root_states", 1105): ("float", R.SLOT_RESET_ROOT_XY, "col"),
    ("_reset_root_states", 1108): ("float", R.SLOT_RESET_ROOT_XY, "col"),
    ("generate_gait_time", 116): ("float", R.SLOT_GAIT_TIME, "i"),
    ("_resample_walk_omnidirectional_command", 171): ("float", R.SLOT_CMD_X, "one"),
    ("_resample_walk_omnidirectional_command", 172): ("float", R.SLOT_CMD_Y, "one"),
    ("_resample_walk_omnidirectional_command", 174): ("float", R.SLOT_CMD_HEADING, "one"),
    ("_resample_walk_omnidirectional_command", 176): ("float", R.SLOT_CMD_YAW, "one"),
    ("_compute_torques", 1071): ("float", R.SLOT_TORQUE_MULT, "substep"),
    ("_add_ext_force", 237): ("float", R.SLOT_EXT_FORCE + 0, "one"),
    ("_add_ext_force", 238): ("float", R.SLOT_EXT_FORCE + 1, "one"),
    ("_add_ext_force", 239): ("float", R.SLOT_EXT_FORCE + 2, "one"),
    ("_add_ext_force", 241): ("float", R.SLOT_EXT_TORQUE, "col"),
    ("_push_robots", 223): ("float", R.SLOT_PUSH_VEL, "col"),
    ("_push_robots", 225): ("float", R.SLOT_PUSH_ANG, "col"),
    ("compute_observations", 472): ("uniform", R.SLOT_OBS_NOISE, "col"),
    ("randomize_lag_props", 608): ("int", R.SLOT_LAG_ACTION, "one"),
    ("randomize_lag_props", 618): ("int", R.SLOT_LAG_DOF, "one"),
    ("randomize_lag_props", 628): ("int", R.SLOT_LAG_IMU, "one"),
    ("_init_buffers", 277): ("int", R.SLOT_LAG_ACTION, "one"),
    ("_init_buffers", 297): ("int", R.SLOT_LAG_DOF, "one"),
    ("_init_buffers", 313): ("int", R.SLOT_LAG_IMU, "one"),
    ("_init_buffers", 569): ("int", R.SLOT_GAIT_START, "one"),
    ("reset_idx", 523): ("int", R.SLOT_GAIT_START, "one"),
    ("_get_env_origins", 1489): ("int", R.SLOT_TERRAIN_LEVEL_INIT, "one"),
    ("_update_terrain_curriculum", 1156): ("int", R.SLOT_TERRAIN_LEVEL_RAND, "one"),
}


def _caller(depth=2):
    f = sys._getframe(depth)
    return f


def _ids_and_ctr(frame, n_rows):
    loc = frame.f_locals
    self = loc.get("self")
    ids = None
    for k in ("env_ids", "envs"):
        if k in loc and isinstance(loc[k], torch.Tensor):
            ids = loc[k].detach().cpu().numpy().astype(np.int64)
            break
    if ids is None or len(ids) != n_rows:
        ids = np.arange(n_rows, dtype=np.int64)
    ctr = int(getattr(self, "common_step_counter", 0)) if self is not None else 0
    return ids, ctr | CTR_SALT, loc


def _site(frame):
    key = (frame.f_code.co_name, frame.f_lineno)
    return key


def _slots(key, loc, ncols):
    kind, base, mode = SITES[key]
    if mode == "col":
        return [base + c for c in range(ncols)]
    if mode == "i":
        return [base + int(loc["i"])]
    if mode == "substep":
        # _compute_torques called from LeggedRobot.step's decimation loop (loop variable `_`)
        sub = int(sys._getframe(4).f_locals.get("_", 0))
        return [base + sub * ncols + c for c in range(ncols)]
    return [base]


def rand_float(lower, upper, shape, device):
    frame = _caller(3)  # _caller <- rand_float <- torch_utils.torch_rand_float <- reference
    key = _site(frame)
    LOG.append((key, tuple(shape)))
    if key not in SITES:
        if DISCOVER:
            return (upper - lower) * torch.rand(*shape, device=device) + lower
        raise KeyError(f"unmapped torch_rand_float site {key}")
    n_rows = shape[0]
    ncols = int(np.prod(shape[1:])) if len(shape) > 1 else 1
    ids, ctr, loc = _ids_and_ctr(frame, n_rows)
    slots = _slots(key, loc, ncols)
    kind = SITES[key][0]
    if kind == "bucket":   # friction / restitution buckets: the "env" key is the bucket index
        ids = np.arange(n_rows, dtype=np.int64)
    if kind == "start_xy":  # per-env start pose jitter: rows are (x, y) of env `i`
        i = int(loc["i"])
        out = np.array([R.rand_float(lower, upper, SEED, i, ctr, SITES[key][1] + r) for r in range(n_rows)])
        return torch.from_numpy(out.reshape(shape).astype(np.float32)).to(device)
    out = np.stack([R.rand_float(lower, upper, SEED, ids, ctr, s) for s in slots], axis=1)
    return torch.from_numpy(out.reshape(shape)).to(device)


def randint(*args, **kw):
    frame = _caller(2)
    key = _site(frame)
    if frame.f_code.co_filename.startswith("/root/reference"):
        LOG.append((key, args))
    if key not in SITES:
        if DISCOVER or not frame.f_code.co_filename.startswith("/root/reference"):
            return _orig_randint(*args, **kw)
        raise KeyError(f"unmapped torch.randint site {key}")
    if len(args) == 3:
        lo, hi, size = args
    else:
        lo, (hi, size) = 0, args
    n_rows = size[0]
    ids, ctr, loc = _ids_and_ctr(frame, n_rows)
    slot = _slots(key, loc, 1)[0]
    out = R.randint(lo, hi, SEED, ids, ctr, slot)
    if len(size) == 2:
        out = out.reshape(n_rows, 1)
    return torch.from_numpy(out).to(kw.get("device", "cpu"))


def randint_like(t, high, **kw):
    frame = _caller(2)
    key = _site(frame)
    if key not in SITES:
        if DISCOVER or not frame.f_code.co_filename.startswith("/root/reference"):
            return _orig_randint_like(t, high, **kw)
        raise KeyError(f"unmapped torch.randint_like site {key}")
    LOG.append((key, tuple(t.shape)))
    ids, ctr, loc = _ids_and_ctr(frame, t.shape[0])
    slot = _slots(key, loc, 1)[0]
    return torch.from_numpy(R.randint(0, int(high), SEED, ids, ctr, slot)).to(t.dtype)


def rand_like(t, **kw):
    frame = _caller(2)
    key = _site(frame)
    if frame.f_code.co_filename.startswith("/root/reference"):
        LOG.append((key, "rand_like"))
    if key not in SITES:
        if DISCOVER or not frame.f_code.co_filename.startswith("/root/reference"):
            return _orig_rand_like(t, **kw)
        raise KeyError(f"unmapped torch.rand_like site {key}")
    LOG.append((key, tuple(t.shape)))
    ids, ctr, loc = _ids_and_ctr(frame, t.shape[0])
    base = SITES[key][1]
    out = np.stack([R.uniform(SEED, ids, ctr, base + c) for c in range(t.shape[1])], axis=1)
    return torch.from_numpy(out).to(t.dtype)


def install():
    torch.randint = randint
    torch.rand_like = rand_like
    torch.randint_like = randint_like


def uninstall():
    torch.randint = _orig_randint
    torch.rand_like = _orig_rand_like
    torch.randint_like = _orig_randint_like
