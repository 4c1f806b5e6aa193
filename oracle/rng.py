"""Counter-based random draws shared by the oracle, the golden-vector harness and the HIP kernels.

TEST INFRASTRUCTURE (oracle/): only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this package.  The product kernels carry their own copy of the same function in
``ti5_isaacgym_amd/csrc/t1_common.h``; ``tests/test_rng.py`` compiles that header for the host and pins the two
against each other.

Why a counter RNG: the reference draws from torch's global generator in call order
(``torch_rand_float`` / ``torch.rand_like`` / ``torch.randint``; e.g. legged_robot.py:1071,
t1_dh_stand_env.py:472, legged_robot.py:608).  A device-side, no-host-sync reset cannot reproduce that
stream, so every draw site is instead keyed by ``(seed, global env id, step counter, slot)`` and the
golden-vector harness (tests/golden/gen_golden.py) routes the *reference's own* draw sites through this
same function.  The reference code then consumes exactly the draws our kernels consume, which is what
makes end-to-end obs/reward parity with DR and noise switched on possible.

Definition (all arithmetic mod 2**32):
    mix(x)      = lowbias32 finaliser (x ^= x>>16; x *= 0x7feb352d; x ^= x>>15; x *= 0x846ca68b; x ^= x>>16)
    h           = mix(seed ^ 0x9E3779B9)
    h           = mix(h ^ env)
    h           = mix(h + ctr * 0x9E3779B1)
    h           = mix(h ^ (slot * 0x85EBCA77))
    uniform     = (h >> 8) * 2**-24                      in [0, 1), exact in fp32
    randint     = lo + (((h >> 8) * (hi - lo)) >> 24)    in [lo, hi)
"""
import numpy as np

M32 = np.uint64(0xFFFFFFFF)
# reset_idx(env_ids) called BETWEEN steps keys its draws on (common_step_counter | BETWEEN_STEP_SALT): the in-step
# resets of the step that produced that counter already used the plain counter, and an env reset in that step and
# reset again before the next one must draw fresh DR / lags / gait / start / commands as the reference's generator
# does (its stream simply advances).  The step counter stays below 2**31 (2400 steps/episode).
BETWEEN_STEP_SALT = 0x80000000


def _u32(x):
    return np.asarray(x, dtype=np.uint64) & M32


def _mix(x):
    x = _u32(x)
    x = x ^ (x >> np.uint64(16))
    x = (x * np.uint64(0x7FEB352D)) & M32
    x = x ^ (x >> np.uint64(15))
    x = (x * np.uint64(0x846CA68B)) & M32
    x = x ^ (x >> np.uint64(16))
    return x


def hash4(seed, env, ctr, slot):
    """Vectorised 32-bit hash; arguments broadcast against each other."""
    h = _mix(_u32(seed) ^ np.uint64(0x9E3779B9))
    h = _mix(h ^ _u32(env))
    h = _mix(h + ((_u32(ctr) * np.uint64(0x9E3779B1)) & M32))
    h = _mix(h ^ ((_u32(slot) * np.uint64(0x85EBCA77)) & M32))
    return h


def uniform(seed, env, ctr, slot):
    """float32 uniform in [0, 1)."""
    h = hash4(seed, env, ctr, slot)
    return ((h >> np.uint64(8)).astype(np.float64) * (1.0 / 16777216.0)).astype(np.float32)


def rand_float(lower, upper, seed, env, ctr, slot):
    """Restates isaacgym.torch_utils.torch_rand_float: (upper - lower) * rand + lower, in fp32, no fma."""
    u = uniform(seed, env, ctr, slot)
    scale = np.float32(upper - lower)
    return (np.float32(scale) * u).astype(np.float32) + np.float32(lower)


def randint(lo, hi, seed, env, ctr, slot):
    h = hash4(seed, env, ctr, slot)
    span = np.uint64(hi - lo)
    return (np.int64(lo) + (((h >> np.uint64(8)) * span) >> np.uint64(24)).astype(np.int64))


# ---------------------------------------------------------------------------------------------
# Slot map: one slot (or slot range) per reference draw site.  Comments give the reference site.
# ---------------------------------------------------------------------------------------------
SLOT_TORQUE_MULT = 1000        # + substep*12 + dof   legged_robot.py:1071 (every substep)
SLOT_CMD_X = 2000              # t1_dh_stand_env.py:171
SLOT_CMD_Y = 2001              # t1_dh_stand_env.py:172
SLOT_CMD_YAW = 2002            # t1_dh_stand_env.py:176
SLOT_CMD_HEADING = 2003        # t1_dh_stand_env.py:174 (heading mode only)
SLOT_EXT_FORCE = 3000          # + axis               t1_dh_stand_env.py:237-239
SLOT_EXT_TORQUE = 3003         # + axis               t1_dh_stand_env.py:241
SLOT_PUSH_VEL = 3100           # + axis (2)           t1_dh_stand_env.py:223
SLOT_PUSH_ANG = 3102           # + axis (3)           t1_dh_stand_env.py:225
SLOT_OBS_NOISE = 4000          # + obs index (47)     t1_dh_stand_env.py:472
SLOT_RESET_DOF = 5000          # + dof                legged_robot.py:1084
SLOT_RESET_ROOT_XY = 5100      # + axis (2)           legged_robot.py:1105 / 1108
SLOT_DR_TORQUE = 5200          # + dof                legged_robot.py:737
SLOT_DR_OFFSET = 5300          # + dof                legged_robot.py:741
SLOT_DR_KP = 5400              # + dof                legged_robot.py:746
SLOT_DR_KD = 5500              # + dof                legged_robot.py:747
SLOT_DR_COULOMB = 5600         # + dof                legged_robot.py:752
SLOT_DR_VISCOUS = 5700         # + dof                legged_robot.py:753
SLOT_DR_ARMATURE = 5800        # + dof                legged_robot.py:780
SLOT_LAG_ACTION = 5900         # legged_robot.py:608
SLOT_LAG_DOF = 5901            # legged_robot.py:618
SLOT_LAG_IMU = 5902            # legged_robot.py:628
SLOT_GAIT_START = 5903         # t1_dh_stand_env.py:523 / :569
SLOT_GAIT_TIME = 5910          # + gait slot (3)      t1_dh_stand_env.py:116
SLOT_TERRAIN_LEVEL_RAND = 5920  # legged_robot.py:1156
# creation-time draws (ctr = 0)
SLOT_PAYLOAD = 6000            # legged_robot.py:699
SLOT_LINK_MASS = 6001          # + link-1 (12)        legged_robot.py:703
SLOT_COM = 6020                # + axis               legged_robot.py:707-709
SLOT_FRICTION_BUCKET = 6030    # randint(0,256)       legged_robot.py:807
SLOT_FRICTION_VALUE = 6031     # env := bucket id     legged_robot.py:809
SLOT_RESTITUTION_VALUE = 6032  # env := bucket id     legged_robot.py:811
SLOT_TERRAIN_LEVEL_INIT = 6040  # legged_robot.py:1489
SLOT_START_XY = 6050           # + axis               legged_robot.py:1382
