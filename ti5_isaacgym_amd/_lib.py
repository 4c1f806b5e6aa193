"""ctypes binding of libt1env_hip.so (include/t1env.h).

The product path has no fallback: if the HIP library is missing or fails to load, importing the env
raises.  Build it with ``python -m ti5_isaacgym_amd.build`` (or ``__graft_entry__.build()``).
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("T1ENV_LIB") or os.path.join(HERE, "_lib", "libt1env_hip.so")  # override: A/B builds

NB, ND, MAXC, NOBS, NPRIV, HIST, CHIST, NREW = 13, 12, 48, 47, 73, 66, 3, 24

f32, i32, u32 = C.c_float, C.c_int32, C.c_uint32
fp, u8p, i32p, i64p = C.POINTER(C.c_float), C.POINTER(C.c_uint8), C.POINTER(C.c_int32), C.POINTER(C.c_int64)


class Model(C.Structure):
    _fields_ = [
        ("joint_offset", (f32 * 3) * NB), ("joint_axis", (f32 * 3) * NB), ("parent", i32 * NB), ("mass", f32 * NB),
        ("com", (f32 * 3) * NB), ("inertia", (f32 * 6) * NB),
        ("q_lower", f32 * ND), ("q_upper", f32 * ND), ("vel_limit", f32 * ND), ("torque_limit", f32 * ND),
        ("default_dof_pos", f32 * ND), ("p_gains", f32 * ND), ("d_gains", f32 * ND),
        ("contact_start", i32 * NB), ("contact_count", i32 * NB), ("contact_point", (f32 * 3) * MAXC),
        ("n_contact", i32),
        ("k_contact", f32), ("d_contact", f32), ("friction_vs", f32), ("k_limit", f32), ("d_limit", f32),
        ("gravity", f32), ("ground_friction", f32), ("ground_restitution", f32), ("base_init_state", f32 * 13),
        ("self_collisions", i32), ("self_capsule", (f32 * 7) * 4), ("bounce_threshold", f32),
    ]


class Config(C.Structure):
    _fields_ = [
        ("num_envs", i32), ("env_offset", i32), ("num_envs_total", i32), ("seed", u32), ("sim_dt", f32),
        ("decimation", i32), ("action_scale", f32), ("clip_actions", f32), ("clip_obs", f32),
        ("max_episode_length", f32), ("episode_length_s", f32), ("cycle_time", f32), ("stand_com_threshold", f32),
        ("target_joint_pos_scale", f32), ("noise_level", f32), ("noise_vec", f32 * NOBS),
        ("reward_scales", f32 * NREW), ("only_positive_rewards", i32),
        ("base_height_target", f32), ("foot_min_dist", f32), ("foot_max_dist", f32), ("knee_min_dist", f32),
        ("knee_max_dist", f32), ("target_feet_height", f32), ("target_feet_height_max", f32),
        ("tracking_sigma", f32), ("max_contact_force", f32),
        ("gait_time_range", (f32 * 2) * 3), ("gait_kind", i32 * 3),
        ("ext_force_max", f32 * 3), ("ext_torque_max", f32), ("push_vel_xy", f32), ("push_ang", f32),
        ("lag_range", i32 * 2), ("dof_lag_range", i32 * 2), ("imu_lag_range", i32 * 2),
        ("torque_mult_range", f32 * 2), ("motor_offset_range", f32 * 2), ("kp_mult_range", f32 * 2),
        ("kd_mult_range", f32 * 2), ("coulomb_range", f32 * 2), ("viscous_range", f32 * 2),
        ("armature_range", (f32 * 2) * ND), ("reset_dof_range", f32), ("terrain_curriculum", i32),
        ("platform", f32), ("env_length", f32), ("num_terrain_rows", i32), ("num_terrain_cols", i32),
        ("lin_vel_obs_scale", f32), ("ang_vel_obs_scale", f32), ("dof_pos_obs_scale", f32),
        ("dof_vel_obs_scale", f32), ("quat_obs_scale", f32),
        ("dr_base_mass", i32), ("dr_link_mass", i32), ("dr_com", i32), ("dr_friction", i32),
        ("added_mass_range", f32 * 2), ("link_mass_range", f32 * 2), ("com_range", (f32 * 2) * 3),
        ("friction_range", f32 * 2), ("restitution_range", f32 * 2), ("custom_origins", i32),
        ("max_init_terrain_level", i32), ("reset_xy_range", f32), ("obs_half", i32),
    ]


BUFFER_FIELDS = [
    ("root_states", fp), ("dof_state", fp), ("rigid_state", fp), ("contact_forces", fp),
    ("obs_buf", fp * 2), ("priv_buf", fp * 2), ("rew_buf", fp), ("reset_buf", u8p), ("time_out_buf", u8p),
    ("episode_length_buf", i64p), ("phase_length_buf", i64p), ("commands", fp), ("torques", fp), ("actions", fp),
    ("last_actions", fp), ("last_last_actions", fp), ("last_dof_vel", fp), ("last_root_vel", fp),
    ("base_lin_vel", fp), ("base_ang_vel", fp), ("projected_gravity", fp), ("base_euler_xyz", fp),
    ("feet_euler_xyz", fp), ("feet_air_time", fp), ("last_contacts", u8p), ("feet_height", fp), ("last_feet_z", fp),
    ("ref_dof_pos", fp), ("gait_time", i32p), ("gait_start", fp), ("ext_forces", fp), ("ext_torques", fp),
    ("applied_force", fp), ("episode_sums", fp), ("kp", fp), ("kd", fp), ("motor_offsets", fp), ("coulomb", fp),
    ("viscous", fp), ("armature", fp), ("friction", fp), ("restitution", fp), ("body_mass", fp),
    ("link_mass_scale", fp), ("com_disp", fp), ("lag_timestep", i32p), ("dof_lag_timestep", i32p),
    ("imu_lag_timestep", i32p), ("act_hist", fp), ("dof_hist", fp), ("imu_hist", fp), ("env_origins", fp),
    ("terrain_levels", i32p), ("terrain_types", i32p), ("terrain_origins", fp), ("extras", fp), ("ep_accum", fp),
    ("contact_vimp", fp),
]


class Buffers(C.Structure):
    _fields_ = BUFFER_FIELDS


class StepArgs(C.Structure):
    _fields_ = [("counter", u32), ("obs_slot", i32), ("ext_force_call", i32), ("ext_force_first", i32),
                ("push_call", i32), ("cmd_ranges", (f32 * 2) * 3)]


class Injected(C.Structure):
    _fields_ = [("root", fp), ("dof", fp), ("rigid", fp), ("contact", fp), ("torque_log", fp)]


class SubstepLog(C.Structure):
    _fields_ = [("root", fp), ("dof", fp), ("torque", fp)]


EXPORTS = ["t1env_create", "t1env_destroy", "t1env_init", "t1env_set_terrain", "t1env_reset_all", "t1env_step",
           "t1env_step_physics_and_rewards", "t1env_step_reset_and_observe", "t1env_step_injected",
           "t1env_set_fused", "t1env_set_timing", "t1env_get_timing", "t1env_last_error", "t1env_version",
           "t1env_measure_heights", "t1env_critic_heights", "t1env_reset_idx", "t1env_set_substep_log"]

# include/t1policy.h: the DH policy's HIP kernels, in the same library
POLICY_EXPORTS = ["t1policy_conv1d_forward", "t1policy_history_rows", "t1policy_conv1d_frag_bytes",
                  "t1policy_conv1d_pack_weights", "t1policy_conv1d_forward_packed", "t1policy_heads_frag_bytes",
                  "t1policy_heads_pack", "t1policy_heads_forward", "t1policy_conv1_bf16_frag_bytes",
                  "t1policy_conv1_bf16_workspace_bytes", "t1policy_conv1_pack_bf16", "t1policy_conv1_forward_bf16",
                  "t1policy_conv1_wgrad_bf16", "t1policy_colsum_workspace_bytes", "t1policy_colsum",
                  "t1policy_slice_sum", "t1policy_linear_wgrad_workspace_bytes", "t1policy_linear_wgrad_bf16",
                  "t1policy_fold_rows", "t1policy_gather_rows", "t1policy_conv1_wgrad_f32",
                  "t1policy_linear_wgrad_f32", "t1policy_gemm_nt_f32", "t1policy_gemm_f32",
                  "t1policy_linear_wgrad_f32x"]

_lib = None


def load():
    """Load the HIP library (raises if it is missing: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libt1env_hip.so not built ({LIB_PATH}); run `python -m ti5_isaacgym_amd.build`")
    lib = C.CDLL(LIB_PATH)
    check_stamp(lib, LIB_PATH)
    P = C.POINTER
    vp = C.c_void_p
    sig = {
        "t1env_create": ([P(Model), P(Config), P(Buffers), P(vp)], C.c_int),
        "t1env_destroy": ([vp], C.c_int),
        "t1env_init": ([vp, vp], C.c_int),
        "t1env_set_terrain": ([vp, vp, i32, i32, f32, f32, f32, i32], C.c_int),
        "t1env_reset_all": ([vp, P(StepArgs), vp], C.c_int),
        "t1env_step": ([vp, vp, P(StepArgs), vp], C.c_int),
        "t1env_step_physics_and_rewards": ([vp, vp, P(StepArgs), vp], C.c_int),
        "t1env_step_reset_and_observe": ([vp, P(StepArgs), vp], C.c_int),
        "t1env_step_injected": ([vp, vp, P(StepArgs), P(Injected), vp], C.c_int),
        "t1env_set_fused": ([vp, i32], C.c_int),
        "t1env_set_substep_log": ([vp, P(SubstepLog)], C.c_int),
        "t1env_set_timing": ([vp, i32], C.c_int),
        "t1env_get_timing": ([vp, C.POINTER(C.c_double), i32p], C.c_int),
        "t1env_last_error": ([], C.c_char_p),
        "t1env_version": ([], C.c_char_p),
        "t1env_measure_heights": ([vp, vp, i32, vp, vp], C.c_int),
        "t1env_reset_idx": ([vp, vp, P(StepArgs), vp], C.c_int),
        "t1env_critic_heights": ([vp, i32, i32, f32, vp, vp, vp, vp], C.c_int),
        "t1policy_conv1d_forward": ([vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp], C.c_int),
        "t1policy_history_rows": ([vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp], C.c_int),
        "t1policy_conv1d_frag_bytes": ([], C.c_int),
        "t1policy_conv1d_pack_weights": ([vp, vp, i32, i32, i32, vp], C.c_int),
        "t1policy_conv1d_forward_packed": ([vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp], C.c_int),
        "t1policy_heads_frag_bytes": ([], C.c_int),
        "t1policy_heads_pack": ([vp, vp, vp, vp], C.c_int),
        "t1policy_heads_forward": ([vp, vp, vp, vp, vp, i32, vp, i32, vp, vp, vp, vp, vp, vp, i32, vp], C.c_int),
        "t1policy_conv1_bf16_frag_bytes": ([], C.c_int),
        "t1policy_conv1_bf16_workspace_bytes": ([], C.c_int),
        "t1policy_conv1_pack_bf16": ([vp, vp, i32, i32, i32, vp], C.c_int),
        "t1policy_conv1_forward_bf16": ([vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp], C.c_int),
        "t1policy_conv1_wgrad_bf16": ([vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp], C.c_int),
        "t1policy_conv1_wgrad_f32": ([vp, vp, vp, vp, vp, i32, i32, i32, i32, i32, i32, vp], C.c_int),
        "t1policy_colsum_workspace_bytes": ([i32, i32], C.c_int),
        "t1policy_colsum": ([vp, i32, i32, i32, vp, vp, vp], C.c_int),
        "t1policy_slice_sum": ([vp, i32, i32, vp, vp], C.c_int),
        "t1policy_linear_wgrad_workspace_bytes": ([i32, i32, i32], C.c_longlong),
        "t1policy_linear_wgrad_bf16": ([vp, vp, i32, i32, i32, vp, C.c_longlong, vp, vp, i32, vp], C.c_int),
        "t1policy_linear_wgrad_f32": ([vp, vp, i32, i32, i32, vp, C.c_longlong, vp, vp, i32, vp], C.c_int),
        "t1policy_linear_wgrad_f32x": ([vp, vp, i32, i32, i32, i32, vp, C.c_longlong, vp, vp, i32, vp], C.c_int),
        "t1policy_gemm_nt_f32": ([vp, vp, vp, vp, vp, i32, i32, i32, i32, vp], C.c_int),
        "t1policy_gemm_f32": ([vp, i32, vp, i32, i32, vp, vp, vp, i32, i32, i32, i32, vp], C.c_int),
        "t1policy_fold_rows": ([vp, vp, i32, i32, i32, i32, i32, i32, vp], C.c_int),
        "t1policy_gather_rows": ([vp, vp, vp, i32, vp, i32, vp], C.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    _lib = lib
    return lib


def check_stamp(lib, path):
    """Refuse a library built from other sources than this tree's (build.source_stamp, compiled into t1env_version):
    a stale product or guard library would otherwise fail later with a missing symbol or, worse, run old code.  Skipped
    when the sources are not present (an installed copy) or T1ENV_SKIP_STAMP=1."""
    from . import build as _build
    if os.environ.get("T1ENV_SKIP_STAMP") == "1" or not _build.DEPS:
        return
    fn = lib.t1env_version
    fn.argtypes, fn.restype = [], C.c_char_p
    ver = fn().decode()
    got = ver.split("src:", 1)[1].strip() if "src:" in ver else None
    want = _build.source_stamp()
    if got != want:
        raise RuntimeError(f"{path} is stale: built from sources {got or '(unstamped)'}, this tree's are {want}; "
                           "rebuild it (python -m ti5_isaacgym_amd.build, or __graft_entry__.build() for the guard "
                           "library too)")


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc}): {load().t1env_last_error().decode()}")
