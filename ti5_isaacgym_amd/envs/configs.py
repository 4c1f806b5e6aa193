"""Config API of the reference, re-stated: nested classes instantiated recursively, same attribute names.

Mirrors humanoid/envs/base/base_config.py (BaseConfig), humanoid/envs/base/legged_robot_config.py
(LeggedRobotCfg / LeggedRobotCfgPPO) and humanoid/envs/t1/t1_dh_stand_config.py (DHT1StandCfg /
DHT1StandCfgPPO) so user code that edits ``cfg.env.num_envs``, ``cfg.terrain.mesh_type``,
``cfg.domain_rand.*``... works unchanged.  Values are the reference's; only what the step path or its
callers read is kept (viewer/CLI-only knobs are dropped).
"""
import inspect


class BaseConfig:
    """Instantiates every nested class recursively (reference base_config.py:3-25)."""

    def __init__(self):
        self._instantiate(self)

    @staticmethod
    def _instantiate(obj):
        for key in dir(obj):
            if key == "__class__":
                continue
            val = getattr(obj, key)
            if inspect.isclass(val):
                inst = val()
                setattr(obj, key, inst)
                BaseConfig._instantiate(inst)


class LeggedRobotCfg(BaseConfig):
    class env:
        num_envs, num_observations, num_privileged_obs, num_actions = 4096, 235, None, 12
        short_frame_stack, env_spacing, send_timeouts, episode_length_s, num_commands = 4, 3, True, 20, 5
        add_stand_bool, add_target_dof_scale = False, False
        # build extension (not in the reference): storage dtype of the obs / critic histories the env returns;
        # "fp16" = BASELINE config 5's fp16 state (values computed in fp32 and rounded once)
        state_dtype = "fp32"

    class terrain:
        mesh_type, horizontal_scale, vertical_scale, border_size, curriculum = "trimesh", 0.1, 0.005, 25, True
        static_friction, dynamic_friction, restitution, measure_heights = 1.0, 1.0, 0.0, False
        measured_points_x = [round(-0.8 + 0.1 * i, 1) for i in range(17)]
        measured_points_y = [round(-0.5 + 0.1 * i, 1) for i in range(11)]
        num_height = len(measured_points_x) * len(measured_points_y)
        selected, terrain_kwargs, max_init_terrain_level = False, None, 5
        terrain_length, terrain_width, num_rows, num_cols, platform = 8.0, 8.0, 10, 20, 3.0
        terrain_dict = {"flat": 0.15, "rough flat": 0.15, "rough slope up": 0.0, "rough slope down": 0.0,
                        "slope up": 0.0, "slope down": 0.0, "stairs up": 0.35, "stairs down": 0.25,
                        "discrete": 0.0, "wave": 0.0}
        terrain_proportions = list(terrain_dict.values())
        rough_flat_range, slope_range, rough_slope_range = [0.005, 0.02], [0, 0.4], [0.005, 0.02]
        stair_width_range, stair_height_range, discrete_height_range = [0.25, 0.25], [0.04, 0.1], [0.05, 0.25]
        slope_treshold = 0.75

    class commands:
        curriculum, max_curriculum, num_commands, resampling_time, heading_command = True, 1, 4, 10, True

        class ranges:
            lin_vel_x, lin_vel_y, ang_vel_yaw, heading = [-1.0, 1.0], [-1.0, 1.0], [-1, 1], [-3.14, 3.14]

    class init_state:
        pos, rot, lin_vel, ang_vel = [0.0, 0.0, 1.0], [0.0, 0.0, 0.0, 1.0], [0.0, 0.0, 0.0], [0.0, 0.0, 0.0]
        default_joint_angles = {"joint_a": 0.0, "joint_b": 0.0}

    class control:
        control_type, action_scale, decimation = "P", 0.5, 4
        stiffness = {"joint_a": 10.0, "joint_b": 15.0}
        damping = {"joint_a": 1.0, "joint_b": 1.5}

    class asset:
        file, name, foot_name = "", "legged_robot", "None"
        penalize_contacts_on, terminate_after_contacts_on = [], []
        disable_gravity, collapse_fixed_joints, fix_base_link, default_dof_drive_mode = False, True, False, 3
        self_collisions, replace_cylinder_with_capsule, flip_visual_attachments = 0, True, True
        density, angular_damping, linear_damping = 0.001, 0, 0
        max_angular_velocity, max_linear_velocity, armature, thickness = 1000, 1000, 0, 0.01

    class domain_rand:
        randomize_friction, friction_range, restitution_range = False, [0.2, 1.3], [0.0, 0.4]
        push_robots, push_interval_s, update_step, push_duration = False, 4, 2000 * 60, [0, 0.1, 0.2, 0.3]
        max_push_vel_xy, max_push_ang_vel = 0.2, 0.2
        add_ext_force, ext_force_max_xy, ext_force_max_z, ext_torque_max = False, 10, 5, 0
        ext_force_interval_s, add_update_step, add_duration = 10, 2000 * 60, [0, 0.1, 0.2, 0.3]
        randomize_base_mass, added_mass_range = False, [-2.5, 2.5]
        randomize_com, com_displacement_range = False, [[-0.05, 0.05]] * 3
        randomize_link_com, randomize_base_inertia, randomize_link_inertia = False, False, False
        randomize_gains, stiffness_multiplier_range, damping_multiplier_range = False, [0.8, 1.2], [0.8, 1.2]
        randomize_torque, torque_multiplier_range = False, [0.8, 1.2]
        randomize_link_mass, added_link_mass_range = False, [0.9, 1.1]
        randomize_motor_offset, motor_offset_range = False, [-0.035, 0.035]
        randomize_joint_friction, randomize_joint_friction_each_joint = False, False
        randomize_joint_damping, randomize_joint_damping_each_joint = False, False
        randomize_joint_armature, randomize_joint_armature_each_joint = False, False
        joint_armature_range = [0.0001, 0.05]
        add_lag, randomize_lag_timesteps, randomize_lag_timesteps_perstep, lag_timesteps_range = False, True, False, [5, 70]
        add_dof_lag, randomize_dof_lag_timesteps, randomize_dof_lag_timesteps_perstep = False, True, False
        dof_lag_timesteps_range = [0, 40]
        add_dof_pos_vel_lag = False
        add_imu_lag, randomize_imu_lag_timesteps, randomize_imu_lag_timesteps_perstep = False, True, False
        imu_lag_timesteps_range = [1, 10]
        randomize_coulomb_friction, joint_coulomb_range, joint_viscous_range = False, [0.1, 0.9], [0.10, 0.70]

    class rewards:
        class scales:
            termination = tracking_lin_vel = tracking_ang_vel = lin_vel_z = ang_vel_xy = orientation = 0.0
            torques = dof_vel = dof_acc = base_height = feet_air_time = collision = 0.0
            feet_stumble = action_rate = stand_still = 0.0
        only_positive_rewards, tracking_sigma, max_contact_force = True, 0.25, 100.0

    class normalization:
        class obs_scales:
            lin_vel, ang_vel, dof_pos, dof_vel, height_measurements = 2.0, 0.25, 1.0, 0.05, 5.0
        clip_observations, clip_actions = 100.0, 100.0

    class noise:
        add_noise, noise_level = True, 1.0

        class noise_scales:
            dof_pos, dof_vel, lin_vel, ang_vel, gravity, height_measurements = 0.01, 1.5, 0.1, 0.2, 0.05, 0.1

    class viewer:
        ref_env, pos, lookat = 0, [22, 3, 6], [0, 3, 0]

    class sim:
        dt, substeps, gravity, up_axis = 0.005, 1, [0.0, 0.0, -9.81], 1

        class physx:
            num_threads, solver_type, num_position_iterations, num_velocity_iterations = 10, 1, 4, 0
            contact_offset, rest_offset, bounce_threshold_velocity = 0.01, 0.0, 0.5
            max_depenetration_velocity, max_gpu_contact_pairs = 1.0, 2 ** 23
            default_buffer_size_multiplier, contact_collection = 5, 2


class LeggedRobotCfgPPO(BaseConfig):
    seed, runner_class_name = 1, "OnPolicyRunner"

    class policy:
        init_noise_std, actor_hidden_dims, critic_hidden_dims = 1.0, [512, 256, 128], [512, 256, 128]

    class algorithm:
        value_loss_coef, use_clipped_value_loss, clip_param, entropy_coef = 1.0, True, 0.2, 0.01
        num_learning_epochs, num_mini_batches, learning_rate, schedule = 5, 4, 1.0e-3, "adaptive"
        gamma, lam, desired_kl, max_grad_norm = 0.99, 0.95, 0.01, 1.0

    class runner:
        policy_class_name, algorithm_class_name, num_steps_per_env, max_iterations = "ActorCritic", "PPO", 24, 1500
        save_interval, experiment_name, run_name, resume, load_run, checkpoint, resume_path = 100, "test", "", False, -1, -1, None


_ANGLE = 0.3


class DHT1StandCfg(LeggedRobotCfg):
    """t1_dh_stand task (reference humanoid/envs/t1/t1_dh_stand_config.py:4-427)."""

    class env(LeggedRobotCfg.env):
        frame_stack, short_frame_stack, c_frame_stack, num_single_obs = 66, 5, 3, 47
        num_observations = frame_stack * num_single_obs
        single_num_privileged_obs = 73
        num_privileged_obs = c_frame_stack * single_num_privileged_obs
        num_actions, num_envs, episode_length_s, use_ref_actions = 12, 4096, 24, False
        single_linvel_index, num_commands = 53, 5

    class safety:
        pos_limit, vel_limit, torque_limit = 1.0, 1.0, 0.85

    class asset(LeggedRobotCfg.asset):
        file = "{LEGGED_GYM_ROOT_DIR}/resources/robots/t1/urdf/t1.urdf"
        name, foot_name, knee_name = "t1", "6_link", "4_link"
        terminate_after_contacts_on, penalize_contacts_on = ["base_link"], ["base_link"]
        self_collisions, flip_visual_attachments, replace_cylinder_with_capsule, fix_base_link = 0, False, False, False

    class terrain(LeggedRobotCfg.terrain):
        mesh_type, curriculum, measure_heights = "trimesh", True, False
        static_friction, dynamic_friction, restitution = 0.6, 0.6, 0
        terrain_length, terrain_width, num_rows, num_cols, max_init_terrain_level, platform = 8, 8, 20, 20, 5, 3
        terrain_dict = {"flat": 0.5, "rough flat": 0.3, "slope up": 0.1, "slope down": 0.1, "rough slope up": 0,
                        "rough slope down": 0, "stairs up": 0, "stairs down": 0, "discrete": 0, "wave": 0}
        terrain_proportions = list(terrain_dict.values())
        rough_flat_range, slope_range, rough_slope_range = [0.005, 0.01], [0, 0.1], [0.005, 0.02]
        stair_width_range, stair_height_range, discrete_height_range = [0.25, 0.25], [0.01, 0.1], [0.0, 0.01]

    class noise(LeggedRobotCfg.noise):
        add_noise, noise_level = True, 1.5

        class noise_scales(LeggedRobotCfg.noise.noise_scales):
            dof_pos, dof_vel, ang_vel, lin_vel, quat, gravity, height_measurements = 0.02, 1.5, 0.2, 0.1, 0.1, 0.05, 0.1

    class init_state(LeggedRobotCfg.init_state):
        pos, init_angle = [0.0, 0.0, 1.1], _ANGLE
        default_joint_angles = {f"leg_{s}{i}_joint": a for s in "lr"
                                for i, a in zip(range(1, 7), (0, 0, -_ANGLE, 2 * _ANGLE, -_ANGLE, 0))}

    class control(LeggedRobotCfg.control):
        control_type, action_scale, decimation = "P", 0.5, 10
        stiffness = {"1_joint": 50, "2_joint": 70, "3_joint": 90, "4_joint": 120, "5_joint": 50, "6_joint": 30}
        damping = {"1_joint": 5, "2_joint": 7, "3_joint": 9, "4_joint": 12, "5_joint": 5, "6_joint": 3}

    class sim(LeggedRobotCfg.sim):
        dt, substeps, up_axis = 0.001, 1, 1

        class physx(LeggedRobotCfg.sim.physx):
            num_threads, solver_type, num_position_iterations, num_velocity_iterations = 10, 1, 4, 0
            contact_offset, rest_offset, bounce_threshold_velocity, max_depenetration_velocity = 0.01, 0.0, 0.5, 1.0
            max_gpu_contact_pairs, default_buffer_size_multiplier, contact_collection = 2 ** 23, 5, 2

    class domain_rand(LeggedRobotCfg.domain_rand):
        randomize_friction, friction_range, restitution_range = True, [0.2, 1.3], [0.0, 0.4]
        push_robots, push_interval_s, update_step = False, 6, 2500 * 24
        push_duration, max_push_vel_xy, max_push_ang_vel = [0, 0.05, 0.1, 0.15, 0.2, 0.25, 0.3], 0.2, 0.2
        add_ext_force, ext_force_max_x, ext_force_max_y, ext_force_max_z, ext_torque_max = True, 600, 400, 5, 0
        ext_force_interval_s, add_update_step, add_duration = 4, 4000 * 24, [0.0, 0.05, 0.1, 0.15]
        randomize_base_mass, added_mass_range = True, [-2.5, 2.5]
        randomize_com, com_displacement_range = True, [[-0.05, 0.05], [-0.05, 0.05], [-0.05, 0.05]]
        randomize_gains, stiffness_multiplier_range, damping_multiplier_range = True, [0.8, 1.2], [0.8, 1.2]
        randomize_torque, torque_multiplier_range = True, [0.8, 1.2]
        randomize_link_mass, added_link_mass_range = True, [0.9, 1.1]
        randomize_motor_offset, motor_offset_range = True, [-0.035, 0.035]
        randomize_joint_armature, randomize_joint_armature_each_joint = True, True
        joint_armature_range = [0.001, 0.05]
        for _i, (_lo, _hi) in enumerate([(0.15 * 0.8, 0.15 * 1.2), (0.15 * 0.8, 0.15 * 1.2), (3.6 * 0.5, 3.6 * 1.0),
                                         (3.6 * 0.5, 3.6 * 1.0), (0.1 * 0.5, 0.1 * 1.1), (0.028 * 0.5, 0.028 * 1.5)] * 2):
            locals()[f"joint_{_i + 1}_armature_range"] = [_lo, _hi]
        del _i, _lo, _hi
        add_lag, randomize_lag_timesteps, randomize_lag_timesteps_perstep, lag_timesteps_range = True, True, False, [0, 30]
        add_dof_lag, randomize_dof_lag_timesteps, randomize_dof_lag_timesteps_perstep = True, True, False
        dof_lag_timesteps_range = [0, 30]
        add_dof_pos_vel_lag = False
        add_imu_lag, randomize_imu_lag_timesteps, randomize_imu_lag_timesteps_perstep = True, True, False
        imu_lag_timesteps_range = [0, 10]
        randomize_coulomb_friction, joint_coulomb_range, joint_viscous_range = True, [0.1, 1.0], [0.1, 0.9]

    class commands(LeggedRobotCfg.commands):
        curriculum, max_curriculum, num_commands, resampling_time = True, 1.5, 4, 25
        gait = ["walk_omnidirectional", "stand", "walk_omnidirectional"]
        gait_time_range = {"walk_sagittal": [2, 6], "walk_lateral": [2, 6], "rotate": [2, 3], "stand": [2, 3],
                           "walk_omnidirectional": [4, 6]}
        stand_time, heading_command, stand_com_threshold, sw_switch = 18, False, 0.05, True

        class ranges:
            lin_vel_x, lin_vel_y, ang_vel_yaw, heading = [-0.5, 0.5], [-0.5, 0.5], [-0.5, 0.5], [-3.14, 3.14]

    class rewards:
        base_height_target, foot_min_dist, foot_max_dist, knee_min_dist, knee_max_dist = 0.965, 0.15, 0.45, 0.12, 0.35
        target_joint_pos_scale, target_feet_height, target_feet_height_max, cycle_time = 0.3, 0.02, 0.08, 0.8
        only_positive_rewards, tracking_sigma, max_contact_force = True, 5, 500

        class scales:
            joint_pos, feet_clearance, feet_contact_number, feet_air_time, foot_slip = 4, 1, 1.2, 1, -0.5
            feet_distance, knee_distance, feet_rotation, feet_contact_forces = 0.2, 0.2, 0.8, -0.01
            tracking_lin_vel, tracking_ang_vel, vel_mismatch_exp, low_speed, track_vel_hard = 1.5, 0.8, 0.5, 0.2, 0.5
            default_joint_pos, orientation, base_height, base_acc = 1, 1, 0.2, 0.2
            action_smoothness, torques, dof_vel, dof_acc, collision, stand_still = -0.03, -2e-7, -2e-5, -5e-7, -1, 2.5

    class normalization:
        class obs_scales:
            lin_vel, ang_vel, dof_pos, dof_vel, quat, height_measurements = 2, 1, 1, 0.05, 1, 5.0
        clip_observations, clip_actions = 100, 100


class DHT1StandCfgPPO(LeggedRobotCfgPPO):
    seed, runner_class_name = 5, "DHOnPolicyRunner"

    class policy:
        init_noise_std = 1.0
        actor_hidden_dims, critic_hidden_dims, state_estimator_hidden_dims = [512, 256, 128], [768, 256, 128], [256, 128, 64]
        kernel_size, filter_size, stride_size, lh_output_dim = [6, 4], [32, 16], [3, 2], 64
        in_channels = DHT1StandCfg.env.frame_stack

    class algorithm(LeggedRobotCfgPPO.algorithm):
        entropy_coef, learning_rate, num_learning_epochs, gamma, lam, num_mini_batches = 0.001, 1e-5, 2, 0.994, 0.9, 4
        if DHT1StandCfg.terrain.measure_heights:   # t1_dh_stand_config.py:460-466
            lin_vel_idx = (DHT1StandCfg.env.single_num_privileged_obs + DHT1StandCfg.terrain.num_height) \
                * (DHT1StandCfg.env.c_frame_stack - 1) + DHT1StandCfg.env.single_linvel_index
        else:
            lin_vel_idx = DHT1StandCfg.env.single_num_privileged_obs * (DHT1StandCfg.env.c_frame_stack - 1) \
                + DHT1StandCfg.env.single_linvel_index

    class runner:
        policy_class_name, algorithm_class_name, num_steps_per_env, max_iterations = "ActorCriticDH", "DHPPO", 24, 30000
        save_interval, experiment_name, run_name, resume, load_run, checkpoint, resume_path = 500, "t1_dh_stand", "ti5", False, -1, -1, None
