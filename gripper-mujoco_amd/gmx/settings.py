"""Canonical settings: what rl/TrainingManager.py applies to `env.mj.set`.

`canonical_settings()` restates TrainingManager.wipe_cpp_settings (804-855),
apply_env_settings (937-1058) with the cpp section of
rl/baseline_settings/baseline_06-09-24_15-38.yaml (lines 76-205), and
create_reward_function(style="sensor_mixed_v1") (1200-1268) with the
set_sensor_* helpers (1082-1198).  Field names are the reference's.
"""
from __future__ import annotations

from ._lib import Settings, default_settings, ACTION_KINDS, SENSORS, BINARY_EVENTS, LINEAR_EVENTS

MAX_EPISODE_STEPS = 250        # baseline yaml env.max_episode_steps


def _set_br(s, name, reward, done, trigger):
    r = getattr(s, name)
    r.reward, r.done, r.trigger = reward, int(done), trigger


def _set_lr(s, name, reward, done, trigger, mn, mx, overshoot):
    # LinearReward::set never updates overshoot (mjclass.h:681 quirk): keep it
    r = getattr(s, name)
    r.reward, r.done, r.trigger, r.min, r.max = reward, int(done), trigger, mn, mx


def wipe(s: Settings) -> Settings:
    """TrainingManager.wipe_cpp_settings (804-855)."""
    s.auto_set_timestep = 1
    s.auto_calibrate_gauges = 1
    s.auto_sim_steps = 1
    s.auto_exceed_lateral_lim = 0
    s.curve_validation = 0
    s.render_on_step = 0
    for a in ACTION_KINDS:
        act = getattr(s, a)
        act.in_use, act.continous, act.value, act.sign = 0, 0, 0.0, 1
    s.use_termination_action = 0
    for n in BINARY_EVENTS:
        _set_br(s, n, 0.0, 0, 1)
    for n in LINEAR_EVENTS:
        r = getattr(s, n)
        r.reward, r.done, r.trigger = 0.0, 0, 1
    s.cap_reward = 0
    s.quit_if_cap_exceeded = 0
    s.reward_cap_lower_bound = -1e6
    s.reward_cap_upper_bound = 1e6
    s.use_HER = 0
    for n in SENSORS:
        sen = getattr(s, n)
        sen.in_use = 0
        sen.use_normalisation = 1
        sen.use_noise = 1
    s.sensor_n_prev_steps = 1
    s.state_n_prev_steps = 1
    s.motor_state_sensor.read_rate = -1
    s.base_state_sensor_XY.read_rate = -1
    s.base_state_sensor_Z.read_rate = -1
    for k in ("sensor_noise_mag", "sensor_noise_mu", "sensor_noise_std", "state_noise_mag",
              "state_noise_mu", "state_noise_std", "base_position_noise"):
        setattr(s, k, 0.0)
    return s


def set_gaussian_noise(sensor, mu, std):
    """Sensor::set_gaussian_noise (mjclass.h:123-128)."""
    sensor.noise_mag, sensor.noise_mu, sensor.noise_std, sensor.noise_overriden = 0.0, mu, std, 1


def canonical_settings(noise: bool = True, seed: int = 0) -> Settings:
    s = wipe(default_settings())
    s.debug = 0                      # MjEnv forces debug off (MjEnv.py:190)
    s.random_seed = seed
    # ---- cpp section of baseline_06-09-24_15-38.yaml ----
    s.XY_distance_threshold = 0.01
    acts = {"base_X": (0, 1, 0.002), "base_Y": (0, 1, 0.002), "base_Z": (1, 1, 0.002),
            "base_yaw": (0, 1, 0.005), "gripper_Z": (1, 1, 0.004),
            "gripper_prismatic_X": (1, -1, 0.002), "gripper_revolute_Y": (1, -1, 0.015)}
    for name, (use, sign, value) in acts.items():
        a = getattr(s, name)
        a.in_use, a.sign, a.value = use, sign, value
    s.base_position_noise = 0.005
    s.cap_reward = 0
    s.continous_actions = 1
    s.fingertip_min_mm = -12.5
    s.gripper_target_height = 0.02
    s.lift_height = 0.015
    s.oob_distance = 0.075
    s.palm_scale_factor = 1.0
    s.randomise_colours = 0
    s.saturation_yield_factor = 1.5
    sens = {"base_state_sensor_XY": (0, 0.0, -1), "base_state_sensor_Z": (1, 0.0, -1),
            "base_state_sensor_yaw": (0, 0.0, -1), "bending_gauge": (1, 20.0, 10),
            "cartesian_contacts_XYZ": (0, 0.0, -1), "motor_state_sensor": (1, 0.0, -1),
            "palm_sensor": (1, 6.0, 10), "wrist_sensor_XY": (0, 5.0, 10), "wrist_sensor_Z": (1, 10.0, 10)}
    for name, (use, norm, rate) in sens.items():
        sen = getattr(s, name)
        sen.in_use, sen.normalise, sen.read_rate = use, norm, rate
    set_gaussian_noise(s.base_state_sensor_Z, 0.1, 0.0)
    set_gaussian_noise(s.cartesian_contacts_XYZ, 0, 0)
    s.sensor_n_prev_steps = 3
    s.sensor_noise_mu = 0.05
    s.sensor_noise_std = 0.025
    s.sensor_sample_mode = 2
    s.stable_finger_force = 1.0
    s.stable_finger_force_lim = 4.0
    s.stable_palm_force = 1.0
    s.stable_palm_force_lim = 4.0
    s.state_n_prev_steps = 3
    s.state_noise_mu = 0.025
    s.state_noise_std = 0.0
    s.state_sample_mode = 4
    s.termination_threshold = 0.9
    s.time_for_action = 0.2
    s.use_termination_action = 0
    # ---- reward: create_reward_function("sensor_mixed_v1") ----
    mBend, gBend, xBend, dBend = 0.0, s.stable_finger_force, s.stable_finger_force_lim, 5.0
    mPalm, gPalm, xPalm, dPalm = 0.0, s.stable_palm_force, s.stable_palm_force_lim, 5.0
    xWrist, dWrist = 6.0, 8.0
    _set_br(s, "step_num", -0.01, 0, 1)
    bonus = 0.002 * 1.0
    _set_br(s, "lifted", bonus, 0, 1)
    _set_br(s, "lifted_to_height", bonus, 0, 1)
    _set_br(s, "object_stable", bonus, 0, 1)
    _set_lr(s, "good_bend_sensor", bonus, 0, 1, mBend, gBend, -1)
    _set_lr(s, "good_palm_sensor", bonus, 0, 1, mPalm, gPalm, -1)
    pen = -0.002 * 1.0
    _set_br(s, "exceed_limits", pen, 0, 1)
    _set_lr(s, "exceed_bend_sensor", pen, 0, 1, xBend, dBend, -1)
    _set_lr(s, "exceed_palm_sensor", pen, 0, 1, xPalm, dPalm, -1)
    _set_lr(s, "exceed_wrist_sensor", pen, 0, 1, xWrist, dWrist, -1)
    _set_lr(s, "action_penalty_sq", pen * 2, 0, 1, 0.1, 3.0, -1)
    scale = 100.0 / MAX_EPISODE_STEPS       # Settings::scale_rewards
    for n in BINARY_EVENTS + LINEAR_EVENTS:
        getattr(s, n).reward *= scale
    _set_br(s, "stable_height", 1.0, 1, 1)
    _set_br(s, "oob", -1.0, 1, 1)
    _set_lr(s, "dangerous_bend_sensor", -1.0, 1, 1, dBend, dBend, -1)
    _set_lr(s, "dangerous_palm_sensor", -1.0, 1, 1, dPalm, dPalm, -1)
    _set_lr(s, "dangerous_wrist_sensor", -1.0, 1, 1, dWrist, dWrist, -1)
    s.object_stable.trigger = 1
    if not noise:
        disable_noise(s)
    return s


def disable_noise(s: Settings) -> Settings:
    """Parity configuration: noise off, base position noise off."""
    for k in ("sensor_noise_mag", "sensor_noise_mu", "sensor_noise_std", "state_noise_mag",
              "state_noise_mu", "state_noise_std", "base_position_noise"):
        setattr(s, k, 0.0)
    for n in SENSORS:
        sen = getattr(s, n)
        sen.noise_overriden = 0
    return s
