"""gmx -- MI355X-native batched gripper env-step (the reference's MjClass hot path).

Host-side mirror of the reference's MjClass / MjEnv step contract over the C ABI
in include/gripper_mi355x.h.  Every env-step runs on the GPU; there is no CPU
fallback (the library raises ImportError when the HIP extension is missing).
"""
from ._lib import (load_library, Settings, ModelParams, Object, Spawn, SpawnParams, default_spawn_params,
                   Calibration, calibrate, CAL_TIMESTEP, CAL_GAUGES, CAL_REFERENCE_RETRY,
                   ModelBlob, ConfigBlob,
                   default_settings, make_object_set, BINARY_EVENTS, LINEAR_EVENTS, ACTION_KINDS,
                   SENSORS, LIB_PATH, env_state_dtype, env_state_view)
from .settings import canonical_settings, disable_noise, MAX_EPISODE_STEPS
from .env import BatchedGripperEnv, spawn_draws, spawn_int, random_fractions
from .policy import DevicePolicy, eps_threshold
from .scripted import GraspScript, in_use_actions

__all__ = ["load_library", "Settings", "ModelParams", "Object", "Spawn", "SpawnParams", "default_spawn_params",
           "Calibration", "calibrate", "CAL_TIMESTEP", "CAL_GAUGES", "CAL_REFERENCE_RETRY",
           "ModelBlob", "ConfigBlob",
           "default_settings", "make_object_set", "canonical_settings", "disable_noise",
           "BatchedGripperEnv", "spawn_draws", "spawn_int", "random_fractions", "MAX_EPISODE_STEPS", "BINARY_EVENTS",
           "LINEAR_EVENTS", "ACTION_KINDS", "SENSORS", "LIB_PATH", "DevicePolicy", "eps_threshold",
           "GraspScript", "in_use_actions", "env_state_dtype", "env_state_view"]
