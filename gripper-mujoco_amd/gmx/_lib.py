"""ctypes binding of the C ABI in include/gripper_mi355x.h.

The struct layouts are generated from the same X-macro list the C side uses
(include/gm_settings.def) and verified against gm_struct_size() at load time,
so a layout drift fails loudly instead of corrupting settings.
"""
from __future__ import annotations

import ctypes as C
import os
import re

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_DIR = os.path.dirname(PKG_DIR)
INCLUDE_DIR = os.path.join(REPO_DIR, "include")
LIB_PATH = os.path.join(PKG_DIR, "lib", "libgm.so")

GM_MAX_SEG = 10
GM_MAX_BODY = 40
GM_MAX_DOF = 44
GM_MAX_QPOS = 48
GM_RING = 64
GM_MAX_GEOM = 40
GM_MAX_PAIR = 80
GM_MAX_CON = 32
GM_MAX_LOCK = 4
GM_MAX_EFC = 4 * GM_MAX_CON + GM_MAX_LOCK
GM_MAX_OBJSET = 64

GEOM_SPHERE, GEOM_CYLINDER, GEOM_BOX = 2, 5, 6

_CTYPE = {"int32_t": C.c_int32, "uint32_t": C.c_uint32, "double": C.c_double, "float": C.c_float}


class Sensor(C.Structure):
    _fields_ = [("in_use", C.c_int32), ("normalise", C.c_float), ("read_rate", C.c_float),
                ("use_normalisation", C.c_int32), ("use_noise", C.c_int32),
                ("raw_value_offset", C.c_float), ("noise_mag", C.c_float), ("noise_mu", C.c_float),
                ("noise_std", C.c_float), ("noise_overriden", C.c_int32), ("prev_steps", C.c_int32),
                ("readings_per_step", C.c_int32), ("total_readings", C.c_int32)]


class Action(C.Structure):
    _fields_ = [("in_use", C.c_int32), ("continous", C.c_int32), ("value", C.c_double),
                ("sign", C.c_int32)]


class BinaryReward(C.Structure):
    _fields_ = [("reward", C.c_float), ("done", C.c_int32), ("trigger", C.c_int32)]


class LinearReward(C.Structure):
    _fields_ = [("reward", C.c_float), ("done", C.c_int32), ("trigger", C.c_int32),
                ("min", C.c_float), ("max", C.c_float), ("overshoot", C.c_float)]


def parse_settings_def(path=None):
    """Return [(kind, name, args...)] in declaration order from gm_settings.def."""
    path = path or os.path.join(INCLUDE_DIR, "gm_settings.def")
    out = []
    pat = re.compile(r"^\s*GM_(XX|SS|AA|BR|LR)\(\s*([A-Za-z0-9_]+)\s*,(.*)\)\s*$")
    with open(path) as f:
        for line in f:
            m = pat.match(line)
            if not m:
                continue
            args = [a.strip() for a in m.group(3).split(",")]
            out.append((m.group(1), m.group(2), args))
    return out


SETTINGS_DEF = parse_settings_def()
BINARY_EVENTS = [n for k, n, _ in SETTINGS_DEF if k == "BR"]
LINEAR_EVENTS = [n for k, n, _ in SETTINGS_DEF if k == "LR"]
ACTION_KINDS = [n for k, n, _ in SETTINGS_DEF if k == "AA"]
SENSORS = [n for k, n, _ in SETTINGS_DEF if k == "SS"]


def _settings_fields():
    fields = []
    for kind, name, args in SETTINGS_DEF:
        if kind == "XX":
            fields.append((name, _CTYPE[args[0]]))
        elif kind == "SS":
            fields.append((name, Sensor))
        elif kind == "AA":
            fields.append((name, Action))
        elif kind == "BR":
            fields.append((name, BinaryReward))
        else:
            fields.append((name, LinearReward))
    return fields


class Settings(C.Structure):
    _fields_ = _settings_fields()


class ModelParams(C.Structure):
    _fields_ = [("n_seg", C.c_int32), ("finger_length", C.c_double), ("finger_width", C.c_double),
                ("finger_thickness", C.c_double), ("finger_E", C.c_double),
                ("hook_length", C.c_double), ("hook_angle_degrees", C.c_double),
                ("fingertip_clearance", C.c_double), ("segment_inertia_scaling", C.c_double),
                ("timestep", C.c_double), ("pgs_iterations", C.c_int32),
                ("collision_half_thickness", C.c_double), ("segment_damping", C.c_double),
                ("segment_damping_power", C.c_double), ("segment_armature", C.c_double),
                ("segment_armature_power", C.c_double), ("mujoco_actuators", C.c_int32), ("pad_params", C.c_int32),
                ("actuator_armature", C.c_double * 4)]


class Object(C.Structure):
    _fields_ = [("type", C.c_int32), ("size", C.c_double * 3), ("mass", C.c_double),
                ("friction", C.c_double)]


class Spawn(C.Structure):
    _fields_ = [("object_index", C.c_int32), ("x", C.c_double), ("y", C.c_double),
                ("zrot", C.c_double)]


class SpawnParams(C.Structure):
    """MjType::SpawnParams (mjclass.h:916-931; bind.cpp:411-430): same field names."""
    _fields_ = [("index", C.c_int32), ("pad", C.c_int32), ("x", C.c_double), ("y", C.c_double),
                ("zrot", C.c_double), ("xrange", C.c_double), ("yrange", C.c_double),
                ("rotrange", C.c_double), ("xmin", C.c_double), ("xmax", C.c_double),
                ("ymin", C.c_double), ("ymax", C.c_double), ("smallest_gap", C.c_double),
                ("xy_increment", C.c_double), ("rot_increment", C.c_double)]


class RolloutParams(C.Structure):
    """gm_rollout_params (include/gripper_mi355x.h)."""
    _fields_ = [("action_mode", C.c_int32), ("max_episode_steps", C.c_int32), ("seed", C.c_uint64),
                ("jitter", C.c_float), ("pad", C.c_int32)]


class Calibration(C.Structure):
    """gm_calibration: the automatic settings of MjClass::configure_settings
    (mjclass.cpp:241-308) found by simulation."""
    _fields_ = [("timestep", C.c_double), ("sim_steps_per_action", C.c_int32), ("n_tested", C.c_int32),
                ("search_timestep", C.c_double), ("yield_load", C.c_double),
                ("bend_gauge_normalise", C.c_double), ("bending_normalise", C.c_float),
                ("sim_gauge_raw_to_N_factor", C.c_float), ("wrist_Z_offset", C.c_float),
                ("gauge_retries", C.c_int32)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


CAL_TIMESTEP, CAL_GAUGES, CAL_REFERENCE_RETRY = 1, 2, 4


def calibrate(model, cfg, objects, what: int = CAL_TIMESTEP | CAL_GAUGES, device: int = 0):
    """Batched device calibration (gm_calibrate): returns (Calibration, trace) where trace
    is the timestep search's [(candidate_dt, unstable), ...] in the reference's order."""
    lib = load_library()
    out = Calibration()
    tdt = (C.c_double * 256)()
    tbad = (C.c_uint8 * 256)()
    rc = lib.gm_calibrate(model.ptr, cfg.ptr, C.cast(objects, C.c_void_p), len(objects), int(device), int(what),
                          C.byref(out), tdt, tbad, 256)
    if rc != 0:
        raise RuntimeError(f"gm_calibrate failed ({rc})")
    n = min(out.n_tested, 256)
    return out, [(float(tdt[i]), bool(tbad[i])) for i in range(n)]


def default_spawn_params() -> "SpawnParams":
    p = SpawnParams()
    load_library().gm_default_spawn_params(C.byref(p))
    return p


_lib = None


def load_library(path: str | None = None):
    """Load libgm.so.  Raises ImportError (loudly) when the HIP extension is missing:
    there is no CPU fallback for the product path."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("GM_LIB") or LIB_PATH   # GM_LIB: developer A/B builds
    # One HIP runtime per process: torch's libc10_hip pulls its bundled libamdhip64 by
    # the unversioned name, so if libgm (NEEDED libamdhip64.so.7) loaded first a second
    # runtime would appear and one of them sees no devices.  Loading torch first makes
    # libgm bind to torch's runtime (same SONAME), so RCCL / torch tensors and our
    # kernels share streams and device pointers.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(p):
        raise ImportError(
            f"gripper-mi355x HIP extension not built: {p} is missing "
            "(run `python -c 'import __graft_entry__ as g; g.build()'` from the repo root)")
    lib = C.CDLL(p)
    _declare(lib)
    sizes = {0: Settings, 3: Object, 4: Spawn, 5: ModelParams, 6: SpawnParams, 7: Calibration}
    for which, cls in sizes.items():
        n = lib.gm_struct_size(which)
        if n < 0 and os.environ.get("GM_LIB"):
            continue   # an older developer build without this struct
        if n != C.sizeof(cls):
            raise ImportError(f"struct layout mismatch for {cls.__name__}: C {n} vs ctypes {C.sizeof(cls)}")
    if path is None:
        _lib = lib
    return lib


def _declare(lib):
    vp, i32, f32p, i32p, u8p, f64p = C.c_void_p, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_int32), \
        C.POINTER(C.c_uint8), C.POINTER(C.c_double)
    sig = {
        "gm_version": (C.c_char_p, []),
        "gm_device_count": (i32, []),
        "gm_struct_size": (C.c_int64, [i32]),
        "gm_model_info": (None, [vp, i32p]),
        "gm_config_info": (None, [vp, i32p]),
        "gm_default_model_params": (None, [vp]),
        "gm_build_model": (i32, [vp, vp]),
        "gm_default_settings": (None, [vp]),
        "gm_configure": (i32, [vp, vp, vp]),
        "gm_model_to_mjcf": (C.c_int64, [vp, C.c_char_p, C.c_int64]),
        "gm_model_from_mjcf": (i32, [C.c_char_p, vp, C.c_char_p, i32]),
        "gm_config_set_base_limits": (i32, [vp, C.c_double, C.c_double, C.c_double, C.c_double]),
        "gm_make_object_set": (i32, [C.c_char_p, C.c_uint64, vp, i32]),
        "gm_create": (i32, [vp, vp, vp, i32, i32, i32, i32, C.c_uint64, C.POINTER(vp)]),
        "gm_destroy": (None, [vp]),
        "gm_last_error": (C.c_char_p, [vp]),
        "gm_n_envs": (i32, [vp]),
        "gm_n_obs": (i32, [vp]),
        "gm_n_actions": (i32, [vp]),
        "gm_update_config": (i32, [vp, vp]),
        "gm_reset": (i32, [vp, u8p, vp]),
        "gm_set_action": (i32, [vp, vp, i32]),
        "gm_set_discrete_action": (i32, [vp, vp, i32]),
        "gm_step": (i32, [vp]),
        "gm_get_obs": (i32, [vp, vp, i32]),
        "gm_get_reward_done": (i32, [vp, vp, vp, i32]),
        "gm_get_event_rows": (i32, [vp, i32p, i32p, f32p]),
        "gm_get_state": (i32, [vp, f64p, f64p, f64p]),
        "gm_set_state": (i32, [vp, f64p, f64p]),
        "gm_env_state_size": (C.c_int64, []),
        "gm_get_env_states": (i32, [vp, vp]),
        "gm_set_env_states": (i32, [vp, vp]),
        "gm_get_target": (i32, [vp, f64p, i32p, i32p, f64p]),
        "gm_get_overflow": (i32, [vp, i32p]),
        "gm_device_obs": (vp, [vp]),
        "gm_device_reward": (vp, [vp]),
        "gm_device_done": (vp, [vp]),
        "gm_device_actions": (vp, [vp]),
        "gm_stream": (vp, [vp]),
        "gm_last_step_ms": (i32, [vp, f32p]),
        "gm_chunk_stats": (i32, [vp, C.POINTER(C.c_uint32), C.POINTER(C.c_uint64)]),
        "gm_dispatch_info": (i32, [vp, C.POINTER(C.c_int32)]),
        "gm_get_outputs": (i32, [vp, vp, vp, vp]),
        "gm_chunk_timeline": (i32, [vp, C.POINTER(C.c_uint64), i32]),
        "gm_debug_substep": (i32, [vp, i32p, f64p, f64p, f64p, i32p, f64p]),
        "gm_step_profiled": (i32, [vp, C.POINTER(C.c_uint64)]),
        "gm_set_stream": (i32, [vp, vp]),
        "gm_spawn_object": (i32, [vp, vp, vp]),
        "gm_default_spawn_params": (None, [vp]),
        "gm_spawn_into_scene": (i32, [vp, u8p, vp, i32, u8p]),
        "gm_set_scene_spawn": (i32, [vp, vp, i32]),
        "gm_calibrate": (i32, [vp, vp, vp, i32, i32, i32, vp, vp, vp, i32]),
        "gm_set_settle_cache": (None, [i32]),
        "gm_autoreset": (i32, [vp, i32, vp, i32, vp]),
        "gm_autoreset_episodes": (i32, [vp, i32, vp, i32, vp, vp]),
        "gm_set_motor_target": (i32, [vp, vp, vp, i32, vp]),
        "gm_random_actions": (i32, [vp, C.c_uint64, vp, i32]),
        "gm_rollout": (i32, [vp, i32, vp, vp]),
        "gm_get_sensor_si": (i32, [vp, vp]),
        "gm_set_random_spawn": (i32, [vp, i32, C.c_uint64, i32, i32]),
        "gm_scripted_actions": (i32, [vp, C.c_uint64, C.c_float, vp, i32]),
        "gm_program_actions": (i32, [vp, C.c_uint64, C.c_float, i32, vp, i32]),
        "gm_chunk_claim_waits": (i32, [vp, vp]),
        "gm_chunk_job_stats": (i32, [vp, vp, vp]),
        "gm_device_reset_mask": (vp, [vp]),
        "gm_policy_create": (i32, [vp, i32p, i32, f32p, C.POINTER(vp)]),
        "gm_policy_destroy": (None, [vp]),
        "gm_policy_pack": (C.c_int64, [i32p, i32, f32p, f32p]),
        "gm_policy_act": (i32, [vp, C.c_float, C.c_uint64, C.c_uint64]),
        "gm_policy_read": (i32, [vp, i32p, f32p]),
        "gm_policy_rollout": (i32, [vp, i32, f32p, C.c_uint64, C.c_uint64, i32, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None and os.environ.get("GM_LIB"):
            continue   # an older developer build without this entry point
        if fn is None:
            raise ImportError(f"libgm is missing {name}")
        fn.restype = res
        fn.argtypes = args


def struct_size(which: int) -> int:
    return int(load_library().gm_struct_size(which))


class ModelBlob:
    """An opaque gm_model (the compiled gripper, what mj_loadXML would return)."""

    def __init__(self, params: ModelParams | None = None):
        lib = load_library()
        if params is None:
            params = ModelParams()
            lib.gm_default_model_params(C.byref(params))
        self.params = params
        self.buf = C.create_string_buffer(struct_size(1))
        rc = lib.gm_build_model(C.byref(params), self.buf)
        if rc != 0:
            raise RuntimeError(f"gm_build_model failed ({rc})")
        info = (C.c_int32 * 20)()
        lib.gm_model_info(self.buf, info)
        self.nlock, self.nM = info[18], info[19]
        (self.nq, self.nv, self.nbody, self.ngeom, self.npair, self.n_seg, self.dof_base,
         self.dof_palm, self.dof_obj) = info[:9]
        self.dof_pris = list(info[9:12])
        self.dof_rev = list(info[12:15])
        self.dof_seg = list(info[15:18])

    @property
    def ptr(self):
        return C.cast(self.buf, C.c_void_p)

    def _read_info(self, lib):
        info = (C.c_int32 * 20)()
        lib.gm_model_info(self.buf, info)
        self.nlock, self.nM = info[18], info[19]
        (self.nq, self.nv, self.nbody, self.ngeom, self.npair, self.n_seg, self.dof_base,
         self.dof_palm, self.dof_obj) = info[:9]
        self.dof_pris = list(info[9:12])
        self.dof_rev = list(info[12:15])
        self.dof_seg = list(info[15:18])

    def to_mjcf(self) -> str:
        """The model as MJCF with the reference's names (gm_model_to_mjcf)."""
        lib = load_library()
        n = lib.gm_model_to_mjcf(self.buf, None, 0)
        out = C.create_string_buffer(n + 1)
        lib.gm_model_to_mjcf(self.buf, out, n + 1)
        return out.value.decode()

    @classmethod
    def from_mjcf(cls, xml: str) -> "ModelBlob":
        """Compile an MJCF (the subset gm_model_from_mjcf reads) into a model."""
        lib = load_library()
        self = cls.__new__(cls)
        self.params = None
        self.buf = C.create_string_buffer(struct_size(1))
        err = C.create_string_buffer(512)
        rc = lib.gm_model_from_mjcf(xml.encode(), self.buf, err, 512)
        if rc != 0:
            raise ValueError(f"gm_model_from_mjcf: {err.value.decode()}")
        self._read_info(lib)
        return self


def env_state_dtype():
    """numpy view of one GmEnvState record (gripper-mujoco_amd/csrc/gm_state.h), C layout
    (align=True); checked against gm_env_state_size() at load."""
    import numpy as np
    nb, nl = len(BINARY_EVENTS), len(LINEAR_EVENTS)
    grip = np.dtype([("x", "f8"), ("y", "f8"), ("z", "f8"), ("th", "f8"),
                     ("sx", "i4"), ("sy", "i4"), ("sz", "i4"), ("pad", "i4")], align=True)
    return np.dtype([
        ("time", "f8"), ("last_step_time", "f8"), ("end", grip), ("next", grip), ("base", "f8", 6),
        ("last_read", "f8", 10), ("qpos", "f8", GM_MAX_QPOS), ("qvel", "f8", GM_MAX_DOF),
        ("qacc_warm", "f8", GM_MAX_DOF),
        ("lock_q", "f8", GM_MAX_LOCK), ("start_qpos", "f8", 7), ("obj_size", "f8", 3), ("obj_mass", "f8"),
        ("obj_inertia", "f8", 3), ("obj_friction", "f8"), ("obj_rbound", "f8"), ("obj_rest_z", "f8"),
        ("obj_invw", "f8", 2),
        ("dt", "f8"), ("tip_force", "f8"),
        ("rand_mu", "f4", (10, 3)), ("lev_value", "f4", nl), ("lev_last", "f4", nl),
        ("cumulative_reward", "f4"), ("grp_peak_lateral", "f4"), ("reward", "f4"),
        ("ring_i", "i4", 37), ("bev_value", "i4", nb), ("bev_last", "i4", nb), ("bev_row", "i4", nb),
        ("bev_abs", "i4", nb), ("lev_row", "i4", nl), ("lev_abs", "i4", nl), ("lock_active", "i4", GM_MAX_LOCK),
        ("old_x", "i4"), ("old_y", "i4"), ("old_z", "i4"), ("num_action_steps", "i4"),
        ("termination_signal_sent", "i4"), ("extra_substeps", "i4"), ("obj_type", "i4"), ("obj_index", "i4"),
        ("done", "i4"), ("overflow", "i4"), ("rng", "u4"), ("cal_steps", "i4"), ("badqacc", "i4"),
        ("episode", "i4"), ("newton_caps", "i4"), ("pad_end", "i4", 1),
        # the sensor windows follow the part the step kernel stages into LDS (GmEnvHot)
        ("ring", "f4", (37, GM_RING))], align=True)


def env_state_view(records):
    """Structured view of raw [n, size] uint8 GmEnvState records."""
    import numpy as np
    dt = env_state_dtype()
    r = np.ascontiguousarray(records, dtype=np.uint8)
    if r.shape[-1] != dt.itemsize:
        raise ValueError(f"GmEnvState is {r.shape[-1]} bytes, numpy view expects {dt.itemsize}")
    return r.reshape(-1, dt.itemsize).view(dt).reshape(r.shape[:-1])


class ConfigBlob:
    """An opaque gm_config: settings + what configure_settings() derives from them."""

    def __init__(self, settings: Settings, model: ModelBlob):
        lib = load_library()
        self.buf = C.create_string_buffer(struct_size(2))
        rc = lib.gm_configure(C.byref(settings), model.buf, self.buf)
        if rc != 0:
            raise RuntimeError(f"gm_configure rejected the settings ({rc})")
        info = (C.c_int32 * 5)()
        lib.gm_config_info(self.buf, info)
        self.n_obs, self.n_actions, self.sim_steps_per_action, self.sensor_fcn, self.state_fcn = info[:5]

    @property
    def ptr(self):
        return C.cast(self.buf, C.c_void_p)


def default_settings() -> Settings:
    s = Settings()
    load_library().gm_default_settings(C.byref(s))
    return s


def make_object_set(name: str, seed: int = 1234):
    arr = (Object * GM_MAX_OBJSET)()
    n = load_library().gm_make_object_set(name.encode(), seed, arr, GM_MAX_OBJSET)
    if n <= 0:
        raise ValueError(f"unknown object set {name!r}")
    out = (Object * n)()
    for i in range(n):
        out[i] = arr[i]
    return out
