"""Drop-in facade for the reference's pybind11 module `bind` (src/bind.cpp:32),
imported by rl/env/MjEnv.py:18 as `from mjpy.bind import MjClass, EventTrack`.

One MjClass is one env (the reference's model: one MjClass per process, bind.cpp:46),
backed by a 1-env context of the MI355X C ABI (include/gripper_mi355x.h); every
action_step() runs on the GPU.  The methods MjEnv calls on the hot path are mirrored
with the reference's names, argument meaning and error behaviour:

  .set (Settings, r/w fields of simsettings.h)      bind.cpp:195
  set_continous_action(i, f) / set_discrete_action   bind.cpp:95-96   (MjEnv.py:594,597)
  action_step()                                      bind.cpp:93      (MjEnv.py:612)
  get_observation_numpy()                            bind.cpp:119-123 (MjEnv.py:823)
  is_done() / reward()                               bind.cpp:115,128 (MjEnv.py:635,1039)
  reset() / hard_reset()                             bind.cpp:53-54   (MjEnv.py:2240,2249)
  spawn_object / spawn_into_scene / default_spawn_params / set_new_base_XY
  set_base_XYZ_limits / set_base_yaw_limit (effective on the device config)
  is_finger_hook_fixed / using_xyz_base_actions / reset_timestep
  get_test_report / add_events / reward(event)
  get_n_actions / get_n_obs / get_N / finger dimension setters and getters
  get_event_state() -> EventTrack                    bind.cpp:525-590 (MjEnv.py:1020)
  __getstate__ / __setstate__ (pickle pair)          bind.cpp:207-241 (MjEnv.py:2088-2105)

Differences the caller can observe are listed in DESIGN.md ("Facade").  There is no
CPU fallback: without the HIP library / a GPU, construction of the env raises.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

import gmx
from gmx._lib import BINARY_EVENTS, LINEAR_EVENTS


class SpawnParams(gmx.SpawnParams):
    """MjType::SpawnParams (mjclass.h:916-931; bind.cpp:411-430): r/w fields with the
    reference's names and defaults, laid out as the C ABI's gm_spawn_params."""

    def __init__(self):
        super().__init__()
        gmx.load_library().gm_default_spawn_params(C.byref(self))


class _BinaryEvent:
    __slots__ = ("value", "last_value", "active_sum", "row", "abs", "percent")

    def __init__(self):
        self.value = False
        self.last_value = 0
        self.active_sum = 0
        self.row = 0
        self.abs = 0
        self.percent = 0.0


class _LinearEvent:
    __slots__ = ("value", "last_value", "active_sum", "row", "abs", "percent")

    def __init__(self):
        self.value = 0.0
        self.last_value = 0.0
        self.active_sum = 0
        self.row = 0
        self.abs = 0
        self.percent = 0.0


class EventTrack:
    """MjType::EventTrack (mjclass.h:575-647): one BinaryEvent / LinearEvent per reward
    name, readable attributes; reset(); calculate_percentage()."""

    def __init__(self):
        for n in BINARY_EVENTS:
            setattr(self, n, _BinaryEvent())
        for n in LINEAR_EVENTS:
            setattr(self, n, _LinearEvent())

    def reset(self):
        self.__init__()

    def calculate_percentage(self):
        """EventTrack::calculate_percentage (mjclass.h:628-645): percent = 100 abs /
        step_num.abs for every event."""
        total = float(self.step_num.abs)
        for n in list(BINARY_EVENTS) + list(LINEAR_EVENTS):
            e = getattr(self, n)
            e.percent = (100.0 * e.abs) / total if total else float("nan")

    def print(self):
        for n in list(BINARY_EVENTS) + list(LINEAR_EVENTS):
            e = getattr(self, n)
            print(f"{n}: row {e.row} abs {e.abs} last {e.last_value}")


class TestReport:
    """MjType::TestReport (mjclass.h:941-950): object name, cumulative reward, event counts."""

    def __init__(self, object_name: str = "", cumulative_reward: float = 0.0, cnt: EventTrack | None = None):
        self.object_name = object_name
        self.cumulative_reward = cumulative_reward
        self.cnt = cnt if cnt is not None else EventTrack()


def _linear_reward(val, mn, mx, overshoot):
    """linear_reward (mjclass.cpp:4866-4894), float arithmetic."""
    f = np.float32
    val, mn, mx, overshoot = f(val), f(mn), f(mx), f(overshoot)
    if val < mn:
        return f(0.0)
    if val > mx:
        if overshoot < mx:
            return f(1.0)
        if val > overshoot:
            return f(0.0)
        mn, mx, val = f(0.0), f(overshoot - mx), f(overshoot - val)
    return f((val - mn) / (mx - mn))


# j_.baseLims defaults (myfunctions.cpp:245-261): x, y, z (m) and yaw (rad)
_BASE_LIMITS_DEFAULT = (500e-3, 500e-3, 30e-3)
_BASE_YAW_DEFAULT = math.pi / 2


class MjClass:
    """MjClass (mjclass.h:1554-1833) on the MI355X hot path, one env."""

    def __init__(self, model_path: str | None = None):
        self.set = gmx.default_settings()
        self.default_spawn_params = SpawnParams()
        self.model_folder_path = model_path or ""
        self.object_set_name = "set6_synthetic"
        self.machine = "mi355x"
        self.current_load_path = ""
        self._params = None          # gm_model_params overrides (finger dimensions)
        self._env = None
        self._pending = None         # continuous action vector buffered between calls
        self._rd = None              # (reward, done) of the current transition, read with the obs
        self._rng = np.random.default_rng(0)
        self._base_limits = _BASE_LIMITS_DEFAULT     # j_.baseLims (reset by hard_reset)
        self._base_yaw = _BASE_YAW_DEFAULT

    # ------------------------------------------------------------ model / lifecycle
    def load(self, file_path: str = ""):
        self.current_load_path = file_path
        self._drop()

    def load_relative(self, file_path: str = ""):
        """The reference loads task MJCF here (bind.cpp:52); the build's model is compiled
        from gm_model_params and the object set named by object_set_name."""
        self.load(file_path)

    def _drop(self):
        self._rd = None              # the cached transition belongs to the env being dropped
        if self._env is not None:
            self._env.close()
            self._env = None

    def _ensure(self):
        self._rd = None              # any call that may change the env drops the cached reward / done
        if self._env is None:
            model_params = self._params
            self._env = gmx.BatchedGripperEnv(1, object_set=self.object_set_name, settings=self.set,
                                              model_params=model_params, seed=int(self.set.random_seed),
                                              max_episode_steps=1 << 30)
            self._rng = np.random.default_rng(int(self.set.random_seed))
            self._push_base_limits(self._env.cfg)
        return self._env

    def _push_base_limits(self, cfg):
        """write j_.baseLims into the context's configuration (update_base_limits)"""
        env = self._env
        x, y, z = self._base_limits
        rc = env.lib.gm_config_set_base_limits(cfg.ptr, x, y, z, self._base_yaw)
        if rc != 0:
            raise RuntimeError(f"base limits rejected ({rc})")
        env._check(env.lib.gm_update_config(env.ctx, cfg.ptr))

    def reset(self):
        """MjClass::reset (mjclass.cpp:434-486): re-apply settings (configure_settings),
        keyframe + equilibrium, noise means, base-Z noise; the object set's first object
        is placed until spawn_object / spawn_into_scene picks one (MjEnv.reset order)."""
        env = self._ensure()
        cfg = gmx.ConfigBlob(self.set, env.model)
        env.lib.gm_config_set_base_limits(cfg.ptr, *self._base_limits, self._base_yaw)
        if env.lib.gm_update_config(env.ctx, cfg.ptr) != 0:
            # the observation layout changed: the reference re-sizes on reset too
            self._drop()
            env = self._ensure()
            cfg = env.cfg
        env.cfg = cfg
        env.n_obs, env.n_actions = cfg.n_obs, cfg.n_actions
        env._obs = np.zeros((1, cfg.n_obs), dtype=np.float32)
        sp = (gmx.Spawn * 1)()
        sp[0].object_index, sp[0].x, sp[0].y, sp[0].zrot = 0, 0.0, 0.0, 0.0
        env.reset(spawn=sp)
        self._pending = None

    def hard_reset(self):
        """Reload from scratch (bind.cpp:54): a fresh device context.  Base limits do not
        persist through a hard reset (myfunctions.cpp:2309-2333; MjEnv re-sets them)."""
        self._drop()
        self._base_limits = _BASE_LIMITS_DEFAULT
        self._base_yaw = _BASE_YAW_DEFAULT
        self.reset()

    def reset_timestep(self):
        """MjEnv.reset(timestep=True) (MjEnv.py:2247): recalibrate the timestep
        (find_highest_stable_timestep, mjclass.cpp:4745-4854, as one batched device job),
        rebuild the model with it (S = ceil(time_for_action / dt)) and reset."""
        env = self._ensure()
        cal, _ = gmx.calibrate(env.model, env.cfg, env.objects, what=gmx.CAL_TIMESTEP)
        self._model_params().timestep = float(cal.timestep)
        self._drop()
        self.reset()
        return float(cal.timestep)

    def step(self):
        raise NotImplementedError("single physics substeps are inside action_step() on the device")

    # ------------------------------------------------------------ actions
    def set_motor_target(self, x: float, y: float, z: float) -> bool:
        """MjClass::set_motor_target (bind.cpp:82, mjclass.cpp:1359-1364)."""
        return bool(self._ensure().set_motor_target([x, y, z])[0])

    def set_continous_action(self, action: int, fraction: float):
        """MjClass::set_continous_action (mjclass.cpp:1517-1526). MjEnv calls it for every
        index in order then action_step(); the vector is applied in that order on the
        device at action_step()."""
        env = self._ensure()
        if self._pending is None:
            self._pending = np.zeros(env.n_actions, dtype=np.float32)
        if action < 0 or action >= env.n_actions:
            print(f"set_continous_action: action {action} out of range")
            return []
        self._pending[action] = fraction
        return []

    def set_discrete_action(self, action: int):
        env = self._ensure()
        env.set_discrete_action(np.array([action], dtype=np.int32))
        return []

    def set_action(self, action: int):
        return self.set_discrete_action(action)

    def action_step(self):
        env = self._ensure()
        if self._pending is not None:
            env.set_action(self._pending.reshape(1, -1))
            self._pending = None
        env.action_step()

    # ------------------------------------------------------------ outputs
    def get_observation_numpy(self):
        # one device read for the transition: the reward and done flag ride along for the
        # is_done() / reward() calls MjEnv.step makes next (dropped by any other call)
        obs, r, d = self._ensure().outputs()
        self._rd = (float(r[0]), bool(d[0]))
        return obs[0]

    def get_observation(self):
        return self.get_observation_numpy().tolist()

    def _reward_done(self):
        """(reward, done) of the current transition, one device read per transition:
        MjEnv.step asks is_done() then reward() (MjEnv.py:616-637) with nothing in between."""
        rd = self._rd
        if rd is None:
            env = self._ensure()
            r, d = env.reward_done()
            rd = self._rd = (float(r[0]), bool(d[0]))
        return rd

    def is_done(self) -> bool:
        return self._reward_done()[1]

    def reward(self, event: "EventTrack | None" = None) -> float:
        """MjClass::reward (mjclass.cpp:3000-3049): the current transition's reward; with
        an EventTrack, calc_rewards over that track (mjclass.cpp:5471-5528: binary
        reward if row >= trigger, linear reward x linear_reward(last_value) likewise)."""
        if event is None:
            return self._reward_done()[0]
        st = self.set
        r = np.float32(0.0)
        for n in BINARY_EVENTS:
            if getattr(event, n).row >= getattr(st, n).trigger:
                r = np.float32(r + np.float32(getattr(st, n).reward))
        for n in LINEAR_EVENTS:
            sr, ev = getattr(st, n), getattr(event, n)
            if ev.row >= sr.trigger:
                frac = _linear_reward(ev.last_value, sr.min, sr.max, sr.overshoot)
                r = np.float32(r + np.float32(np.float32(sr.reward) * frac))
        return float(r)

    def add_events(self, e1: "EventTrack", e2: "EventTrack") -> "EventTrack":
        """MjClass::add_events (mjclass.cpp:4692-4715): abs and active_sum summed, linear
        last_value summed, everything else default."""
        out = EventTrack()
        for n in BINARY_EVENTS:
            a, b, o = getattr(e1, n), getattr(e2, n), getattr(out, n)
            o.abs, o.active_sum = a.abs + b.abs, a.active_sum + b.active_sum
        for n in LINEAR_EVENTS:
            a, b, o = getattr(e1, n), getattr(e2, n), getattr(out, n)
            o.abs, o.active_sum = a.abs + b.abs, a.active_sum + b.active_sum
            o.last_value = float(np.float32(np.float32(a.last_value) + np.float32(b.last_value)))
        return out

    def get_test_report(self) -> TestReport:
        """MjClass::get_test_report (mjclass.cpp:3800-3809)."""
        env = self._ensure()
        st = gmx.env_state_view(env.env_states())[0]
        return TestReport(self.get_current_object_name(), float(st["cumulative_reward"]), self.get_event_state())

    def get_event_state(self) -> EventTrack:
        rows, absc, lastv = self._ensure().event_rows()
        t = EventTrack()
        for i, n in enumerate(list(BINARY_EVENTS) + list(LINEAR_EVENTS)):
            e = getattr(t, n)
            e.row, e.abs = int(rows[0, i]), int(absc[0, i])
            e.last_value = float(lastv[0, i]) if i >= len(BINARY_EVENTS) else int(lastv[0, i])
            e.value = e.last_value
            e.active_sum = int(e.row != 0)
        return t

    def get_n_actions(self) -> int:
        return int(self._config().n_actions)

    def get_n_obs(self) -> int:
        return int(self._config().n_obs)

    def _config(self):
        if self._env is not None:
            return self._env.cfg
        return gmx.ConfigBlob(self.set, gmx.ModelBlob(self._params))

    # ------------------------------------------------------------ objects / spawning
    def get_number_of_objects(self) -> int:
        return len(gmx.make_object_set(self.object_set_name, int(self.set.random_seed)))

    def get_object_name(self, idx: int) -> str:
        o = gmx.make_object_set(self.object_set_name, int(self.set.random_seed))[idx]
        kind = {2: "sphere", 5: "cylinder", 6: "cube"}.get(o.type, "object")
        return f"{kind}_{idx}"

    def get_current_object_name(self) -> str:
        return self.get_object_name(self._spawned if hasattr(self, "_spawned") else 0)

    def spawn_object(self, idx: int, x: float = 0.0, y: float = 0.0, zrot: float = 0.0):
        """MjClass::spawn_object (mjclass.cpp:2352-2420)."""
        env = self._ensure()
        sp = (gmx.Spawn * 1)()
        sp[0].object_index, sp[0].x, sp[0].y, sp[0].zrot = int(idx), float(x), float(y), float(zrot)
        env._check(env.lib.gm_spawn_object(env.ctx, None, sp))
        self._spawned = int(idx)

    def spawn_into_scene(self, index, xpos=None, ypos=None, zrot=None, xrange=None, yrange=None,
                         rotrange=None) -> bool:
        """MjClass::spawn_into_scene (mjclass.cpp:2422-2654; the four bind.cpp:100-103
        overloads): default_spawn_params with the given overrides, the shuffled xy /
        rotation grid search with Box2d rejection against the fingertips and the scene
        bounds, run on the device.  Returns False when no free pose exists."""
        env = self._ensure()
        p = SpawnParams()
        C.memmove(C.byref(p), C.byref(self.default_spawn_params), C.sizeof(p))
        p.index = int(index)
        if xpos is not None: p.x = float(xpos)
        if ypos is not None: p.y = float(ypos)
        if zrot is not None: p.zrot = float(zrot)
        if xrange is not None: p.xrange = float(xrange)
        if yrange is not None: p.yrange = float(yrange)
        if rotrange is not None: p.rotrange = float(rotrange)
        ok = bool(env.spawn_into_scene(p)[0])
        if ok:
            self._spawned = int(index)
        return ok

    def set_new_base_XY(self, x: float, y: float) -> bool:
        """MjClass::set_new_base_XY -> luke::set_base_to_XY_position (mjclass.cpp:1394-1402,
        myfunctions.cpp:2568-2608): the base XY target is clamped to the base limits, then
        the qpos snap needs XY base joints -- this gripper (like the reference's canonical
        one) has base Z only, so, as the reference does, it raises after setting the target."""
        env = self._ensure()
        rec = env.env_states()
        st = gmx.env_state_view(rec)[0]
        lx, ly, _ = self._base_limits
        tx = min(max(float(x), -lx), lx)
        ty = min(max(float(y), -ly), ly)
        st["base"][0], st["base"][1] = tx, ty
        env.set_env_states(rec)
        raise RuntimeError("luke::set_base_to_XY_position() cannot move XY because these motions are not in use")

    def set_scene_grasp_target(self, num_objects: int):
        return None

    def reset_goal(self):
        return None

    # ------------------------------------------------------------ gripper dimensions
    def _model_params(self):
        if self._params is None:
            p = gmx.ModelParams()
            gmx.load_library().gm_default_model_params(C.byref(p))
            self._params = p
        return self._params

    def get_N(self) -> int:
        return int(self._model_params().n_seg)

    def set_finger_thickness(self, t: float):
        self._model_params().finger_thickness = float(t)
        self._drop()

    def set_finger_width(self, w: float):
        self._model_params().finger_width = float(w)
        self._drop()

    def set_finger_modulus(self, E: float):
        self._model_params().finger_E = float(E)
        self._drop()

    def get_finger_thickness(self) -> float:
        return float(self._model_params().finger_thickness)

    def get_finger_width(self) -> float:
        return float(self._model_params().finger_width)

    def get_finger_modulus(self) -> float:
        return float(self._model_params().finger_E)

    def get_finger_length(self) -> float:
        return float(self._model_params().finger_length)

    def get_finger_hook_length(self) -> float:
        return float(self._model_params().hook_length)

    def get_finger_hook_angle_degrees(self) -> float:
        return float(self._model_params().hook_angle_degrees)

    def get_fingertip_clearance(self) -> float:
        return float(self._model_params().fingertip_clearance)

    def get_finger_rigidity(self) -> float:
        p = self._model_params()
        return float(p.finger_E * p.finger_width * p.finger_thickness ** 3 / 12.0)

    def yield_load(self, thickness: float | None = None, width: float | None = None) -> float:
        """MjClass::yield_load (bind.cpp:191-192; calc_yield_point_load, myfunctions.cpp:
        3587-3606): end load that yields the finger, float arithmetic as the reference."""
        p = self._model_params()
        t = p.finger_thickness if thickness is None else float(thickness)
        w = p.finger_width if width is None else float(width)
        I = (w * t ** 3) / 12.0
        ys = 215e6                       # j_.dim.yield_stress (myfunctions.cpp:216)
        M_max = np.float32((ys * I) / (0.5 * t))
        return float(np.float32(float(M_max) / p.finger_length))

    def calibrate(self, what: int = 3):
        """The automatic settings configure_settings derives by simulation
        (find_highest_stable_timestep, calibrate_simulated_sensors; mjclass.cpp:241-291),
        as one batched device job.  Returns the gm_calibration fields as a dict."""
        env = self._ensure()
        cal, trace = gmx.calibrate(env.model, env.cfg, env.objects, what=what)
        out = cal.as_dict()
        out["search_trace"] = trace
        return out

    def set_base_XYZ_limits(self, x: float, y: float, z: float):
        """MjClass::set_base_XYZ_limits (mjclass.cpp:3847-3852): symmetric base limits,
        effective immediately on the device (base action clamps, base state normalisation)."""
        self._base_limits = (float(x), float(y), float(z))
        if self._env is not None:
            self._push_base_limits(self._env.cfg)

    def set_base_yaw_limit(self, yaw: float):
        """MjClass::set_base_yaw_limit (mjclass.cpp:3854-3859)."""
        self._base_yaw = float(yaw)
        if self._env is not None:
            self._push_base_limits(self._env.cfg)

    def is_finger_hook_fixed(self) -> bool:
        """MjClass::is_finger_hook_fixed (mjclass.cpp:3941-3946): the hook is a fixed part
        of the last finger link in this gripper model."""
        return True

    def using_xyz_base_actions(self) -> bool:
        """MjClass::using_xyz_base_actions (mjclass.cpp:3955-3960): the base moves in Z only."""
        return False

    def get_base_limits(self):
        """(x, y, z, yaw) symmetric base limits currently applied."""
        return (*self._base_limits, self._base_yaw)

    # ------------------------------------------------------------ pickling (bind.cpp:207-241)
    def __getstate__(self):
        return {"set": bytes(self.set), "params": bytes(self._params) if self._params is not None else None,
                "base_limits": self._base_limits, "base_yaw": self._base_yaw,
                "object_set_name": self.object_set_name, "model_folder_path": self.model_folder_path,
                "machine": self.machine, "default_spawn_params": bytes(self.default_spawn_params)}

    def __setstate__(self, st):
        self.__init__(st.get("model_folder_path"))
        self.set = gmx.Settings.from_buffer_copy(st["set"])
        if st.get("params") is not None:
            self._params = gmx.ModelParams.from_buffer_copy(st["params"])
        self.object_set_name = st["object_set_name"]
        self.machine = st["machine"]
        if st.get("base_limits") is not None:
            self._base_limits = tuple(st["base_limits"])
            self._base_yaw = float(st["base_yaw"])
        if st.get("default_spawn_params") is not None:
            C.memmove(C.byref(self.default_spawn_params), st["default_spawn_params"], C.sizeof(SpawnParams))
