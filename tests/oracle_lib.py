"""ctypes wrapper of oracle/liboracle.so (the fp64 CPU restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker / CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np
from gmx._lib import GM_MAX_CON, GM_MAX_DOF, GM_MAX_EFC  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")


# every source the oracle is compiled from (oracle/Makefile's liboracle.so prerequisites)
ORACLE_DEPS = [os.path.join(ORACLE_DIR, f) for f in ("oracle.c", "physics.c", "oracle.h", "Makefile")] + \
    [os.path.join(REPO, "gripper-mujoco_amd", "csrc", f) for f in ("gm_math.h", "gm_state.h")] + \
    [os.path.join(REPO, "include", f) for f in ("gripper_mi355x.h", "gm_settings.def")]


def build_oracle():
    stale = not os.path.exists(ORACLE_LIB) or any(
        os.path.exists(d) and os.path.getmtime(d) > os.path.getmtime(ORACLE_LIB) for d in ORACLE_DEPS)
    if stale:
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, os.path.join(ORACLE_DIR, "liboracle.so")], check=True)
    return ORACLE_LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build_oracle()
        _lib = load(ORACLE_LIB)
    return _lib


ORACLE_LIBM = os.path.join(ORACLE_DIR, "liboracle_libm.so")


def lib_libm():
    """The same oracle built with glibc's sin / cos in place of gm_math.h's shared kernel
    (oracle/Makefile liboracle_libm.so; -DGM_LIBM_TRIG): an independent check that the
    shared trigonometry is not what makes device and oracle agree."""
    stale = not os.path.exists(ORACLE_LIBM) or any(
        os.path.exists(d) and os.path.getmtime(d) > os.path.getmtime(ORACLE_LIBM) for d in ORACLE_DEPS)
    if stale:
        subprocess.run(["make", "-s", "-C", ORACLE_DIR, ORACLE_LIBM], check=True)
    return load(ORACLE_LIBM)


def load(path):
    if True:
        L = C.CDLL(path)
        vp, i32, f32p, f64p, i32p = C.c_void_p, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_double), C.POINTER(C.c_int32)
        sig = {
            "or_create": (vp, [vp, vp, vp, i32, C.c_int64]),
            "or_destroy": (None, [vp]),
            "or_sizeof": (C.c_size_t, []),
            "or_reset": (None, [vp, vp]),
            "or_set_action": (None, [vp, f32p]),
            "or_driver_actions": (None, [vp, i32, C.c_uint64, C.c_float, C.c_int64, f32p]),
            "or_set_discrete_action": (None, [vp, C.c_int32]),
            "or_step": (None, [vp]),
            "or_get_obs": (i32, [vp, f32p]),
            "or_is_done": (i32, [vp]),
            "or_reward": (C.c_float, [vp]),
            "or_get_state": (None, [vp, f64p, f64p, f64p]),
            "or_set_state": (None, [vp, f64p, f64p]),
            "or_get_target": (None, [vp, f64p, i32p, i32p, f64p]),
            "or_get_event_rows": (None, [vp, i32p, i32p, f32p]),
            "or_overflow": (i32, [vp]),
            "or_get_eq": (None, [vp, f64p]),
            "or_debug_substep": (None, [vp, i32p, f64p, f64p, f64p, f64p]),
            "or_state_size": (C.c_size_t, []),
            "or_import_state": (i32, [vp, vp]),
            "or_export_state": (None, [vp, vp]),
            "or_batch_step": (i32, [vp, vp, vp, i32, i32, vp, vp, vp, vp, vp, vp, i32]),
            "or_batch_substep": (i32, [vp, vp, vp, i32, i32, vp, vp, vp, vp, vp, vp, vp, i32]),
            "or_gauge_reading": (C.c_float, [vp, f64p]),
            "or_minstd_next_canonical_float": (C.c_double, [C.POINTER(C.c_uint32)]),
            "or_minstd_next_canonical_double": (C.c_double, [C.POINTER(C.c_uint32)]),
            "or_grip_step_sequence": (i32, [f64p, i32, f64p]),
            "or_sample": (i32, [i32, f32p, i32, i32, i32, f32p]),
            "or_bench": (C.c_double, [vp, vp, vp, i32, i32, i32, C.c_uint64, i32, i32, i32]),
            "or_polyfit_eval": (C.c_float, [f64p, f64p, i32, i32, C.c_double]),
            "or_gauge_points": (None, [vp, f64p, f64p, f64p]),
            "or_ring_trace": (None, [f32p, i32, i32, f32p]),
            "or_spawn_into_scene": (i32, [vp, vp]),
            "or_std_shuffle": (C.c_uint32, [C.c_uint32, i32, i32p]),
            "or_box2d_overlaps": (i32, [f64p, f64p, C.c_double]),
            "or_calibrate": (i32, [vp, vp, vp, i32, i32, vp, vp, vp, i32]),
            "or_get_stats": (None, [vp, C.POINTER(C.c_int64)]),
            "or_set_default_solver": (None, [i32]),
            "or_set_default_weld_locks": (None, [i32]),
            "or_set_solver": (None, [vp, i32]),
            "or_dynamics": (None, [vp, f64p, f64p, f64p, f64p, f64p]),
            "or_set_settle_cache": (None, [i32]),
            "or_set_motor_target": (i32, [vp, C.c_double, C.c_double, C.c_double]),
            "or_get_sensor_si": (None, [vp, f32p]),
            "or_want_forces": (None, [vp, i32]),
            "or_last_forces": (None, [vp, f64p, f64p]),
            "or_collide": (i32, [i32, f64p, f64p, f64p, i32, f64p, f64p, f64p, C.c_double, i32, f64p]),
        }
        for n, (r, a) in sig.items():
            f = getattr(L, n)
            f.restype = r
            f.argtypes = a
    return L


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


class OracleEnv:
    """One reference MjClass, fp64 CPU restatement."""

    def __init__(self, model, cfg, objects, env_id: int = 0):
        L = lib()
        self.L = L
        self.model = model
        self.cfg = cfg
        self.objects = objects
        self.env_id = int(env_id)
        self.h = L.or_create(model.ptr, cfg.ptr, C.cast(objects, C.c_void_p), len(objects), env_id)
        if not self.h:
            raise RuntimeError("or_create failed")
        self.n_obs = cfg.n_obs
        self.n_actions = cfg.n_actions

    def __del__(self):
        try:
            if self.h:
                self.L.or_destroy(self.h)
        except Exception:
            pass

    def reset(self, spawn):
        self.L.or_reset(self.h, C.byref(spawn))

    def spawn_into_scene(self, params) -> bool:
        """MjClass::spawn_into_scene(SpawnParams) (mjclass.cpp:2475-2654)."""
        return bool(self.L.or_spawn_into_scene(self.h, C.byref(params)))

    def set_action(self, a):
        a = _f32(a)
        self.L.or_set_action(self.h, a.ctypes.data_as(C.POINTER(C.c_float)))

    def driver_actions(self, mode: int = 3, seed: int = 0, jitter: float = 0.2, gid: int | None = None):
        """The rollout drivers' fractions for this env's current state (or_driver_actions:
        0 scripted mix, 1 random, 3 grasp program, 4 program / scripted mix)."""
        out = np.zeros(max(self.n_actions, 1), dtype=np.float32)
        self.L.or_driver_actions(self.h, int(mode), int(seed), float(jitter), int(self.env_id if gid is None else gid),
                                 out.ctypes.data_as(C.POINTER(C.c_float)))
        return out[:self.n_actions]

    def set_discrete_action(self, a: int):
        self.L.or_set_discrete_action(self.h, int(a))

    def action_step(self):
        self.L.or_step(self.h)

    def observation(self):
        out = np.zeros(max(self.n_obs, 1), dtype=np.float32)
        n = self.L.or_get_obs(self.h, out.ctypes.data_as(C.POINTER(C.c_float)))
        return out[:n]

    def is_done(self):
        return bool(self.L.or_is_done(self.h))

    def reward(self):
        return float(self.L.or_reward(self.h))

    def step(self, a):
        self.set_action(a)
        self.action_step()
        obs = self.observation()
        d = self.is_done()
        r = self.reward()
        return obs, r, d

    def state(self):
        q = np.zeros(self.model.nq); v = np.zeros(self.model.nv); t = np.zeros(1)
        self.L.or_get_state(self.h, q.ctypes.data_as(C.POINTER(C.c_double)), v.ctypes.data_as(C.POINTER(C.c_double)),
                            t.ctypes.data_as(C.POINTER(C.c_double)))
        return q, v, float(t[0])

    def set_state(self, q, v):
        q = np.ascontiguousarray(q, dtype=np.float64); v = np.ascontiguousarray(v, dtype=np.float64)
        self.L.or_set_state(self.h, q.ctypes.data_as(C.POINTER(C.c_double)), v.ctypes.data_as(C.POINTER(C.c_double)))

    def target(self):
        e = np.zeros(4); es = np.zeros(3, dtype=np.int32); ns = np.zeros(3, dtype=np.int32); b = np.zeros(3)
        self.L.or_get_target(self.h, e.ctypes.data_as(C.POINTER(C.c_double)), es.ctypes.data_as(C.POINTER(C.c_int32)),
                             ns.ctypes.data_as(C.POINTER(C.c_int32)), b.ctypes.data_as(C.POINTER(C.c_double)))
        return e, es, ns, b

    def event_rows(self):
        from gmx import BINARY_EVENTS, LINEAR_EVENTS
        W = len(BINARY_EVENTS) + len(LINEAR_EVENTS)
        rows = np.zeros(W, dtype=np.int32); absc = np.zeros(W, dtype=np.int32); lv = np.zeros(W, dtype=np.float32)
        self.L.or_get_event_rows(self.h, rows.ctypes.data_as(C.POINTER(C.c_int32)),
                                 absc.ctypes.data_as(C.POINTER(C.c_int32)), lv.ctypes.data_as(C.POINTER(C.c_float)))
        return rows, absc, lv

    def eq(self):
        q = np.zeros(self.model.nq)
        self.L.or_get_eq(self.h, q.ctypes.data_as(C.POINTER(C.c_double)))
        return q

    def set_motor_target(self, x, y, z) -> bool:
        """MjClass::set_motor_target (bind.cpp:82): Gripper::set_xyz_m on the target."""
        return bool(self.L.or_set_motor_target(self.h, float(x), float(y), float(z)))

    def sensor_si(self):
        """[finger1, finger2, finger3 gauge, palm, wrist Z] latest sim_sensors_SI_ readings (N)."""
        out = np.zeros(5, dtype=np.float32)
        self.L.or_get_sensor_si(self.h, out.ctypes.data_as(C.POINTER(C.c_float)))
        return out

    def overflow(self):
        return int(self.L.or_overflow(self.h))

    def debug_substep(self):
        n = C.c_int32()
        con = np.zeros((GM_MAX_CON, 16), dtype=np.float64)
        f = np.zeros(GM_MAX_EFC, dtype=np.float64)
        qacc = np.zeros(self.model.nv)
        d = C.POINTER(C.c_double)
        self.L.or_debug_substep(self.h, C.byref(n), con.ctypes.data_as(d), f.ctypes.data_as(d), qacc.ctypes.data_as(d),
                                None)
        return n.value, con, f, qacc

    def import_state(self, rec):
        """Load one device GmEnvState record (uint8 row of BatchedGripperEnv.env_states())."""
        r = np.ascontiguousarray(rec, dtype=np.uint8)
        rc = self.L.or_import_state(self.h, r.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"or_import_state failed ({rc})")

    def export_state(self):
        out = np.zeros(int(self.L.or_state_size()), dtype=np.uint8)
        self.L.or_export_state(self.h, out.ctypes.data)
        return out


def set_default_solver(pgs_sweeps: int):
    """Constraint solver of every oracle env created from now on: 0 = the engine's Newton
    solver (the default), k > 0 = the dense PGS cross-check run to k sweeps."""
    lib().or_set_default_solver(int(pgs_sweeps))


class pgs_solver:
    """with pgs_solver(800): ... -- oracle envs created inside use dense PGS"""

    def __init__(self, sweeps: int):
        self.sweeps = sweeps

    def __enter__(self):
        set_default_solver(self.sweeps)

    def __exit__(self, *exc):
        set_default_solver(0)


class weld_locks:
    """with weld_locks(): ... -- oracle envs created inside hold their stopped motors with
    the reference's weld equalities (rows along the slide axis with the weld's
    regulariser) instead of the engine's 1-row joint locks"""

    def __enter__(self):
        lib().or_set_default_weld_locks(1)

    def __exit__(self, *exc):
        lib().or_set_default_weld_locks(0)


def solver_stats(env) -> dict:
    """Newton iteration statistics accumulated by one OracleEnv."""
    st = np.zeros(6, dtype=np.int64)
    lib().or_get_stats(env.h, st.ctypes.data_as(C.POINTER(C.c_int64)))
    return dict(solves=int(st[0]), iterations=int(st[1]), line_search_evals=int(st[2]), max_iterations=int(st[3]),
                max_contacts=int(st[4]), rows=int(st[5]))


def n_threads():
    return max(1, min(16, os.cpu_count() or 1))


def batch_step(model, cfg, objects, states, actions=None, discrete=None, threads=None):
    """One env-step of the oracle for every device state record (threaded).  Returns
    (obs [n, n_obs], reward [n], done [n], states_after [n, size])."""
    st = np.array(states, dtype=np.uint8, copy=True, order="C")
    n = st.shape[0]
    obs = np.zeros((n, max(cfg.n_obs, 1)), dtype=np.float32)
    rew = np.zeros(n, dtype=np.float32)
    done = np.zeros(n, dtype=np.uint8)
    ca = None if actions is None else np.ascontiguousarray(actions, dtype=np.float32)
    da = None if discrete is None else np.ascontiguousarray(discrete, dtype=np.int32)
    rc = lib().or_batch_step(model.ptr, cfg.ptr, C.cast(objects, C.c_void_p), len(objects), n, st.ctypes.data,
                             None if ca is None else ca.ctypes.data, None if da is None else da.ctypes.data,
                             obs.ctypes.data, rew.ctypes.data, done.ctypes.data, threads or n_threads())
    if rc != 0:
        raise RuntimeError(f"or_batch_step failed ({rc})")
    return obs[:, :cfg.n_obs], rew, done, st


def batch_substep(model, cfg, objects, states, threads=None):
    """One MjClass::step with diagnostics for every device state record (threaded).
    Returns (ncon, nefc, contact [n,GM_MAX_CON,16], efc [n,GM_MAX_EFC], qacc [n,GM_MAX_DOF], wrench [n,6],
    states_after)."""
    st = np.array(states, dtype=np.uint8, copy=True, order="C")
    n = st.shape[0]
    ncon = np.zeros(n, dtype=np.int32); nefc = np.zeros(n, dtype=np.int32)
    con = np.zeros((n, GM_MAX_CON, 16)); efc = np.zeros((n, GM_MAX_EFC)); qacc = np.zeros((n, GM_MAX_DOF)); w = np.zeros((n, 6))
    rc = lib().or_batch_substep(model.ptr, cfg.ptr, C.cast(objects, C.c_void_p), len(objects), n, st.ctypes.data,
                                ncon.ctypes.data, nefc.ctypes.data, con.ctypes.data, efc.ctypes.data, qacc.ctypes.data,
                                w.ctypes.data, threads or n_threads())
    if rc != 0:
        raise RuntimeError(f"or_batch_substep failed ({rc})")
    return ncon, nefc, con, efc, qacc, w, st


def gauge_reading(model, finger_q):
    q = np.ascontiguousarray(finger_q, dtype=np.float64)
    return float(lib().or_gauge_reading(model.ptr, q.ctypes.data_as(C.POINTER(C.c_double))))


def grip_step_sequence(cmds):
    cmds = np.ascontiguousarray(cmds, dtype=np.float64).reshape(-1, 4)
    out = np.zeros((len(cmds), 15))
    lib().or_grip_step_sequence(cmds.ctypes.data_as(C.POINTER(C.c_double)), len(cmds),
                                out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def sample(mode, recent_first, prev_steps, rps):
    w = _f32(recent_first)
    out = np.zeros(64, dtype=np.float32)
    n = lib().or_sample(mode, w.ctypes.data_as(C.POINTER(C.c_float)), len(w), prev_steps, rps,
                        out.ctypes.data_as(C.POINTER(C.c_float)))
    return out[:n]


def canonical_floats(seed, n):
    s = C.c_uint32(seed)
    return np.array([lib().or_minstd_next_canonical_float(C.byref(s)) for _ in range(n)])


def bench(model, cfg, objects, n_envs, n_steps, seed=1234, n_threads=1, scripted=True, max_episode_steps=250):
    return float(lib().or_bench(model.ptr, cfg.ptr, C.cast(objects, C.c_void_p), len(objects), n_envs, n_steps,
                                seed, n_threads, 1 if scripted else 0, max_episode_steps))


def polyfit_eval(X, Y, order, x):
    X = np.ascontiguousarray(X, dtype=np.float64); Y = np.ascontiguousarray(Y, dtype=np.float64)
    return float(lib().or_polyfit_eval(X.ctypes.data_as(C.POINTER(C.c_double)),
                                       Y.ctypes.data_as(C.POINTER(C.c_double)), len(X), order, x))


def gauge_points(model, finger_q):
    q = np.ascontiguousarray(finger_q, dtype=np.float64)
    X = np.zeros(16); Y = np.zeros(16)
    lib().or_gauge_points(model.ptr, q.ctypes.data_as(C.POINTER(C.c_double)),
                          X.ctypes.data_as(C.POINTER(C.c_double)), Y.ctypes.data_as(C.POINTER(C.c_double)))
    return X[:model.n_seg + 1], Y[:model.n_seg + 1]


def ring_trace(adds, n_reads):
    a = _f32(adds)
    out = np.zeros((len(a), n_reads), dtype=np.float32)
    lib().or_ring_trace(a.ctypes.data_as(C.POINTER(C.c_float)), len(a), n_reads,
                        out.ctypes.data_as(C.POINTER(C.c_float)))
    return out


def std_shuffle(seed, n):
    """libstdc++ std::shuffle of [0, n) with minstd_rand0(seed); returns (perm, next draw)."""
    out = np.zeros(max(n, 1), dtype=np.int32)
    nxt = lib().or_std_shuffle(seed, n, out.ctypes.data_as(C.POINTER(C.c_int32)))
    return out[:n].tolist(), int(nxt)


def calibrate(model, cfg, objects, what=3):
    """or_calibrate: the sequential reference calibration; returns (Calibration, trace)."""
    import gmx
    out = gmx.Calibration()
    tdt = (C.c_double * 256)()
    tbad = (C.c_uint8 * 256)()
    rc = lib().or_calibrate(model.ptr, cfg.ptr, C.cast(objects, C.c_void_p), len(objects), what, C.byref(out),
                            tdt, tbad, 256)
    if rc != 0:
        raise RuntimeError(f"or_calibrate failed ({rc})")
    n = min(out.n_tested, 256)
    return out, [(float(tdt[i]), bool(tbad[i])) for i in range(n)]


def box2d_overlaps(a5, b5, gap):
    """luke::Box2d::overlapsWith for boxes given as (cx, cy, w, h, rot)."""
    a = np.ascontiguousarray(a5, dtype=np.float64); b = np.ascontiguousarray(b5, dtype=np.float64)
    return bool(lib().or_box2d_overlaps(a.ctypes.data_as(C.POINTER(C.c_double)),
                                        b.ctypes.data_as(C.POINTER(C.c_double)), gap))


def minstd_raw(seed, n):
    """minstd_rand0 raw outputs via the oracle's canonical draw state (16807 x mod 2^31-1)."""
    s = C.c_uint32(seed)
    out = []
    for _ in range(n):
        lib().or_minstd_next_canonical_float(C.byref(s))
        out.append(s.value)
    return out


def canonical_doubles(seed, n):
    s = C.c_uint32(seed)
    return np.array([lib().or_minstd_next_canonical_double(C.byref(s)) for _ in range(n)])
