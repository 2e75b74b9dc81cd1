"""Batched env: the reference's MjEnv.step / reset contract (rl/env/MjEnv.py:2170-2263)
for n_envs envs at once, every env-step executed by the fused device kernel.

Step order matches MjEnv.step: actions -> action_step -> observation -> (terminated,
truncated) -> reward.  Truncation at max_episode_steps is tracked on the host exactly
as MjEnv._is_done does (MjEnv.py:616-637).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import (GM_MAX_CON, GM_MAX_DOF, GM_MAX_EFC, load_library, ModelBlob, ConfigBlob, ModelParams, Spawn, SpawnParams, make_object_set,
                   BINARY_EVENTS, LINEAR_EVENTS, RolloutParams)
from .settings import canonical_settings, MAX_EPISODE_STEPS


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return x ^ (x >> np.uint64(31))


def spawn_int(seed, gid, episode, k, lo, hi):
    """gm_spawn_int (csrc/gm_state.h) vectorised: uniform integer in [lo, hi] from draw k of
    splitmix64(seed, global env id, episode) -- bit-identical to the device draw."""
    with np.errstate(over="ignore"):
        gid = np.asarray(gid, dtype=np.int64).astype(np.uint64)
        ep = np.asarray(episode, dtype=np.int64).astype(np.uint32).astype(np.uint64)
        kk = np.asarray(k, dtype=np.int64).astype(np.uint64)
        x = (np.uint64(seed) + gid * np.uint64(0xD1B54A32D192ED03) + ep * np.uint64(0x8CB92BA72F3D8DD7)
             + kk * np.uint64(0x9E3779B97F4A7C15)) & _M64
        h = _splitmix64(x)
        span = np.uint64(hi - lo + 1)
        return lo + (((h >> np.uint64(32)) * span) >> np.uint64(32)).astype(np.int64)


def random_fractions(seed, gid, episode, step, n_actions):
    """gm_random_fraction (csrc/gm_state.h) vectorised over envs: [n, n_actions] uniform
    fractions in [-1, 1) for episode step `step` -- bit-identical to gm_random_actions."""
    with np.errstate(over="ignore"):
        gid = np.asarray(gid, dtype=np.int64).astype(np.uint64).reshape(-1, 1)
        ep = np.asarray(episode, dtype=np.int64).astype(np.uint32).astype(np.uint64).reshape(-1, 1)
        kk = np.asarray(step, dtype=np.int64).astype(np.uint32).astype(np.uint64).reshape(-1, 1)
        ii = np.arange(n_actions, dtype=np.uint64).reshape(1, -1)
        x = (np.uint64(seed) * np.uint64(0xA24BAED4963EE407) + gid * np.uint64(0xD1B54A32D192ED03)
             + ep * np.uint64(0x8CB92BA72F3D8DD7) + kk * np.uint64(0x9E3779B97F4A7C15)
             + ii * np.uint64(0xF1357AEA2E62A9C5)) & _M64
        h = _splitmix64(x)
        return ((h >> np.uint64(40)).astype(np.float32) * np.float32(2.0 / 16777216.0) - np.float32(1.0)).astype(np.float32)


def spawn_draws(seed, gids, episodes, n_objects, position_noise_mm: int = 10, rotation_noise_deg: int = 5):
    """MjEnv._spawn_object's generator draws (MjEnv.py:1177-1267) for each (global env id,
    episode): object index and the "old method" pose (integer mm offsets; z rotation one of
    {0, 60, 120} deg plus integer-degree noise).  The device makes the same draws in
    gm_reset / gm_autoreset (gm_set_random_spawn), so they are shard-independent."""
    nm, nd = int(position_noise_mm), int(rotation_noise_deg)
    idx = spawn_int(seed, gids, episodes, 0, 0, n_objects - 1)
    x = spawn_int(seed, gids, episodes, 1, -nm, nm) * 1e-3
    y = spawn_int(seed, gids, episodes, 2, -nm, nm) * 1e-3
    noise = spawn_int(seed, gids, episodes, 3, -nd, nd)
    opt = spawn_int(seed, gids, episodes, 4, 0, 2)
    rot = (60 * opt + noise) * (np.pi / 180.0)
    return idx, x, y, rot


class BatchedGripperEnv:
    def __init__(self, n_envs: int, object_set: str = "set6_synthetic", settings=None,
                 model_params: ModelParams | None = None, device: int = 0, seed: int = 1234,
                 env_offset: int = 0, max_episode_steps: int = MAX_EPISODE_STEPS, lib=None,
                 model_blob: ModelBlob | None = None, objects=None):
        self.lib = lib if lib is not None else load_library()
        self.n_envs = int(n_envs)
        self.model = model_blob if model_blob is not None else ModelBlob(model_params)
        self.settings = settings if settings is not None else canonical_settings(seed=seed)
        self.cfg = ConfigBlob(self.settings, self.model)
        # an explicit gm_object array (e.g. the force-measurement spheres) or a named set
        self.objects = objects if objects is not None else make_object_set(object_set, seed)
        self.max_episode_steps = max_episode_steps
        self.device = device
        self.seed = int(seed)
        self.env_offset = int(env_offset)
        self._episode = np.zeros(self.n_envs, dtype=np.int64)   # mirrors GmEnvState::episode
        self._ctx = C.c_void_p()
        rc = self.lib.gm_create(self.model.ptr, self.cfg.ptr, self.objects, len(self.objects), self.n_envs,
                                int(env_offset), int(device), int(seed), C.byref(self._ctx))
        if rc != 0:
            msg = self.lib.gm_last_error(self._ctx).decode() if self._ctx else ""
            raise RuntimeError(f"gm_create failed ({rc}) {msg}")
        # resets without a spawn table draw MjEnv._spawn_object's object / pose on the device
        self._check(self.lib.gm_set_random_spawn(self._ctx, 1, self.seed, 10, 5))
        self.n_obs = self.lib.gm_n_obs(self._ctx)
        self.n_actions = self.lib.gm_n_actions(self._ctx)
        self.current_step = np.zeros(self.n_envs, dtype=np.int64)
        self._obs = np.zeros((self.n_envs, self.n_obs), dtype=np.float32)
        self._rew = np.zeros(self.n_envs, dtype=np.float32)
        self._done = np.zeros(self.n_envs, dtype=np.uint8)

    # ------------------------------------------------------------ plumbing
    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(self.lib.gm_last_error(self._ctx).decode() or f"gm error {rc}")

    def close(self):
        if self._ctx:
            self.lib.gm_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def ctx(self):
        return self._ctx

    @property
    def stream(self) -> int:
        return self.lib.gm_stream(self._ctx)

    # ------------------------------------------------------------ env API
    def make_spawn(self, mask=None, idx=None, x=None, y=None, rot=None):
        """An explicit spawn table for the next reset: MjEnv._spawn_object's draws for each
        env's global id and next episode (spawn_draws), with optional overrides."""
        n = self.n_envs
        gids = self.env_offset + np.arange(n)
        self._sync_episode()
        si, sx, sy, sr = spawn_draws(self.seed, gids, self._episode + 1, len(self.objects))
        if idx is not None: si = np.broadcast_to(np.asarray(idx), (n,))
        if x is not None: sx = np.broadcast_to(np.asarray(x, dtype=np.float64), (n,))
        if y is not None: sy = np.broadcast_to(np.asarray(y, dtype=np.float64), (n,))
        if rot is not None: sr = np.broadcast_to(np.asarray(rot, dtype=np.float64), (n,))
        arr = (Spawn * n)()
        for e in range(n):
            arr[e].object_index = int(si[e]); arr[e].x = float(sx[e]); arr[e].y = float(sy[e]); arr[e].zrot = float(sr[e])
        return arr

    def _sync_episode(self):
        """The device owns GmEnvState::episode (gm_autoreset and gm_set_env_states move it
        without the host seeing): re-read it before drawing a spawn table."""
        from ._lib import env_state_view
        self._episode[:] = env_state_view(self.env_states())["episode"]

    def reset(self, mask=None, spawn=None):
        """MjClass::reset + spawn for masked envs; returns the observation (MjEnv.reset).
        spawn=None: the object and pose are drawn on the device (gm_set_random_spawn)."""
        if mask is not None:
            m = np.ascontiguousarray(np.asarray(mask, dtype=np.uint8))
            self._check(self.lib.gm_reset(self._ctx, m.ctypes.data_as(C.POINTER(C.c_uint8)), spawn))
            self.current_step[m.astype(bool)] = 0
            self._episode[m.astype(bool)] += 1
        else:
            self._check(self.lib.gm_reset(self._ctx, None, spawn))
            self.current_step[:] = 0
            self._episode += 1
        return self.observation()

    def spawn_into_scene(self, params, mask=None):
        """MjClass::spawn_into_scene(SpawnParams) on the device (mjclass.cpp:2475-2654).
        params: one SpawnParams (shared) or a sequence of n_envs.  Returns ok[n_envs]
        (True where the object was placed)."""
        if isinstance(params, SpawnParams):
            arr, n = (SpawnParams * 1)(params), 1
        else:
            arr = (SpawnParams * len(params))(*params)
            n = len(params)
        ok = np.zeros(self.n_envs, dtype=np.uint8)
        m = None
        if mask is not None:
            m = np.ascontiguousarray(np.asarray(mask, dtype=np.uint8))
        self._check(self.lib.gm_spawn_into_scene(self._ctx, None if m is None else m.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                 arr, n, ok.ctypes.data_as(C.POINTER(C.c_uint8))))
        return ok.astype(bool)

    def set_scene_spawn(self, params, max_tries: int = 3):
        """Resets place objects with spawn_into_scene (MjEnv._spawn_object: up to max_tries
        attempts, then the spawn table pose); params=None restores plain spawn_object."""
        self._check(self.lib.gm_set_scene_spawn(self._ctx, None if params is None else C.byref(params), int(max_tries)))

    def scripted_actions(self, seed: int, jitter: float = 0.2) -> np.ndarray:
        """The device scripted grasp mix for every env's current episode step
        (gm_scripted_actions; gmx.GraspScript is its host mirror)."""
        out = np.zeros((self.n_envs, self.n_actions), dtype=np.float32)
        self._check(self.lib.gm_scripted_actions(self._ctx, int(seed), float(jitter), out.ctypes.data, 0))
        return out

    def program_actions(self, seed: int = 0, jitter: float = 0.2, mode: int = 3) -> np.ndarray:
        """The device grasp-lift-hold program (mode 3) or the benchmark's program / scripted
        mix (mode 4) for every env's current state (gm_program_actions)."""
        out = np.zeros((self.n_envs, self.n_actions), dtype=np.float32)
        self._check(self.lib.gm_program_actions(self._ctx, int(seed), float(jitter), int(mode), out.ctypes.data, 0))
        return out

    def set_action(self, actions):
        a = np.ascontiguousarray(np.asarray(actions, dtype=np.float32).reshape(self.n_envs, self.n_actions))
        self._check(self.lib.gm_set_action(self._ctx, a.ctypes.data, 0))

    def set_discrete_action(self, actions):
        a = np.ascontiguousarray(np.asarray(actions, dtype=np.int32).reshape(self.n_envs))
        self._check(self.lib.gm_set_discrete_action(self._ctx, a.ctypes.data, 0))

    def action_step(self):
        self._check(self.lib.gm_step(self._ctx))

    def rollout(self, n_steps: int, action_mode: int = 0, seed: int = 1234, jitter: float = 0.2,
                max_episode_steps: int | None = None, records_dev_ptr: int | None = None):
        """gm_rollout: n_steps env-steps of every env in one launch with the device driver
        (0: scripted grasp mix, 1: uniform random actions, 3: the grasp program, 4: the
        benchmark's program / scripted mix) and the device auto-reset; equal bit
        for bit to n_steps rounds of driver actions -> set_action -> step -> autoreset.
        records_dev_ptr: device [n_steps x n_envs] gm_episode_end records (or None)."""
        mx = self.max_episode_steps if max_episode_steps is None else max_episode_steps
        p = RolloutParams()
        p.action_mode, p.max_episode_steps, p.seed, p.jitter = int(action_mode), int(mx), int(seed), float(jitter)
        self._check(self.lib.gm_rollout(self._ctx, int(n_steps), C.byref(p), C.c_void_p(records_dev_ptr or 0)))

    def set_motor_target(self, xyz, mask=None):
        """MjClass::set_motor_target(x, y, z) (bind.cpp:82) for every env (xyz: 3 values, or
        [n_envs, 3]); returns the reference's in-limits flags per env."""
        t = np.ascontiguousarray(np.asarray(xyz, dtype=np.float64).reshape(-1, 3))
        if t.shape[0] not in (1, self.n_envs):
            raise ValueError(f"xyz must be 3 values or [{self.n_envs}, 3]")
        ok = np.ones(self.n_envs, dtype=np.uint8)
        m = None if mask is None else np.ascontiguousarray(np.asarray(mask, dtype=np.uint8).reshape(self.n_envs))
        self._check(self.lib.gm_set_motor_target(self._ctx, None if m is None else m.ctypes.data, t.ctypes.data,
                                                 t.shape[0], ok.ctypes.data))
        return ok.astype(bool)

    def sensor_si(self):
        """Latest sim_sensors_SI_ readings [n_envs, 5]: finger 1..3 gauges, palm, wrist Z (N)."""
        out = np.zeros((self.n_envs, 5), dtype=np.float32)
        self._check(self.lib.gm_get_sensor_si(self._ctx, out.ctypes.data))
        return out

    def observation(self):
        self._check(self.lib.gm_get_obs(self._ctx, self._obs.ctypes.data, 0))
        return self._obs.copy()

    def outputs(self):
        """(obs, reward, done) of the last env-step, one device read (gm_get_outputs)."""
        self._check(self.lib.gm_get_outputs(self._ctx, self._obs.ctypes.data, self._rew.ctypes.data,
                                            self._done.ctypes.data))
        return self._obs.copy(), self._rew.copy(), self._done.astype(bool)

    def reward_done(self):
        self._check(self.lib.gm_get_reward_done(self._ctx, self._rew.ctypes.data, self._done.ctypes.data, 0))
        return self._rew.copy(), self._done.astype(bool)

    def step(self, actions, discrete: bool = False):
        """Returns (obs, reward, terminated, truncated) like MjEnv.step."""
        self.current_step += 1
        if discrete:
            self.set_discrete_action(actions)
        else:
            self.set_action(actions)
        self.action_step()
        obs, rew, term = self.outputs()
        trunc = self.current_step >= self.max_episode_steps
        term = np.where(trunc, False, term)
        return obs, rew, term, trunc

    # ------------------------------------------------------------ device (zero-copy) path
    def step_device(self, actions_dev_ptr: int):
        """actions already on the device (e.g. a torch tensor's data_ptr() written on
        this context's stream); obs/reward/done stay on the device."""
        self._check(self.lib.gm_set_action(self._ctx, C.c_void_p(actions_dev_ptr), 1))
        self._check(self.lib.gm_step(self._ctx))

    def set_stream(self, stream_handle: int | None):
        """Launch on an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream)."""
        self._check(self.lib.gm_set_stream(self._ctx, C.c_void_p(stream_handle or 0)))

    def upload_spawn(self, spawn):
        """Copy a host gm_spawn array once; returns the device pointer kept alive by self."""
        import torch
        raw = np.frombuffer(bytes(spawn), dtype=np.uint8)
        self._spawn_dev = torch.from_numpy(raw.copy()).to(f"cuda:{self.device}")
        return self._spawn_dev.data_ptr()

    def autoreset_device(self, spawn_dev_ptr: int, returns_dev_ptr: int | None = None,
                         max_episode_steps: int | None = None, episodes_dev_ptr: int | None = None):
        """Episode boundary on the device: done/truncated envs report their return (and, with
        episodes_dev_ptr, the gm_episode_end record: return, length, success) and are reset
        + respawned (MjEnv.py:616-637, 2222-2263)."""
        mx = self.max_episode_steps if max_episode_steps is None else max_episode_steps
        self._check(self.lib.gm_autoreset_episodes(self._ctx, int(mx), C.c_void_p(spawn_dev_ptr), 1,
                                                   C.c_void_p(returns_dev_ptr or 0),
                                                   C.c_void_p(episodes_dev_ptr or 0)))

    def device_buffers(self):
        return (self.lib.gm_device_obs(self._ctx), self.lib.gm_device_reward(self._ctx),
                self.lib.gm_device_done(self._ctx))

    def last_step_ms(self) -> float:
        v = C.c_float()
        self._check(self.lib.gm_last_step_ms(self._ctx, C.byref(v)))
        return float(v.value)

    def chunk_stats(self) -> dict:
        """The last gm_step's chunked-dispatch counters (include/gripper_mi355x.h gm_chunk_stats)."""
        v = (C.c_uint32 * 7)()
        t = (C.c_uint64 * 5)()
        self._check(self.lib.gm_chunk_stats(self._ctx, v, t))
        span = (t[2] - t[0]) * 1e-5 if t[2] > t[0] else 0.0   # ms
        return dict(started=v[0], finished=v[1], yields=v[2], resumes=v[3], every=v[4], workgroups=v[5], steals=v[6],
                    span_ms=span, fresh_empty_ms=(t[1] - t[0]) * 1e-5 if t[1] >= t[0] and span else 0.0,
                    busy=(t[3] / (v[5] * (t[2] - t[0]))) if span and v[5] else 0.0,
                    poll=(t[4] / (v[5] * (t[2] - t[0]))) if span and v[5] else 0.0)

    def claim_waits(self) -> dict:
        """The last chunked launch's claims that found their ring slot still empty, and the
        polls they made (gm_chunk_claim_waits)."""
        v = (C.c_uint32 * 2)()
        self._check(self.lib.gm_chunk_claim_waits(self._ctx, v))
        return dict(waiting_claims=int(v[0]), polls=int(v[1]))

    def job_stats(self):
        """The last chunked launch's jobs (gm_chunk_job_stats): per env the shader clocks / 64
        its job ran for and the job's yields, as two numpy arrays."""
        import numpy as np
        clk = np.zeros(self.n_envs, dtype=np.uint32)
        yl = np.zeros(self.n_envs, dtype=np.int32)
        self._check(self.lib.gm_chunk_job_stats(self._ctx, clk.ctypes.data_as(C.c_void_p),
                                                 yl.ctypes.data_as(C.c_void_p)))
        return clk, yl

    def chunk_timeline(self):
        """When each workgroup of the last chunked launch finished its last work, ms after the
        launch's first pick, its XCD, and per env [start, finish] ms (gm_chunk_timeline)."""
        import numpy as np
        info = self.dispatch_info()
        G = info["grid"]
        buf = (C.c_uint64 * max(1, G + 2 * self.n_envs))()
        n = self.lib.gm_chunk_timeline(self._ctx, buf, G + 2 * self.n_envs)
        if n < 0:
            raise RuntimeError(f"gm_chunk_timeline failed ({n})")
        t = (C.c_uint64 * 5)()
        v = (C.c_uint32 * 7)()
        self._check(self.lib.gm_chunk_stats(self._ctx, v, t))
        raw = np.frombuffer(buf, dtype=np.uint64, count=n)
        wg = raw[:G]
        ends = ((wg & np.uint64((1 << 60) - 1)).astype(np.float64) - float(t[0])) * 1e-5
        ev = (raw[G:].astype(np.float64).reshape(-1, 2) - float(t[0])) * 1e-5
        return ends, (wg >> np.uint64(60)).astype(np.int32), ev

    def dispatch_info(self) -> dict:
        """How gm_step / gm_rollout dispatch this context (include/gripper_mi355x.h gm_dispatch_info)."""
        v = (C.c_int32 * 4)()
        self._check(self.lib.gm_dispatch_info(self._ctx, v))
        return dict(chunk=v[0], grid=v[1], waves_per_env=v[2], last_launch_env_steps=v[3])

    # ------------------------------------------------------------ inspection
    def state(self):
        """fp64 qpos [n, nq], qvel [n, nv], time [n] (mjData's precision)."""
        q = np.zeros((self.n_envs, self.model.nq), dtype=np.float64)
        v = np.zeros((self.n_envs, self.model.nv), dtype=np.float64)
        t = np.zeros(self.n_envs, dtype=np.float64)
        self._check(self.lib.gm_get_state(self._ctx, q.ctypes.data_as(C.POINTER(C.c_double)),
                                          v.ctypes.data_as(C.POINTER(C.c_double)),
                                          t.ctypes.data_as(C.POINTER(C.c_double))))
        return q, v, t

    def set_state(self, qpos, qvel):
        q = np.ascontiguousarray(np.asarray(qpos, dtype=np.float64))
        v = np.ascontiguousarray(np.asarray(qvel, dtype=np.float64))
        self._check(self.lib.gm_set_state(self._ctx, q.ctypes.data_as(C.POINTER(C.c_double)),
                                          v.ctypes.data_as(C.POINTER(C.c_double))))

    def env_states(self) -> np.ndarray:
        """The whole per-env state as raw GmEnvState records, [n_envs, state_size] uint8
        (checkpoint / resume, and the oracle hand-off of the parity tests)."""
        sz = int(self.lib.gm_env_state_size())
        out = np.zeros((self.n_envs, sz), dtype=np.uint8)
        self._check(self.lib.gm_get_env_states(self._ctx, out.ctypes.data))
        return out

    def set_env_states(self, states):
        a = np.ascontiguousarray(np.asarray(states, dtype=np.uint8))
        if a.shape != (self.n_envs, int(self.lib.gm_env_state_size())):
            raise ValueError(f"expected {(self.n_envs, int(self.lib.gm_env_state_size()))} state records, got {a.shape}")
        self._check(self.lib.gm_set_env_states(self._ctx, a.ctypes.data))

    def target(self):
        e = np.zeros((self.n_envs, 4)); es = np.zeros((self.n_envs, 3), dtype=np.int32)
        ns = np.zeros((self.n_envs, 3), dtype=np.int32); b = np.zeros((self.n_envs, 3))
        self._check(self.lib.gm_get_target(self._ctx, e.ctypes.data_as(C.POINTER(C.c_double)),
                                           es.ctypes.data_as(C.POINTER(C.c_int32)),
                                           ns.ctypes.data_as(C.POINTER(C.c_int32)),
                                           b.ctypes.data_as(C.POINTER(C.c_double))))
        return e, es, ns, b

    def event_rows(self):
        W = len(BINARY_EVENTS) + len(LINEAR_EVENTS)
        rows = np.zeros((self.n_envs, W), dtype=np.int32)
        absc = np.zeros((self.n_envs, W), dtype=np.int32)
        lastv = np.zeros((self.n_envs, W), dtype=np.float32)
        self._check(self.lib.gm_get_event_rows(self._ctx, rows.ctypes.data_as(C.POINTER(C.c_int32)),
                                               absc.ctypes.data_as(C.POINTER(C.c_int32)),
                                               lastv.ctypes.data_as(C.POINTER(C.c_float))))
        return rows, absc, lastv

    def overflow(self):
        o = np.zeros(self.n_envs, dtype=np.int32)
        self._check(self.lib.gm_get_overflow(self._ctx, o.ctypes.data_as(C.POINTER(C.c_int32))))
        return o

    def debug_substep(self, full: bool = False):
        """One MjClass::step on every env with fp64 diagnostics: (ncon, contact [n, GM_MAX_CON, 16],
        efc_force [n, GM_MAX_EFC], qacc [n, GM_MAX_DOF]) and, with full=True, also nefc [n] and
        the object's cfrc_ext wrench [n, 6]."""
        n = self.n_envs
        ncon = np.zeros(n, dtype=np.int32)
        nefc = np.zeros(n, dtype=np.int32)
        con = np.zeros((n, GM_MAX_CON, 16), dtype=np.float64)
        f = np.zeros((n, GM_MAX_EFC), dtype=np.float64)
        qacc = np.zeros((n, GM_MAX_DOF), dtype=np.float64)
        w = np.zeros((n, 6), dtype=np.float64)
        d = C.POINTER(C.c_double)
        self._check(self.lib.gm_debug_substep(self._ctx, ncon.ctypes.data_as(C.POINTER(C.c_int32)),
                                              con.ctypes.data_as(d), f.ctypes.data_as(d), qacc.ctypes.data_as(d),
                                              nefc.ctypes.data_as(C.POINTER(C.c_int32)), w.ctypes.data_as(d)))
        if full:
            return ncon, con, f, qacc, nefc, w
        return ncon, con, f, qacc

    PHASES = ("kinematics", "crb_rne", "mass_forces", "  n:QF+bodies", "  n:scans+composites", "collision",
              "newton_solve", "  n:H_assembly", "integrate", "update_all", "monitor_sensors",
              "  n:setup", "  n:warm_start", "  n:jar+line_search", "  n:factor", "  k:A_hinge", "  k:B_chains",
              "  crb:chains", "e:sense", "e:update_env", "e:get_obs", "e:done_reward", "substep_body", "env_step",
              "  n:solve", "t:start", "t:end", "cu")   # 25-27: timeline (100 MHz clock) and CU id, not clocks
    # counter columns past the clocks
    PH_NEFC, PH_MPR, PH_NEWTON, PH_LS = 28, 29, 30, 31
    N_PHASE = 32

    def step_profiled(self):
        """One env-step with per-phase shader-clock counters (lane 0, summed over substeps)."""
        ph = np.zeros((self.n_envs, self.N_PHASE), dtype=np.uint64)
        self._check(self.lib.gm_step_profiled(self._ctx, ph.ctypes.data_as(C.POINTER(C.c_uint64))))
        return ph
