"""Scripted grasp mix: a deterministic per-env action schedule that drives the batch
through every phase of a reference episode -- approach, finger contact, squeeze (the
bending gauges load up), palm press, lift -- so that parity tests and the benchmark see
grasp-phase physics, not only the early free-motion steps of random actions.

Actions are continuous fractions in [-1, 1] for the in-use actions of the settings
(MjClass::set_continous_action order, mjclass.cpp:1517-1526).  For the canonical
baseline (gripper_prismatic_X sign -1, gripper_revolute_Y sign -1, gripper_Z, base_Z):
+1 prismatic closes the fingers, -1 revolute tilts the tips inward (squeeze), +1
gripper_Z lowers the palm, -1 base_Z lifts the base (MjClass::set_action,
mjclass.cpp:1528-1630; Target::base_min/max, myfunctions.cpp:245-261).

The draws are counter-based (splitmix64 of seed, global env id, episode, draw; see
gm_state.h gm_spawn_int), so this host class and the device kernel behind
gm_scripted_actions produce the same actions bit for bit, whatever the sharding.
"""
from __future__ import annotations

import numpy as np

from ._lib import ACTION_KINDS
from .env import spawn_int


def in_use_actions(settings) -> list[str]:
    names = [k for k in ACTION_KINDS if getattr(settings, k).in_use]
    if settings.use_termination_action:
        names.append("termination")
    return names


class GraspScript:
    """`actions(k, episode)` gives the [n, n_act] action rows for per-env episode step
    counters k and episode numbers (first episode after gm_create = 1)."""

    def __init__(self, settings, n_envs: int, seed: int = 0, jitter: float = 0.2, env_offset: int = 0):
        self.names = in_use_actions(settings)
        self.n = int(n_envs)
        self.seed = int(seed)
        self.jitter = np.float32(jitter)
        self.gids = int(env_offset) + np.arange(self.n, dtype=np.int64)

    def phases(self, episode):
        s, g = self.seed, self.gids
        close_n = spawn_int(s, g, episode, 16, 34, 45)
        tilt_n = spawn_int(s, g, episode, 17, 0, 25)
        tilt_dir = np.where(spawn_int(s, g, episode, 18, 0, 4) < 4, -1.0, 1.0).astype(np.float32)
        palm_n = spawn_int(s, g, episode, 19, 0, 15)
        return close_n, tilt_n, tilt_dir, palm_n

    def actions(self, k, episode=1) -> np.ndarray:
        k = np.broadcast_to(np.asarray(k, dtype=np.int64), (self.n,))
        ep = np.broadcast_to(np.asarray(episode, dtype=np.int64), (self.n,))
        close_n, tilt_n, tilt_dir, palm_n = self.phases(ep)
        t1 = close_n
        t2 = t1 + tilt_n
        t3 = t2 + palm_n
        a = np.zeros((self.n, len(self.names)), dtype=np.float32)
        for i, name in enumerate(self.names):
            if name == "gripper_prismatic_X":
                a[k < t1, i] = 1.0
            elif name == "gripper_revolute_Y":
                m = (k >= t1) & (k < t2)
                a[m, i] = tilt_dir[m]
            elif name == "gripper_Z":
                a[(k >= t2) & (k < t3), i] = 1.0
            elif name == "base_Z":
                a[k >= t3, i] = -1.0
            if self.jitter > 0:
                u = spawn_int(self.seed, self.gids, ep, 32 + 8 * k + i, 0, 1 << 20).astype(np.float32)
                a[:, i] += self.jitter * (u * np.float32(2.0 / (1 << 20)) - np.float32(1.0))
        return np.clip(a, np.float32(-1.0), np.float32(1.0))
