"""Scripted grasp mix: a deterministic per-env action schedule that drives the batch
through every phase of a reference episode -- approach, finger contact, squeeze (the
bending gauges load up), palm press, lift -- so that parity tests and the benchmark see
grasp-phase physics, not only the early free-motion steps of random actions.

Actions are continuous fractions in [-1, 1] for the in-use actions of the settings, by
name (MjClass::set_continous_action order, mjclass.cpp:1517-1526).  For the canonical
baseline (gripper_prismatic_X sign -1, gripper_revolute_Y sign -1, gripper_Z, base_Z):
+1 prismatic closes the fingers, -1 revolute tilts the tips inward (squeeze), +1
gripper_Z lowers the palm, -1 base_Z lifts the base (MjClass::set_action,
mjclass.cpp:1528-1630; Target::base_min/max, myfunctions.cpp:245-261).
"""
from __future__ import annotations

import numpy as np

from ._lib import ACTION_KINDS


def in_use_actions(settings) -> list[str]:
    names = [k for k in ACTION_KINDS if getattr(settings, k).in_use]
    if settings.use_termination_action:
        names.append("termination")
    return names


class GraspScript:
    """Per-env phase lengths drawn once from `seed`; `actions(k)` gives the [n, n_act]
    action rows for per-env episode step counters k (so envs can be staggered)."""

    def __init__(self, settings, n_envs: int, seed: int = 0, jitter: float = 0.2):
        self.names = in_use_actions(settings)
        self.n = int(n_envs)
        rng = np.random.default_rng(seed)
        self.close_n = rng.integers(34, 46, size=self.n)
        self.tilt_n = rng.integers(0, 26, size=self.n)
        self.tilt_dir = np.where(rng.random(self.n) < 0.8, -1.0, 1.0)
        self.palm_n = rng.integers(0, 16, size=self.n)
        self.jitter = float(jitter)
        self._rng = np.random.default_rng(seed + 1)

    def _col(self, name):
        return self.names.index(name) if name in self.names else None

    def actions(self, k) -> np.ndarray:
        k = np.broadcast_to(np.asarray(k), (self.n,))
        a = np.zeros((self.n, len(self.names)), dtype=np.float32)
        c_pris, c_rev = self._col("gripper_prismatic_X"), self._col("gripper_revolute_Y")
        c_z, c_bz = self._col("gripper_Z"), self._col("base_Z")
        t1 = self.close_n
        t2 = t1 + self.tilt_n
        t3 = t2 + self.palm_n
        closing = k < t1
        tilting = (k >= t1) & (k < t2)
        pressing = (k >= t2) & (k < t3)
        lifting = k >= t3
        if c_pris is not None:
            a[closing, c_pris] = 1.0
        if c_rev is not None:
            a[tilting, c_rev] = self.tilt_dir[tilting]
        if c_z is not None:
            a[pressing, c_z] = 1.0
        if c_bz is not None:
            a[lifting, c_bz] = -1.0
        if self.jitter > 0:
            a += self._rng.uniform(-self.jitter, self.jitter, size=a.shape).astype(np.float32)
        return np.clip(a, -1.0, 1.0)
