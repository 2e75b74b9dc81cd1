"""On-device DQN action selection for the batched env.

Mirrors the reference's policy side of the rollout:
  - VariableNetwork (rl/networks.py:7-41): Linear + ReLU per hidden layer, a final
    Linear, Softmax(dim=1); canonical layers [n_obs, 150, 100, 50, n_actions]
    (launch_training.py:850-857);
  - Agent_DQN.select_action (rl/agents/DQN.py:184-209): eps_threshold =
    eps_end + (eps_start - eps_end) exp(-decay_num / eps_decay); a uniform random
    action with that probability, otherwise the argmax of the network output.
The forward pass and the choice run in one HIP kernel (gm_policy_kernel, f32 MFMA) on
the env's device observations and the chosen actions are applied on the device.
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from ._lib import load_library

CANONICAL_HIDDEN = (150, 100, 50)


def eps_threshold(decay_num: int, eps_start: float = 0.9, eps_end: float = 0.05, eps_decay: int = 1000) -> float:
    """Agent_DQN.select_action's exploration threshold (DQN.py:195-198; defaults DQN.py:75-77)."""
    return eps_end + (eps_start - eps_end) * math.exp(-1.0 * decay_num / float(eps_decay))


def init_params(sizes, seed: int = 0) -> np.ndarray:
    """nn.Linear's default init (kaiming-uniform weights, U(+-1/sqrt(fan_in)) biases) for
    every layer, flattened in state_dict order: W0 [out x in], b0, W1, b1, ..."""
    rng = np.random.default_rng(seed)
    parts = []
    for i in range(len(sizes) - 1):
        fan_in, fan_out = sizes[i], sizes[i + 1]
        bound = 1.0 / math.sqrt(fan_in)
        parts.append(rng.uniform(-bound, bound, size=(fan_out, fan_in)).astype(np.float32).ravel())
        parts.append(rng.uniform(-bound, bound, size=fan_out).astype(np.float32))
    return np.concatenate(parts).astype(np.float32)


def params_from_state_dict(state_dict) -> tuple[list[int], np.ndarray]:
    """(sizes, flat params) from a VariableNetwork state_dict (linear.i.weight / .bias)."""
    ws = sorted((k for k in state_dict if k.endswith(".weight")), key=lambda k: int(k.split(".")[1]))
    sizes = [int(state_dict[ws[0]].shape[1])]
    parts = []
    for k in ws:
        w = np.asarray(state_dict[k].detach().cpu().numpy() if hasattr(state_dict[k], "detach") else state_dict[k],
                       dtype=np.float32)
        b = state_dict[k[:-len("weight")] + "bias"]
        b = np.asarray(b.detach().cpu().numpy() if hasattr(b, "detach") else b, dtype=np.float32)
        sizes.append(int(w.shape[0]))
        parts += [w.ravel(), b.ravel()]
    return sizes, np.concatenate(parts).astype(np.float32)


def pack(sizes, params) -> np.ndarray:
    """The device layout of the parameters (gm_policy_pack; testable without a GPU)."""
    lib = load_library()
    sz = np.ascontiguousarray(sizes, dtype=np.int32)
    pr = np.ascontiguousarray(params, dtype=np.float32)
    i32p, f32p = C.POINTER(C.c_int32), C.POINTER(C.c_float)
    n = lib.gm_policy_pack(sz.ctypes.data_as(i32p), len(sz), pr.ctypes.data_as(f32p), None)
    if n < 0:
        raise ValueError("unsupported network sizes")
    out = np.zeros(n, dtype=np.float32)
    lib.gm_policy_pack(sz.ctypes.data_as(i32p), len(sz), pr.ctypes.data_as(f32p), out.ctypes.data_as(f32p))
    return out


class DevicePolicy:
    """A VariableNetwork DQN policy bound to a BatchedGripperEnv (discrete actions)."""

    def __init__(self, env, sizes=None, params=None, seed: int = 0):
        self.env = env
        self.lib = env.lib
        if sizes is None:
            sizes = [env.n_obs, *CANONICAL_HIDDEN, env.n_actions]
        self.sizes = [int(x) for x in sizes]
        self.params = init_params(self.sizes, seed) if params is None else np.ascontiguousarray(params, np.float32)
        sz = np.ascontiguousarray(self.sizes, dtype=np.int32)
        self._p = C.c_void_p()
        rc = self.lib.gm_policy_create(env.ctx, sz.ctypes.data_as(C.POINTER(C.c_int32)), len(sz),
                                       self.params.ctypes.data_as(C.POINTER(C.c_float)), C.byref(self._p))
        if rc != 0:
            raise RuntimeError(self.lib.gm_last_error(env.ctx).decode() or f"gm_policy_create failed ({rc})")

    def act(self, eps: float = 0.0, seed: int = 0, decision: int = 0):
        """select_action for every env from its current observation, applied on the device."""
        rc = self.lib.gm_policy_act(self._p, C.c_float(eps), C.c_uint64(seed), C.c_uint64(decision))
        if rc != 0:
            raise RuntimeError(self.lib.gm_last_error(self.env.ctx).decode() or f"gm_policy_act failed ({rc})")

    def rollout(self, eps, seed: int = 0, decision0: int = 0, max_episode_steps: int | None = None,
                records_dev_ptr: int | None = None):
        """gm_policy_rollout: len(eps) rounds of act(eps[k], seed, decision0 + k) -> env step ->
        auto-reset, fused into one persistent launch (bit for bit the per-step sequence).
        records_dev_ptr: device [len(eps) x n_envs] gm_episode_end records (or None)."""
        e = np.ascontiguousarray(np.atleast_1d(eps), dtype=np.float32)
        mx = self.env.max_episode_steps if max_episode_steps is None else max_episode_steps
        rc = self.lib.gm_policy_rollout(self._p, len(e), e.ctypes.data_as(C.POINTER(C.c_float)), C.c_uint64(seed),
                                        C.c_uint64(decision0), int(mx), C.c_void_p(records_dev_ptr or 0))
        if rc != 0:
            raise RuntimeError(self.lib.gm_last_error(self.env.ctx).decode() or f"gm_policy_rollout failed ({rc})")

    def read(self):
        n, a = self.env.n_envs, self.env.n_actions
        acts = np.zeros(n, dtype=np.int32)
        q = np.zeros((n, a), dtype=np.float32)
        rc = self.lib.gm_policy_read(self._p, acts.ctypes.data_as(C.POINTER(C.c_int32)),
                                     q.ctypes.data_as(C.POINTER(C.c_float)))
        if rc != 0:
            raise RuntimeError(self.lib.gm_last_error(self.env.ctx).decode())
        return acts, q

    def close(self):
        if self._p:
            self.lib.gm_policy_destroy(self._p)
            self._p = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
