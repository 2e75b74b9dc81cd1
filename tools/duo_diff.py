"""Developer probe: which record fields differ between dispatch variants of the same batch
(one-shot / chunked x one-wave / DUO) after a few random env-steps.
usage: python tools/duo_diff.py [n] [steps]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd')]
import numpy as np
import gmx

n = int(sys.argv[1]) if len(sys.argv) > 1 else 37
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 4


def make(env_vars):
    old = {k: os.environ.get(k) for k in env_vars}
    os.environ.update(env_vars)
    try:
        env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=gmx.canonical_settings(seed=77), seed=77)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    env.reset()
    return env


variants = {"oneshot-1w": {"GM_CHUNK_SUBSTEPS": "0", "GM_DUO": "0"}, "oneshot-duo": {"GM_CHUNK_SUBSTEPS": "0", "GM_DUO": "1"},
            "chunk-1w": {"GM_DUO": "0"}, "chunk-duo": {"GM_DUO": "1"}, "chunk-duo-b": {"GM_DUO": "1"}}
envs = {k: make(v) for k, v in variants.items()}
rng = np.random.default_rng(n)
for t in range(steps):
    a = rng.uniform(-1, 1, size=(n, envs["oneshot-1w"].n_actions)).astype(np.float32)
    for e in envs.values():
        e.step(a)
    ref = gmx.env_state_view(envs["oneshot-1w"].env_states())
    for k, e in envs.items():
        v = gmx.env_state_view(e.env_states())
        bad = []
        for f in v.dtype.names:
            x, y = np.asarray(v[f]), np.asarray(ref[f])
            if not np.array_equal(x, y):
                envs_bad = np.where((x != y).reshape(n, -1).any(axis=1))[0]
                if x.dtype.kind == "f":
                    d = float(np.nanmax(np.abs(x.astype(np.float64) - y.astype(np.float64))))
                else:
                    d = None
                bad.append((f, len(envs_bad), envs_bad[:4].tolist(), d))
        print(f"step {t} {k}: {len(bad)} fields differ from oneshot-1w", bad[:12], flush=True)
