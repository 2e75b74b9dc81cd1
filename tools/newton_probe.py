"""CPU probe of the constraint solver on grasp-phase states (oracle only, no GPU).

Rolls n envs of the C3 workload (set6-like objects, device-style spawn draws, the scripted
grasp mix) on the CPU oracle with the engine's Newton solver, reports the Newton
iteration / line-search statistics and the contact counts, and at a few snapshot steps
compares one env-step of Newton against the dense PGS cross-check run to many sweeps
from the same states (the regularised problem has one optimum: both must land on it).

    python tools/newton_probe.py [n_envs] [steps]
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "gripper-mujoco_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import gmx  # noqa: E402
import oracle_lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 48
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    snaps = [int(s) for s in sys.argv[3].split(",")] if len(sys.argv) > 3 else [25, 40, 55]
    L = oracle_lib.lib()
    L.or_get_stats.argtypes = [C.c_void_p, C.POINTER(C.c_int64)]
    L.or_set_default_solver.argtypes = [C.c_int]
    settings = gmx.canonical_settings(noise=False, seed=1234)
    model = gmx.ModelBlob()
    cfg = gmx.ConfigBlob(settings, model)
    objects = gmx.make_object_set("set6_synthetic", 1234)
    envs = [oracle_lib.OracleEnv(model, cfg, objects, e) for e in range(n)]
    si, sx, sy, sr = gmx.env.spawn_draws(1234, np.arange(n), np.ones(n, dtype=np.int64), len(objects))
    sp = gmx.default_spawn_params()
    for e, o in enumerate(envs):
        s = gmx.Spawn(int(si[e]), float(sx[e]), float(sy[e]), float(sr[e]))
        o.reset(s)
        sp.index = int(si[e])
        for _ in range(3):
            if o.spawn_into_scene(sp):
                break
    script = gmx.GraspScript(settings, n, seed=1234)
    t0 = time.time()
    for k in range(steps):
        a = script.actions(k)
        if k in snaps:
            recs = np.stack([o.export_state() for o in envs])
            res = {}
            for sweeps in (0, 200, 800, 3000):
                L.or_set_default_solver(sweeps)
                obs, _, _, _ = oracle_lib.batch_step(model, cfg, objects, recs, actions=a)
                res[sweeps] = obs
            L.or_set_default_solver(0)
            ref = res[0]
            big = np.abs(ref) >= 1e-3
            msg = []
            for sw in (200, 800, 3000):
                d = np.abs(res[sw] - ref)
                rel = np.where(big, d / np.where(big, np.abs(ref), 1), d).max(axis=1)
                msg.append(f"pgs{sw}: max {rel.max():.2e} n>1e-4 {(rel > 1e-4).sum()}")
            print(f"step {k}: Newton vs " + "; ".join(msg), flush=True)
        for e, o in enumerate(envs):
            o.step(a[e])
    dt = time.time() - t0
    st = np.zeros((n, 6), dtype=np.int64)
    for e, o in enumerate(envs):
        L.or_get_stats(o.h, st[e].ctypes.data_as(C.POINTER(C.c_int64)))
    solves = st[:, 0].sum()
    print(f"{n} envs x {steps} steps in {dt:.1f} s; Newton iterations/solve {st[:, 1].sum() / solves:.3f} "
          f"(max {st[:, 3].max()}), line-search evals/solve {st[:, 2].sum() / solves:.3f}, "
          f"mean rows {st[:, 5].sum() / solves:.1f}, max contacts {st[:, 4].max()}")


if __name__ == "__main__":
    main()
