"""Developer probe: how many constraint rows change between consecutive Newton points of
the oracle's solver on the C3 benchmark mix -- the case for (or against) an incremental
rank-1 factor update in place of the refactor each extra point pays.
Builds oracle/physics.c with -DOR_NEWTON_STATS into /tmp (the tree's oracle is untouched).
usage: python tools/newton_active_set_probe.py [n_envs] [n_steps]"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "gripper-mujoco_amd")]
import gmx  # noqa: E402
import oracle_lib  # noqa: E402

n_envs = int(sys.argv[1]) if len(sys.argv) > 1 else 64
n_steps = int(sys.argv[2]) if len(sys.argv) > 2 else 250
so = "/tmp/liboracle_nstats.so"
subprocess.run(["gcc", "-O2", "-mavx", "-ffp-contract=off", "-std=c11", "-fPIC", "-shared", "-DOR_NEWTON_STATS",
                "-I" + os.path.join(REPO, "include"), os.path.join(REPO, "oracle", "oracle.c"), "-o", so, "-lm",
                "-pthread"], check=True)
oracle_lib._lib = oracle_lib.load(so)
s = gmx.canonical_settings(seed=1234)
model = gmx.ModelBlob()
cfg = gmx.ConfigBlob(s, model)
objs = gmx.make_object_set("set6_synthetic", 1234)
oracle_lib.bench(model, cfg, objs, n_envs, n_steps, seed=1234, n_threads=8, scripted=True)
st = (C.c_longlong * 40)()
oracle_lib._lib.or_newton_stats(st)
a = np.array(st[:], dtype=np.int64)
pts, solves = int(a[33]), int(a[34])
extra = pts - solves
h = a[:31]
c = np.cumsum(h) / max(extra, 1)
print(f"{n_envs} envs x {n_steps} env-steps of the C3 benchmark mix: {solves} solves, {pts} Newton points "
      f"({pts / solves:.4f} per solve), {a[35] / solves:.2f} rows per solve")
print(f"extra points {extra}: rows changed since the previous point, histogram "
      f"{ {i: int(h[i]) for i in range(31) if h[i]} }")
print(f"rows entering {a[31]}, leaving {a[32]}, mean changed per extra point {(a[31] + a[32]) / max(extra, 1):.2f}; "
      f"share with <= 1 / 2 / 4 changed rows: {c[1]:.3f} / {c[2]:.3f} / {c[4]:.3f}")
