"""Fit the invented segment-hinge numerics (damping law, armature law) to the reference's
measured stable timesteps (tests/golden/mujoco_timesteps.json <- rl/juypter/thesis_plots/
mujoco_timesteps.csv: 4 inertia scalings x 3 (thickness, width) x N = 5..10, 72 points).
Every evaluation runs find_highest_stable_timestep on the CPU oracle for all 72 points.

    python tools/fit_timesteps.py [maxiter]
"""
import ctypes as C
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "gripper-mujoco_amd"), os.path.join(REPO, "tests")]
import gmx  # noqa: E402
import oracle_lib  # noqa: E402

GOLDEN = os.path.join(REPO, "tests", "golden", "mujoco_timesteps.json")


def cases():
    out = []
    for name, col in json.load(open(GOLDEN))["columns"].items():
        kv = dict(x.strip().split("=") for x in name.split(","))
        for n, ms in col.items():
            out.append((int(n), float(kv["t"]), float(kv["w"]), float(kv["inertia"]), ms))
    return out


def search(n, t, w, s, params):
    p = gmx.ModelParams()
    gmx.load_library().gm_default_model_params(C.byref(p))
    p.n_seg, p.finger_thickness, p.finger_width = n, t * 1e-3, w * 1e-3
    p.segment_inertia_scaling, p.timestep = s, 1.0e-3
    for k, v in params.items():
        setattr(p, k, v)
    model = gmx.ModelBlob(p)
    cfg = gmx.ConfigBlob(gmx.canonical_settings(noise=False, seed=1), model)
    objs = gmx.make_object_set("set1_synthetic", 1)
    try:
        cal, _ = oracle_lib.calibrate(model, cfg, objs, 1)
    except RuntimeError:     # unstable at every candidate down to 50 us
        return 0.05
    return cal.search_timestep * 1e3


def evaluate(params, cs, ex):
    res = np.array(list(ex.map(lambda c: search(*c[:4], params), cs)))
    ref = np.array([c[4] for c in cs])
    return res, np.log(res / ref)


def main():
    maxiter = int(sys.argv[1]) if len(sys.argv) > 1 else 60
    cs = cases()
    ex = ThreadPoolExecutor(max_workers=os.cpu_count() or 8)
    names = ["segment_damping", "segment_damping_power", "segment_armature", "segment_armature_power"]
    # log-parametrised coefficients, linear powers
    def unpack(x):
        return {"segment_damping": float(np.exp(x[0])), "segment_damping_power": float(x[1]),
                "segment_armature": float(np.exp(x[2])), "segment_armature_power": float(x[3])}
    hist = []

    def f(x):
        params = unpack(x)
        _, lr = evaluate(params, cs, ex)
        obj = float(np.sqrt(np.mean(lr ** 2)))
        hist.append((obj, float(np.abs(lr).max()), params))
        print(f"{len(hist):3d} rms {obj:.4f} max {np.abs(lr).max():.4f} {params}", flush=True)
        return obj
    from scipy.optimize import minimize
    x0 = np.array([np.log(0.05), 1.0, np.log(1e-6), 1.0])
    t = time.time()
    r = minimize(f, x0, method="Nelder-Mead", options={"maxiter": maxiter, "xatol": 1e-3, "fatol": 1e-4})
    best = unpack(r.x)
    res, lr = evaluate(best, cs, ex)
    print("best", best, "rms", np.sqrt(np.mean(lr ** 2)), "max", np.abs(lr).max(), f"{time.time() - t:.0f} s")
    for c, v, l in zip(cs, res, lr):
        print(f"N={c[0]} t={c[1]} w={c[2]} s={c[3]:>5}: ref {c[4]:.3f} engine {v:.3f} ({np.expm1(l):+.1%})")


if __name__ == "__main__":
    main()
