"""Developer probe: the C1 line (one env, 200 random-action steps through the mjpy.bind
facade) split into the step kernel's time (HIP events, gm_last_step_ms) and the host
round trip around it.  usage: python tools/c1_probe.py"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd')]
import numpy as np
import gmx
from mjpy.bind import MjClass

acts = np.random.default_rng(1234).uniform(-1, 1, size=(200, 4)).astype(np.float32)
mj = MjClass()
mj.set = gmx.canonical_settings(seed=1234)
mj.object_set_name = "set1_synthetic"
mj.reset()
na = mj.get_n_actions()
env = mj._env
print("dispatch", env.dispatch_info(), flush=True)
for rep in range(2):
    ks = []
    t0 = time.perf_counter()
    for t in range(200):
        for i in range(na):
            mj.set_continous_action(i, float(acts[t, i]))
        mj.action_step()
        mj.get_observation_numpy()
        mj.is_done()
        mj.reward()
        ks.append(env.last_step_ms())
    wall = (time.perf_counter() - t0) / 200 * 1e3
    print(f"rep {rep}: facade {wall:.3f} ms/step, step kernel {np.mean(ks):.3f} ms (min {np.min(ks):.3f}), host {wall - np.mean(ks):.3f} ms",
          flush=True)
    mj.reset()
