"""Developer timing probe: one fused env-step launch at several batch sizes."""
import sys, time, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd')]
import numpy as np
import gmx
for n in [int(x) for x in (sys.argv[1:] or ["256", "4096"])]:
    env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", seed=1)
    env.reset()
    rng = np.random.default_rng(0)
    a = rng.uniform(-1, 1, size=(n, env.n_actions)).astype(np.float32)
    env.step(a)
    ts = []
    for k in range(3):
        t = time.time(); env.step(a); ts.append(time.time() - t)
    print(f"n={n} wall/step {min(ts)*1e3:.2f} ms  kernel {env.last_step_ms():.2f} ms  env-steps/s {n/min(ts):.0f}", flush=True)
    print("overflow envs:", int(env.overflow().sum()), "finite:", bool(np.isfinite(env.observation()).all()), flush=True)
    env.close()
