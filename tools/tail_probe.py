"""Developer probe: per-env cost spread of the fused env-step kernel and the makespan
of in-order vs cost-sorted dispatch over the resident slots (list scheduling)."""
import sys, os, heapq
sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd')]
import numpy as np
import gmx
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
slots = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
s = gmx.canonical_settings(noise=True, seed=5)
env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=s, seed=5)
env.reset()
rng = np.random.default_rng(0)
for t in range(3):
    env.step(rng.uniform(-1, 1, size=(n, env.n_actions)).astype(np.float32))


def makespan(cost, order):
    h = [0.0] * slots
    for e in order:
        t = heapq.heappop(h)
        heapq.heappush(h, t + cost[e])
    return max(h)


prev = None
for t in range(6):
    a = rng.uniform(-1, 1, size=(n, env.n_actions)).astype(np.float32)
    env.set_action(a)
    ph = env.step_profiled().astype(np.float64)
    env.step(a)
    ms = env.last_step_ms()
    c = ph[:, 23]
    line = (f"step {t}: kernel {ms:.2f} ms  env cycles mean {c.mean():.3e} p10 {np.percentile(c,10):.3e} "
            f"p90 {np.percentile(c,90):.3e} max {c.max():.3e}  ideal(sum/slots) {c.sum()/slots:.3e}  "
            f"in-order {makespan(c, range(n)):.3e}  sorted-oracle {makespan(c, np.argsort(-c)):.3e}")
    if prev is not None:
        line += f"  sorted-by-prev {makespan(c, np.argsort(-prev)):.3e}  corr(prev) {np.corrcoef(prev, c)[0,1]:.3f}"
    print(line, flush=True)
    prev = c
