"""Developer probe: per-env cost spread and dispatch makespan on the bench's own workload
(steady-state C3 batch: staggered episodes, scripted grasp mix, device auto-reset).
Prints, per env-step, the mean / p90 / max env cost (shader clocks on lane 0), the ideal
makespan sum/slots, and the list-scheduling makespan of in-order, previous-cost-sorted
and perfectly sorted dispatch over the resident slots."""
import ctypes as C
import heapq
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'), os.path.join(os.path.dirname(__file__), '..')]
import numpy as np
import gmx

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
slots = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
seed, MAX_EP = 1234, 250
env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=gmx.canonical_settings(seed=seed), seed=seed)
import bench  # noqa: E402  (the bench's spawn parameters)
env.set_scene_spawn(bench.mjenv_spawn_params(gmx), max_tries=3)
env.reset()
d_act = env.lib.gm_device_actions(env.ctx)
t_start = gmx.spawn_int(seed, np.arange(n), 0, 99, 0, MAX_EP - 1)
ret = np.zeros(n, dtype=np.float32)


def drive(profiled=False):
    env.lib.gm_scripted_actions(env.ctx, seed, 0.2, d_act, 1)
    env.lib.gm_set_action(env.ctx, d_act, 1)
    ph = env.step_profiled() if profiled else env.lib.gm_step(env.ctx)
    env.autoreset_device(0, 0, max_episode_steps=MAX_EP)
    return ph


for t in range(MAX_EP):
    m = t_start == t
    if m.any():
        env.lib.gm_reset(env.ctx, np.ascontiguousarray(m.astype(np.uint8)).ctypes.data_as(C.POINTER(C.c_uint8)), None)
    drive()


def makespan(cost, order):
    h = [0.0] * slots
    for e in order:
        heapq.heappush(h, heapq.heappop(h) + cost[e])
    return max(h)


prev = None
dump = []
for t in range(8):
    ph = drive(profiled=True).astype(np.float64)
    dump.append(ph.copy())   # all phase slots
    c, nefc, mpr, nwt = ph[:, 23], ph[:, env.PH_NEFC], ph[:, env.PH_MPR], ph[:, env.PH_NEWTON]
    line = (f"step {t}: env cycles mean {c.mean():.3e} p90 {np.percentile(c, 90):.3e} "
            f"max {c.max():.3e}  ideal {c.sum() / slots:.3e}  in-order {makespan(c, range(n)):.3e}  "
            f"sorted-oracle {makespan(c, np.argsort(-c)):.3e}")
    if prev is not None:
        pc, pn, pm, pw = prev
        X = np.stack([np.ones(n), pn, pm, pw], axis=1)
        beta = np.linalg.lstsq(X, pc, rcond=None)[0]
        pred = X @ beta
        line += (f"  by-prev-cost {makespan(c, np.argsort(-pc)):.3e} (corr {np.corrcoef(pc, c)[0, 1]:.3f})"
                 f"  by-work-model {makespan(c, np.argsort(-pred)):.3e} (corr {np.corrcoef(pred, c)[0, 1]:.3f},"
                 f" beta {beta[0]:.3g} {beta[1]:.3g} {beta[2]:.3g} {beta[3]:.3g})")
    print(line, flush=True)
    # the launch's real timeline (100 MHz constant clock, start / end of every env's wave)
    t0, t1 = ph[:, 25], ph[:, 26]
    base = t0.min()
    t0, t1 = (t0 - base) * 10e-9, (t1 - base) * 10e-9
    span = t1.max()
    busy = (t1 - t0).sum()
    ev = np.concatenate([np.stack([t0, np.ones(n)], 1), np.stack([t1, -np.ones(n)], 1)])
    ev = ev[np.argsort(ev[:, 0], kind="stable")]
    conc = np.cumsum(ev[:, 1])
    dt = np.diff(ev[:, 0], append=span)
    full = dt[conc >= 0.95 * conc.max()].sum()
    print(f"        timeline: span {span * 1e3:.3f} ms, wave-busy {busy / (conc.max() * span):.3f} of "
          f"{int(conc.max())} peak-resident slots x span; >=95% resident for {full * 1e3:.3f} ms; "
          f"shader clock {np.median(c / np.maximum(t1 - t0, 1e-9)) / 1e6:.0f} MHz; "
          f"mean env {np.mean(t1 - t0) * 1e3:.3f} ms, max {np.max(t1 - t0) * 1e3:.3f} ms, "
          f"last start {t0.max() * 1e3:.3f} ms", flush=True)
    prev = (c, nefc, mpr, nwt)

if len(sys.argv) > 3:
    np.save(sys.argv[3], np.stack(dump))   # [step, env, (phases 0-7, total, nefc sum, mpr substeps)]

# the chunked dispatch gm_step runs (the profiled steps above use the one-shot kernel)
for t in range(3):
    drive()
    print("chunked dispatch:", {k: (round(v, 3) if isinstance(v, float) else v) for k, v in env.chunk_stats().items()},
          f"kernel {env.last_step_ms():.3f} ms", flush=True)

# which phases carry the spread: per-phase mean / std over envs (shader clocks per env-step)
ph = drive(profiled=True).astype(np.float64)
tot = ph[:, 23]
hi = tot >= np.percentile(tot, 95)
print("phase spread over envs (mean, std, mean of the 5% costliest envs):")
for k, name in enumerate(env.PHASES):
    print(f"  {name:18s} mean {ph[:, k].mean():10.0f} std {ph[:, k].std():10.0f} top5% {ph[hi, k].mean():10.0f}")
print(f"  {'total':18s} mean {tot.mean():10.0f} std {tot.std():10.0f} top5% {tot[hi].mean():10.0f}")
