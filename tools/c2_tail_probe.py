"""Developer probe: C2's step is its slowest env's step (one env per CU).  Per-env env-step
clocks on the bench's C2 workload (256 envs, one cylinder, scripted grasp mix, steady state)
and what the slowest envs do: Newton points, line-search evaluations, rows, MPR substeps.
usage: python tools/c2_tail_probe.py [envs] [object_set] [steps]"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'), os.path.join(os.path.dirname(__file__), '..')]
import numpy as np
import gmx
import bench

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
oset = sys.argv[2] if len(sys.argv) > 2 else "cylinder"
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
seed, MAX_EP, S = 1234, 250, 63
env = gmx.BatchedGripperEnv(n, object_set=oset, settings=gmx.canonical_settings(seed=seed), seed=seed)
env.set_scene_spawn(bench.mjenv_spawn_params(gmx), max_tries=3)
env.reset()
d_act = env.lib.gm_device_actions(env.ctx)
t_start = gmx.spawn_int(seed, np.arange(n), 0, 99, 0, MAX_EP - 1)


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
print(f"n={n} {oset}: per-env env-step clocks (whole env-step on one wave), {steps} profiled steps", flush=True)
for t in range(steps):
    ph = drive(True).astype(np.float64)
    cyc = ph[:, 23]
    order = np.argsort(cyc)
    newton, ls, nefc, mpr = (ph[:, env.PH_NEWTON], ph[:, env.PH_LS], ph[:, env.PH_NEFC], ph[:, env.PH_MPR])
    top = order[-3:][::-1]
    print(f"step {t}: mean {cyc.mean():.3e} p50 {np.median(cyc):.3e} p90 {np.percentile(cyc, 90):.3e} "
          f"max {cyc.max():.3e} (max/mean {cyc.max() / cyc.mean():.2f}); Newton points per substep mean "
          f"{newton.mean() / S:.2f}, of the 3 slowest " + ", ".join(
              f"[{cyc[i]:.2e} cyc: {newton[i] / S:.2f} pts, {ls[i] / S:.2f} ls, {nefc[i] / S:.1f} rows, "
              f"{mpr[i] / S:.2f} mpr]" for i in top), flush=True)
    # the clocks the slowest env spends per phase against the mean env
    if t == steps - 1:
        i = top[0]
        for k, name in enumerate(env.PHASES[:25]):
            if k in (22, 23) or name.startswith("e:"):
                continue
            print(f"  {name:18s} slowest {ph[i, k] / S:9.0f}  mean {ph[:, k].mean() / S:9.0f} cyc/substep")
