"""Developer probe: the C3 rollout launch's makespan is bounded by its longest jobs (an env's
R env-steps run back to back on one wave).  Per-env clocks summed over R profiled env-steps
of the bench's steady-state C3 workload: the job-cost spread, and what the heaviest jobs do
(Newton points, line-search evaluations, rows, MPR substeps) per phase against the mean.
usage: python tools/c3_jobs_probe.py [envs] [R]"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'), os.path.join(os.path.dirname(__file__), '..')]
import numpy as np
import gmx
import bench

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
R = int(sys.argv[2]) if len(sys.argv) > 2 else 10
seed, MAX_EP, S = 1234, 250, 63
env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=gmx.canonical_settings(seed=seed), seed=seed)
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
acc = None
for t in range(R):
    ph = drive(True).astype(np.float64)
    acc = ph if acc is None else acc + ph
cyc = acc[:, 23]
order = np.argsort(cyc)
q = np.percentile(cyc, [50, 90, 99])
print(f"n={n} R={R}: job clocks mean {cyc.mean():.3e} p50 {q[0]:.3e} p90 {q[1]:.3e} p99 {q[2]:.3e} max {cyc.max():.3e} "
      f"(max/mean {cyc.max() / cyc.mean():.2f}, p99/mean {q[2] / cyc.mean():.2f}); 2 jobs per slot -> mean slot load "
      f"{2 * cyc.mean():.3e}", flush=True)
sub = R * S
for name, idx in (("top 1%", order[-max(1, n // 100):]), ("top 10%", order[-max(1, n // 10):]), ("all", order)):
    print(f"{name:8s}: Newton pts/substep {acc[idx, env.PH_NEWTON].mean() / sub:.3f}, ls {acc[idx, env.PH_LS].mean() / sub:.3f}, "
          f"rows {acc[idx, env.PH_NEFC].mean() / sub:.1f}, mpr {acc[idx, env.PH_MPR].mean() / sub:.3f}", flush=True)
top = order[-max(1, n // 100):]
for k, name in enumerate(env.PHASES[:25]):
    if k in (22, 23) or name.startswith("e:"):
        continue
    print(f"  {name:20s} top1% {acc[top, k].mean() / sub:9.0f}  mean {acc[:, k].mean() / sub:9.0f} cyc/substep", flush=True)
