"""Developer probe: is the C3 rollout launch bounded by its heaviest job?  Runs the bench's
steady-state C3 workload (scripted mix, 4096 envs, 10-env-step gm_rollout launches), takes the
envs that finished last in a timed launch, and re-runs each one's 10-step job ALONE from the
same pre-launch state (a 1-env context with env_offset = the env's id, so its driver draws
and resets are the batch's; GM_DUO=0: one wave, nothing else on the GPU) -- the job's pure
serial time, checked bit-identical against the batch's result.
usage: python tools/heavy_job_probe.py [n_last]"""
import ctypes as C
import hashlib
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'), os.path.join(os.path.dirname(__file__), '..')]
import numpy as np
import torch
import gmx
import bench

k_last = int(sys.argv[1]) if len(sys.argv) > 1 else 6
n, R, seed, MAX_EP = 4096, 10, 1234, 250
settings = gmx.canonical_settings(seed=seed)
env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=settings, seed=seed)
env.set_scene_spawn(bench.mjenv_spawn_params(gmx), max_tries=3)
env.reset()
d_act = env.lib.gm_device_actions(env.ctx)
t_start = gmx.spawn_int(seed, np.arange(n), 0, 99, 0, MAX_EP - 1)
for t in range(MAX_EP):
    m = t_start == t
    if m.any():
        env.lib.gm_reset(env.ctx, np.ascontiguousarray(m.astype(np.uint8)).ctypes.data_as(C.POINTER(C.c_uint8)), None)
    env.lib.gm_scripted_actions(env.ctx, seed, 0.2, d_act, 1)
    env.lib.gm_set_action(env.ctx, d_act, 1)
    env.lib.gm_step(env.ctx)
    env.autoreset_device(0, 0, max_episode_steps=MAX_EP)
for _ in range(2):
    env.rollout(R, 0, seed, 0.2, MAX_EP)
torch.cuda.synchronize()
pre = env.env_states().copy()
env.rollout(R, 0, seed, 0.2, MAX_EP)
torch.cuda.synchronize()
launch = env.last_step_ms()
post = env.env_states().copy()
ends, xcd, ev = env.chunk_timeline()
cs = env.chunk_stats()
print(f"batch launch {launch:.2f} ms (busy {cs['busy']:.3f}); work ends p50 {np.median(ends):.2f} p99 "
      f"{np.percentile(ends, 99):.2f} max {ends.max():.2f} ms", flush=True)
clk, yl = env.job_stats()
busy_ms = clk.astype(np.float64) * 64 / 2.4e6          # shader clocks at 2.4 GHz
life = ev[:, 1] - ev[:, 0]
print(f"jobs: busy (s_memtime at 2.4 GHz) mean {busy_ms.mean():.1f} p99 {np.percentile(busy_ms, 99):.1f} max "
      f"{busy_ms.max():.1f} ms; life mean {life.mean():.1f} ms; yields per job mean {yl.mean():.2f} max {yl.max()}", flush=True)
hv = np.argsort(-busy_ms)[:4]
print("   busiest jobs (env: start/finish ms, busy ms, yields): " + "  ".join(
    f"{int(e)}: {ev[e, 0]:.1f}/{ev[e, 1]:.1f}, {busy_ms[e]:.1f}, {int(yl[e])}" for e in hv), flush=True)
last = np.argsort(ev[:, 1])[-k_last:][::-1]
print("   last jobs (env: start/finish ms, busy ms, yields): " + "  ".join(
    f"{int(e)}: {ev[e, 0]:.1f}/{ev[e, 1]:.1f}, {busy_ms[e]:.1f}, {int(yl[e])}" for e in last), flush=True)
objs = env.objects
os.environ["GM_DUO"] = "0"
for e in list(last) + [int(x) for x in hv[:2]]:
    solo = gmx.BatchedGripperEnv(1, object_set=None, objects=objs, settings=settings, seed=seed, env_offset=int(e),
                                 model_blob=env.model)
    solo.set_scene_spawn(bench.mjenv_spawn_params(gmx), max_tries=3)
    times = []
    for rep in range(3):
        solo.set_env_states(pre[e:e + 1])
        solo.rollout(R, 0, seed, 0.2, MAX_EP)
        torch.cuda.synchronize()
        times.append(solo.last_step_ms())
    same = hashlib.sha1(solo.env_states().tobytes()).hexdigest() == hashlib.sha1(post[e:e + 1].tobytes()).hexdigest()
    print(f"env {int(e)}: in the batch start {ev[e, 0]:.1f} finish {ev[e, 1]:.1f} ms (life {ev[e, 1] - ev[e, 0]:.1f}); "
          f"busy {busy_ms[e]:.1f} ms, {int(yl[e])} yields; alone on one wave {min(times):.1f} ms "
          f"({', '.join(f'{x:.1f}' for x in times)}); identical final state: {same}",
          flush=True)
    solo.close()
env.close()
