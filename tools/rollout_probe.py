"""Developer probe: the bench's steady-state C3 workload stepped (a) per step (driver,
set_action, step, autoreset: 5 launches per env-step) and (b) as gm_rollout launches of R
env-steps; wall ms per env-step for each, plus the chunked queue's busy fraction.
usage: python tools/rollout_probe.py [envs] [R] [launches]"""
import ctypes as C
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'), os.path.join(os.path.dirname(__file__), '..')]
import numpy as np
import torch
import gmx
import bench

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
R = int(sys.argv[2]) if len(sys.argv) > 2 else 10
L = int(sys.argv[3]) if len(sys.argv) > 3 else 2
seed, MAX_EP = 1234, 250
env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=gmx.canonical_settings(seed=seed), seed=seed)
env.set_scene_spawn(bench.mjenv_spawn_params(gmx), max_tries=3)
env.reset()
d_act = env.lib.gm_device_actions(env.ctx)
t_start = gmx.spawn_int(seed, np.arange(n), 0, 99, 0, MAX_EP - 1)


def drive():
    env.lib.gm_scripted_actions(env.ctx, seed, 0.2, d_act, 1)
    env.lib.gm_set_action(env.ctx, d_act, 1)
    env.lib.gm_step(env.ctx)
    env.autoreset_device(0, 0, max_episode_steps=MAX_EP)


for t in range(MAX_EP):
    m = t_start == t
    if m.any():
        env.lib.gm_reset(env.ctx, np.ascontiguousarray(m.astype(np.uint8)).ctypes.data_as(C.POINTER(C.c_uint8)), None)
    drive()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(R * L):
    drive()
torch.cuda.synchronize()
ps = (time.perf_counter() - t0) / (R * L) * 1e3
rec = torch.zeros((R, n, 3), dtype=torch.int32, device="cuda")
env.rollout(R, 0, seed, 0.2, MAX_EP, rec.data_ptr())     # warm (costs in the new job scale)
torch.cuda.synchronize()
t0 = time.perf_counter()
ks = []
for _ in range(L):
    env.rollout(R, 0, seed, 0.2, MAX_EP, rec.data_ptr())
    ks.append(env.last_step_ms())
torch.cuda.synchronize()
ro = (time.perf_counter() - t0) / (R * L) * 1e3
cs = env.chunk_stats()
print(f"n={n} per-step {ps:.3f} ms/step | rollout R={R}: {ro:.3f} ms/step (kernel {np.mean(ks) / R:.3f} ms/step)"
      f" busy {cs['busy']:.3f} poll {cs['poll']:.3f} yields {cs['yields']} span {cs['span_ms']:.2f} ms fresh-empty {cs['fresh_empty_ms']:.2f} ms"
      f" episodes ended {int((rec[:, :, 1] > 0).sum())}", flush=True)
