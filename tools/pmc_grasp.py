"""Developer probe: the bench's C3 steady-state workload (set6_synthetic, scene spawn,
staggered pre-roll over the episode, scripted grasp mix) for PMC counter passes; the
analysis takes the last `steps` gm_step_kernel dispatches.
usage: python tools/pmc_grasp.py [envs] [steps] [object_set]"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'), os.path.join(os.path.dirname(__file__), '..')]
import numpy as np
import gmx
import bench

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
oset = sys.argv[3] if len(sys.argv) > 3 else "set6_synthetic"
seed, MAX_EP = 1234, 250
env = gmx.BatchedGripperEnv(n, object_set=oset, settings=gmx.canonical_settings(seed=seed), seed=seed)
env.set_scene_spawn(bench.mjenv_spawn_params(gmx), max_tries=3)
env.reset()
d_act = env.lib.gm_device_actions(env.ctx)
t_start = gmx.spawn_int(seed, np.arange(n), 0, 99, 0, MAX_EP - 1)
for t in range(MAX_EP + steps):
    if t < MAX_EP:
        m = t_start == t
        if m.any():
            env.lib.gm_reset(env.ctx, np.ascontiguousarray(m.astype(np.uint8)).ctypes.data_as(C.POINTER(C.c_uint8)), None)
    env.lib.gm_scripted_actions(env.ctx, seed, 0.2, d_act, 1)
    env.lib.gm_set_action(env.ctx, d_act, 1)
    env.lib.gm_step(env.ctx)
    env.autoreset_device(0, 0, max_episode_steps=MAX_EP)
env.observation()   # (a host read-back: the stream has drained)
print("done")
