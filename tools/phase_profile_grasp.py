"""Developer probe: per-phase cycle breakdown of the fused env-step kernel on the bench's
own workload (C3 set6_synthetic, scene spawn, steady state after the staggered pre-roll,
scripted grasp mix), as opposed to tools/phase_profile.py's random actions from reset.
usage: python tools/phase_profile_grasp.py [envs] [object_set]  (C2: 256 cylinder)"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'), os.path.join(os.path.dirname(__file__), '..')]
import numpy as np
import gmx
import bench

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
oset = sys.argv[2] if len(sys.argv) > 2 else "set6_synthetic"
seed, MAX_EP = 1234, 250
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
tot = np.zeros(env.N_PHASE)
for t in range(3):
    tot += drive(True).astype(np.float64).mean(axis=0)
tot /= 3
S = 63
TOP = [0, 1, 2, 5, 6, 8, 9, 10]
allc = tot[TOP].sum()
print(f"n={n} {oset} grasp workload: mean cycles per env-step (lane 0) total {allc:.3e}  per substep {allc / S:.3e}")
for k, name in enumerate(env.PHASES):
    if k in (22, 23, 25, 26, 27) or name == "-":
        continue
    if name.startswith("e:"):
        print(f"  {name:18s} {tot[k]:10.0f} cyc/env-step  (= {tot[k] / S:.0f} per substep)")
    else:
        print(f"  {name:18s} {tot[k] / S:10.0f} cyc/substep  {100 * tot[k] / allc:5.1f}%")
print(f"  whole env-step on one wave {tot[23]:.3e} cyc")
print(f"  rows per substep {tot[env.PH_NEFC] / S:.1f}; Newton iterations per solve {tot[env.PH_NEWTON] / S:.3f}; "
      f"line-search evals per solve {tot[env.PH_LS] / S:.3f}; substeps running MPR {tot[env.PH_MPR] / S:.3f}")
