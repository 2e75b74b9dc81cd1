"""Developer probe: per-env, per-env-step clocks (whole env-step on one wave) and work
counters of the bench's steady-state C3 workload over T profiled env-steps, saved for the
dispatch-cost predictor study (tools/cost_predictor.py).
usage: python tools/c3_cost_dump.py [envs] [T] [out.npz]"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'), os.path.join(os.path.dirname(__file__), '..')]
import numpy as np
import gmx
import bench

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
T = int(sys.argv[2]) if len(sys.argv) > 2 else 40
out = sys.argv[3] if len(sys.argv) > 3 else "gpurun_out/c3_costs.npz"
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
cyc = np.zeros((T, n)); nefc = np.zeros((T, n)); mpr = np.zeros((T, n)); newton = np.zeros((T, n)); ls = np.zeros((T, n))
for t in range(T):
    ph = drive(True).astype(np.float64)
    cyc[t], nefc[t], mpr[t], newton[t], ls[t] = ph[:, 23], ph[:, env.PH_NEFC], ph[:, env.PH_MPR], ph[:, env.PH_NEWTON], ph[:, env.PH_LS]
    if t % 10 == 0:
        print(f"step {t}", flush=True)
np.savez_compressed(out, cyc=cyc, nefc=nefc, mpr=mpr, newton=newton, ls=ls)
print("saved", out, cyc.shape, flush=True)
