"""Developer A/B probe: the bench's steady-state C3 workload for a given segment count N,
mean kernel time over `steps` env-steps (10) and a digest of the final fp64 env states.  usage: python tools/quick_bench_n.py N [envs] [steps] [object_set]
(object_set "cylinder" with 256 envs is the C2 workload)."""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'), os.path.join(os.path.dirname(__file__), '..')]
import numpy as np
import gmx
import bench

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
oset = sys.argv[4] if len(sys.argv) > 4 else "set6_synthetic"
seed, MAX_EP = 1234, 250
p = gmx.ModelParams()
gmx.load_library().gm_default_model_params(C.byref(p))
p.n_seg = N
p.timestep = 3.187e-3 if N <= 8 else 2.2e-3
if os.environ.get("GM_MJ") is not None:       # 0: the folded actuator scheme (r01-r03 physics)
    p.mujoco_actuators = int(os.environ["GM_MJ"])
    if p.mujoco_actuators == 0:
        p.actuator_armature[1] = 0.0
        p.segment_damping, p.segment_damping_power = 0.24, 1.0
env = gmx.BatchedGripperEnv(n, object_set=oset, settings=gmx.canonical_settings(seed=seed), seed=seed,
                            model_params=p)
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
ms = []
for t in range(steps):
    drive()
    ms.append(env.last_step_ms())
import hashlib  # noqa: E402
st = env.env_states()
digest = hashlib.sha1(np.ascontiguousarray(st).tobytes()).hexdigest()[:12]   # bit-identity across builds
cs = env.chunk_stats() if hasattr(env, "chunk_stats") else {}
print(f"N={N} n={n} {oset} lib={os.environ.get('GM_LIB', 'default')} kernel ms mean {np.mean(ms):.3f} min {np.min(ms):.3f}"
      f" state sha1 {digest} yields {cs.get('yields', '-')} resumes {cs.get('resumes', '-')}"
      f" span {cs.get('span_ms', 0):.3f} fresh-empty {cs.get('fresh_empty_ms', 0):.3f} busy {cs.get('busy', 0):.3f}"
      f" poll {cs.get('poll', 0):.3f}", flush=True)
