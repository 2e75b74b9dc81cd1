"""Developer probe: the tail of a gm_rollout launch on the bench's steady-state C3 workload.
Per-workgroup end of work (gm_chunk_timeline) of the timed launch: when each wave ran out of
work for good, against the launch span and the queue's busy fraction.
usage: python tools/tail_timeline.py [envs] [R]"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), '..', 'gripper-mujoco_amd'), os.path.join(os.path.dirname(__file__), '..')]
import numpy as np
import torch
import gmx
import bench

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
R = int(sys.argv[2]) if len(sys.argv) > 2 else 10
seed, MAX_EP = 1234, 250
env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=gmx.canonical_settings(seed=seed), seed=seed)
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
rec = torch.zeros((R, n, 3), dtype=torch.int32, device="cuda")
for it in range(3):
    env.rollout(R, 0, seed, 0.2, MAX_EP, rec.data_ptr())
    torch.cuda.synchronize()
    cs = env.chunk_stats()
    ends, xcd, ev = env.chunk_timeline()
    ex = np.sort(ends)
    span = cs["span_ms"]
    q = np.percentile(ex, [1, 10, 25, 50, 75, 90, 99, 100])
    # wave-time lost to the tail: each workgroup idle from its exit to the last exit
    idle = float((ex[-1] - ex).sum() / (len(ex) * ex[-1]))
    print(f"n={n} R={R} launch {env.last_step_ms():.2f} ms span {span:.2f} busy {cs['busy']:.3f} poll {cs['poll']:.3f} "
          f"yields {cs['yields']} steals {cs['steals']} fresh-empty {cs['fresh_empty_ms']:.2f} ms | work ends (ms) p1/10/25/50/75/90/99/100 "
          + " ".join(f"{x:.2f}" for x in q) + f" | tail idle {idle:.3f}", flush=True)
    # the envs that finished last: when they started, how long they ran, their cost rank
    last = np.argsort(ev[:, 1])[-8:][::-1]
    dur = ev[:, 1] - ev[:, 0]
    rank = np.empty(n, int)
    rank[np.argsort(-dur)] = np.arange(n)
    print("   last envs (start, finish, duration ms; duration rank): " + "  ".join(
        f"{ev[e, 0]:.1f}/{ev[e, 1]:.1f}/{dur[e]:.1f}#{rank[e]}" for e in last), flush=True)
    print(f"   durations: mean {dur.mean():.1f} p90 {np.percentile(dur, 90):.1f} p99 {np.percentile(dur, 99):.1f} max {dur.max():.1f} ms;"
          f" starts after 15 ms: {int((ev[:, 0] > 15).sum())}, of those ending after the p99 work end: "
          f"{int(((ev[:, 0] > 15) & (ev[:, 1] > q[6])).sum())}", flush=True)
    print("   per XCD: work-end median / max (ms) " + "  ".join(
        f"{g}:{np.median(ends[xcd == g]):.1f}/{ends[xcd == g].max():.1f}" for g in range(8) if (xcd == g).any()), flush=True)
