#!/usr/bin/env python3
"""Batched env-step throughput of the MI355X gripper hot path (BASELINE.json metric).

A "step" is one MjEnv.step-equivalent for every env of the batch (MjEnv.py:2170-2220):
set actions (MjClass::set_continous_action x n_actions), action_step() = S = 63 physics
substeps + sense_gripper_state + update_env, then observation, done and reward
(mjclass.cpp:1483-1508, 1632-1959, 3000-3049), followed by the episode-boundary
bookkeeping (return hand-off, reset + respawn of done/truncated envs, MjEnv.py:616-637).
Everything runs on the device; inputs (pre-drawn random actions, a spawn table) are
resident in HBM before the timed region starts.

Workload = BASELINE.json configs[2] ("C3"): 4096 envs per GPU, 20-object synthetic
set6-like mixed set, randomised spawn, random actions U[-1,1]^4.  N GPUs run N x 4096
envs sharded by env id (weak scaling); the only collective is an RCCL all-gather of
the per-env episode returns each step.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Rank 0 prints one JSON line.  `roofline.achieved` = algorithmic bytes per launch of
the fused step kernel (SURVEY.md 8d per-env-substep working set, constants frozen from
the model below) / the kernel's average duration from HIP events recorded on the
stream it is launched on.  `cpu_baseline` times the fp64 CPU oracle (a restatement of
the reference path; the reference bind.so needs MuJoCo 2.1.5 and cannot be built).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "gripper-mujoco_amd"))

METRIC = "env-steps/sec (batched rollout) at 4096 envs; obs max-rel-err vs C++ ref"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md "HBM")
NCON_NOMINAL = 12              # SURVEY.md 8d nominal contacts per env-substep


def algorithmic_bytes_per_substep(model, ncon: int = NCON_NOMINAL) -> dict:
    """fp32 working set crossing the north-star stage boundaries per
    env-substep, with this model's frozen sizes."""
    nefc = model.nlock + 4 * ncon
    parts = {
        "state_in_out": 2 * (model.nq + model.nv) * 4,
        "ctrl": 8 * 4,
        "fk_poses": (model.nbody * 16 + model.ngeom * 12) * 4,
        "cinert_cdof": (model.nbody * 10 + model.nv * 6) * 4,
        "mass_ldl": 2 * model.nM * 4,
        "force_vectors": 4 * model.nv * 4,
        "contacts": ncon * 60,
        "constraints": nefc * 68,
        "qacc_qfrc_constraint": 2 * model.nv * 4,
        "cfrc_ext": model.nbody * 24,
    }
    return {"bytes": sum(parts.values()), "ncon": ncon, "nefc": nefc, "parts": parts}


def mjenv_spawn_params(gmx):
    """default_spawn_params as MjEnv._spawn_object sets them (MjEnv.py:1211-1215):
    +-10 mm xy on the 2 mm grid, +-pi/2 rotation on the pi/30 grid; resets place the
    object with spawn_into_scene on the device (3 tries, then the spawn-table pose)."""
    import math
    p = gmx.default_spawn_params()
    p.xrange = p.yrange = 10e-3
    p.rotrange = math.pi / 2.0
    return p


def load_traffic(n_envs: int):
    """HBM bytes per launch of gm_step_kernel from the committed rocprofv3 PMC pass
    (profiles/*pmc_traffic.json, FETCH_SIZE x2 + WRITE_SIZE per the gfx950 guide)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if int(d.get("n_envs", -1)) == n_envs:
            return float(d["bytes_per_launch"]), d.get("source")
    except (OSError, ValueError, KeyError):
        pass
    return None, None


def _rel_abs(obs, ref):
    import numpy as np
    ref = np.asarray(ref, dtype=np.float64)
    d = np.abs(np.asarray(obs, dtype=np.float64) - ref)
    big = np.abs(ref) >= 1e-3
    rel = float((d[big] / np.abs(ref[big])).max()) if big.any() else 0.0
    ab = float(d[~big].max()) if (~big).any() else 0.0
    return rel, ab


def obs_parity(gmx):
    """obs max-rel-err of the GPU path vs the fp64 oracle (noise off; SURVEY.md 8d: rel
    over |ref| >= 1e-3, abs elsewhere) on two probes: a 20-step contact-free rollout of
    4 envs, and the first env-step of 3 envs closing on an object (contact-rich, from the
    identical reset state; longer contact-rich rollouts separate chaotically)."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    s = gmx.canonical_settings(noise=False, seed=5)
    out = {}
    # contact-free rollout
    env = gmx.BatchedGripperEnv(4, object_set="set1_synthetic", settings=s, seed=5)
    xs = np.array([0.055, 0.058, 0.06, 0.062])
    sp = env.make_spawn(x=xs, y=xs, idx=0)
    env.reset(spawn=sp)
    orc = []
    for e in range(4):
        o = oracle_lib.OracleEnv(env.model, env.cfg, env.objects, e)
        o.reset(sp[e])
        orc.append(o)
    rng = np.random.default_rng(1234)
    rel = ab = 0.0
    for _ in range(20):
        a = rng.uniform(-1, 1, size=(4, env.n_actions)).astype(np.float32)
        obs, _, _, _ = env.step(a)
        for e in range(4):
            r, b = _rel_abs(obs[e], orc[e].step(a[e])[0])
            rel, ab = max(rel, r), max(ab, b)
    env.close()
    out["contact_free_rollout"] = {"max_rel": rel, "max_abs_small": ab, "envs": 4, "steps": 20}
    # contact-rich first step
    env = gmx.BatchedGripperEnv(3, object_set="set1_synthetic", settings=s, seed=5)
    sp = env.make_spawn(x=0.0, y=0.0)
    env.reset(spawn=sp)
    a = np.array([[1.0, 0.0, 1.0, 0.5]] * 3, dtype=np.float32)
    obs, _, _, _ = env.step(a)
    rel = ab = 0.0
    for e in range(3):
        o = oracle_lib.OracleEnv(env.model, env.cfg, env.objects, e)
        o.reset(sp[e])
        r, b = _rel_abs(obs[e], o.step(a[e])[0])
        rel, ab = max(rel, r), max(ab, b)
    env.close()
    out["contact_rich_first_step"] = {"max_rel": rel, "max_abs_small": ab, "envs": 3, "steps": 1}
    return out


def cpu_baseline(gmx, n_envs: int, n_steps: int, n_threads: int):
    """The fp64 CPU oracle on the host cores: envs are independent (one env
    per thread, as the reference runs one env per process), spread over n_threads."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    s = gmx.canonical_settings(seed=1234)
    model = gmx.ModelBlob()
    cfg = gmx.ConfigBlob(s, model)
    objs = gmx.make_object_set("set6_synthetic", 1234)
    t = time.time()
    v = oracle_lib.bench(model, cfg, objs, n_envs, n_steps, seed=1234, n_threads=n_threads)
    return {"value": round(v, 2), "unit": "env-steps/s", "cores": n_threads, "kind": "port",
            "sample": f"fp64 C oracle (oracle/oracle.c, gcc -O2 -mavx), {n_threads} thread(s), {n_envs} envs x "
                      f"{n_steps} env-steps of the C3 workload (set6_synthetic, random actions, "
                      f"resets at done), {time.time() - t:.1f} s wall"}


def policy_rollout(gmx, torch, dev, stream, n: int, steps: int, seed: int, env_offset: int):
    """C5: the C3 workload with discrete actions chosen on the device by the
    DQN policy (VariableNetwork [63,150,100,50,8], eps-greedy) -- policy, env-step and
    auto-reset with no host round trip.  Returns env-steps/s and the policy kernel's
    share of the step (HIP events on the shared stream)."""
    s = gmx.canonical_settings(seed=seed)
    s.continous_actions = 0
    env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=s, seed=seed, env_offset=env_offset,
                                device=dev.index)
    env.set_stream(stream.cuda_stream)
    env.set_scene_spawn(mjenv_spawn_params(gmx), max_tries=3)
    spawn = env.make_spawn()
    env.reset(spawn=spawn)
    spawn_ptr = env.upload_spawn(spawn)
    pol = gmx.DevicePolicy(env, seed=seed)
    returns = torch.full((n,), float("nan"), device=dev)
    evp = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]

    def one(t, k):
        if k is not None:
            evp[k][0].record(stream)
        pol.act(eps=gmx.eps_threshold(t), seed=seed, decision=t)
        if k is not None:
            evp[k][1].record(stream)
        env.lib.gm_step(env.ctx)
        env.autoreset_device(spawn_ptr, returns.data_ptr())

    one(0, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        one(1 + k, k)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    pol_ms = sum(a.elapsed_time(b) for a, b in evp) / steps
    out = {"value": round(n * steps / el, 1), "unit": "env-steps/s", "envs": n, "steps": steps,
           "ms_per_step": round(el / steps * 1e3, 3), "policy_select_ms": round(pol_ms, 4),
           "network": pol.sizes, "dtype": "f32 policy (MFMA) + f64 env"}
    pol.close()
    env.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--cpu-envs", type=int, default=40, help="envs per CPU thread in the baseline")
    ap.add_argument("--cpu-steps", type=int, default=250)
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host threads for the CPU baseline (the GPU box's CPU share is 16)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-policy", action="store_true", help="skip the C5 on-device DQN rollout line item")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N>1 with torch.distributed.run",
              file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    import gmx
    from gmx.shard import shard_range, gather_returns, max_over_ranks
    settings = gmx.canonical_settings(seed=args.seed)
    n = args.envs
    first_env, _ = shard_range(rank, world, n)
    env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=settings, seed=args.seed,
                                env_offset=first_env, device=local_rank)
    stream = torch.cuda.Stream(dev)          # a real (non-null) stream shared by torch and the ctx
    torch.cuda.set_stream(stream)
    env.set_stream(stream.cuda_stream)
    S = env.cfg.sim_steps_per_action
    env.set_scene_spawn(mjenv_spawn_params(gmx), max_tries=3)
    spawn = env.make_spawn()
    env.reset(spawn=spawn)
    spawn_ptr = env.upload_spawn(spawn)

    K, W = args.steps, args.warmup
    g = torch.Generator(device=dev)
    g.manual_seed(args.seed + 7919 * rank)
    actions = torch.rand((W + K, n, env.n_actions), generator=g, device=dev) * 2 - 1
    returns = torch.full((n,), float("nan"), device=dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
    episodes = torch.zeros((), device=dev, dtype=torch.int64)

    def one_step(i, timed):
        env.lib.gm_set_action(env.ctx, actions[i].data_ptr(), 1)
        if timed is not None:
            ev[timed][0].record(stream)
        env.lib.gm_step(env.ctx)
        if timed is not None:
            ev[timed][1].record(stream)
        env.autoreset_device(spawn_ptr, returns.data_ptr())
        episodes.add_(torch.isfinite(gather_returns(returns, world)).sum())

    for i in range(W):
        one_step(i, None)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K):
        one_step(W + k, k)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, dev)

    kern_ms = [a.elapsed_time(b) for a, b in ev]
    kern_avg_s = sum(kern_ms) / len(kern_ms) / 1e3
    finite = bool(torch.isfinite(torch.as_tensor(env.observation())).all())
    overflow = int(env.overflow().sum())

    if rank == 0:
        B = algorithmic_bytes_per_substep(env.model)
        bytes_per_launch = n * S * B["bytes"]
        achieved = bytes_per_launch / kern_avg_s / 1e9
        traffic, traffic_src = load_traffic(n)
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "kernel": "gm_step_kernel", "kernel_avg_ms": round(kern_avg_s * 1e3, 4),
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "traffic_source": traffic_src}
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(gmx, args.cpu_envs * args.cpu_threads // 4, args.cpu_steps, args.cpu_threads)
            cpu["single_thread"] = cpu_baseline(gmx, args.cpu_envs, args.cpu_steps, 1)["value"]
        parity = None if args.no_parity else obs_parity(gmx)
        c5 = None if (args.no_policy or world > 1) else policy_rollout(gmx, torch, dev, stream, n, max(3, K // 2), args.seed,
                                                        first_env)
        value = world * n * K / elapsed
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world,
            "steps": K, "warmup": W, "ms_per_step": round(elapsed / K * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic",
            "config": {"workload": "C3: set6_synthetic 20 mixed objects, randomised spawn (spawn_into_scene "
                                   "grid search on the device), random actions U[-1,1]^4, canonical "
                                   "sensor/reward config, device auto-reset",
                       "envs_per_gpu": n, "global_envs": world * n, "substeps_per_env_step": S,
                       "parallelism": f"env-shard x{world}",
                       "B_substep_bytes": B["bytes"], "B_substep_ncon": B["ncon"], "B_substep_nefc": B["nefc"],
                       "model": {"nq": env.model.nq, "nv": env.model.nv, "nbody": env.model.nbody,
                                 "ngeom": env.model.ngeom, "nM": env.model.nM, "nlock": env.model.nlock},
                       "dtype_detail": "f64 dynamics, collision and PGS; f32 sensor windows / observations (as the reference)"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "obs_max_rel_err": parity,
            "c5_device_policy_rollout": c5,
            "episodes_finished": int(episodes.item()),
            "overflow_envs": overflow, "finite": finite,
        }
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
