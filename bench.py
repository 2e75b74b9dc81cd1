#!/usr/bin/env python3
"""Batched env-step throughput of the MI355X gripper hot path (BASELINE.json metric).

A "step" is one MjEnv.step-equivalent for every env of the batch (MjEnv.py:2170-2220):
set actions (MjClass::set_continous_action x n_actions), action_step() = S = 63 physics
substeps + sense_gripper_state + update_env, then observation, done and reward
(mjclass.cpp:1483-1508, 1632-1959, 3000-3049), followed by the episode-boundary
bookkeeping (return hand-off, reset + respawn of done/truncated envs, MjEnv.py:616-637).
Everything runs on the device: the actions come from a device driver reading each env's
episode step (gm_scripted_actions), resets draw their object and pose on the device.  The
headline drives R = --rollout env-steps per launch with gm_rollout (the same sequence fused
per env in one persistent launch, bit-identical to the per-step calls); `per_step_api`
reports the same workload through the per-step launches.

Workload = BASELINE.json configs[2] ("C3"): 4096 envs per GPU, 20-object synthetic
set6-like mixed set, randomised spawn (MjEnv._spawn_object: object drawn per episode,
spawn_into_scene grid search), at STEADY STATE: before the timed region
(and independent of --warmup) the batch is pre-rolled untimed so that the envs are spread
uniformly over episode steps 1..250, driven by the benchmark mix (gm_program_actions mode
4): in 1 episode of 4 per env the closed-loop grasp-lift-hold program (close, squeeze, lift,
palm onto the object, hold -- it reaches the reference's successful_grasp on spheres), the
scripted grasp mix (close, squeeze, palm press, lift, with jitter) in the others, so grasp
contacts, lifts, successes, done flags and resets all fall inside the timed window.  N GPUs
run N x 4096 envs sharded by env id (weak scaling); the only collective is an RCCL
all-gather of the per-env episode-end records (return, length, success) of every env-step
(SURVEY.md 8e): a launch of R env-steps is followed by its R per-env-step gathers.

    python bench.py [--gpus N --steps K --warmup W]       (defaults: N 1, K 30, W 2)
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
import numpy as np
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "gripper-mujoco_amd"))

METRIC = "env-steps/sec (batched rollout) at 4096 envs; obs max-rel-err vs C++ ref"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md "HBM")
NCON_NOMINAL = 12              # SURVEY.md 8d nominal contacts per env-substep
MAX_EP = 250                   # baseline yaml env.max_episode_steps
DRIVER_MODE = 4                # gm_program_actions: grasp program in 1 episode of 4, scripted mix otherwise


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
    object with spawn_into_scene on the device (3 tries, then the drawn fallback pose)."""
    import math
    p = gmx.default_spawn_params()
    p.xrange = p.yrange = 10e-3
    p.rotrange = math.pi / 2.0
    return p


def load_traffic(n_envs: int, steps_per_launch: int):
    """HBM bytes per launch of gm_step_kernel from the committed rocprofv3 PMC passes
    (profiles/pmc_traffic.json, FETCH_SIZE x2 + WRITE_SIZE per the gfx950 guide), for the
    same batch and the same env-steps per launch as this run's timed launches."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if int(d.get("n_envs", -1)) == n_envs and int(d.get("env_steps_per_launch", 1)) == steps_per_launch:
            return float(d["bytes_per_launch"]), d.get("source")
    except (OSError, ValueError, KeyError):
        pass
    return None, None


FP64_VECTOR_PEAK_TFS = 78.6    # half the FP32 vector peak (157.3 TF, MI355X_MICROARCH.md); not in the guide


def load_compute(n_envs: int, substeps: int, steps_per_launch: int, launch_s: float):
    """The bound that applies to the step kernel (VALU issue / dependent latency, not HBM):
    fp64 VALU work per env-substep and lane utilisation from the committed rocprofv3 SQ
    counter pass of the same workload (profiles/pmc_sq_c3.json), and the fp64 rate they give
    at this run's launch time."""
    path = os.path.join(REPO, "profiles", "pmc_sq_c3.json")
    try:
        with open(path) as f:
            d = json.load(f)
        pe = d["per_env_substep"]
        util = float(d["valu_lane_utilisation"])
    except (OSError, ValueError, KeyError):
        return None
    fma, add, mul = pe["SQ_INSTS_VALU_FMA_F64"], pe["SQ_INSTS_VALU_ADD_F64"], pe["SQ_INSTS_VALU_MUL_F64"]
    flop_substep = (2 * fma + add + mul) * 64 * util          # active lanes per wave instruction
    flop_launch = flop_substep * n_envs * substeps * steps_per_launch
    rate = flop_launch / launch_s / 1e12
    return {"bound": "fp64 VALU issue / dependent latency (2 waves per SIMD, LDS-resident working set)",
            "valu_insts_per_env_substep": pe["SQ_INSTS_VALU"],
            "fp64_fma_add_mul_per_env_substep": [fma, add, mul],
            "salu_insts_per_env_substep": pe.get("SQ_INSTS_SALU"),
            "lds_insts_per_env_substep": pe.get("SQ_INSTS_LDS"),
            "valu_lane_utilisation": util,
            "wave_cycle_fractions": d.get("wave_cycle_fractions"),
            "lds_bank_conflict_cycles_per_launch": d.get("per_launch", {}).get("SQ_LDS_BANK_CONFLICT"),
            "fp64_flop_per_launch": flop_launch, "achieved_fp64_tflops": round(rate, 3),
            "fp64_vector_peak_tflops": FP64_VECTOR_PEAK_TFS, "frac": round(rate / FP64_VECTOR_PEAK_TFS, 4),
            "source": d.get("source", path)}


def obs_parity(gmx, env, seed: int):
    """obs max-rel-err of the GPU path vs the fp64 oracle ON THE BENCHMARK'S OWN STATES
    (rel over |ref| >= 1e-3, abs elsewhere): the whole batch's fp64 state
    after the timed window is handed to the oracle (gm_get_env_states -> or_import_state),
    and both run the next env-step of the benchmark mix (the device's driver actions).  Done
    flags and event rows are compared bit for bit."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    rec = env.env_states()
    a = env.program_actions(seed, 0.2, 4)
    env.set_action(a)
    env.action_step()
    obs = env.observation()
    rew, done = env.reward_done()
    after = env.env_states()
    t = time.time()
    obs_o, rew_o, done_o, after_o = oracle_lib.batch_step(env.model, env.cfg, env.objects, rec, actions=a)
    ref = obs_o.astype(np.float64)
    d = np.abs(obs.astype(np.float64) - ref)
    big = np.abs(ref) >= 1e-3
    rel = np.where(big, d / np.where(big, np.abs(ref), 1.0), 0.0).max(axis=1)
    ab = np.where(big, 0.0, d).max(axis=1)
    dv, ov = gmx.env_state_view(after), gmx.env_state_view(after_o)
    # where the worst relative error sits (env, observation index, values)
    relm = np.where(big, d / np.where(big, np.abs(ref), 1.0), 0.0)
    we, wi = np.unravel_index(int(np.argmax(relm)), relm.shape)
    worst = {"env": int(we), "obs_index": int(wi), "ref": float(ref[we, wi]), "gpu": float(obs[we, wi]),
             "abs_diff": float(d[we, wi]),
             "env_qpos_max_abs_diff": float(np.abs(dv["qpos"][we] - ov["qpos"][we]).max())}
    return {"max_rel": float(rel.max()), "max_abs_small": float(ab.max()), "worst": worst,
            "envs_over_1e-4": int(((rel > 1e-4) | (ab > 1e-4)).sum()), "envs": int(env.n_envs),
            "p99_rel": float(np.percentile(rel, 99)),
            "done_mismatch": int((done.astype(np.uint8) != done_o).sum()),
            "event_row_mismatch_envs": int(((dv["bev_row"] != ov["bev_row"]).any(axis=1) |
                                            (dv["lev_row"] != ov["lev_row"]).any(axis=1)).sum()),
            "reward_max_abs_diff": float(np.abs(rew - rew_o).max()),
            "states": "the benchmark batch after the timed window (steady state, noise on), one env-step",
            "oracle_s": round(time.time() - t, 2)}


def steady_env(gmx, torch, dev, stream, n: int, object_set: str, seed: int, env_offset: int, mode: int = 0):
    """A batch at steady state: env e (global id) starts its episode at pre-roll step t_e, so
    after MAX_EP untimed per-step drives the batch covers episode steps 1..MAX_EP uniformly.
    Returns (env, per-step drive)."""
    import ctypes
    s = gmx.canonical_settings(seed=seed)
    env = gmx.BatchedGripperEnv(n, object_set=object_set, settings=s, seed=seed, env_offset=env_offset,
                                device=dev.index)
    env.set_stream(stream.cuda_stream)
    env.set_scene_spawn(mjenv_spawn_params(gmx), max_tries=3)
    env.reset()
    d_act = env.lib.gm_device_actions(env.ctx)

    def drive():
        if mode == 0:
            env.lib.gm_scripted_actions(env.ctx, seed, 0.2, d_act, 1)
        else:
            env.lib.gm_random_actions(env.ctx, seed, d_act, 1)
        env.lib.gm_set_action(env.ctx, d_act, 1)
        env.lib.gm_step(env.ctx)
        env.autoreset_device(0, None, max_episode_steps=MAX_EP)

    t_start = gmx.spawn_int(seed, env_offset + np.arange(n), 0, 99, 0, MAX_EP - 1)
    for t in range(MAX_EP):
        m = (t_start == t)
        if m.any():
            env.lib.gm_reset(env.ctx, np.ascontiguousarray(m.astype(np.uint8)).ctypes.data_as(
                ctypes.POINTER(ctypes.c_uint8)), None)
        drive()
    return env, drive


def time_both(env, drive, torch, steps: int, R: int, seed: int, mode: int):
    """Wall ms per env-step of the same workload driven per step (5 launches per env-step)
    and as gm_rollout launches of R env-steps."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        drive()
    torch.cuda.synchronize()
    per_step = (time.perf_counter() - t0) / steps
    out = {"per_step_api_ms": round(per_step * 1e3, 3)}
    if R > 0:
        n_l = max(1, steps // R)
        env.rollout(R, mode, seed, 0.2, MAX_EP)          # untimed: the dispatch costs in the job's scale
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n_l):
            env.rollout(R, mode, seed, 0.2, MAX_EP)
        torch.cuda.synchronize()
        out["rollout_ms"] = round((time.perf_counter() - t0) / (n_l * R) * 1e3, 3)
        out["rollout_steps_per_launch"] = R
    return out


def c2_line(gmx, torch, dev, stream, steps: int, seed: int, env_offset: int, R: int):
    """C2 (BASELINE.json configs[1]): 256 envs, one cylinder (r 20 mm, h 60 mm), the same
    steady-state scripted workload as the headline, per-step API and rollout launches."""
    n = 256
    env, drive = steady_env(gmx, torch, dev, stream, n, "cylinder", seed, env_offset)
    t = time_both(env, drive, torch, steps, R, seed, 0)
    env.close()
    ms = t.get("rollout_ms", t["per_step_api_ms"])
    return {"value": round(n / ms * 1e3, 1), "unit": "env-steps/s", "envs": n, "steps": steps, "ms_per_step": ms,
            **t, "workload": "C2: 256 envs, one cylinder, steady-state scripted grasp mix"}


def c3_random_line(gmx, torch, dev, stream, steps: int, seed: int, env_offset: int, n: int, R: int):
    """C3 with synthetic random actions (BASELINE.json north_star: "throughput on synthetic
    random-action rollouts"): every env draws U[-1,1)^4 each env-step on the device
    (gm_random_actions: a counter-based hash of seed 1234 -- TrainDQN.profile's seed,
    TrainDQN.py:2520 -- env id, episode and step); same set6 objects, scene spawn, auto-reset
    and steady-state pre-roll as the scripted headline."""
    env, drive = steady_env(gmx, torch, dev, stream, n, "set6_synthetic", seed, env_offset, mode=1)
    t = time_both(env, drive, torch, steps, R, seed, 1)
    caps = int(gmx.env_state_view(env.env_states())["newton_caps"].sum())
    env.close()
    ms = t.get("rollout_ms", t["per_step_api_ms"])
    return {"value": round(n / ms * 1e3, 1), "unit": "env-steps/s", "envs": n, "steps": steps, "ms_per_step": ms,
            **t, "newton_cap_hits": caps,
            "workload": "C3 with random actions U[-1,1)^4 (device counter-based draws, seed 1234), set6_synthetic, "
                        "scene spawn, auto-reset, steady state after a staggered pre-roll"}


def c3_scripted_line(gmx, torch, dev, stream, steps: int, seed: int, env_offset: int, n: int, R: int):
    """C3 driven by the scripted grasp mix alone (mode 0: close / squeeze / palm / lift with
    jitter in every episode) -- the r05 headline's workload, reported beside the headline so
    the two rounds compare like with like: the r06 headline's mix (mode 4) adds the grasp
    program's lifted, multi-contact holds (more constraint rows per substep)."""
    env, drive = steady_env(gmx, torch, dev, stream, n, "set6_synthetic", seed, env_offset, mode=0)
    t = time_both(env, drive, torch, steps, R, seed, 0)
    env.close()
    ms = t.get("rollout_ms", t["per_step_api_ms"])
    return {"value": round(n / ms * 1e3, 1), "unit": "env-steps/s", "envs": n, "steps": steps, "ms_per_step": ms,
            **t, "workload": "C3 with the scripted grasp mix only (the r05 headline's workload), set6_synthetic, "
                             "scene spawn, auto-reset, steady state after a staggered pre-roll"}


def c1_line(gmx, seed: int, n_steps: int = 200):
    """C1 (BASELINE.json configs[0]): 1 env, one 200-step random-action episode, actions
    U[-1,1]^4 from np.random.default_rng(1234) (TrainDQN.py:2520).  Device: the mjpy.bind
    facade in MjEnv.step's call order (set_continous_action per index, action_step,
    get_observation_numpy, is_done, reward; MjEnv.py:585-637); CPU: the fp64 oracle on one
    core, the same actions from the same reset.  set1_nocuboid_525 is absent, so the
    synthetic set1 (box, cylinder, sphere) stands in."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    from mjpy.bind import MjClass
    acts = np.random.default_rng(1234).uniform(-1, 1, size=(n_steps, 4)).astype(np.float32)
    mj = MjClass()
    mj.set = gmx.canonical_settings(seed=seed)
    mj.object_set_name = "set1_synthetic"
    mj.reset()
    na = mj.get_n_actions()
    env = mj._env
    o = oracle_lib.OracleEnv(env.model, env.cfg, env.objects, env_id=0)
    sp = gmx.Spawn()
    sp.object_index, sp.x, sp.y, sp.zrot = 0, 0.0, 0.0, 0.0
    o.reset(sp)
    obs_d = []
    t0 = time.perf_counter()
    for t in range(n_steps):
        for i in range(na):
            mj.set_continous_action(i, float(acts[t, i]))
        mj.action_step()
        obs_d.append(mj.get_observation_numpy())
        mj.is_done()
        mj.reward()
    dev_s = time.perf_counter() - t0
    obs_o = []
    t0 = time.perf_counter()
    for t in range(n_steps):
        ob, _, _ = o.step(acts[t, :na])
        obs_o.append(ob)
    cpu_s = time.perf_counter() - t0
    a = np.asarray(obs_d, dtype=np.float64)
    b = np.asarray(obs_o, dtype=np.float64)
    d = np.abs(a - b)
    big = np.abs(b) >= 1e-3
    rel = float((d[big] / np.abs(b[big])).max(initial=0.0))
    mj._drop()
    return {"device": {"value": round(n_steps / dev_s, 1), "unit": "env-steps/s", "ms_per_step": round(dev_s / n_steps * 1e3, 3),
                       "path": "mjpy.bind.MjClass facade (one env, host round trip per call, as MjEnv drives it)"},
            "cpu_oracle_1_core": {"value": round(n_steps / cpu_s, 1), "unit": "env-steps/s", "cores": 1, "kind": "port"},
            "steps": n_steps, "actions": "np.random.default_rng(1234).uniform(-1, 1, (200, 4))",
            "object_set": "set1_synthetic",
            "obs_max_rel_err_over_episode": rel,
            "obs_max_abs_err_small_over_episode": float(np.where(big, 0.0, d).max(initial=0.0))}


def host_cpu_quota():
    """CPUs this process may use: its affinity mask and the cgroup v2 CPU quota (cpu.max)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return aff, quota


def host_cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(gmx, n_envs: int, n_steps: int, n_threads: int):
    """The fp64 CPU oracle on the host cores: envs are independent (one env
    per thread, as the reference runs one env per process), spread over n_threads; the
    same workload as the GPU line (the benchmark mix, device-identical spawn draws and
    driver decisions, resets at done / 250 steps)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_lib
    s = gmx.canonical_settings(seed=1234)
    model = gmx.ModelBlob()
    cfg = gmx.ConfigBlob(s, model)
    objs = gmx.make_object_set("set6_synthetic", 1234)
    t = time.time()
    v = oracle_lib.bench(model, cfg, objs, n_envs, n_steps, seed=1234, n_threads=n_threads, scripted=True)
    aff, quota = host_cpu_quota()
    return {"value": round(v, 2), "unit": "env-steps/s", "cores": n_threads, "kind": "port",
            "cpu_model": host_cpu_model(), "host_cpus_visible": os.cpu_count(),
            "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "cores_note": "the GPU box gives a 1-GPU job a share of 16 host CPUs (OMP_NUM_THREADS / MAX_JOBS are "
                          "16 there and worker pools must stay within it); the other visible CPUs belong to "
                          "other jobs, so 16 threads is every core this job may use",
            "sample": f"fp64 C oracle (oracle/oracle.c, gcc -O2 -mavx), {n_threads} thread(s), {n_envs} envs x "
                      f"{n_steps} env-steps of the C3 workload (set6_synthetic, the benchmark mix: grasp program / "
                      f"scripted grasp mix, resets at "
                      f"done / 250 steps), {time.time() - t:.1f} s wall"}


def policy_rollout(gmx, torch, dev, stream, n: int, steps: int, seed: int, env_offset: int, R: int = 10):
    """C5: the C3 workload with discrete actions chosen on the device by the
    DQN policy (VariableNetwork [63,150,100,50,8], eps-greedy) -- policy, env-step and
    auto-reset with no host round trip.  Returns env-steps/s and the policy kernel's
    share of the step (HIP events on the shared stream), driven per step (gm_policy_act,
    gm_step, gm_autoreset_episodes) and fused into gm_policy_rollout launches of R env-steps
    (each env's wave selects its own action; bit for bit the per-step sequence)."""
    s = gmx.canonical_settings(seed=seed)
    s.continous_actions = 0
    env = gmx.BatchedGripperEnv(n, object_set="set6_synthetic", settings=s, seed=seed, env_offset=env_offset,
                                device=dev.index)
    env.set_stream(stream.cuda_stream)
    env.set_scene_spawn(mjenv_spawn_params(gmx), max_tries=3)
    env.reset()
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
        env.autoreset_device(0, returns.data_ptr())

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
    if R > 0:
        t = 1 + steps
        pol.rollout([gmx.eps_threshold(t + i) for i in range(R)], seed=seed, decision0=t)   # untimed: costs
        t += R
        n_l = 2
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n_l):
            pol.rollout([gmx.eps_threshold(t + i) for i in range(R)], seed=seed, decision0=t)
            t += R
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out["fused_rollout"] = {"value": round(n * n_l * R / el, 1), "ms_per_step": round(el / (n_l * R) * 1e3, 3),
                                "steps_per_launch": R, "launches": n_l}
    pol.close()
    env.close()
    return out


def measure(drive, episodes, K: int, W: int, world: int, dev, sync):
    """The contract's timed region, independent of what steps the envs (the device here,
    the oracle in tests/test_distributed.py): W untimed warmup drives, then EXACTLY K
    drives bracketed by sync + barrier + sync on both sides; the wall time is the MAX over
    ranks.  Every env-step's episode-end records (return, length, success per env:
    gm_episode_end) are all-gathered -- the one collective, SURVEY.md 8e, once per env-step
    also when a drive runs R env-steps in one launch -- and the finished episodes, their
    successes and their lengths summed over the whole job.  drive(k) takes the timed index k
    (None when untimed); `episodes` is the [R, n, 3] (or [n, 3]) int32 record buffer the
    drive's auto-reset writes (length 0 where an env's episode did not end)."""
    import torch
    import torch.distributed as dist
    from gmx.shard import gather_episodes, max_over_ranks, unpack_episodes
    tally = torch.zeros(3, device=dev, dtype=torch.int64)   # episodes, successes, length sum

    recs = episodes if episodes.dim() == 3 else episodes.unsqueeze(0)

    def step(k=None):
        drive(k)
        for r in range(recs.shape[0]):          # one gather per env-step of the drive
            _, length, success = unpack_episodes(gather_episodes(recs[r], world))
            tally[0] += (length > 0).sum()
            tally[1] += success.sum()
            tally[2] += length.sum()

    # warmup counts episodes too, so every kernel the timed loop launches (incl. torch's
    # reductions for the tally) is loaded before the clock starts
    for _ in range(max(W, 1)):
        step()
    tally.zero_()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(K):
        step(k)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    t = [int(x) for x in tally.tolist()]
    return max_over_ranks(elapsed, dev), {"episodes": t[0], "successes": t[1], "length_sum": t[2]}


def headline(world: int, n: int, K: int, W: int, elapsed: float, ep: dict) -> dict:
    """The contract fields of rank 0's JSON line: value = env-steps of ALL ranks / the
    slowest rank's wall time (weak scaling: n envs per rank)."""
    return {"metric": METRIC, "value": round(world * n * K / elapsed, 1), "unit": "env-steps/s", "n_gpus": world,
            "steps": K, "warmup": W, "ms_per_step": round(elapsed / K * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f64", "data": "synthetic",
            "config": {"envs_per_gpu": n, "global_envs": world * n, "parallelism": f"env-shard x{world}"},
            "episodes_finished": ep["episodes"],
            # from the all-gathered episode-end records (gm_episode_end: return, length, success)
            "episode_successes": ep["successes"],
            "mean_episode_length": round(ep["length_sum"] / ep["episodes"], 2) if ep["episodes"] else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
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
    ap.add_argument("--no-c2", action="store_true", help="skip the C2 (256 envs, one cylinder) line item")
    ap.add_argument("--no-random", action="store_true", help="skip the C3 random-action line item")
    ap.add_argument("--no-scripted", action="store_true",
                    help="skip the C3 scripted-mix-only line item (the r05 headline's workload)")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 (1 env, 200 random steps) line item")
    ap.add_argument("--no-preroll", dest="preroll", action="store_false",
                    help="skip the steady-state pre-roll (profiling runs only; the headline needs it)")
    ap.add_argument("--rollout", type=int, default=10,
                    help="env-steps per gm_rollout launch for the headline (0: the per-step API's launches)")
    ap.add_argument("--c2-rollout", type=int, default=30,
                    help="env-steps per gm_rollout launch for the C2 line (its 256 envs: a launch lasts as long as "
                         "its slowest env's job, so longer jobs average each env's heavy and light env-steps; "
                         "profiles/r06_bench_window.txt)")
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
    from gmx.shard import shard_range
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
    env.reset()
    import math
    K, W = args.steps, args.warmup
    # the headline drives R env-steps per launch (gm_rollout: driver actions, env-step and
    # auto-reset fused per env in one persistent launch); R divides K so exactly K are timed
    R = math.gcd(K, args.rollout) if args.rollout > 0 else 1
    rollout = args.rollout > 0
    n_drives, w_drives = K // R, -(-W // R)
    episodes = torch.zeros((R, n, 3), dtype=torch.int32, device=dev)   # gm_episode_end [R][n]
    d_act = env.lib.gm_device_actions(env.ctx)

    def drive_ps(timed=None, rec=None):
        """one MjEnv.step-equivalent for the whole batch through the per-step API, all on the
        device (driver actions, set_action, step, auto-reset: five launches)"""
        env.lib.gm_program_actions(env.ctx, args.seed, 0.2, DRIVER_MODE, d_act, 1)
        env.lib.gm_set_action(env.ctx, d_act, 1)
        if timed is not None:
            ev[timed][0].record(stream)
        env.lib.gm_step(env.ctx)
        if timed is not None:
            ev[timed][1].record(stream)
        env.autoreset_device(0, None, max_episode_steps=MAX_EP, episodes_dev_ptr=rec)

    def drive(timed=None):
        """R env-steps of the whole batch: one gm_rollout launch (or one per-step round)"""
        if not rollout:
            drive_ps(timed, episodes.data_ptr())
            return
        if timed is not None:
            ev[timed][0].record(stream)
        env.rollout(R, DRIVER_MODE, args.seed, 0.2, MAX_EP, episodes.data_ptr())
        if timed is not None:
            ev[timed][1].record(stream)

    # steady state: env e (global id) starts its episode at pre-roll step t_e, so after
    # MAX_EP untimed steps the batch covers episode steps 1..MAX_EP uniformly
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(max(K, 1))]
    gids = first_env + np.arange(n)
    t_start = gmx.spawn_int(args.seed, gids, 0, 99, 0, MAX_EP - 1)
    for t in range(MAX_EP if args.preroll else 0):
        m = (t_start == t)
        if m.any():
            env.lib.gm_reset(env.ctx, np.ascontiguousarray(m.astype(np.uint8)).ctypes.data_as(
                __import__("ctypes").POINTER(__import__("ctypes").c_uint8)), None)
        drive_ps()
    elapsed, ep_stats = measure(drive, episodes, n_drives, w_drives, world, dev, torch.cuda.synchronize)
    steps_view = gmx.env_state_view(env.env_states())["num_action_steps"]

    kern_ms = [a.elapsed_time(b) for a, b in ev[:n_drives]]
    kern_launch_s = sum(kern_ms) / len(kern_ms) / 1e3
    kern_avg_s = kern_launch_s / R                      # the kernel's time per env-step
    # the same workload through the per-step API (five launches per env-step), for reference
    per_step_api = None
    if rollout and rank == 0 and world == 1:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(K):
            drive_ps(k)
        torch.cuda.synchronize()
        ps_s = (time.perf_counter() - t0) / K
        ps_k = sum(a.elapsed_time(b) for a, b in ev[:K]) / K
        per_step_api = {"ms_per_step": round(ps_s * 1e3, 3), "value": round(n / ps_s, 1), "unit": "env-steps/s",
                        "step_kernel_ms": round(ps_k, 4),
                        "path": "gm_program_actions + gm_set_action + gm_step + gm_autoreset_episodes per env-step"}
    finite = bool(torch.isfinite(torch.as_tensor(env.observation())).all())
    overflow = int(env.overflow().sum())
    parity = None if (args.no_parity or rank != 0) else obs_parity(gmx, env, args.seed)
    # contact load of the batch state (one probing substep after the timed window)
    ncon_m, _, _, _, nefc_m, _ = env.debug_substep(full=True)
    # the constraint solver's work on the same states (one profiled env-step after it):
    # Newton iterations and exact-line-search evaluations per substep solve
    ph = env.step_profiled().astype(np.float64)
    n_solves = float(n * S)
    solver = {"method": "primal Newton (mj_solNewton) with exact line search, warm-started",
              "iterations_per_solve": round(ph[:, env.PH_NEWTON].sum() / n_solves, 4),
              "max_iterations_in_env_step": int(ph[:, env.PH_NEWTON].max()),
              "line_search_evals_per_solve": round(ph[:, env.PH_LS].sum() / n_solves, 4),
              "rows_per_solve": round(ph[:, env.PH_NEFC].sum() / n_solves, 3),
              # solves that hit GM_NEWTON_MAXIT or a line search that hit GM_NEWTON_MAXLS,
              # over every substep this batch ran (pre-roll, warmup, timed, probes)
              "newton_cap_hits": int(gmx.env_state_view(env.env_states())["newton_caps"].sum()),
              "states": "the batch after the timed window, one profiled env-step"}

    if rank == 0:
        B = algorithmic_bytes_per_substep(env.model)
        Bm = algorithmic_bytes_per_substep(env.model, ncon=int(round(float(ncon_m.mean()))))
        # bytes and traffic both per LAUNCH (R env-steps of every env); per env-step = / R
        bytes_per_env_step = n * S * B["bytes"]
        bytes_per_launch = bytes_per_env_step * R
        achieved = bytes_per_launch / kern_launch_s / 1e9
        traffic, traffic_src = load_traffic(n, R)
        roof = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                "per": "launch (R env-steps of the whole batch): achieved = algorithmic_bytes_per_launch / "
                       "kernel_launch_ms; traffic = PMC HBM bytes per launch",
                "kernel": "gm_step_kernel", "kernel_avg_ms": round(kern_avg_s * 1e3, 4),
                # one launch runs R env-steps of every env (gm_rollout); per-step = launch / R
                "kernel_launch_ms": round(kern_launch_s * 1e3, 4), "env_steps_per_launch": R,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "algorithmic_bytes_per_env_step": bytes_per_env_step,
                "traffic_per_env_step": None if traffic is None else traffic / R,
                "compute": load_compute(n, S, R, kern_launch_s),
                "traffic_source": traffic_src,
                "traffic_measured_in_this_run": False,   # PMC counters need their own rocprofv3 pass
                # the same roofline with the per-substep bytes at the batch's measured mean
                # contact count instead of SURVEY.md 8d's nominal 12
                "achieved_at_measured_ncon": round(n * S * Bm["bytes"] / kern_avg_s / 1e9, 2),
                "frac_at_measured_ncon": round(n * S * Bm["bytes"] / kern_avg_s / 1e9 / HBM_PEAK_GBS, 5),
                "measured_ncon": Bm["ncon"]}
        cpu = None
        if world == 1 and not args.no_cpu:
            cpu = cpu_baseline(gmx, args.cpu_envs * args.cpu_threads // 4, args.cpu_steps, args.cpu_threads)
            cpu["single_thread"] = cpu_baseline(gmx, args.cpu_envs, args.cpu_steps, 1)["value"]
        c2 = None if (args.no_c2 or world > 1) else c2_line(gmx, torch, dev, stream, K, args.seed, first_env,
                                                            math.gcd(K, args.c2_rollout) if rollout and args.c2_rollout > 0 else 0)
        c3r = None if (args.no_random or world > 1) else c3_random_line(gmx, torch, dev, stream, K, args.seed, first_env, n,
                                                                        R if rollout else 0)
        c3s = None if (args.no_scripted or world > 1) else c3_scripted_line(gmx, torch, dev, stream, K, args.seed,
                                                                             first_env, n, R if rollout else 0)
        c1 = None if (args.no_c1 or world > 1) else c1_line(gmx, args.seed)
        c5 = None if (args.no_policy or world > 1) else policy_rollout(gmx, torch, dev, stream, n, max(3, K // 2), args.seed,
                                                        first_env, R if rollout else 0)
        out = headline(world, n, K, W, elapsed, ep_stats)
        out["warmup_steps_run"] = max(w_drives, 1) * R
        out["config"].update({"workload": "C3: set6_synthetic 20 mixed objects, randomised spawn (object drawn per "
                                   "episode, spawn_into_scene grid search on the device), steady state: envs "
                                   "staggered over episode steps 1..250 by an untimed pre-roll, benchmark mix "
                                   "(1 episode in 4: the closed-loop grasp-lift-hold program; otherwise the "
                                   "scripted grasp mix: close / squeeze / palm / lift + jitter), canonical "
                                   "sensor/reward "
                                   "config, device auto-reset at done / 250 steps; driven as gm_rollout launches "
                                   f"of {R} env-steps (driver actions, env-step, episode-end record and reset "
                                   "fused per env; bit-identical to the per-step API, tests/test_rollout.py)"
                                   if rollout else "the per-step API",
                       "substeps_per_env_step": S,
                       "B_substep_bytes": B["bytes"], "B_substep_ncon": B["ncon"], "B_substep_nefc": B["nefc"],
                       "measured_contacts": {"mean_ncon": round(float(ncon_m.mean()), 3),
                                             "mean_nefc": round(float(nefc_m.mean()), 3),
                                             "max_ncon": int(ncon_m.max()), "max_nefc": int(nefc_m.max()),
                                             "B_substep_bytes_at_mean_ncon": Bm["bytes"],
                                             "episode_step_spread": [int(steps_view.min()), int(steps_view.max()),
                                                                     round(float(steps_view.mean()), 1)]},
                       "model": {"nq": env.model.nq, "nv": env.model.nv, "nbody": env.model.nbody,
                                 "ngeom": env.model.ngeom, "nM": env.model.nM, "nlock": env.model.nlock},
                       "dtype_detail": "f64 dynamics, collision and constraint solver; f32 sensor windows / observations (as the reference)"})
        out.update({
            "roofline": roof,
            "constraint_solver": solver,
            "cpu_baseline": cpu,
            "obs_max_rel_err": parity,
            "per_step_api": per_step_api,
            "c2_single_cylinder_256": c2,
            "c3_random_actions": c3r,
            "c3_scripted_mix_only": c3s,
            "c1_single_env_200_steps": c1,
            "c5_device_policy_rollout": c5,
            "overflow_envs": overflow, "finite": finite,
        })
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
