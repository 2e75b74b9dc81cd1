"""The multi-GPU path on CPU: world_size-2 gloo.  Each rank owns a contiguous shard of
global env ids (gmx.shard), steps its envs (here through the fp64 oracle, the stand-in
for a rank's device), and the per-env episode returns are all-gathered.  The gathered
result must equal a single-process run over all envs: results do not depend on the
number of ranks, because every env's RNG stream is keyed by its global id."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N_PER_RANK = 2
STEPS = 6


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_envs(env_ids, steps, records=False):
    """Cumulative reward per env after `steps` random-action env-steps (oracle); with
    records=True the episode-end record of each env's first episode instead (return,
    length, successful_grasp), packed as gm_episode_end ([n, 3] int32)."""
    import gmx
    import oracle_lib
    s = gmx.canonical_settings(noise=True, seed=11)
    model = gmx.ModelBlob()
    cfg = gmx.ConfigBlob(s, model)
    objs = gmx.make_object_set("set1_synthetic", 11)
    out, recs = [], []
    i_succ = list(gmx.BINARY_EVENTS).index("successful_grasp")
    for g in env_ids:
        e = oracle_lib.OracleEnv(model, cfg, objs, int(g))
        sp = gmx.Spawn()
        sp.object_index = int(g) % len(objs)
        # env 1 spawns its object out of bounds: its episode ends (done) at the first step
        sp.x, sp.y, sp.zrot = (0.09 if int(g) == 1 else 0.0), 0.0, 0.0
        e.reset(sp)
        rng = np.random.default_rng(1000 + int(g))
        tot = 0.0
        rec = None
        for k in range(steps):
            _, r, d = e.step(rng.uniform(-1, 1, size=cfg.n_actions).astype(np.float32))
            tot = np.float32(tot + np.float32(r))
            if rec is None and (d or k + 1 == steps):
                rec = (tot, k + 1, int(e.event_rows()[2][i_succ] > 0))
        out.append(tot)
        recs.append(rec)
    if records:
        import torch
        from gmx.shard import pack_episodes
        r = np.array(recs, dtype=np.float64)
        return pack_episodes(torch.tensor(r[:, 0], dtype=torch.float32), torch.tensor(r[:, 1]),
                             torch.tensor(r[:, 2])).numpy()
    return np.array(out, dtype=np.float32)


def worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gmx.shard import shard_range, gather_episodes, gather_returns, max_over_ranks
        lo, hi = shard_range(rank, world, N_PER_RANK)
        ret = torch.from_numpy(run_envs(range(lo, hi), STEPS))
        allr = gather_returns(ret, world)
        rec = torch.from_numpy(run_envs(range(lo, hi), STEPS, records=True))
        allrec = gather_episodes(rec, world)
        t = max_over_ranks(0.5 + rank)
        if rank == 0:
            q.put((allr.numpy().tolist(), allrec.numpy().tolist(), t))
    finally:
        dist.destroy_process_group()


def test_shard_range():
    from gmx.shard import shard_range
    assert shard_range(0, 2, 4096) == (0, 4096)
    assert shard_range(1, 2, 4096) == (4096, 8192)
    with pytest.raises(ValueError):
        shard_range(2, 2, 4)


def test_two_rank_gather_matches_single_process(gm):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, got_rec, tmax = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = run_envs(range(world * N_PER_RANK), STEPS)
    np.testing.assert_array_equal(np.array(got, dtype=np.float32), ref)
    # the episode-end records (return, length, success), bit for bit in global env order
    ref_rec = run_envs(range(world * N_PER_RANK), STEPS, records=True)
    np.testing.assert_array_equal(np.array(got_rec, dtype=np.int32), ref_rec)
    from gmx.shard import unpack_episodes
    r, length, _ = unpack_episodes(torch.from_numpy(ref_rec))
    assert length[1] == 1 and length[0] == STEPS      # env 1's episode ended at once (oob)
    assert r.isfinite().all()
    assert tmax == 1.5


# ---------------------------------------------------------------- bench.py's timed loop
BENCH_N, BENCH_K, BENCH_W, BENCH_EP = 2, 4, 1, 2


class OracleRollout:
    """A rank's envs stepped by the oracle behind the same drive(k) / returns interface
    the device path gives bench.measure: each drive is one env-step of every env; an env
    whose episode ends (done, or BENCH_EP steps) hands its return over and is reset."""

    def __init__(self, env_ids, sleep_s=0.0):
        import gmx
        import oracle_lib
        s = gmx.canonical_settings(noise=True, seed=11)
        self.model = gmx.ModelBlob()
        self.cfg = gmx.ConfigBlob(s, self.model)
        self.objs = gmx.make_object_set("set1_synthetic", 11)
        self.ids = [int(g) for g in env_ids]
        self.envs = [oracle_lib.OracleEnv(self.model, self.cfg, self.objs, g) for g in self.ids]
        self.rng = [np.random.default_rng(2000 + g) for g in self.ids]
        self.steps = [0] * len(self.ids)
        self.ret = [np.float32(0)] * len(self.ids)
        from gmx.shard import new_episode_records
        self.episodes = new_episode_records(len(self.ids))
        self.ended = 0          # episodes ended inside the timed drives
        self.succeeded = 0
        self.length_sum = 0
        self.i_succ = list(gmx.BINARY_EVENTS).index("successful_grasp")
        self.sleep_s = sleep_s
        for i in range(len(self.ids)):
            self._reset(i)

    def _reset(self, i):
        import gmx
        sp = gmx.Spawn()
        sp.object_index = self.ids[i] % len(self.objs)
        sp.x, sp.y, sp.zrot = 0.0, 0.0, 0.0
        self.envs[i].reset(sp)
        self.steps[i] = 0
        self.ret[i] = np.float32(0)

    def drive(self, k=None):
        import time
        from gmx.shard import pack_episodes
        n = len(self.envs)
        ret = torch.full((n,), float("nan"))
        length = torch.zeros(n, dtype=torch.int32)
        succ = torch.zeros(n, dtype=torch.int32)
        for i, e in enumerate(self.envs):
            _, r, d = e.step(self.rng[i].uniform(-1, 1, size=self.cfg.n_actions).astype(np.float32))
            self.ret[i] = np.float32(self.ret[i] + np.float32(r))
            self.steps[i] += 1
            if d or self.steps[i] >= BENCH_EP:
                ret[i] = float(self.ret[i])
                length[i] = self.steps[i]
                succ[i] = int(e.event_rows()[2][self.i_succ] > 0)
                if k is not None:
                    self.ended += 1
                    self.succeeded += int(succ[i])
                    self.length_sum += int(length[i])
                self._reset(i)
        self.episodes.copy_(pack_episodes(ret, length, succ))
        if self.sleep_s:
            time.sleep(self.sleep_s)


def bench_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from gmx.shard import shard_range
        lo, hi = shard_range(rank, world, BENCH_N)
        ro = OracleRollout(range(lo, hi), sleep_s=0.25 if rank == 1 else 0.0)   # rank 1 is the slow one
        elapsed, ep = bench.measure(ro.drive, ro.episodes, BENCH_K, BENCH_W, world, torch.device("cpu"),
                                    lambda: None)
        line = bench.headline(world, BENCH_N, BENCH_K, BENCH_W, elapsed, ep)
        q.put((rank, line, ep, elapsed, (ro.ended, ro.succeeded, ro.length_sum)))
    finally:
        dist.destroy_process_group()


def test_bench_timed_loop_two_ranks(gm):
    """bench.py's measure/headline over 2 gloo ranks: the all-gathered episode count covers
    both ranks, the wall time is the slowest rank's, and rank 0's line carries the contract
    fields with value = all ranks' env-steps / that time."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=240)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    line, ep, elapsed, _ = res[0]
    ended = res[0][3][0] + res[1][3][0]
    assert ep == res[1][1]                             # every rank tallies the whole job's records
    assert ep["episodes"] == ended > 0
    assert ep["successes"] == res[0][3][1] + res[1][3][1]
    assert ep["length_sum"] == res[0][3][2] + res[1][3][2]
    assert elapsed == res[1][2] >= BENCH_K * 0.25     # the max over ranks: rank 1 slept 0.25 s per drive
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data"):
        assert key in line, key
    assert line["n_gpus"] == world and line["steps"] == BENCH_K and line["warmup"] == BENCH_W
    assert line["scaling"] == "weak" and line["higher_is_better"] is True
    assert line["value"] == round(world * BENCH_N * BENCH_K / elapsed, 1)
    assert line["ms_per_step"] == round(elapsed / BENCH_K * 1e3, 3)
    assert line["config"]["global_envs"] == world * BENCH_N and line["config"]["envs_per_gpu"] == BENCH_N
    assert line["episodes_finished"] == ended
    assert line["episode_successes"] == ep["successes"]
    assert line["mean_episode_length"] == round(ep["length_sum"] / ended, 2)


# ---------------------------------------------------------------- successes through the collective
SUCC_STEPS = 110


def program_records(env_ids):
    """Each env's first episode under the grasp-lift-hold program (oracle or_driver_actions,
    mode 3), centred set6 objects: spheres for even global ids (carried on the hooks to
    successful_grasp), boxes for odd ones (squeezed, not carried); the gm_episode_end
    record of each, packed [n, 3] int32."""
    import gmx
    import oracle_lib
    from gmx.shard import pack_episodes
    s = gmx.canonical_settings(noise=False, seed=5)
    model = gmx.ModelBlob()
    cfg = gmx.ConfigBlob(s, model)
    objs = gmx.make_object_set("set6_synthetic", 1234)
    spheres = [i for i in range(len(objs)) if objs[i].type == 2 and objs[i].size[0] > 0.02]
    boxes = [i for i in range(len(objs)) if objs[i].type == 6]
    i_succ = list(gmx.BINARY_EVENTS).index("successful_grasp")
    recs = []
    for g in env_ids:
        e = oracle_lib.OracleEnv(model, cfg, objs, int(g))
        sp = gmx.Spawn()
        sp.object_index = spheres[int(g) // 2 % len(spheres)] if int(g) % 2 == 0 else boxes[0]
        sp.x, sp.y, sp.zrot = 0.0, 0.0, 0.0
        e.reset(sp)
        tot, rec = np.float32(0.0), None
        for k in range(SUCC_STEPS):
            e.set_action(e.driver_actions(mode=3, seed=5, gid=int(g)))
            e.action_step()
            d, r = e.is_done(), e.reward()
            tot = np.float32(tot + np.float32(r))
            if d or k + 1 == SUCC_STEPS:
                rec = (tot, k + 1, int(e.event_rows()[0][i_succ] > 0))
                break
        recs.append(rec)
    r = np.array(recs, dtype=np.float64)
    return pack_episodes(torch.tensor(r[:, 0], dtype=torch.float32), torch.tensor(r[:, 1]),
                         torch.tensor(r[:, 2])).numpy()


def succ_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gmx.shard import shard_range, gather_episodes
        lo, hi = shard_range(rank, world, N_PER_RANK)
        allrec = gather_episodes(torch.from_numpy(program_records(range(lo, hi))), world)
        if rank == 0:
            q.put(allrec.numpy().tolist())
    finally:
        dist.destroy_process_group()


def test_two_rank_gather_carries_program_successes(gm):
    """The episode-end collective with real successes in it: 2 gloo ranks x 2 envs under the
    grasp program; the gathered records equal a single-process run, the sphere envs' success
    bytes are 1 with their +1 return, the box envs' 0."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=succ_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = program_records(range(world * N_PER_RANK))
    np.testing.assert_array_equal(np.array(got, dtype=np.int32), ref)
    from gmx.shard import unpack_episodes
    r, length, success = unpack_episodes(torch.from_numpy(ref))
    assert success.tolist() == [1, 0, 1, 0], success
    assert (r[success.bool()] > 0.5).all() and (length[success.bool()] < SUCC_STEPS).all()


def test_bench_cli_contract():
    """bench.py's command line (the driver's contract): --gpus / --steps / --warmup, the
    headline's and the C2 line's rollout lengths, and the side-line switches; --help needs
    no GPU."""
    import subprocess
    import sys
    import os
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--help"], capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    for opt in ("--gpus", "--steps", "--warmup", "--rollout", "--c2-rollout", "--no-scripted", "--no-random",
                "--no-c2", "--no-c1", "--no-policy", "--no-cpu", "--no-parity"):
        assert opt in out.stdout, opt
