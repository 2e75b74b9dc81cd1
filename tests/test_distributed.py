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


def run_envs(env_ids, steps):
    """Cumulative reward per env after `steps` random-action env-steps (oracle)."""
    import gmx
    import oracle_lib
    s = gmx.canonical_settings(noise=True, seed=11)
    model = gmx.ModelBlob()
    cfg = gmx.ConfigBlob(s, model)
    objs = gmx.make_object_set("set1_synthetic", 11)
    out = []
    for g in env_ids:
        e = oracle_lib.OracleEnv(model, cfg, objs, int(g))
        sp = gmx.Spawn()
        sp.object_index = int(g) % len(objs)
        sp.x, sp.y, sp.zrot = 0.0, 0.0, 0.0
        e.reset(sp)
        rng = np.random.default_rng(1000 + int(g))
        tot = 0.0
        for _ in range(steps):
            _, r, _ = e.step(rng.uniform(-1, 1, size=cfg.n_actions).astype(np.float32))
            tot += r
        out.append(tot)
    return np.array(out, dtype=np.float32)


def worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gmx.shard import shard_range, gather_returns, max_over_ranks
        lo, hi = shard_range(rank, world, N_PER_RANK)
        ret = torch.from_numpy(run_envs(range(lo, hi), STEPS))
        allr = gather_returns(ret, world)
        t = max_over_ranks(0.5 + rank)
        if rank == 0:
            q.put((allr.numpy().tolist(), t))
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
    got, tmax = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = run_envs(range(world * N_PER_RANK), STEPS)
    np.testing.assert_array_equal(np.array(got, dtype=np.float32), ref)
    assert tmax == 1.5
