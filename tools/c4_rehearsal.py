"""C4 rehearsal on ONE GPU: the 8-rank env-shard job (32768 envs, 4096 per
rank, global env ids rank * 4096 + i) run as 8 processes sharing cuda:0, the episode-end
collective over gloo (the 8-GPU node runs it over RCCL; this box has one GPU).  Checks the
sharded data path at full size, not scaling: every rank steps its shard with gm_rollout
(the headline's driver, R env-steps per launch), the [32768 x 3] episode-end records are
all-gathered every launch, and rank 0 then re-runs shard 7 alone in its own context and
requires its records and final state digest to equal what rank 7 produced bit for bit
(results independent of the sharding: every env's streams are keyed by its global id).
usage: python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1
       --master-port P tools/c4_rehearsal.py [launches] [R]"""
import hashlib
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gripper-mujoco_amd"))

N_PER_RANK = 4096
MAX_EP = 8          # short episodes: truncations (and resets) inside the launches


def run_shard(gmx, torch, bench, rank, world, launches, R, seed, gather):
    from gmx.shard import shard_range
    lo, _ = shard_range(rank, world, N_PER_RANK)
    env = gmx.BatchedGripperEnv(N_PER_RANK, object_set="set6_synthetic", settings=gmx.canonical_settings(seed=seed),
                                seed=seed, env_offset=lo, device=0)
    env.set_scene_spawn(bench.mjenv_spawn_params(gmx), max_tries=3)
    env.reset()
    rec = torch.zeros((R, N_PER_RANK, 3), dtype=torch.int32, device="cuda:0")
    out = []
    t_run = 0.0
    for _ in range(launches):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        env.rollout(R, 0, seed, 0.2, MAX_EP, rec.data_ptr())
        torch.cuda.synchronize()
        t_run += time.perf_counter() - t0
        host = rec.cpu()
        out.append(gather(host) if gather else host)
    digest = hashlib.sha1(env.env_states().tobytes()).hexdigest()
    env.close()
    return out, digest, t_run


def main():
    import torch
    import torch.distributed as dist
    import bench
    import gmx
    launches = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    seed = 1234

    def gather(host):   # [R, n, 3] per rank -> [R, world * n, 3] in global env order
        parts = [torch.empty_like(host) for _ in range(world)]
        dist.all_gather(parts, host.contiguous())
        return torch.cat(parts, dim=1)

    dist.barrier()
    t0 = time.perf_counter()
    recs, digest, t_run = run_shard(gmx, torch, bench, rank, world, launches, R, seed, gather)
    wall = time.perf_counter() - t0
    digests = [None] * world
    dist.all_gather_object(digests, digest)
    times = [None] * world
    dist.all_gather_object(times, (t_run, wall))
    if rank == 0:
        allrec = torch.stack(recs)                         # [launches, R, world * n, 3]
        from gmx.shard import unpack_episodes
        _, length, success = unpack_episodes(allrec.reshape(-1, 3))
        # shard 7 alone, in this process's own context: bit for bit rank 7's records and state
        solo, solo_digest, _ = run_shard(gmx, torch, bench, world - 1, world, launches, R, seed, None)
        lo = (world - 1) * N_PER_RANK
        same = all(torch.equal(allrec[k, :, lo:lo + N_PER_RANK], solo[k]) for k in range(launches))
        line = {"what": "C4 rehearsal: 8 ranks x 4096 envs sharing ONE MI355X (gloo all-gather of the episode-end "
                        "records); a data-path check at full size, NOT a scaling measurement",
                "ranks": world, "global_envs": world * N_PER_RANK, "launches": launches, "env_steps_per_launch": R,
                "records_gathered": int(allrec.shape[0] * allrec.shape[1] * allrec.shape[2]),
                "episodes_finished": int((length > 0).sum()), "successes": int(success.sum()),
                "shard7_solo_records_equal": bool(same), "shard7_solo_state_digest_equal": solo_digest == digests[-1],
                "distinct_rank_digests": len(set(digests)),
                "per_rank_rollout_s": [round(t[0], 3) for t in times], "per_rank_wall_s": [round(t[1], 3) for t in times]}
        print(json.dumps(line))
        ok = same and solo_digest == digests[-1] and len(set(digests)) == world and int((length > 0).sum()) > 0
        dist.destroy_process_group()
        sys.exit(0 if ok else 1)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
