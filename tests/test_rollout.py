"""gm_rollout: n env-steps of every env in ONE persistent launch with the synthetic driver and
the auto-reset on the device must equal, bit for bit, n rounds of the per-step API
(driver actions -> gm_set_action -> gm_step -> gm_autoreset_episodes): the same code on the
same state in the same order per env (include/gripper_mi355x.h gm_rollout).  Checked on the
whole fp64 state record, observations, rewards, done flags and every episode-end record, in
both driver modes, with episodes short enough that resets (and their spawn searches) happen
inside the launch.  The random driver's host mirror (gmx.random_fractions) equals the device
draws."""
import hashlib
import os

import numpy as np
import pytest

from conftest import gpu_available

N, K, MAX_EP, SEED = 96, 14, 6, 77


# the hand-off heavy dispatch: a preemption test every substep, no margins, many yields, so
# envs change waves inside and across the env-steps of the launch (the carry's step index,
# steps left and per-step counters)
# (on 24 workgroups: with a wave slot per env nothing would ever wait in the queue)
HANDOFF = {"GM_CHUNK_SUBSTEPS": "1", "GM_CHUNK_MARGIN": "0", "GM_CHUNK_YIELDS": "60", "GM_CHUNK_CMARGIN": "0",
           "GM_CHUNK_GRID": "24"}


def make_env(gm, env_vars=None, n=N):
    import bench
    s = gm.canonical_settings(noise=True, seed=SEED)          # noise on: the RNG streams matter
    old = {k: os.environ.get(k) for k in (env_vars or {})}
    os.environ.update(env_vars or {})
    try:
        env = gm.BatchedGripperEnv(n, object_set="set6_synthetic", settings=s, seed=SEED)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    env.set_scene_spawn(bench.mjenv_spawn_params(gm), max_tries=3)
    env.reset()
    return env


def per_step(gm, env, mode, records, steps=K, max_ep=MAX_EP):
    import torch
    d_act = env.lib.gm_device_actions(env.ctx)
    for k in range(steps):
        if mode == 0:
            env.lib.gm_scripted_actions(env.ctx, SEED, 0.2, d_act, 1)
        elif mode == 1:
            env.lib.gm_random_actions(env.ctx, SEED, d_act, 1)
        else:
            env.lib.gm_program_actions(env.ctx, SEED, 0.2, mode, d_act, 1)
        env.lib.gm_set_action(env.ctx, d_act, 1)
        env.lib.gm_step(env.ctx)
        env.autoreset_device(0, None, max_episode_steps=max_ep, episodes_dev_ptr=records[k].data_ptr())
    torch.cuda.synchronize()


def snapshot(env, records):
    import torch
    torch.cuda.synchronize()
    st = env.env_states()
    rew, done = env.reward_done()
    return (hashlib.sha1(np.ascontiguousarray(st).tobytes()).hexdigest(), st, env.observation(), rew, done,
            records.cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("mode,dispatch", [(0, "default"), (1, "default"), (0, "handoff-heavy"), (3, "default"),
                                           (4, "handoff-heavy")])
def test_rollout_equals_per_step_api(gm, mode, dispatch):
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    from gmx.shard import unpack_episodes
    ra = torch.zeros((K, N, 3), dtype=torch.int32, device="cuda")
    rb = torch.zeros((K, N, 3), dtype=torch.int32, device="cuda")
    a = make_env(gm)
    b = make_env(gm, HANDOFF if dispatch == "handoff-heavy" else None)
    try:
        per_step(gm, a, mode, ra)
        # (the hand-off test needs dispatch costs, which a context records from its first
        # env-step on: b takes that one through the per-step API too)
        k0 = 1 if dispatch == "handoff-heavy" else 0
        per_step(gm, b, mode, rb, steps=k0)
        b.rollout(K - k0, action_mode=mode, seed=SEED, jitter=0.2, max_episode_steps=MAX_EP,
                  records_dev_ptr=rb[k0:].data_ptr())
        sa, sb = snapshot(a, ra), snapshot(b, rb)
        va, vb = gm.env_state_view(sa[1]), gm.env_state_view(sb[1])
        for f in va.dtype.names:
            np.testing.assert_array_equal(va[f], vb[f], err_msg=f)
        assert sa[0] == sb[0]
        np.testing.assert_array_equal(sa[2], sb[2])
        np.testing.assert_array_equal(sa[3], sb[3])
        np.testing.assert_array_equal(sa[4], sb[4])
        np.testing.assert_array_equal(sa[5], sb[5])
        # the launch really crossed episode boundaries: resets with their spawn searches
        _, length, _ = unpack_episodes(torch.from_numpy(sa[5].reshape(-1, 3)))
        assert int((length > 0).sum()) >= N, int((length > 0).sum())
        assert int(va["episode"].min()) >= 2
        if dispatch == "handoff-heavy":
            st = b.chunk_stats()
            assert st["yields"] > N, st
            # idle waves resumed yielded envs of other XCDs (cross-XCD hand-offs)
            assert st["steals"] > 0, st
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_random_actions_match_host_mirror(gm):
    if not gpu_available():
        pytest.skip("no GPU")
    env = make_env(gm)
    try:
        out = np.zeros((N, env.n_actions), dtype=np.float32)
        env.lib.gm_random_actions(env.ctx, SEED, out.ctypes.data, 0)
        v = gm.env_state_view(env.env_states())
        ref = gm.random_fractions(SEED, np.arange(N), v["episode"], v["num_action_steps"], env.n_actions)
        np.testing.assert_array_equal(out, ref)
        assert out.min() >= -1.0 and out.max() < 1.0 and out.std() > 0.4
    finally:
        env.close()


@pytest.mark.gpu
def test_rollout_equals_per_step_api_full_size(gm):
    """The identity at the headline batch (4096 envs on every XCD's queue, yields and
    cross-XCD resumptions under the default dispatch), 3-step episodes so every env resets
    inside the launch."""
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    n, k, mx = 4096, 5, 3
    ra = torch.zeros((k, n, 3), dtype=torch.int32, device="cuda")
    rb = torch.zeros((k, n, 3), dtype=torch.int32, device="cuda")
    a, b = make_env(gm, n=n), make_env(gm, n=n)
    try:
        per_step(gm, a, 0, ra, steps=k, max_ep=mx)
        per_step(gm, b, 0, rb, steps=1, max_ep=mx)     # (b's dispatch costs from one env-step)
        b.rollout(k - 1, action_mode=0, seed=SEED, jitter=0.2, max_episode_steps=mx, records_dev_ptr=rb[1:].data_ptr())
        sa, sb = snapshot(a, ra), snapshot(b, rb)
        assert sa[0] == sb[0]
        for i in range(2, 6):
            np.testing.assert_array_equal(sa[i], sb[i])
        assert int((sa[5][..., 1] > 0).sum()) >= n
        st = b.chunk_stats()
        assert st["finished"] == n and st["yields"] > 0, st
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_program_rollout_equals_per_step_api_through_the_lift(gm):
    """The grasp program (mode 3) is closed-loop: its fractions read each env's targets,
    joint positions and SI sensor windows.  Over 110 env-steps (close, squeeze, lift, palm,
    hold, successes and their resets) the fused launch equals the per-step calls bit for bit,
    under the hand-off heavy dispatch (envs move between waves mid env-step)."""
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    n, k, mx = 256, 110, 250
    ra = torch.zeros((k, n, 3), dtype=torch.int32, device="cuda")
    rb = torch.zeros((k, n, 3), dtype=torch.int32, device="cuda")
    a, b = make_env(gm, n=n), make_env(gm, HANDOFF, n=n)
    try:
        per_step(gm, a, 3, ra, steps=k, max_ep=mx)
        per_step(gm, b, 3, rb, steps=1, max_ep=mx)
        b.rollout(k - 1, action_mode=3, seed=SEED, jitter=0.2, max_episode_steps=mx, records_dev_ptr=rb[1:].data_ptr())
        sa, sb = snapshot(a, ra), snapshot(b, rb)
        assert sa[0] == sb[0]
        for i in range(2, 6):
            np.testing.assert_array_equal(sa[i], sb[i])
        # the program got through the chain in this window: successes in the records
        assert int((sa[5][..., 2] & 0xFF).sum()) > 0
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_work_queue_claims_never_park_tiny_grid_4096(gm):
    """Regression test of the work queue's claim protocol (claim_bucket, gm_kernels.hip): a
    4096-env rollout on a deliberately tiny persistent grid (16 workgroups) with the hand-off
    heavy knobs -- thousands of yields and resumptions, every wave contending for the same
    bucket slots -- equals the per-step calls bit for bit, and no claim parks: a claimed slot
    always has its producer in flight, so the claims that find their slot empty poll only
    briefly (the r05 race parked a wave on a slot only a future yield would fill: one rank
    took 50 s instead of 0.6 s)."""
    if not gpu_available():
        pytest.skip("no GPU")
    import time
    import torch
    n, k, mx = 4096, 3, 250
    tiny = dict(HANDOFF, GM_CHUNK_GRID="16")
    ra = torch.zeros((k, n, 3), dtype=torch.int32, device="cuda")
    rb = torch.zeros((k, n, 3), dtype=torch.int32, device="cuda")
    a, b = make_env(gm, n=n), make_env(gm, tiny, n=n)
    try:
        assert b.dispatch_info()["grid"] == 16
        per_step(gm, a, 0, ra, steps=k, max_ep=mx)
        per_step(gm, b, 0, rb, steps=1, max_ep=mx)
        t0 = time.time()
        b.rollout(k - 1, action_mode=0, seed=SEED, jitter=0.2, max_episode_steps=mx, records_dev_ptr=rb[1:].data_ptr())
        torch.cuda.synchronize()
        wall = time.time() - t0
        st, cw = b.chunk_stats(), b.claim_waits()
        print(f"tiny grid: {wall:.2f} s, {st}, {cw}")
        sa, sb = snapshot(a, ra), snapshot(b, rb)
        assert sa[0] == sb[0]
        for i in range(2, 6):
            np.testing.assert_array_equal(sa[i], sb[i])
        assert st["finished"] == n and st["yields"] > n and st["resumes"] == st["yields"], st
        assert b.dispatch_info()["last_launch_env_steps"] == k - 1
        # no parked claim: the waits are the producer's two-instruction window
        assert cw["polls"] <= 64 * cw["waiting_claims"] + 64, cw
        assert wall < 60.0, wall
    finally:
        a.close()
        b.close()
