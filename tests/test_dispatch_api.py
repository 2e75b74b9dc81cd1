"""The dispatch diagnostics and host-transfer entry points of the C ABI (r05):
gm_chunk_timeline (per-workgroup end of work, per-env start / finish of the last chunked
launch), gm_chunk_stats' cross-XCD resumptions, gm_get_outputs (observation, reward and
done in one read) and gm_set_action's pinned staging (the call returns before the upload;
the caller's array may be reused at once)."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu


def make(gm, n, seed=3):
    env = gm.BatchedGripperEnv(n, object_set="set6_synthetic", settings=gm.canonical_settings(seed=seed), seed=seed)
    env.set_scene_spawn(gm.default_spawn_params(), max_tries=3)
    env.reset()
    return env


def test_chunk_timeline_is_consistent(gm):
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    n = 3000                                   # past the DUO capacity (1024) and the grid (2048)
    env = make(gm, n)
    try:
        assert env.dispatch_info()["waves_per_env"] == 1
        rec = torch.zeros((4, n, 3), dtype=torch.int32, device="cuda")
        env.rollout(4, action_mode=1, seed=3, records_dev_ptr=rec.data_ptr())
        torch.cuda.synchronize()
        st = env.chunk_stats()
        ends, xcd, ev = env.chunk_timeline()
        assert st["finished"] == n and st["started"] == n
        assert len(ends) == st["workgroups"] and ev.shape == (n, 2)
        assert ((xcd >= 0) & (xcd < 8)).all() and len(np.unique(xcd)) > 1
        assert (ev[:, 0] >= -1e-3).all() and (ev[:, 1] > ev[:, 0]).all()        # every env started, then finished
        span = st["span_ms"]
        assert ev[:, 1].max() <= span + 1e-2 and ends.max() <= span + 1e-2
        # the workgroups ran out of work no later than the last env finished
        assert abs(ends.max() - ev[:, 1].max()) < 0.5
        assert st["steals"] >= 0 and st["resumes"] == st["yields"]
    finally:
        env.close()


def test_get_outputs_equals_separate_reads(gm):
    if not gpu_available():
        pytest.skip("no GPU")
    env = make(gm, 64)
    try:
        a = np.random.default_rng(1).uniform(-1, 1, size=(64, env.n_actions)).astype(np.float32)
        env.set_action(a)
        env.action_step()
        obs, rew, done = env.outputs()
        np.testing.assert_array_equal(obs, env.observation())
        r2, d2 = env.reward_done()
        np.testing.assert_array_equal(rew, r2)
        np.testing.assert_array_equal(done, d2)
    finally:
        env.close()


def test_set_action_staging_reuses_caller_array(gm):
    """Back-to-back host set_action calls with one caller array rewritten in between give
    what two synchronised contexts give."""
    if not gpu_available():
        pytest.skip("no GPU")
    a = make(gm, 128)
    b = make(gm, 128)
    try:
        rng = np.random.default_rng(2)
        buf = np.zeros((128, a.n_actions), dtype=np.float32)
        for t in range(4):
            acts = rng.uniform(-1, 1, size=buf.shape).astype(np.float32)
            buf[:] = acts
            a.set_action(buf)
            buf[:] = 0.0                      # the caller reuses its array at once
            a.action_step()
            b.set_action(acts.copy())
            b.action_step()
            oa, ra, da = a.outputs()
            ob, rb, db = b.outputs()
            np.testing.assert_array_equal(oa, ob)
            np.testing.assert_array_equal(ra, rb)
        np.testing.assert_array_equal(a.env_states(), b.env_states())
    finally:
        a.close()
        b.close()
