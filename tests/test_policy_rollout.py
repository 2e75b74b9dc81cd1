"""gm_policy_rollout: the DQN policy's rollout fused into one persistent launch (each env's own
wave runs select_action on its observation before each env-step) must equal, bit for bit,
the per-step sequence gm_policy_act (the batched MFMA kernel) -> gm_step ->
gm_autoreset_episodes (include/gripper_mi355x.h).  Checked on the whole fp64 state record,
observations, rewards, done flags and every episode-end record, with an eps schedule that
mixes greedy and random choices, episodes short enough to reset inside the launch, and the
hand-off heavy dispatch (envs change waves and XCDs mid env-step)."""
import hashlib
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

N, K, MAX_EP, SEED, PSEED, DEC0 = 96, 12, 5, 41, 9, 1000

HANDOFF = {"GM_CHUNK_SUBSTEPS": "1", "GM_CHUNK_MARGIN": "0", "GM_CHUNK_YIELDS": "60", "GM_CHUNK_CMARGIN": "0",
           "GM_CHUNK_GRID": "24"}


def make_env(gm, env_vars=None, n=N):
    import bench
    s = gm.canonical_settings(noise=True, seed=SEED)
    s.continous_actions = 0                                  # the DQN policy's discrete actions
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


def eps_schedule(k0, k1):
    # alternating mostly-greedy and mostly-random env-steps
    return np.array([0.9 if k % 3 == 0 else 0.2 for k in range(k0, k1)], dtype=np.float32)


def per_step(env, pol, records, k0, k1, max_ep=MAX_EP):
    import torch
    acts = []
    for k in range(k0, k1):
        pol.act(float(eps_schedule(k, k + 1)[0]), seed=PSEED, decision=DEC0 + k)
        acts.append(pol.read()[0])
        env.lib.gm_step(env.ctx)
        env.autoreset_device(0, None, max_episode_steps=max_ep, episodes_dev_ptr=records[k].data_ptr())
    torch.cuda.synchronize()
    return acts


def snapshot(env, records):
    import torch
    torch.cuda.synchronize()
    st = env.env_states()
    rew, done = env.reward_done()
    return (hashlib.sha1(np.ascontiguousarray(st).tobytes()).hexdigest(), st, env.observation(), rew, done,
            records.cpu().numpy())


@pytest.mark.parametrize("dispatch", ["default", "handoff-heavy", "one-shot"])
def test_policy_rollout_equals_per_step(gm, dispatch):
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    from gmx.policy import DevicePolicy
    from gmx.shard import unpack_episodes
    ra = torch.zeros((K, N, 3), dtype=torch.int32, device="cuda")
    rb = torch.zeros((K, N, 3), dtype=torch.int32, device="cuda")
    a = make_env(gm)
    b = make_env(gm, {"handoff-heavy": HANDOFF, "one-shot": {"GM_CHUNK_SUBSTEPS": "0"}}.get(dispatch))
    pa = DevicePolicy(a, seed=3)
    pb = DevicePolicy(b, seed=3)
    try:
        acts = per_step(a, pa, ra, 0, K)
        # the hand-off dispatch needs the dispatch costs a context records from its first
        # env-step on: b takes that one through the per-step API too
        k0 = 1 if dispatch == "handoff-heavy" else 0
        per_step(b, pb, rb, 0, k0)
        pb.rollout(eps_schedule(k0, K), seed=PSEED, decision0=DEC0 + k0, max_episode_steps=MAX_EP,
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
        # the policy chose varied actions and the launch crossed episode boundaries
        assert len(np.unique(np.concatenate(acts))) >= 4
        _, length, _ = unpack_episodes(torch.from_numpy(sa[5].reshape(-1, 3)))
        assert int((length > 0).sum()) >= N, int((length > 0).sum())
        assert int(va["episode"].min()) >= 2
        if dispatch == "handoff-heavy":
            st = b.chunk_stats()
            assert st["yields"] > N and st["steals"] > 0, st
        assert (b.dispatch_info()["chunk"] == 0) == (dispatch == "one-shot")
    finally:
        pa.close()
        pb.close()
        a.close()
        b.close()


def test_policy_rollout_greedy_differs_from_random(gm):
    """eps = 0 (greedy) and eps = 1 (uniform) fused rollouts take different actions."""
    if not gpu_available():
        pytest.skip("no GPU")
    from gmx.policy import DevicePolicy
    a, b = make_env(gm), make_env(gm)
    pa, pb = DevicePolicy(a, seed=3), DevicePolicy(b, seed=3)
    try:
        pa.rollout(np.zeros(4, np.float32), seed=PSEED, max_episode_steps=0)
        pb.rollout(np.ones(4, np.float32), seed=PSEED, max_episode_steps=0)
        assert not np.array_equal(a.observation(), b.observation())
    finally:
        pa.close()
        pb.close()
        a.close()
        b.close()



def test_policy_rollout_equals_per_step_full_size(gm):
    """The same identity at the headline batch (4096 envs, every XCD's queue busy), with
    3-step episodes so every env resets inside the launch."""
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    from gmx.policy import DevicePolicy
    n, k, mx = 4096, 4, 3
    ra = torch.zeros((k, n, 3), dtype=torch.int32, device="cuda")
    rb = torch.zeros((k, n, 3), dtype=torch.int32, device="cuda")
    a, b = make_env(gm, n=n), make_env(gm, n=n)
    pa, pb = DevicePolicy(a, seed=5), DevicePolicy(b, seed=5)
    try:
        per_step(a, pa, ra, 0, k, max_ep=mx)
        per_step(b, pb, rb, 0, 1, max_ep=mx)         # (b's dispatch costs from one env-step)
        pb.rollout(eps_schedule(1, k), seed=PSEED, decision0=DEC0 + 1, max_episode_steps=mx,
                   records_dev_ptr=rb[1:].data_ptr())
        sa, sb = snapshot(a, ra), snapshot(b, rb)
        assert sa[0] == sb[0]
        for i in range(2, 6):
            np.testing.assert_array_equal(sa[i], sb[i])
        assert int((sa[5][..., 1] > 0).sum()) >= n      # every env's episode ended inside
    finally:
        pa.close()
        pb.close()
        a.close()
        b.close()
