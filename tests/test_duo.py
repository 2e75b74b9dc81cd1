"""DUO workgroups (gm_step_kernel<CL, false, true>): for batches whose envs all fit
resident with two waves each, the second wave of an env's workgroup runs the collider
while the first forms the inertia and forces (gm_kernels.hip physics_substep_body /
duo_helper).  The same code runs on the same LDS image in the same order per env, so the
results must equal the one-wave kernel's bit for bit: checked on grasp rollouts (scripted
mix, mixed objects, cylinder) through the per-step API in both dispatch modes (chunked and
one-shot), and through gm_rollout with resets inside the launch."""
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu


def make_env(gm, n, object_set, seed, env_vars):
    s = gm.canonical_settings(noise=True, seed=seed)
    old = {k: os.environ.get(k) for k in env_vars}
    os.environ.update(env_vars)
    try:
        env = gm.BatchedGripperEnv(n, object_set=object_set, settings=s, seed=seed)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    env.set_scene_spawn(gm.default_spawn_params(), max_tries=3)
    env.reset()
    return env


def grasp(gm, env, steps, seed):
    script = gm.GraspScript(env.settings, env.n_envs, seed=seed)
    out = []
    for k in range(steps):
        obs, rew, done, _ = env.step(script.actions(k))
        out.append((obs.copy(), np.asarray(rew).copy(), np.asarray(done).copy()))
    return out


@pytest.mark.parametrize("object_set,chunk", [("set6_synthetic", "16"), ("cylinder", "16"), ("set6_synthetic", "0")])
def test_duo_equals_one_wave(gm, object_set, chunk):
    if not gpu_available():
        pytest.skip("no GPU")
    n, steps, seed = 256, 40, 21
    a = make_env(gm, n, object_set, seed, {"GM_DUO": "1", "GM_CHUNK_SUBSTEPS": chunk})
    b = make_env(gm, n, object_set, seed, {"GM_DUO": "0", "GM_CHUNK_SUBSTEPS": chunk})
    try:
        assert a.dispatch_info()["waves_per_env"] == 2 and b.dispatch_info()["waves_per_env"] == 1
        ra, rb = grasp(gm, a, steps, seed), grasp(gm, b, steps, seed)
        for k, ((oa, wa, da), (ob, wb, db)) in enumerate(zip(ra, rb)):
            np.testing.assert_array_equal(oa, ob, err_msg=f"obs, step {k}")
            np.testing.assert_array_equal(wa, wb, err_msg=f"reward, step {k}")
            np.testing.assert_array_equal(da, db, err_msg=f"done, step {k}")
        sa, sb = a.env_states(), b.env_states()
        va, vb = gm.env_state_view(sa), gm.env_state_view(sb)
        for f in va.dtype.names:
            np.testing.assert_array_equal(va[f], vb[f], err_msg=f)
        # the batch really collided: finger-object contacts
        i_oc = gm.BINARY_EVENTS.index("object_contact")
        assert (va["bev_abs"][:, i_oc] > 0).sum() > 64
    finally:
        a.close()
        b.close()


def test_duo_rollout_equals_one_wave(gm):
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    n, steps, seed = 128, 12, 5
    ra = torch.zeros((steps, n, 3), dtype=torch.int32, device="cuda")
    rb = torch.zeros((steps, n, 3), dtype=torch.int32, device="cuda")
    a = make_env(gm, n, "set6_synthetic", seed, {"GM_DUO": "1"})
    b = make_env(gm, n, "set6_synthetic", seed, {"GM_DUO": "0"})
    try:
        a.rollout(steps, action_mode=1, seed=seed, jitter=0.2, max_episode_steps=5, records_dev_ptr=ra.data_ptr())
        b.rollout(steps, action_mode=1, seed=seed, jitter=0.2, max_episode_steps=5, records_dev_ptr=rb.data_ptr())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(a.env_states(), b.env_states())
        np.testing.assert_array_equal(a.observation(), b.observation())
        np.testing.assert_array_equal(ra.cpu().numpy(), rb.cpu().numpy())
        assert int(gm.env_state_view(a.env_states())["episode"].min()) >= 2
    finally:
        a.close()
        b.close()


def test_dispatch_defaults(gm):
    """DUO is the default exactly when every env's two waves fit resident."""
    if not gpu_available():
        pytest.skip("no GPU")
    small = make_env(gm, 64, "set6_synthetic", 1, {})
    big = make_env(gm, 4096, "set6_synthetic", 1, {})
    try:
        assert small.dispatch_info()["waves_per_env"] == 2
        assert big.dispatch_info()["waves_per_env"] == 1
    finally:
        small.close()
        big.close()


@pytest.mark.parametrize("n_seg,dt", [(5, 6.76e-3), (10, 2.1e-3)])
def test_duo_other_segment_counts(gm, n_seg, dt):
    """The DUO instances for other chain lengths (CL = 7, 12: N = 10 takes the collider's
    second 64-pair batch on the helper wave) equal the one-wave kernel bit for bit."""
    if not gpu_available():
        pytest.skip("no GPU")
    import ctypes as C
    p = gm.ModelParams()
    gm.load_library().gm_default_model_params(C.byref(p))
    p.n_seg, p.timestep = n_seg, dt
    n, steps, seed = 128, 25, 9
    envs = []
    for v in ("1", "0"):
        old = os.environ.get("GM_DUO")
        os.environ["GM_DUO"] = v
        try:
            e = gm.BatchedGripperEnv(n, object_set="set6_synthetic", settings=gm.canonical_settings(noise=True, seed=seed),
                                     seed=seed, model_params=p)
        finally:
            if old is None:
                os.environ.pop("GM_DUO", None)
            else:
                os.environ["GM_DUO"] = old
        e.set_scene_spawn(gm.default_spawn_params(), max_tries=3)
        e.reset()
        envs.append(e)
    a, b = envs
    try:
        assert a.dispatch_info()["waves_per_env"] == 2 and b.dispatch_info()["waves_per_env"] == 1
        ra, rb = grasp(gm, a, steps, seed), grasp(gm, b, steps, seed)
        for k, ((oa, wa, da), (ob, wb, db)) in enumerate(zip(ra, rb)):
            np.testing.assert_array_equal(oa, ob, err_msg=f"obs, step {k}")
            np.testing.assert_array_equal(wa, wb, err_msg=f"reward, step {k}")
        np.testing.assert_array_equal(a.env_states(), b.env_states())
    finally:
        a.close()
        b.close()
