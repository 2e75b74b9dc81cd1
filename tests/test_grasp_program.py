"""The grasp-lift-hold program (gm_state.h gm_program_fraction; device action modes 3 / 4,
gm_program_actions; oracle or_driver_actions) takes an episode through the reference's
whole success chain (mjclass.cpp:1148-1210 update_env, 1295-1322 the successful_grasp
macro, 3000-3049 reward / is_done):

    lifted -> lifted_to_height -> target_height -> object_stable -> stable_height
    -> successful_grasp, done = 1, reward +1 (stable_height's binary reward in the
    canonical sensor_mixed_v1 set, gmx.settings)

CPU (the fp64 oracle): centred spheres of the set6 object set succeed -- the fixed hooks meet
a sphere under its widest section and carry it (the gripper's own mechanism) -- and the chain
fires in the reference's order.  Boxes and cylinders are squeezed but not carried: friction
alone cannot hold them against MuJoCo's soft-constraint creep ("Holding
an object"); their test pins that the chain stops at object contact.

GPU (-m gpu): at the headline batch (4096 C3 envs, randomised spawn), the device program
reaches successful_grasp in at least 10 % of the envs; every success transition is re-run by
the oracle from the device's fp64 pre-step state (actions, done, reward, event rows and the
episode-end record bit-exact), the fused rollout equals the per-step API, and the mode-4
benchmark mix carries successes into the episode-end records.
"""
import numpy as np
import pytest

from conftest import gpu_available

SEED = 5
GM_PROG_G_SQUEEZE = 1.5        # gm_state.h
CHAIN = ("lifted", "lifted_to_height", "target_height", "object_stable", "stable_height", "successful_grasp")


@pytest.fixture(scope="module")
def scene(gm):
    import oracle_lib as ol
    s = gm.canonical_settings(noise=False, seed=SEED)
    model = gm.ModelBlob()
    cfg = gm.ConfigBlob(s, model)
    objs = gm.make_object_set("set6_synthetic", 1234)
    return ol, model, cfg, objs


def run_program(gm, ol, model, cfg, objs, idx, steps=200, x=0.0, y=0.0, rot=0.0):
    """One centred episode of object idx on the oracle under the program; returns the
    per-step trace (first step each chain event fires, rewards, done step)."""
    env = ol.OracleEnv(model, cfg, objs, 0)
    sp = gm.Spawn()
    sp.object_index, sp.x, sp.y, sp.zrot = idx, x, y, rot
    env.reset(sp)
    B = gm.BINARY_EVENTS
    first = {}
    rewards, done_at = [], None
    env.gauge_peak = 0.0
    for t in range(steps):
        a = env.driver_actions(mode=3, seed=SEED)
        env.set_action(a)
        env.action_step()
        d = env.is_done()
        r = env.reward()
        rewards.append(r)
        env.gauge_peak = max(env.gauge_peak, float(env.sensor_si()[:3].max()))
        rows, _, _ = env.event_rows()
        for n in CHAIN + ("object_contact",):
            if rows[B.index(n)] > 0 and n not in first:
                first[n] = t
        if d:
            done_at = t
            break
    return first, rewards, done_at, env


def test_program_succeeds_on_centred_spheres(gm, scene):
    ol, model, cfg, objs = scene
    spheres = [i for i in range(len(objs)) if objs[i].type == 2 and objs[i].size[0] > 0.02]
    assert len(spheres) >= 3
    ok = 0
    for idx in spheres[:3]:
        first, rewards, done_at, env = run_program(gm, ol, model, cfg, objs, idx)
        assert done_at is not None, (idx, first)
        # every event of the chain fired, in the reference's order
        assert all(n in first for n in CHAIN), (idx, first)
        assert first["lifted"] <= first["lifted_to_height"] <= first["target_height"] <= first["stable_height"]
        assert first["object_stable"] <= first["stable_height"] == first["successful_grasp"] == done_at
        # stable_height's +1 (reward 1.0, done) on the final step, the shaped terms before it small
        assert rewards[-1] > 0.95, rewards[-1]
        assert max(rewards[:-1]) < 0.1
        rows, _, _ = env.event_rows()
        assert rows[gm.BINARY_EVENTS.index("successful_grasp")] == 1
        ok += 1
    assert ok == 3


def test_program_chain_stops_at_contact_for_box_and_cylinder(gm, scene):
    """Boxes / cylinders: squeezed (object contact, gauges loaded) but not carried -- the
    friction-only hold creeps ("Holding an object")."""
    ol, model, cfg, objs = scene
    for typ in (6, 5):
        idx = next(i for i in range(len(objs)) if objs[i].type == typ)
        first, rewards, done_at, env = run_program(gm, ol, model, cfg, objs, idx, steps=120)
        assert "object_contact" in first, (typ, first)
        assert "successful_grasp" not in first and "stable_height" not in first, (typ, first)
        assert env.gauge_peak > GM_PROG_G_SQUEEZE, (typ, env.gauge_peak)   # the squeeze loaded the gauges


def test_program_fraction_is_shared_and_stateless(gm, scene):
    """The oracle's driver is the shared gm_state.h function: the same state gives the same
    fractions whatever came before (stateless), and mode 4 picks the program for exactly
    the episodes gm_program_episode selects, the scripted mix otherwise."""
    ol, model, cfg, objs = scene
    env = ol.OracleEnv(model, cfg, objs, 7)
    sp = gm.Spawn()
    sp.object_index, sp.x, sp.y, sp.zrot = 2, 0.0, 0.0, 0.0
    env.reset(sp)
    for _ in range(40):
        env.set_action(env.driver_actions(mode=3, seed=SEED))
        env.action_step()
    st = env.export_state()
    a1 = env.driver_actions(mode=3, seed=SEED)
    env2 = ol.OracleEnv(model, cfg, objs, 7)
    env2.import_state(st)
    np.testing.assert_array_equal(env2.driver_actions(mode=3, seed=SEED), a1)
    # at most one action moves per step (a phase), all fractions in [-1, 1]
    assert (np.abs(a1) > 0).sum() <= 1 and np.abs(a1).max() <= 1.0
    # mode 4 = program in the selected episodes, scripted mix (mode 0) in the rest
    from gmx.env import spawn_int
    for gid in range(12):
        prog = spawn_int(SEED, np.array([gid]), np.array([int(gm.env_state_view(st[None])["episode"][0])]),
                         21, 0, 3)[0] == 0
        ref = env2.driver_actions(mode=3 if prog else 0, seed=SEED, gid=gid)
        np.testing.assert_array_equal(env2.driver_actions(mode=4, seed=SEED, gid=gid), ref)


# ---------------------------------------------------------------------------- GPU
N_GPU, STEPS_GPU = 4096, 150


@pytest.mark.gpu
def test_gpu_program_succeeds_bit_exact_vs_oracle_4096(gm):
    """4096 C3 envs (set6, randomised spawn with the spawn_into_scene search) under the device
    program: >= 10 % reach successful_grasp; every success transition is re-run by the oracle
    from the device's pre-step fp64 state, bit-exact."""
    if not gpu_available():
        pytest.skip("no GPU")
    import bench
    import oracle_lib
    s = gm.canonical_settings(noise=False, seed=SEED)
    env = gm.BatchedGripperEnv(N_GPU, object_set="set6_synthetic", settings=s, seed=SEED)
    try:
        env.set_scene_spawn(bench.mjenv_spawn_params(gm), max_tries=3)
        env.reset()
        isg = gm.BINARY_EVENTS.index("successful_grasp")
        success_env = np.zeros(N_GPU, dtype=bool)
        ever_done = np.zeros(N_GPU, dtype=bool)
        n_act_checked = 0
        for t in range(STEPS_GPU):
            pre = env.env_states()
            acts = env.program_actions(seed=SEED, mode=3)
            if t in (0, 40, 80):
                # the oracle's driver picks the device's actions from the same states
                sub = np.arange(0, N_GPU, 16)
                for j in sub:
                    oe = oracle_lib.OracleEnv(env.model, env.cfg, env.objects, int(j))
                    oe.import_state(pre[j])
                    np.testing.assert_array_equal(oe.driver_actions(mode=3, seed=SEED, gid=int(j)), acts[j])
                n_act_checked += len(sub)
            obs, rew, term, trunc = env.step(acts)
            post = env.env_states()
            vpost = gm.env_state_view(post)
            succ = term & (vpost["bev_last"][:, isg] > 0) & ~ever_done
            idx = np.nonzero(succ)[0]
            if len(idx):
                # the oracle re-runs each success transition from the device's pre-step state
                o_obs, o_rew, o_done, o_st = oracle_lib.batch_step(env.model, env.cfg, env.objects, pre[idx], acts[idx])
                np.testing.assert_array_equal(o_done, np.ones(len(idx), dtype=np.uint8))
                np.testing.assert_allclose(o_rew, rew[idx], rtol=1e-5, atol=1e-6)
                vo = gm.env_state_view(o_st)
                for f in ("bev_value", "bev_row", "bev_abs", "bev_last", "num_action_steps", "done"):
                    np.testing.assert_array_equal(vo[f], vpost[f][idx], err_msg=f)
                np.testing.assert_allclose(vo["cumulative_reward"], vpost["cumulative_reward"][idx], rtol=1e-6)
                assert (o_rew > 0.95).all(), o_rew.min()
                success_env[idx] = True
            ever_done |= term
            if term.any():
                env.reset(mask=term)      # next episodes run on; only first episodes are counted
        n_succ = int(success_env.sum())
        print(f"program successes {n_succ} / {N_GPU} first episodes; done {int(ever_done.sum())}")
        assert n_succ >= 0.10 * N_GPU, n_succ
        assert n_act_checked >= 3 * 256
    finally:
        env.close()


@pytest.mark.gpu
def test_gpu_bench_mix_records_successes(gm):
    """The benchmark's mode-4 mix through the fused rollout: the episode-end records carry
    successes (the collective's success byte), and each one is an episode the program drove."""
    if not gpu_available():
        pytest.skip("no GPU")
    import torch
    import bench
    from gmx.shard import unpack_episodes
    s = gm.canonical_settings(noise=True, seed=SEED)
    n, steps = 4096, 200
    env = gm.BatchedGripperEnv(n, object_set="set6_synthetic", settings=s, seed=SEED)
    try:
        env.set_scene_spawn(bench.mjenv_spawn_params(gm), max_tries=3)
        env.reset()
        rec = torch.zeros((steps, n, 3), dtype=torch.int32, device="cuda")
        env.rollout(steps, action_mode=4, seed=SEED, jitter=0.2, max_episode_steps=250, records_dev_ptr=rec.data_ptr())
        torch.cuda.synchronize()
        ret, length, success = unpack_episodes(rec.reshape(-1, 3).cpu())
        n_succ = int(success.sum())
        print(f"mode-4 rollout: {int((length > 0).sum())} episodes, {n_succ} successes")
        assert n_succ > 0.02 * n, n_succ
        assert (ret[success.bool()] > 0.5).all()
    finally:
        env.close()
