"""The mjpy.bind facade (drop-in for the reference's pybind11 `bind` module, MjEnv.py:18):
host-side surface on the CPU, and an MjEnv-style episode on the GPU checked against the
fp64 oracle step by step."""
import pickle

import numpy as np
import pytest

from conftest import gpu_available


def test_facade_surface_without_gpu(gm):
    from mjpy.bind import MjClass, EventTrack
    mj = MjClass()
    for name in ("set_continous_action", "set_discrete_action", "action_step", "get_observation_numpy",
                 "is_done", "reward", "reset", "hard_reset", "spawn_object", "spawn_into_scene",
                 "get_n_actions", "get_n_obs", "get_N", "set_finger_thickness", "set_base_XYZ_limits",
                 "get_event_state", "get_number_of_objects", "get_object_name", "load_relative"):
        assert callable(getattr(mj, name))
    assert hasattr(mj.default_spawn_params, "xrange")
    t = EventTrack()
    assert hasattr(t, "lifted") and hasattr(t, "exceed_limits")


def test_facade_settings_drive_sizes(gm):
    from mjpy.bind import MjClass
    mj = MjClass()
    mj.set = gm.canonical_settings(seed=2)
    assert mj.get_n_obs() == 63 and mj.get_n_actions() == 4
    assert mj.get_N() == 8
    mj.set_finger_thickness(1.0e-3)
    assert mj.get_finger_thickness() == pytest.approx(1.0e-3)


def test_facade_pickle_roundtrip(gm):
    from mjpy.bind import MjClass
    mj = MjClass()
    mj.set = gm.canonical_settings(seed=9)
    mj.object_set_name = "set1_synthetic"
    mj.default_spawn_params.xrange = 7e-3
    mj2 = pickle.loads(pickle.dumps(mj))
    assert bytes(mj2.set) == bytes(mj.set)
    assert mj2.object_set_name == "set1_synthetic"
    assert mj2.default_spawn_params.xrange == 7e-3


def test_facade_spawn_params_defaults(gm):
    """MjType::SpawnParams member defaults (mjclass.h:916-931)."""
    import math
    from mjpy.bind import MjClass
    p = MjClass().default_spawn_params
    assert (p.index, p.x, p.y, p.zrot, p.xrange, p.yrange, p.rotrange) == (-1, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)
    assert (p.xmin, p.xmax, p.ymin, p.ymax) == (-100, 100, -100, 100)
    assert p.smallest_gap == 1e-3 and p.xy_increment == 2e-3 and p.rot_increment == math.pi / 30.0


def test_facade_without_gpu_fails_loudly(gm):
    if gpu_available():
        pytest.skip("a GPU is present")
    from mjpy.bind import MjClass
    mj = MjClass()
    with pytest.raises(RuntimeError):
        mj.reset()


@pytest.mark.gpu
def test_facade_spawn_into_scene_matches_oracle(gm):
    """MjEnv._spawn_object's call (MjEnv.py:1211-1223): default_spawn_params with 10 mm
    xy noise and pi/2 rotation range, spawn_into_scene(idx) -> True, pose as the oracle."""
    import oracle_lib
    from mjpy.bind import MjClass
    mj = MjClass()
    mj.set = gm.canonical_settings(noise=False, seed=6)
    mj.reset()
    mj.default_spawn_params.xrange = mj.default_spawn_params.yrange = 10e-3
    mj.default_spawn_params.rotrange = np.pi / 2.0
    assert mj.spawn_into_scene(2) is True
    env = mj._env
    o = oracle_lib.OracleEnv(env.model, env.cfg, env.objects, 0)
    sp = gm.Spawn()
    sp.object_index, sp.x, sp.y, sp.zrot = 0, 0.0, 0.0, 0.0
    o.reset(sp)
    p = gm.default_spawn_params()
    p.index, p.xrange, p.yrange, p.rotrange = 2, 10e-3, 10e-3, np.pi / 2.0
    assert o.spawn_into_scene(p)
    q, _, _ = env.state()
    qo, _, _ = o.state()
    qa = env.model.nq - 7
    np.testing.assert_array_equal(q[0][qa:qa + 7], qo[qa:qa + 7])


@pytest.mark.gpu
def test_facade_episode_matches_oracle(gm):
    """MjEnv._set_action / _take_action / _next_observation / _is_done / _reward order
    (MjEnv.py:585-637, 2170-2220) through the facade vs the oracle, noise off."""
    import oracle_lib
    from mjpy.bind import MjClass
    mj = MjClass()
    mj.set = gm.canonical_settings(noise=False, seed=4)
    mj.object_set_name = "set1_synthetic"
    mj.reset()
    mj.spawn_object(0, 0.06, 0.06, 0.0)
    env = mj._env
    o = oracle_lib.OracleEnv(env.model, env.cfg, env.objects, 0)
    sp = gm.Spawn()
    sp.object_index, sp.x, sp.y, sp.zrot = 0, 0.06, 0.06, 0.0
    o.reset(sp)
    rng = np.random.default_rng(3)
    for t in range(10):
        a = rng.uniform(-1, 1, size=mj.get_n_actions()).astype(np.float32)
        for i, f in enumerate(a):
            mj.set_continous_action(i, float(f))
        mj.action_step()
        obs = mj.get_observation_numpy()
        done = mj.is_done()
        r = mj.reward()
        ro, rr, rd = o.step(a)
        d = np.abs(obs - ro)
        big = np.abs(ro) >= 1e-3
        assert (d[big] / np.abs(ro[big])).max(initial=0) <= 1e-4 and d[~big].max(initial=0) <= 1e-4
        assert done == rd
        assert r == pytest.approx(rr, rel=1e-4, abs=1e-6)
    ev = mj.get_event_state()
    assert isinstance(ev.lifted.row, int)


@pytest.mark.gpu
def test_facade_hard_reset_drops_the_cached_transition(gm):
    """get_observation_numpy caches the transition's (reward, done) for MjEnv's next
    is_done() / reward(); a hard_reset (a fresh context) must not answer with the old env's
    done flag."""
    if not gpu_available():
        pytest.skip("no GPU")
    from mjpy.bind import MjClass
    mj = MjClass()
    mj.set = gm.canonical_settings(noise=False, seed=4)
    mj.set.step_num.done = 1          # every env-step ends the episode
    mj.set.step_num.trigger = 1
    mj.object_set_name = "set1_synthetic"
    mj.reset()
    for i in range(mj.get_n_actions()):
        mj.set_continous_action(i, 0.0)
    mj.action_step()
    mj.get_observation_numpy()
    assert mj.is_done()
    mj.hard_reset()
    assert not mj.is_done()
    mj._drop()
