"""The drop-in facade under MjEnv's exact call sequences (rl/env/MjEnv.py), against the
oracle driven through the same sequence:

- _load_xml (MjEnv.py:417-448): load_relative, get_number_of_objects, the gripper
  dimension getters incl. is_finger_hook_fixed / using_xyz_base_actions, then
  set_base_XYZ_limits / set_base_yaw_limit (MjEnv's 300, 200 mm, pi/4; Z set to 20 mm);
- reset (2222-2263): mj.reset() then _spawn_object (1177-1267): generator-drawn object
  index, default_spawn_params ranges, spawn_into_scene up to 3 tries, the "old method"
  spawn_object fallback;
- step (2170-2220): set_continous_action(i, a_i) for every i, action_step,
  get_observation_numpy, is_done (with MjEnv's truncation), reward;
- test-mode reporting (1291): get_test_report at the end of an episode;
- _add_events / _calc_rewards (530-540): add_events, reward(event).
The base limits must reach the device: a base-Z action sequence that runs into the
20 mm limit clamps where the oracle (same limits) clamps.
"""
import math

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

BASE_LIM = (300e-3, 200e-3, 20e-3)    # MjEnv base_lim_{X,Y}_mm defaults, Z tightened to 20 mm
BASE_YAW = math.pi / 4


class MjEnvReplay:
    """The subset of MjEnv's control flow that touches the bind module, verbatim in
    order (parameters at MjEnv's defaults: object_position_noise_mm 10,
    object_rotation_noise_deg 5, max_episode_steps as given)."""

    def __init__(self, mj, max_episode_steps, seed):
        self.mj = mj
        self.max_episode_steps = max_episode_steps
        self.gen = np.random.default_rng(seed)
        self.current_step = 0
        self.cumulative_reward = 0.0

    def load_xml(self):
        mj = self.mj
        mj.load_relative("task/gripper_task_0.xml")
        self.num_objects = mj.get_number_of_objects()
        self.params = dict(object_set_name=mj.object_set_name, num_segments=mj.get_N(),
                           finger_width=mj.get_finger_width(), finger_thickness=mj.get_finger_thickness(),
                           finger_modulus=mj.get_finger_modulus(), finger_length=mj.get_finger_length(),
                           finger_hook_angle_degrees=mj.get_finger_hook_angle_degrees(),
                           fixed_finger_hook=mj.is_finger_hook_fixed(),
                           fingertip_clearance=mj.get_fingertip_clearance(),
                           XY_base_actions=mj.using_xyz_base_actions(),
                           finger_hook_length=mj.get_finger_hook_length())
        mj.set_base_XYZ_limits(*BASE_LIM)
        mj.set_base_yaw_limit(BASE_YAW)

    def spawn_object(self):
        g = self.gen
        obj_idx = int(g.integers(0, self.num_objects))
        self.mj.default_spawn_params.xrange = 10 * 1e-3
        self.mj.default_spawn_params.yrange = 10 * 1e-3
        self.mj.default_spawn_params.rotrange = np.pi / 2.0
        spawned, count = False, 0
        while not spawned and count < 3:
            spawned = self.mj.spawn_into_scene(obj_idx)
            count += 1
        fallback = None
        if not spawned:
            x_mm = int(g.integers(-10, 11)); y_mm = int(g.integers(-10, 11))
            noise = int(g.integers(-5, 6)); opt = int(g.integers(0, 3))
            z = ([0, 60, 120][opt] + noise) * (np.pi / 180.0)
            self.mj.spawn_object(obj_idx, x_mm * 1e-3, y_mm * 1e-3, z)
            fallback = (x_mm * 1e-3, y_mm * 1e-3, z)
        return obj_idx, spawned, fallback

    def reset(self):
        self.current_step = 0
        self.cumulative_reward = 0.0
        self.mj.reset()
        spawn = self.spawn_object()
        return self.mj.get_observation_numpy(), spawn

    def step(self, action):
        self.current_step += 1
        for i in range(len(action)):
            self.mj.set_continous_action(i, action[i])
        self.mj.action_step()
        obs = self.mj.get_observation_numpy()
        truncated = self.current_step >= self.max_episode_steps
        terminated = False if truncated else self.mj.is_done()
        reward = self.mj.reward()
        self.cumulative_reward += reward
        return obs, reward, terminated, truncated


def oracle_twin(gm, ol, mj, spawn_log, env_id=0):
    """The oracle with the facade's model, configuration (incl. base limits) and objects."""
    env = mj._env
    cfg = gm.ConfigBlob(mj.set, env.model)
    gm.load_library().gm_config_set_base_limits(cfg.ptr, *BASE_LIM, BASE_YAW)
    o = ol.OracleEnv(env.model, cfg, env.objects, env_id=env_id)
    o._cfg_keep = cfg
    return o


def oracle_reset(gm, o, spawn):
    obj_idx, spawned, fallback = spawn
    sp = gm.Spawn()
    sp.object_index, sp.x, sp.y, sp.zrot = 0, 0.0, 0.0, 0.0
    o.reset(sp)
    p = gm.default_spawn_params()
    p.index, p.xrange, p.yrange, p.rotrange = obj_idx, 10e-3, 10e-3, np.pi / 2.0
    ok = False
    for _ in range(3):
        ok = o.spawn_into_scene(p)
        if ok:
            break
    assert ok == spawned
    if fallback is not None:
        sp.object_index, sp.x, sp.y, sp.zrot = obj_idx, *fallback
        o.L.or_spawn(o.h, __import__("ctypes").byref(sp))


def obs_ok(a, b):
    a = np.asarray(a, dtype=np.float64); b = np.asarray(b, dtype=np.float64)
    big = np.abs(b) >= 1e-3
    d = np.abs(a - b)
    return (d[big] / np.abs(b[big])).max(initial=0) <= 1e-4 and d[~big].max(initial=0) <= 1e-4


def test_mjenv_sequences_through_facade(gm):
    if not gpu_available():
        pytest.skip("no GPU")
    import ctypes
    import oracle_lib as ol
    from mjpy.bind import MjClass
    ol.lib().or_spawn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    mj = MjClass()
    mj.set = gm.canonical_settings(noise=False, seed=17)
    mj.object_set_name = "set1_synthetic"
    rep = MjEnvReplay(mj, max_episode_steps=16, seed=99)
    rep.load_xml()
    assert rep.params["fixed_finger_hook"] is True and rep.params["XY_base_actions"] is False
    assert mj.get_base_limits() == (*BASE_LIM, BASE_YAW)
    rng = np.random.default_rng(3)
    o = None
    tracks = []
    for episode in range(2):
        obs, spawn = rep.reset()
        if o is None:
            o = oracle_twin(gm, ol, mj, spawn)
        oracle_reset(gm, o, spawn)
        np.testing.assert_array_equal(obs, o.observation())
        cum_o = 0.0
        for t in range(rep.max_episode_steps):
            a = rng.uniform(-1, 1, size=mj.get_n_actions()).astype(np.float32)
            if t >= 2:
                a[-1] = -1.0            # base_Z up into the 20 mm limit (clamped on both sides)
            obs, r, term, trunc = rep.step(a)
            ob_o, r_o, d_o = o.step(a)
            last_r_o = r_o                   # oracle calc_rewards over the track so far
            cum_o += r_o
            assert obs_ok(obs, ob_o), (episode, t)
            assert abs(r - r_o) <= 1e-6 + 1e-5 * abs(r_o), (episode, t, r, r_o)
            assert term == (d_o and not trunc)
            if term or trunc:
                break
        e_dev, es, ns, base = mj._env.target()
        _, _, _, base_o = o.target()
        assert base[0][2] == pytest.approx(-BASE_LIM[2]) and base_o[2] == pytest.approx(-BASE_LIM[2])
        report = mj.get_test_report()
        assert report.object_name == mj.get_object_name(spawn[0])
        assert report.cumulative_reward == pytest.approx(cum_o, rel=1e-5, abs=1e-6)
        rows_o, abs_o, _ = o.event_rows()
        nb = len(gm.BINARY_EVENTS)
        for i, n in enumerate(gm.BINARY_EVENTS):
            assert getattr(report.cnt, n).abs == abs_o[i]
        for i, n in enumerate(gm.LINEAR_EVENTS):
            assert getattr(report.cnt, n).row == rows_o[nb + i]
        tracks.append(report.cnt)
    total = mj.add_events(tracks[0], tracks[1])
    assert total.step_num.abs == tracks[0].step_num.abs + tracks[1].step_num.abs == 2 * rep.max_episode_steps
    # reward(event) == calc_rewards over the same track, computed by the oracle for the
    # last transition of the last episode
    ev = mj.get_event_state()
    assert mj.reward(ev) == pytest.approx(last_r_o, rel=1e-6, abs=1e-7)
    with pytest.raises(RuntimeError):
        mj.set_new_base_XY(0.01, 0.02)       # base XY joints are not in use (reference throws)
