"""MjClass::spawn_into_scene (mjclass.cpp:2475-2654): shuffled xy / rotation grids on the
env's RNG stream, Box2d rejection against the scene bounds and the initial fingertip
boxes (Env::reset, mjclass.h:895-904; get_finger_hook_locations, myfunctions.cpp:3717-3761).

CPU tests pin the oracle's restatement (its std::shuffle and Box2d pieces are pinned
bit-exactly in test_oracle_golden.py); the gpu test checks the device search against
the oracle pose for pose, bit-exact (grid indices, success flags, RNG stream position).
"""
import math

import numpy as np
import pytest

import oracle_lib
from conftest import gpu_available


@pytest.fixture(scope="module")
def world(gm):
    s = gm.canonical_settings(noise=False, seed=11)
    model = gm.ModelBlob()
    cfg = gm.ConfigBlob(s, model)
    objs = gm.make_object_set("set6_synthetic", 11)
    return gm, model, cfg, objs


def fresh(world, env_id=0):
    gm, model, cfg, objs = world
    e = oracle_lib.OracleEnv(model, cfg, objs, env_id)
    sp = gm.Spawn()
    sp.object_index, sp.x, sp.y, sp.zrot = 0, 0.0, 0.0, 0.0
    e.reset(sp)
    return e


def mjenv_params(gm, index):
    """default_spawn_params as MjEnv._spawn_object sets them (MjEnv.py:1213-1215):
    object_position_noise_mm = 10, rotrange = pi / 2."""
    p = gm.default_spawn_params()
    p.index = index
    p.xrange = p.yrange = 10e-3
    p.rotrange = np.pi / 2.0
    return p


def bbox(o):
    if o.type == 0:  # GM_GEOM_BOX
        return 2 * o.size[0], 2 * o.size[1]
    return 2 * o.size[0], 2 * o.size[0]


def tip_boxes(model, end_x, base_x=0.0, base_y=0.0):
    """get_finger_hook_locations + Env::reset, restated independently of the oracle."""
    P = model.params
    hook_x = 0.5 * P.hook_length * math.sin(P.hook_angle_degrees * (math.pi / 180.0))
    out = []
    for ang in (0.0, math.pi * (2.0 / 3.0), 2 * math.pi * (2.0 / 3.0)):
        x = -(end_x - hook_x) * math.sin(ang) + base_x
        y = -(end_x - hook_x) * math.cos(ang) + base_y
        out.append((x, y, P.finger_width, P.hook_length, -ang))
    return out


def obj_pose(e, model):
    q, _, _ = e.state()
    qa = model.nq - 7
    return q[qa:qa + 7]


def test_default_mjenv_spawn_lands_on_grid(world):
    gm, model, cfg, objs = world
    for idx in range(len(objs)):
        e = fresh(world, env_id=idx)
        p = mjenv_params(gm, idx)
        assert e.spawn_into_scene(p)
        x, y = obj_pose(e, model)[:2]
        kx, ky = (x + p.xrange) / p.xy_increment, (y + p.yrange) / p.xy_increment
        assert abs(kx - round(kx)) < 1e-9 and abs(ky - round(ky)) < 1e-9
        assert abs(x) <= p.xrange + 1e-12 and abs(y) <= p.yrange + 1e-12


def test_accepted_poses_clear_fingertips_and_bounds(world):
    """A wide grid reaching the fingertips: every accepted pose passes the rules the
    reference applies, re-checked here with an independent fingertip construction."""
    gm, model, cfg, objs = world
    accepted = 0
    for trial in range(24):
        idx = trial % len(objs)
        e = fresh(world, env_id=100 + trial)
        end_x = e.target()[0][0]
        p = mjenv_params(gm, idx)
        p.xrange = p.yrange = 0.075
        p.xy_increment = 5e-3
        p.xmin, p.xmax, p.ymin, p.ymax = -0.09, 0.09, -0.09, 0.09
        p.smallest_gap = 5e-3
        ok = e.spawn_into_scene(p)
        if not ok:
            continue
        accepted += 1
        pose = obj_pose(e, model)
        x, y = pose[:2]
        # rotation: spawn_object composes q = (sin(-z/2), 0, 0, cos(-z/2)) in (w, x, y, z) slots
        zrot = -2.0 * math.atan2(pose[3], pose[6])
        w, h = bbox(objs[idx])
        ob = (x, y, w, h, zrot)
        for tb in tip_boxes(model, end_x):
            assert not oracle_lib.box2d_overlaps(ob, tb, p.smallest_gap)
        c, s = math.cos(zrot), math.sin(zrot)
        for sx, sy in ((-1, -1), (1, -1), (1, 1), (-1, 1)):
            cx = x + sx * w / 2 * c - sy * h / 2 * s
            cy = y + sx * w / 2 * s + sy * h / 2 * c
            assert p.xmin - 1e-9 <= cx <= p.xmax + 1e-9 and p.ymin - 1e-9 <= cy <= p.ymax + 1e-9
    assert accepted >= 20


def test_no_free_pose_returns_false_and_keeps_the_object(world):
    gm, model, cfg, objs = world
    e = fresh(world)
    before = obj_pose(e, model).copy()
    p = mjenv_params(gm, 3)
    p.xmin, p.xmax, p.ymin, p.ymax = -1e-3, 1e-3, -1e-3, 1e-3   # no object fits
    assert not e.spawn_into_scene(p)
    np.testing.assert_array_equal(obj_pose(e, model), before)


def test_search_is_deterministic_per_stream(world):
    gm, model, cfg, objs = world
    poses = []
    for _ in range(2):
        e = fresh(world, env_id=7)
        assert e.spawn_into_scene(mjenv_params(gm, 2))
        poses.append(obj_pose(e, model))
    np.testing.assert_array_equal(poses[0], poses[1])
    other = fresh(world, env_id=8)
    assert other.spawn_into_scene(mjenv_params(gm, 2))


@pytest.mark.gpu
def test_gpu_spawn_into_scene_matches_oracle(world):
    """Device search vs oracle, env by env: same success flags, the same grid pose
    (object qpos, fp64 readback), and the same RNG position afterwards (the next
    reset's noise draws give identical observations)."""
    if not gpu_available():
        pytest.skip("no GPU")
    gm, model, cfg, objs = world
    n = 64
    s = gm.canonical_settings(noise=True, seed=11)
    env = gm.BatchedGripperEnv(n, object_set="set6_synthetic", settings=s, seed=11)
    sp = env.make_spawn(idx=0, x=0.0, y=0.0, rot=0.0)
    env.reset(spawn=sp)
    params = []
    for e in range(n):
        p = mjenv_params(gm, e % len(env.objects))
        if e % 2:
            p.xrange = p.yrange = 0.075
            p.xy_increment = 5e-3
            p.xmin, p.xmax, p.ymin, p.ymax = -0.09, 0.09, -0.09, 0.09
            p.smallest_gap = 5e-3
        if e % 16 == 5:
            p.xmin, p.xmax = -1e-3, 1e-3
        params.append(p)
    ok = env.spawn_into_scene(params)
    q, _, _ = env.state()
    qa = env.model.nq - 7
    oracles = []
    for e in range(n):
        o = oracle_lib.OracleEnv(env.model, env.cfg, env.objects, env_id=e)
        o.reset(sp[e])
        ok_ref = o.spawn_into_scene(params[e])
        assert bool(ok[e]) == ok_ref, e
        qo, _, _ = o.state()
        np.testing.assert_array_equal(q[e][qa:qa + 7], qo[qa:qa + 7], err_msg=f"env {e}")
        oracles.append(o)
    assert (~ok).sum() >= n // 16
    # RNG stream position: the sensor noise of the next env-step comes from the same
    # stream on both sides (a different position would differ by the noise magnitude)
    a = np.zeros((n, env.n_actions), dtype=np.float32)
    obs, _, _, _ = env.step(a)
    for e in range(0, n, 4):
        ro, _, _ = oracles[e].step(a[e])
        np.testing.assert_allclose(obs[e], ro, rtol=1e-4, atol=1e-4, err_msg=f"env {e}")
    env.close()


def grid_params(gm, index, grid):
    """MjEnv's spawn params; large grids (31 x 31 = 961 xy points, 181 rotations); or grids
    at exactly the reset kernel's LDS shuffle-buffer capacity, where an off-by-one would
    overrun them (32 x 32 = GM_SPAWN_MAX_XY = 1024 xy points, GM_SPAWN_MAX_ROT = 256
    rotations: an even count, so the shuffle's leading single swap runs at the bound)."""
    p = mjenv_params(gm, index)
    if grid == "max":
        p.xrange = p.yrange = 15e-3
        p.xy_increment = 1e-3
        p.rot_increment = np.pi / 180.0
    elif grid == "exact":
        p.xrange = p.yrange = 15.5e-3   # 2 r / inc + 1 = 32.0 exactly (the host check bounds the product)
        p.xy_increment = 1e-3
        p.rot_increment = np.pi / 255.3
    return p


def grid_counts(p):
    """spawn_into_scene's grid sizes, truncated as the device and the oracle do (double)"""
    nx = int(2 * p.xrange / p.xy_increment + 1)
    ny = int(2 * p.yrange / p.xy_increment + 1)
    return nx * ny, int(2 * p.rotrange / p.rot_increment + 1)


@pytest.mark.gpu
@pytest.mark.parametrize("grid", ["mjenv", "max", "exact"])
def test_gpu_reset_with_scene_spawn_matches_oracle(world, grid):
    """gm_set_scene_spawn: resets place objects the MjEnv._spawn_object way
    (MjEnv.py:1177-1267) on the device -- reset, then spawn_into_scene(spawn[e].index) --
    pose for pose, and leave the RNG stream where the oracle's is (sensor noise on: the
    next env-step's observations agree)."""
    if not gpu_available():
        pytest.skip("no GPU")
    gm, model, cfg, objs = world
    n = 32
    s = gm.canonical_settings(noise=True, seed=12)
    env = gm.BatchedGripperEnv(n, object_set="set6_synthetic", settings=s, seed=12)
    p = grid_params(gm, 0, grid)
    nxy, nr = grid_counts(p)
    if grid == "max":
        assert 900 < nxy <= 1024 and 150 < nr <= 256, (nxy, nr)
    elif grid == "exact":
        assert (nxy, nr) == (1024, 256), (nxy, nr)
    env.set_scene_spawn(p, max_tries=3)
    sp = env.make_spawn()
    env.reset(spawn=sp)
    q, _, _ = env.state()
    qa = env.model.nq - 7
    oracles = []
    for e in range(n):
        o = oracle_lib.OracleEnv(env.model, env.cfg, env.objects, env_id=e)
        o.reset(sp[e])
        pe = grid_params(gm, sp[e].object_index, grid)
        assert o.spawn_into_scene(pe)
        qo, _, _ = o.state()
        np.testing.assert_array_equal(q[e][qa:qa + 7], qo[qa:qa + 7], err_msg=f"env {e}")
        oracles.append(o)
    a = np.zeros((n, env.n_actions), dtype=np.float32)
    obs, _, _, _ = env.step(a)
    for e in range(0, n, 4):
        ro, _, _ = oracles[e].step(a[e])
        np.testing.assert_allclose(obs[e], ro, rtol=1e-4, atol=1e-4, err_msg=f"env {e}")
    env.set_scene_spawn(None)
    env.close()
