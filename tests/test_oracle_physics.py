"""Physical invariants of the fp64 oracle's engine: these pin
the restated MuJoCo pipeline where no reference vector can (MuJoCo 2.1.5 and the MJCF
are absent: physics parity against MuJoCo itself is unpinned)."""
import numpy as np
import pytest

import oracle_lib

G = 9.81


@pytest.fixture(scope="module")
def world(gm):
    s = gm.canonical_settings(noise=False, seed=3)
    model = gm.ModelBlob()
    cfg = gm.ConfigBlob(s, model)
    objs = gm.make_object_set("set1_synthetic", 3)
    return gm, model, cfg, objs


def make_env(world, idx=0, x=0.0, y=0.0, env_id=0):
    gm, model, cfg, objs = world
    e = oracle_lib.OracleEnv(model, cfg, objs, env_id)
    sp = gm.Spawn()
    sp.object_index, sp.x, sp.y, sp.zrot = idx, x, y, 0.0
    e.reset(sp)
    return e


def test_deterministic(world):
    a = make_env(world, 1)
    b = make_env(world, 1)
    rng = np.random.default_rng(0)
    for _ in range(5):
        act = rng.uniform(-1, 1, size=4).astype(np.float32)
        oa, ra, da = a.step(act)
        ob, rb, db = b.step(act)
        np.testing.assert_array_equal(oa, ob)
        assert ra == rb and da == db


def test_semi_implicit_euler_free_fall(world):
    """Object lifted clear of everything: v_k = -g h k, z_k = z0 - g h^2 k(k+1)/2."""
    _, model, cfg, _ = world
    e = make_env(world, 0)
    q, v, _ = e.state()
    qa = model.dof_obj            # every earlier joint is 1-dof, so qposadr == dofadr here
    q = q.copy(); v = np.zeros_like(v)
    q[qa + 2] = 0.5
    e.set_state(q, v)
    h = 3.187e-3
    for k in range(1, 11):
        e.debug_substep()
        q2, v2, _ = e.state()
        assert v2[model.dof_obj + 2] == pytest.approx(-G * h * k, rel=1e-12)
        assert q2[qa + 2] == pytest.approx(0.5 - G * h * h * k * (k + 1) / 2, rel=1e-12)


def test_resting_object_contact_forces_carry_its_weight(world):
    """Contact-force-sum invariant (objecthandler.cpp:994-1032): a box resting on the
    ground, clear of the fingers, is held up by normal forces summing to m g."""
    gm, model, cfg, objs = world
    box = [i for i, o in enumerate(objs) if o.type == 6][0]
    e = make_env(world, box)
    zero = np.zeros(cfg.n_actions, dtype=np.float32)
    for _ in range(10):
        e.step(zero)
    n, con, f, _ = e.debug_substep()
    obj_geom = model.ngeom - 1
    ground_rows = [c for c in range(n) if int(con[c][13]) == 0 and int(con[c][14]) == obj_geom]
    assert ground_rows, "box should touch the ground"
    assert len(ground_rows) == n, "box should touch nothing but the ground"
    # constraint rows: active motor locks first, then 4 pyramid edges per contact;
    # a contact's normal force is the sum of its edge forces (mj_contactForce)
    nefc = int(np.max(np.nonzero(f)[0]) + 1)
    r0 = nefc - 4 * n
    total = sum(float(f[r0 + 4 * c: r0 + 4 * c + 4].sum()) for c in ground_rows)
    m = objs[box].mass
    assert total == pytest.approx(m * G, rel=2e-2)


def test_gripper_at_rest_reads_near_zero_bend(world):
    """With no contact the finger gauges read only the settled self-weight bend."""
    e = make_env(world, 2)
    obs = None
    for _ in range(3):
        obs, _, _ = e.step(np.zeros(4, dtype=np.float32))
    assert np.all(np.abs(obs[:21]) < 0.05)


def test_motor_locks_equal_the_reference_weld():
    """The reference holds a stopped motor with a weld equality between the slide's two
    bodies (myfunctions.cpp:1177-1279): 6 rows, of which only the translational ones
    along the slide axis have a nonzero Jacobian, each with its own impedance and the
    weld's regulariser (the bodies' translational body_invweight0).  The engine folds
    them into one row on the slide dof; an oracle variant that keeps the weld's rows
    separate gives the same rollout (scripted grasps on set6 objects)."""
    import gmx
    import oracle_lib as ol
    n, steps = 12, 45
    settings = gmx.canonical_settings(noise=False, seed=1234)
    model = gmx.ModelBlob()
    cfg = gmx.ConfigBlob(settings, model)
    objs = gmx.make_object_set("set6_synthetic", 1234)

    def roll(weld):
        if weld:
            with ol.weld_locks():
                envs = [ol.OracleEnv(model, cfg, objs, e) for e in range(n)]
        else:
            envs = [ol.OracleEnv(model, cfg, objs, e) for e in range(n)]
        si, sx, sy, sr = gmx.env.spawn_draws(1234, np.arange(n), np.ones(n, dtype=np.int64), len(objs))
        for e, o in enumerate(envs):
            o.reset(gmx.Spawn(int(si[e]), float(sx[e]), float(sy[e]), float(sr[e])))
        script = gmx.GraspScript(settings, n, seed=1234)
        obs, done = [], []
        for k in range(steps):
            a = script.actions(k)
            out = [o.step(a[e]) for e, o in enumerate(envs)]
            obs.append([x[0] for x in out])
            done.append([x[2] for x in out])
        st = gmx.env_state_view(np.stack([o.export_state() for o in envs]))
        return np.array(obs), np.array(done), st

    o1, d1, s1 = roll(False)
    o2, d2, s2 = roll(True)
    assert (s1["lock_active"].sum() > 0) and (s1["lock_active"] == s2["lock_active"]).all()
    np.testing.assert_array_equal(d1, d2)
    np.testing.assert_allclose(o1, o2, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(s1["qpos"], s2["qpos"], rtol=0, atol=1e-9)
