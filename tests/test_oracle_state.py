"""CPU: the oracle's fp64 state hand-off (GmEnvState import / export) is lossless -- an
oracle env resumed from an exported record continues bit-for-bit like the original.
This is what lets the GPU parity tests start the oracle from exactly the device state
at any phase of an episode (grasp, squeeze, lift)."""
import numpy as np

import oracle_lib


def test_export_import_resumes_bit_exact(gm, model):
    s = gm.canonical_settings(noise=True, seed=11)   # noise on: RNG stream must carry over too
    cfg = gm.ConfigBlob(s, model)
    objs = gm.make_object_set("set6_synthetic", 1234)
    sc = gm.GraspScript(s, 1, seed=3, jitter=0.3)
    a = oracle_lib.OracleEnv(model, cfg, objs, env_id=7)
    sp = gm.Spawn(); sp.object_index = 4; sp.x = 0.004; sp.y = -0.003; sp.zrot = 0.2
    a.reset(sp)
    for k in range(40):
        a.step(sc.actions(k)[0])
    rec = a.export_state()
    assert rec.size == oracle_lib.lib().or_state_size()
    b = oracle_lib.OracleEnv(model, cfg, objs, env_id=0)
    b.import_state(rec)
    np.testing.assert_array_equal(b.export_state(), rec)
    for k in range(40, 52):
        act = sc.actions(k)[0]
        oa, ra, da = a.step(act)
        ob, rb, db = b.step(act)
        np.testing.assert_array_equal(oa, ob)
        assert ra == rb and da == db
    np.testing.assert_array_equal(a.export_state(), b.export_state())


def test_batch_step_matches_single_env(gm, model):
    s = gm.canonical_settings(noise=False, seed=2)
    cfg = gm.ConfigBlob(s, model)
    objs = gm.make_object_set("set6_synthetic", 1234)
    sc = gm.GraspScript(s, 3, seed=5)
    recs, envs = [], []
    for e in range(3):
        o = oracle_lib.OracleEnv(model, cfg, objs, env_id=e)
        sp = gm.Spawn(); sp.object_index = e; sp.x = 0.0; sp.y = 0.0; sp.zrot = 0.0
        o.reset(sp)
        for k in range(36):
            o.step(sc.actions(k)[e])
        recs.append(o.export_state()); envs.append(o)
    acts = sc.actions(36)
    obs, rew, done, after = oracle_lib.batch_step(model, cfg, objs, np.stack(recs), actions=acts, threads=2)
    for e, o in enumerate(envs):
        ob, r, d = o.step(acts[e])
        np.testing.assert_array_equal(obs[e], ob)
        assert rew[e] == np.float32(r) and bool(done[e]) == d
        np.testing.assert_array_equal(after[e], o.export_state())
