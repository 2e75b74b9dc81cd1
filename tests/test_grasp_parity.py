"""GPU parity on grasp-phase states at the BASELINE configs (C3: 4096 envs, set6-like
mixed objects, randomised spawn; C2: 256 envs, one cylinder).

A scripted grasp mix (gmx.GraspScript: close, squeeze, palm press, lift, with jitter)
drives the whole batch on the device.  At several episode phases the fp64 device state
of every env is handed to the CPU oracle verbatim (gm_get_env_states ->
or_import_state), both run the same env-step, and the results are compared:

- observations: max rel-err <= 1e-4 over |ref| >= 1e-3, abs <= 1e-4 elsewhere
  (BASELINE.json north star) for every env;
- done flags, event rows / abs counters, stepper step counts: bit-exact;
- reward: |d| <= 1e-6 + 1e-5 |r| (a float sum of the same terms);
- one MjClass::step (substep) from the same states: contact pair ids bit-exact, contact
  geometry, constraint forces, accelerations and the object's cfrc_ext to ~1e-12 (both
  sides fp64; the device physics fuses multiply-adds, the oracle does not), and the
  contact-force-sum invariant of
  ObjectHandler::check_contact_forces (objecthandler.cpp:994-1032, tol 1e-5).

The batch is asserted to contain the hard cases: finger-object contacts, constraint
problems with nefc > 32 (multi-contact box manifolds), event rows that fire, and done == 1.
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu

OBS_RTOL = 1e-4
OBS_ATOL = 1e-4
SNAPS = (22, 38, 45, 52, 60, 68)


def obs_err(a, b):
    """per-env (max rel over |ref| >= 1e-3, max abs elsewhere)"""
    a = np.asarray(a, dtype=np.float64); b = np.asarray(b, dtype=np.float64)
    big = np.abs(b) >= 1e-3
    d = np.abs(a - b)
    rel = np.where(big, d / np.where(big, np.abs(b), 1.0), 0.0).max(axis=1)
    ab = np.where(big, 0.0, d).max(axis=1)
    return rel, ab


@pytest.fixture(scope="module")
def ol():
    if not gpu_available():
        pytest.skip("no GPU")
    import oracle_lib
    return oracle_lib


def rollout(gm, n_envs, object_set, seed, steps=max(SNAPS) + 1, snaps=SNAPS, tweak=None, model_params=None):
    settings = gm.canonical_settings(noise=False, seed=seed)
    if tweak is not None:
        tweak(settings)
    env = gm.BatchedGripperEnv(n_envs, object_set=object_set, settings=settings, seed=seed, model_params=model_params)
    env.set_scene_spawn(gm.default_spawn_params(), max_tries=3)
    env.reset()
    script = gm.GraspScript(settings, n_envs, seed=seed)
    out = []
    for k in range(steps):
        a = script.actions(k)
        if k in snaps:
            # the device driver (gm_scripted_actions) is the host script bit for bit
            np.testing.assert_array_equal(env.scripted_actions(seed), a)
        rec = env.env_states() if k in snaps else None
        obs, rew, _, _ = env.step(a)
        if rec is not None:
            _, done = env.reward_done()
            out.append(dict(k=k, rec=rec, a=a, obs=obs, rew=rew, done=done, after=env.env_states()))
    return env, out


def compare_step(gm, ol, env, snap):
    obs_o, rew_o, done_o, after_o = ol.batch_step(env.model, env.cfg, env.objects, snap["rec"], actions=snap["a"])
    dv, ov = gm.env_state_view(snap["after"]), gm.env_state_view(after_o)
    rel, ab = obs_err(snap["obs"], obs_o)
    bad_obs = np.where((rel > OBS_RTOL) | (ab > OBS_ATOL))[0]
    # every env meets the bound: both sides run the same tree-ordered factor and solves,
    # the same sin/cos (gm_math.h) and the same converged Newton solve; they differ only by
    # the device's fused multiply-adds in the physics (~1e-12 per substep)
    assert bad_obs.size == 0, (
        f"step {snap['k']}: {bad_obs.size} envs exceed the obs bound, worst rel {rel.max():.3e} abs {ab.max():.3e} "
        f"(envs {bad_obs[:8]})")
    np.testing.assert_array_equal(snap["done"].astype(np.uint8), done_o, err_msg=f"done flags, step {snap['k']}")
    for f in ("bev_row", "bev_abs", "lev_row", "lev_abs", "num_action_steps", "old_x", "old_y", "old_z",
              "lock_active", "rng", "ring_i", "newton_caps"):
        np.testing.assert_array_equal(dv[f], ov[f], err_msg=f"{f}, step {snap['k']}")
    for g in ("end", "next"):
        for f in ("sx", "sy", "sz"):
            np.testing.assert_array_equal(dv[g][f], ov[g][f], err_msg=f"{g}.{f}, step {snap['k']}")
    np.testing.assert_allclose(snap["rew"], rew_o, rtol=1e-5, atol=1e-6, err_msg=f"reward, step {snap['k']}")
    # the physical state after 63 substeps: reported, bounded loosely (contact-rich
    # trajectories are chaotic at the ulp level; the obs bound above is the contract)
    dq = np.abs(dv["qpos"] - ov["qpos"]).max(axis=1)
    return dict(k=snap["k"], obs_rel=float(rel.max()), obs_abs=float(ab.max()), n_over=int(bad_obs.size),
                qpos_max=float(dq.max()), qpos_p99=float(np.percentile(dq, 99)), done=int(done_o.sum()))


def compare_substep(gm, ol, env, snap):
    env.set_env_states(snap["rec"])
    ncon, con, efc, qacc, nefc, w = env.debug_substep(full=True)
    after_d = env.env_states()
    ncon_o, nefc_o, con_o, efc_o, qacc_o, w_o, after_o = ol.batch_substep(env.model, env.cfg, env.objects, snap["rec"])
    np.testing.assert_array_equal(ncon, ncon_o, err_msg="contact counts")
    np.testing.assert_array_equal(nefc, nefc_o, err_msg="constraint row counts")
    np.testing.assert_array_equal(con[:, :, 13:15], con_o[:, :, 13:15], err_msg="contact pair ids")
    np.testing.assert_allclose(con[:, :, :13], con_o[:, :, :13], rtol=0, atol=1e-9, err_msg="contact geometry")
    fs = np.maximum(1.0, np.abs(efc_o).max(axis=1, keepdims=True))
    np.testing.assert_allclose(efc / fs, efc_o / fs, rtol=0, atol=1e-7, err_msg="efc_force")
    qs = np.maximum(1.0, np.abs(qacc_o).max(axis=1, keepdims=True))
    np.testing.assert_allclose(qacc / qs, qacc_o / qs, rtol=0, atol=1e-7, err_msg="qacc")
    np.testing.assert_allclose(w, w_o, rtol=0, atol=1e-7, err_msg="object cfrc_ext")
    # ObjectHandler::check_contact_forces: sum of the object's contact forces (global
    # frame, force on the object) == cfrc_ext force part, within 1e-5
    obj = env.model.ngeom - 1            # the live object's geom is the model's last (gm_build_model)
    fsum = np.zeros((env.n_envs, 3))
    for e in range(env.n_envs):
        for c in range(ncon[e]):
            g1, g2 = int(con[e, c, 13]), int(con[e, c, 14])
            s = 1.0 if g2 == obj else (-1.0 if g1 == obj else 0.0)
            if s == 0.0:
                continue
            Fr = con[e, c, 4:13].reshape(3, 3)
            fe = efc[e]
            base = nefc[e] - 4 * ncon[e] + 4 * c
            f_loc = np.array([fe[base:base + 4].sum(), con[e, c, 15] * (fe[base] - fe[base + 1]),
                              con[e, c, 15] * (fe[base + 2] - fe[base + 3])])
            fsum[e] += s * (Fr.T @ f_loc)
    assert np.abs(fsum - w[:, :3]).max() <= 1e-5, "contact-force sum differs from cfrc_ext"
    dv, ov = gm.env_state_view(after_d), gm.env_state_view(after_o)
    np.testing.assert_allclose(dv["qpos"], ov["qpos"], rtol=0, atol=1e-9, err_msg="qpos after one substep")
    # box-box manifolds (mjc_BoxBox): a finger/palm box against a box object with >= 2
    # contacts in one pair
    is_box = gm.env_state_view(snap["rec"])["obj_type"] == 6
    n_bb = 0
    for e in np.where(is_box)[0]:
        pairs = {}
        for c in range(ncon[e]):
            g1, g2 = int(con[e, c, 13]), int(con[e, c, 14])
            if (g1 == obj or g2 == obj) and 0 not in (g1, g2):
                pairs[(g1, g2)] = pairs.get((g1, g2), 0) + 1
        n_bb += any(v >= 2 for v in pairs.values())
    return dict(k=snap["k"], ncon_max=int(ncon.max()), nefc_max=int(nefc.max()), n_big=int((nefc > 32).sum()),
                n_boxbox_manifold_envs=int(n_bb),
                efc_err=float(np.abs((efc - efc_o) / fs).max()), qacc_err=float(np.abs((qacc - qacc_o) / qs).max()))


def check_config(gm, ol, n_envs, object_set, seed):
    env, snaps = rollout(gm, n_envs, object_set, seed)
    rep = []
    for sn in snaps:
        rep.append(compare_step(gm, ol, env, sn))
    sub = [compare_substep(gm, ol, env, sn) for sn in snaps]
    last = gm.env_state_view(snaps[-1]["after"])
    ev = {n: int((last["bev_row"][:, i] > 0).sum() + (last["bev_abs"][:, i] > 0).sum())
          for i, n in enumerate(gm.BINARY_EVENTS)}
    print(f"\n{object_set} x{n_envs}: step parity {rep}\nsubstep parity {sub}\nenvs with events {ev}")
    env.close()
    return rep, sub, last


def test_c3_grasp_states_4096(gm, ol):
    rep, sub, last = check_config(gm, ol, 4096, "set6_synthetic", seed=1234)
    i_oc = gm.BINARY_EVENTS.index("object_contact")
    assert (last["bev_abs"][:, i_oc] > 0).sum() > 1000, "too few envs reached finger-object contact"
    assert sum(r["done"] for r in rep) > 0, "no env reached done == 1"
    assert sum(s["n_big"] for s in sub) > 0, "no constraint problem with nefc > 32 was checked"
    assert sum(s["n_boxbox_manifold_envs"] for s in sub) > 100, "too few multi-point box-box grasps were checked"
    # every constraint solve of the rollout converged: no Newton solve ran out of
    # iterations (GM_NEWTON_MAXIT) and no line search out of evaluations (GM_NEWTON_MAXLS)
    assert int(last["newton_caps"].sum()) == 0, f"{int((last['newton_caps'] > 0).sum())} envs hit a solver cap"


def test_c2_single_cylinder_256(gm, ol):
    rep, sub, last = check_config(gm, ol, 256, "cylinder", seed=77)
    i_oc = gm.BINARY_EVENTS.index("object_contact")
    assert (last["bev_abs"][:, i_oc] > 0).sum() > 64


def test_long_sensor_history_512(gm, ol):
    """Histories beyond the canonical 3 steps (sensor and state windows of 8 previous
    steps, 17 readings deep, on the GM_RING = 64 windows): the observation, events and
    done flags still match the oracle on grasp states."""
    def longer(s):
        s.sensor_n_prev_steps = 8
        s.state_n_prev_steps = 8
    env, snaps = rollout(gm, 512, "set6_synthetic", 4321, steps=53, snaps=(12, 30, 52), tweak=longer)
    assert env.cfg.n_obs > gm.ConfigBlob(gm.canonical_settings(seed=1), env.model).n_obs
    rep = [compare_step(gm, ol, env, sn) for sn in snaps]
    print("long history", rep)
    env.close()


def test_ten_segment_fingers_256(gm, ol):
    """N = 10 finger segments (the top of the reference's range: 44 dofs, 75 candidate
    pairs -> the collision phase's second 64-pair batch) at the timestep the search gives
    for it, on grasp states: same bounds as the canonical N = 8 batch."""
    import ctypes as C
    p = gm.ModelParams()
    gm.load_library().gm_default_model_params(C.byref(p))
    p.n_seg, p.timestep = 10, 2.1e-3
    env, snaps = rollout(gm, 256, "set6_synthetic", 99, steps=53, snaps=(20, 38, 52), model_params=p)
    assert env.model.nv == 44 and env.cfg.sim_steps_per_action == 96
    rep = [compare_step(gm, ol, env, sn) for sn in snaps]
    sub = [compare_substep(gm, ol, env, sn) for sn in snaps]
    print("N=10", rep, sub)
    last = gm.env_state_view(snaps[-1]["after"])
    i_oc = gm.BINARY_EVENTS.index("object_contact")
    assert (last["bev_abs"][:, i_oc] > 0).sum() > 32
    env.close()


def test_c3_newton_matches_converged_pgs_4096(gm, ol):
    """The constraint solve is converged: the device's Newton solver and the oracle's dense
    PGS run to 800 sweeps (MuJoCo's PGS contract, a different algorithm on the same
    regularised problem, which has one optimum) give the same observations, 1e-4 for every
    env of the C3 batch on grasp states."""
    env, snaps = rollout(gm, 4096, "set6_synthetic", 1234, steps=53, snaps=(52,))
    sn = snaps[0]
    with ol.pgs_solver(800):
        obs_p, rew_p, done_p, _ = ol.batch_step(env.model, env.cfg, env.objects, sn["rec"], actions=sn["a"])
    rel, ab = obs_err(sn["obs"], obs_p)
    bad = np.where((rel > OBS_RTOL) | (ab > OBS_ATOL))[0]
    print(f"\nNewton (device) vs PGS-800 (oracle): max rel {rel.max():.3e}, abs {ab.max():.3e}, over {bad.size}")
    assert bad.size == 0, (bad[:8], rel.max(), ab.max())
    np.testing.assert_array_equal(sn["done"].astype(np.uint8), done_p)
    env.close()


@pytest.mark.parametrize("n_seg", [5, 6, 7, 9])
def test_other_segment_counts_256(gm, ol, n_seg):
    """N = 5, 6, 7, 9 segments (CL = 7, 8, 9, 11 builds of the step kernel) on grasp
    states, same bounds as the canonical batch.  N = 5, 6 run at the timestep the
    reference's search gives them; N = 7, 9 at a timestep inside their stable range
    (between their neighbours' searched steps)."""
    import ctypes as C
    p = gm.ModelParams()
    gm.load_library().gm_default_model_params(C.byref(p))
    p.n_seg, p.timestep = n_seg, {5: 6.76e-3, 6: 4.94e-3, 7: 3.9e-3, 9: 2.6e-3}[n_seg]
    env, snaps = rollout(gm, 256, "set6_synthetic", 40 + n_seg, steps=41, snaps=(20, 40), model_params=p)
    assert env.model.nv == 3 * (n_seg + 2) + 8
    rep = [compare_step(gm, ol, env, sn) for sn in snaps]
    sub = [compare_substep(gm, ol, env, sn) for sn in snaps]
    print(f"N={n_seg}", rep, sub)
    env.close()


def test_capped_newton_substep_matches_oracle_256(gm, ol):
    """A Newton solve that runs out of iterations (gm_model.newton_maxit = 1) on grasp
    states: mj_Euler integrates qfrc_smooth + J^T efc of the unconverged forces, not M qacc
    (the residual path of gm_newton.hip newton_solve / euler_damping).  Device and oracle
    take one substep from the same states: qpos and qvel after it to ~1e-9 (scaled), the
    capped-solve counters bit-exact, and most contact envs really capped."""
    import indep_physics as ip
    env, snaps = rollout(gm, 256, "set6_synthetic", 5, steps=53, snaps=(40, 52))
    capped = gm.ModelBlob(env.model.params)
    ip.GmModel.from_buffer(capped.buf).newton_maxit = 1
    cenv = gm.BatchedGripperEnv(256, settings=env.settings, seed=5, model_blob=capped, objects=env.objects)
    try:
        n_capped = 0
        rng = np.random.default_rng(8)
        for sn in snaps:
            # joint velocities kicked by N(0, 0.1): the warm start's active set is then not
            # the optimum's, and one iteration leaves the solve unconverged
            rec = np.array(sn["rec"], copy=True)
            rv = gm.env_state_view(rec)
            rv["qvel"][:, :env.model.nv] += rng.normal(0.0, 0.1, size=(len(rec), env.model.nv))
            cenv.set_env_states(rec)
            cenv.debug_substep(full=True)
            after_d = cenv.env_states()
            *_, after_o = ol.batch_substep(cenv.model, cenv.cfg, cenv.objects, rec)
            dv, ov, v0 = gm.env_state_view(after_d), gm.env_state_view(after_o), gm.env_state_view(rec)
            np.testing.assert_array_equal(dv["newton_caps"], ov["newton_caps"], err_msg="newton_caps")
            n_capped += int((ov["newton_caps"] > v0["newton_caps"]).sum())
            np.testing.assert_allclose(dv["qpos"], ov["qpos"], rtol=0, atol=1e-9, err_msg="qpos after a capped substep")
            vs = np.maximum(1.0, np.abs(ov["qvel"]).max(axis=1, keepdims=True))
            np.testing.assert_allclose(dv["qvel"] / vs, ov["qvel"] / vs, rtol=0, atol=1e-9,
                                       err_msg="qvel after a capped substep")
        assert n_capped > 100, n_capped
    finally:
        cenv.close()
        env.close()
