"""Automatic calibration (MjClass::configure_settings auto flags, mjclass.cpp:241-308):
find_highest_stable_timestep (mjclass.cpp:4745-4854) and calibrate_simulated_sensors
(4643-4676, tip load via validate_curve_under_force 4023-4105).

The oracle runs the reference's sequential procedure; the device runs every search
candidate as its own env in one launch and replays the sequence (gm_calibrate).  The
engine integrates like MuJoCo 2.1.5's Euler (joint springs explicit, joint damping
implicit), so the search is a real one: it climbs in coarse steps until a candidate
goes unstable (mjWARN_BADQACC) and combs down in fine steps.  Its result is pinned to
the reference's own measured stable timesteps (rl/juypter/thesis_plots/
mujoco_timesteps.csv -> tests/golden/mujoco_timesteps.json).
"""
import json
import math
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle_lib
from conftest import gpu_available


@pytest.fixture(scope="module")
def world(gm):
    s = gm.canonical_settings(noise=False, seed=1)
    model = gm.ModelBlob()
    cfg = gm.ConfigBlob(s, model)
    objs = gm.make_object_set("set1_synthetic", 1)
    return gm, model, cfg, objs, s


def reference_search(stable):
    """find_highest_stable_timestep's control flow (mjclass.cpp:4751-4816) in float32
    over a stability predicate; returns (found, candidates)."""
    f = np.float32
    coarse, fine, start, maxdt = f(0.5e-3), f(50e-6), f(1.0e-3), f(20.0e-3)
    nxt, coarse_pass, seen = start, True, []
    while True:
        ok = stable(nxt)
        seen.append((float(nxt), not ok))
        if not ok:
            coarse_pass = False
            nxt = f(nxt - fine)
        elif coarse_pass:
            nxt = f(nxt + coarse)
        else:
            return nxt, seen
        if nxt < fine:
            raise RuntimeError("no stable timestep")
        if nxt > maxdt:
            nxt, coarse_pass = maxdt, False


def final_timestep(found):
    found = np.float32(found)
    factor = np.float32(0.8 if found <= 3.0e-3 else 0.75 if found < 5.0e-3 else 0.65)
    t = np.float32(found * factor)
    return float(np.float32(int(float(t) * 1e6) * 1e-6))


def test_oracle_timestep_search_follows_reference_sequence(world):
    gm, model, cfg, objs, s = world
    cal, trace = oracle_lib.calibrate(model, cfg, objs, 1)
    flags = {dt: bad for dt, bad in trace}
    found, seen = reference_search(lambda dt: not flags[float(dt)])
    assert seen == trace
    assert cal.search_timestep == float(found)
    assert cal.timestep == final_timestep(found)
    assert abs(cal.timestep * 1e6 - round(cal.timestep * 1e6)) < 1e-3      # whole microseconds
    assert cal.sim_steps_per_action == math.ceil(s.time_for_action / cal.timestep)


def test_oracle_gauge_calibration(world):
    """calibrate_simulated_sensors: saturation load = saturation_yield_factor x yield load
    (float, calc_yield_point_load); the gauge reads the settled bend of finger 0; the
    settled reading does not depend on the timestep the 50 s run used."""
    gm, model, cfg, objs, s = world
    from mjpy.bind import MjClass
    cal, _ = oracle_lib.calibrate(model, cfg, objs, 2)
    y = MjClass().yield_load()
    assert cal.yield_load == pytest.approx(y, rel=1e-7)
    assert cal.bend_gauge_normalise == pytest.approx(float(np.float32(s.saturation_yield_factor) * np.float32(y)), rel=1e-7)
    assert cal.bending_normalise > 0            # the load bends the finger outward (+ gauge)
    assert cal.sim_gauge_raw_to_N_factor == pytest.approx(cal.bend_gauge_normalise / cal.bending_normalise, rel=1e-6)
    assert cal.wrist_Z_offset == 0.0 and cal.gauge_retries == 0
    both, _ = oracle_lib.calibrate(model, cfg, objs, 3)
    assert both.bending_normalise == pytest.approx(cal.bending_normalise, rel=2e-3)


def test_configure_gauge_normalise_is_the_settled_simulation(world):
    """gm_configure's auto_calibrate_gauges value (the static equilibrium of the finger's
    joint chain under the saturation tip load, solved directly) equals what the reference's
    procedure reads after 50 s of simulation (the oracle's or_calibrate)."""
    import ctypes as C
    gm, model, cfg, objs, s = world
    cs = gm.Settings.from_buffer_copy(cfg.buf[:C.sizeof(gm.Settings)])
    cal, _ = oracle_lib.calibrate(model, cfg, objs, 2)
    assert cs.bending_gauge.normalise == pytest.approx(cal.bending_normalise, rel=1e-5)


@pytest.mark.gpu
def test_gpu_calibration_matches_oracle(world):
    """The batched device search simulates every candidate as one env and replays the
    reference's sequence: same candidates, same flags, same timestep bit for bit; the
    device gauge run matches the oracle's settled reading."""
    if not gpu_available():
        pytest.skip("no GPU")
    gm, model, cfg, objs, s = world
    dev, tr_d = gm.calibrate(model, cfg, objs, what=gm.CAL_TIMESTEP | gm.CAL_GAUGES)
    ref, tr_o = oracle_lib.calibrate(model, cfg, objs, 3)
    assert tr_d == tr_o
    assert dev.timestep == ref.timestep and dev.search_timestep == ref.search_timestep
    assert dev.sim_steps_per_action == ref.sim_steps_per_action and dev.n_tested == ref.n_tested
    assert dev.yield_load == ref.yield_load and dev.bend_gauge_normalise == ref.bend_gauge_normalise
    assert dev.bending_normalise == pytest.approx(ref.bending_normalise, rel=1e-4)
    g, _ = gm.calibrate(model, cfg, objs, what=gm.CAL_GAUGES)
    assert g.timestep == model_timestep(model) and g.bending_normalise == pytest.approx(ref.bending_normalise, rel=2e-3)


def model_timestep(model):
    return model.params.timestep


# ---------------------------------------------------------------- the reference's own data
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mujoco_timesteps.json")
# The operating point of every reference baseline is segment_inertia_scaling = 50
# (rl/baseline_settings/*.yaml); its three (t, w) columns are pinned to this band.  The
# segment damping law (0.24 / N, gm_host_model.cpp) is the one invented model numeric the
# fit sets; the other inertia columns are reported in DESIGN.md, not asserted.
CSV_BAND = 0.08


def search_ms(gm, n_seg, t_mm, w_mm, inertia, device=False):
    import ctypes as C
    p = gm.ModelParams()
    gm.load_library().gm_default_model_params(C.byref(p))
    p.n_seg, p.finger_thickness, p.finger_width = n_seg, t_mm * 1e-3, w_mm * 1e-3
    # the search's own start value: the one-time settle before it runs at a stable step
    p.segment_inertia_scaling, p.timestep = inertia, 1.0e-3
    model = gm.ModelBlob(p)
    cfg = gm.ConfigBlob(gm.canonical_settings(noise=False, seed=1), model)
    objs = gm.make_object_set("set1_synthetic", 1)
    if device:
        cal, trace = gm.calibrate(model, cfg, objs, what=gm.CAL_TIMESTEP)
    else:
        cal, trace = oracle_lib.calibrate(model, cfg, objs, 1)
    return cal.search_timestep * 1e3, trace


def csv_cases():
    cols = json.load(open(GOLDEN))["columns"]
    out = []
    for name, col in cols.items():
        kv = dict(x.strip().split("=") for x in name.split(","))
        if float(kv["inertia"]) != 50.0:
            continue
        for n, ms in col.items():
            out.append((int(n), float(kv["t"]), float(kv["w"]), 50.0, ms))
    return out


def test_timestep_search_reproduces_reference_csv(world):
    """find_highest_stable_timestep on the oracle for N = 5..10 at the three inertia-x50
    (t, w) columns of the reference's mujoco_timesteps.csv: every point within 8 %, and
    the search really combs down (an unstable candidate precedes the answer)."""
    gm = world[0]
    cases = csv_cases()
    assert len(cases) == 18
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:   # ctypes drops the GIL
        res = list(ex.map(lambda c: search_ms(gm, *c[:4]), cases))
    worst = 0.0
    for (n, t, w, i, ref), (ms, trace) in zip(cases, res):
        assert any(bad for _, bad in trace), f"N={n} t={t} w={w}: no unstable candidate, search degenerate"
        rel = ms / ref - 1.0
        worst = max(worst, abs(rel))
        assert abs(rel) <= CSV_BAND, f"N={n} t={t} w={w}: {ms:.3f} ms vs reference {ref:.3f} ms ({rel:+.1%})"
    print(f"worst |rel| vs mujoco_timesteps.csv (inertia x50): {worst:.3f}")


@pytest.mark.gpu
def test_gpu_timestep_search_matches_oracle_over_segments(world):
    """The batched device search equals the oracle's sequential one, candidate for
    candidate, for N = 5..10 (t = 0.9 mm, w = 28 mm, inertia x50)."""
    if not gpu_available():
        pytest.skip("no GPU")
    gm = world[0]
    for n in range(5, 11):
        ms_d, tr_d = search_ms(gm, n, 0.9, 28.0, 50.0, device=True)
        ms_o, tr_o = search_ms(gm, n, 0.9, 28.0, 50.0)
        assert tr_d == tr_o and ms_d == ms_o, n


# Stated bands over the whole CSV (4 inertia scalings x 3 (t, w) x N = 5..10).  Only the
# baselines' x50 column is pinned (within 8 %, the test above).  The engine's stable step
# barely depends on the inertia scaling: with the segment damping implicit in mj_Euler the
# limiting proximal-hinge mode is damping-limited (h < 2 c / k, independent of the mass),
# where MuJoCo's moved 2.9x from x1 to x100 -- the absent MJCF's inertia distribution
# (tools/fit_timesteps.py).  So the low-scaling columns sit high and
# x100 low, measured under MuJoCo's actuator order (the default model):
CSV_BANDS = {1.0: (2.0, 3.5), 10.0: (1.45, 2.25), 50.0: (0.92, 1.08), 100.0: (0.70, 0.87)}


def test_timestep_search_all_72_points_within_stated_bands(world):
    gm = world[0]
    cols = json.load(open(GOLDEN))["columns"]
    cases = []
    for name, col in cols.items():
        kv = dict(x.strip().split("=") for x in name.split(","))
        for n, ms in col.items():
            cases.append((int(n), float(kv["t"]), float(kv["w"]), float(kv["inertia"]), ms))
    assert len(cases) == 72
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(lambda c: search_ms(gm, *c[:4])[0], cases))
    got = {}
    for (n, t, w, s, ref), ms in zip(cases, res):
        lo, hi = CSV_BANDS[s]
        assert lo <= ms / ref <= hi, f"N={n} t={t} w={w} x{s:g}: {ms:.3f} ms vs reference {ref:.3f} ms"
        got[(n, t, w, s)] = ms
    # the reference's ordering in N holds everywhere (more segments -> smaller stable
    # step); its ordering in the inertia scaling does not (the damping-limited mode above)
    for (n, t, w, s), ms in got.items():
        if n < 10:
            assert got[(n + 1, t, w, s)] < ms, (n, t, w, s)



@pytest.mark.xfail(strict=True, reason="open fidelity gap (DESIGN.md section 2): the reference's stable "
                   "timestep grows 2.9x from inertia x1 to x100; this engine's stays damping-limited, "
                   "so x1 and x10 sit 2.0-3.5x / 1.45-2.25x above the CSV and x100 0.70-0.87x below")
def test_timestep_search_keeps_the_references_inertia_ordering(world):
    """mujoco_timesteps.csv orders every (t, w, N) column by the segment inertia scaling:
    x1 < x10 < x50 < x100 (more rotational inertia per segment, larger stable step).  Kept
    as a strict xfail so the regression the r04 actuator order introduced stays visible
    (it passes -- and so fails this marker -- once a model change restores the ordering)."""
    gm = world[0]
    ms = [search_ms(gm, 8, 0.9, 28.0, s)[0] for s in (1.0, 10.0, 50.0, 100.0)]
    ref = json.load(open(GOLDEN))["columns"]
    col = [ref[f"t=0.9, w=28.0, inertia={s}"]["8"] for s in (1, 10, 50, 100)]
    assert col == sorted(col)
    assert ms == sorted(ms) and ms[3] / ms[0] > 2.0, ms

# validate_curve_under_force's retry branch (mjclass.cpp:4073-4090), forced: at a 4.8 ms
# model step with a 50x saturation load the loaded 50 s settle reaches mjWARN_BADQACC, the
# run is repeated at 0.8x the step and settles.
RETRY_DT, RETRY_SAT = 4.8e-3, 50.0


def retry_world(gm):
    import ctypes as C
    p = gm.ModelParams()
    gm.load_library().gm_default_model_params(C.byref(p))
    p.timestep = RETRY_DT
    model = gm.ModelBlob(p)
    s = gm.canonical_settings(noise=False, seed=1)
    s.saturation_yield_factor = RETRY_SAT
    return model, gm.ConfigBlob(s, model), gm.make_object_set("set1_synthetic", 1), p


def test_gauge_calibration_retry_is_forced_on_the_oracle(world):
    """The retry runs the whole loaded settle again at 0.8x the step (the engine's
    intentional fix of the reference's resume-without-load): the
    result equals a first-try calibration at that reduced step."""
    import ctypes as C
    gm = world[0]
    model, cfg, objs, p = retry_world(gm)
    cal, _ = oracle_lib.calibrate(model, cfg, objs, 2)
    assert cal.gauge_retries == 1
    assert cal.timestep == pytest.approx(0.8 * RETRY_DT, rel=1e-12)
    p.timestep = 0.8 * RETRY_DT
    model2 = gm.ModelBlob(p)
    s = gm.canonical_settings(noise=False, seed=1)
    s.saturation_yield_factor = RETRY_SAT
    cal2, _ = oracle_lib.calibrate(model2, gm.ConfigBlob(s, model2), objs, 2)
    assert cal2.gauge_retries == 0
    assert cal.bending_normalise == cal2.bending_normalise


@pytest.mark.gpu
def test_gpu_gauge_calibration_retry_matches_oracle(world):
    if not gpu_available():
        pytest.skip("no GPU")
    gm = world[0]
    model, cfg, objs, _ = retry_world(gm)
    dev, _ = gm.calibrate(model, cfg, objs, what=gm.CAL_GAUGES)
    ref, _ = oracle_lib.calibrate(model, cfg, objs, 2)
    assert dev.gauge_retries == ref.gauge_retries == 1
    assert dev.timestep == ref.timestep
    assert dev.bending_normalise == pytest.approx(ref.bending_normalise, rel=1e-4)


def model_search_ms(gm, n_seg, **overrides):
    """search_ms at t 0.9 mm, w 28 mm, inertia x50 with gm_model_params overrides"""
    import ctypes as C
    p = gm.ModelParams()
    gm.load_library().gm_default_model_params(C.byref(p))
    p.n_seg, p.finger_thickness, p.finger_width = n_seg, 0.9e-3, 28e-3
    p.segment_inertia_scaling, p.timestep = 50.0, 1.0e-3
    for k, v in overrides.items():
        if k == "revolute_armature":
            p.actuator_armature[1] = v
        else:
            setattr(p, k, v)
    model = gm.ModelBlob(p)
    cfg = gm.ConfigBlob(gm.canonical_settings(noise=False, seed=1), model)
    cal, trace = oracle_lib.calibrate(model, cfg, gm.make_object_set("set1_synthetic", 1), 1)
    return cal.search_timestep * 1e3, trace


def test_mujoco_actuator_order_needs_the_revolute_motor_inertia(world):
    """MuJoCo 2.1.5's actuator path (the default, gm_model_params.mujoco_actuators): the
    PD forces explicit, the constraint solve on M + armature, the joint damping implicit
    in mj_Euler.  The revolute motor's explicit kd = 1 on the bare finger link (~1.5e-5
    kg m^2) is unstable at every timestep the search tries, down to 50 us; the motor's
    reflected inertia (actuator armature 0.01 kg m^2, DESIGN.md "Model spec") makes the
    explicit path stable and the search lands on the reference's 4.3 ms."""
    gm = world[0]
    with pytest.raises(RuntimeError):
        model_search_ms(gm, 8, revolute_armature=0.0)
    assert model_search_ms(gm, 8)[0] == pytest.approx(4.3, rel=0.08)
    # the rounds-1-3 scheme (PD gains and joint damping folded into the solve's matrix,
    # the r03 damping law) stays available and stable
    ms, _ = model_search_ms(gm, 8, mujoco_actuators=0, revolute_armature=0.0, segment_damping=0.24,
                            segment_damping_power=1.0)
    assert ms == pytest.approx(4.35, rel=0.08)


def test_gauge_calibration_reference_retry_on_the_oracle(world):
    """GM_CAL_REFERENCE_RETRY: validate_curve_under_force's retry as the reference runs it
    (mjclass.cpp:4073-4090) -- after the unstable step reset() wipes the tip load and the
    step loop resumes at 0.8x the timestep, so the remaining steps run unloaded from the
    reset pose and the gauge reads an (almost) unloaded finger: a normalisation far below
    the engine's default retry (which reruns the loaded settle)."""
    gm = world[0]
    model, cfg, objs, _ = retry_world(gm)
    fixed, _ = oracle_lib.calibrate(model, cfg, objs, gm.CAL_GAUGES)
    ref, _ = oracle_lib.calibrate(model, cfg, objs, gm.CAL_GAUGES | gm.CAL_REFERENCE_RETRY)
    assert fixed.gauge_retries == ref.gauge_retries == 1
    assert ref.timestep == fixed.timestep == pytest.approx(0.8 * RETRY_DT, rel=1e-12)
    assert abs(ref.bending_normalise) < 0.2 * abs(fixed.bending_normalise), (ref.bending_normalise,
                                                                            fixed.bending_normalise)


@pytest.mark.gpu
def test_gpu_gauge_calibration_reference_retry_matches_oracle(world):
    if not gpu_available():
        pytest.skip("no GPU")
    gm = world[0]
    model, cfg, objs, _ = retry_world(gm)
    what = gm.CAL_GAUGES | gm.CAL_REFERENCE_RETRY
    dev, _ = gm.calibrate(model, cfg, objs, what=what)
    ref, _ = oracle_lib.calibrate(model, cfg, objs, what)
    assert dev.gauge_retries == ref.gauge_retries == 1
    assert dev.timestep == ref.timestep
    assert dev.bending_normalise == pytest.approx(ref.bending_normalise, rel=1e-4, abs=1e-6)


def thick_model(gm):
    import ctypes as C
    p = gm.ModelParams()
    gm.load_library().gm_default_model_params(C.byref(p))
    p.finger_thickness = 1.0e-3          # stiffer fingers: a different equilibrium
    return gm.ModelBlob(p)


def test_settle_cache_first_call_quirk_on_the_oracle(world):
    """calibrate_reset's function-static first_call (myfunctions.cpp:1441-1519): with the
    process-wide cache on (or_set_settle_cache) the first env's 400-substep settle is reused
    by a later env whose model has the same joint count but stiffer fingers; with it off
    each env settles its own model."""
    gm = world[0]
    model = gm.ModelBlob()
    objs = gm.make_object_set("set1_synthetic", 1)
    cfg = gm.ConfigBlob(gm.canonical_settings(noise=False, seed=1), model)
    m2 = thick_model(gm)
    cfg2 = gm.ConfigBlob(gm.canonical_settings(noise=False, seed=1), m2)
    L = oracle_lib.lib()
    try:
        L.or_set_settle_cache(1)
        a = oracle_lib.OracleEnv(model, cfg, objs, 0)
        b = oracle_lib.OracleEnv(m2, cfg2, objs, 0)
        ea, eb = a.eq(), b.eq()
        np.testing.assert_array_equal(ea, eb)
    finally:
        L.or_set_settle_cache(0)
    c = oracle_lib.OracleEnv(m2, cfg2, objs, 0)
    assert np.abs(c.eq() - ea).max() > 1e-6



def seg_model(gm, n_seg, thickness=None):
    import ctypes as C
    p = gm.ModelParams()
    gm.load_library().gm_default_model_params(C.byref(p))
    p.n_seg = n_seg
    if thickness is not None:
        p.finger_thickness = thickness
    return gm.ModelBlob(p)


def test_settle_cache_recalibrates_on_changed_joint_count(world):
    """calibrate_reset's changed-joint-count branch (myfunctions.cpp:1453-1468): a model with
    a different number of gripper joints sets first_call = true, settles, and its settle is
    the one kept.  Sequence N=8, N=6 (stiff), N=6 (default), N=8 (stiff): the second N=6 env
    takes the stiff N=6 settle, and the last N=8 env settles its own model rather than
    reusing the first N=8 settle."""
    gm = world[0]
    objs = gm.make_object_set("set1_synthetic", 1)
    cfg_of = lambda m: gm.ConfigBlob(gm.canonical_settings(noise=False, seed=1), m)
    m8, m6s, m6, m8s = seg_model(gm, 8), seg_model(gm, 6, 1.0e-3), seg_model(gm, 6), seg_model(gm, 8, 1.0e-3)
    own = {}
    for name, m in (("m6", m6), ("m8s", m8s)):
        own[name] = oracle_lib.OracleEnv(m, cfg_of(m), objs, 0).eq()     # cache off: own settle
    L = oracle_lib.lib()
    try:
        L.or_set_settle_cache(1)
        a = oracle_lib.OracleEnv(m8, cfg_of(m8), objs, 0).eq()
        b = oracle_lib.OracleEnv(m6s, cfg_of(m6s), objs, 0).eq()
        c = oracle_lib.OracleEnv(m6, cfg_of(m6), objs, 0).eq()
        d = oracle_lib.OracleEnv(m8s, cfg_of(m8s), objs, 0).eq()
    finally:
        L.or_set_settle_cache(0)
    np.testing.assert_array_equal(c, b)                  # same joint count: the cached N=6 settle
    assert np.abs(c - own["m6"]).max() > 1e-6           # ... not its own
    np.testing.assert_array_equal(d, own["m8s"])         # changed count: settles its own model
    assert np.abs(d - a).max() > 1e-6                    # ... not the stale first N=8 settle

@pytest.mark.gpu
def test_gpu_settle_cache_first_call_quirk_matches_oracle(world):
    """gm_set_settle_cache(1): the device shares the first context's settle the same way;
    the later context's reset state equals the oracle's under the same switch."""
    if not gpu_available():
        pytest.skip("no GPU")
    gm = world[0]
    objs_name = "set1_synthetic"
    m1 = gm.ModelBlob()
    m2 = thick_model(gm)
    s = gm.canonical_settings(noise=False, seed=1)
    lib = gm.load_library()
    L = oracle_lib.lib()
    try:
        lib.gm_set_settle_cache(1)
        L.or_set_settle_cache(1)
        e1 = gm.BatchedGripperEnv(2, object_set=objs_name, settings=s, seed=1, model_blob=m1)
        o1 = oracle_lib.OracleEnv(m1, e1.cfg, e1.objects, 0)
        e2 = gm.BatchedGripperEnv(2, object_set=objs_name, settings=s, seed=1, model_blob=m2)
        o2 = oracle_lib.OracleEnv(m2, e2.cfg, e2.objects, 0)
        sp = e2.make_spawn(idx=0, x=0.0, y=0.0, rot=0.0)
        obs = e2.reset(spawn=sp)
        o2.reset(sp[0])
        q, _, _ = e2.state()
        qo, _, _ = o2.state()
        np.testing.assert_allclose(q[0], qo, rtol=0, atol=1e-12)
        np.testing.assert_allclose(obs[0], o2.observation(), rtol=1e-5, atol=1e-6)
        # the shared equilibrium: the stiff model reset to the first model's settled pose
        np.testing.assert_allclose(o2.eq(), o1.eq(), rtol=0, atol=0)
        e1.close(); e2.close()
    finally:
        lib.gm_set_settle_cache(0)
        L.or_set_settle_cache(0)
