"""Automatic calibration (MjClass::configure_settings auto flags, mjclass.cpp:241-308):
find_highest_stable_timestep (mjclass.cpp:4745-4854) and calibrate_simulated_sensors
(4643-4676, tip load via validate_curve_under_force 4023-4105).

The oracle runs the reference's sequential procedure; the device runs every search
candidate as its own env in one launch and replays the sequence (gm_calibrate).  With
this engine's implicit spring / damper / PD terms every candidate up to the 20 ms cap is
stable, so the fine-comb branch of the search is not reached by a physical model here.
"""
import math

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
