"""The CPU oracle against the reference's own golden vectors.

Fixtures in tests/golden/ come from the reference's compilable sources
(src/gripper.cpp, src/slidingwindow.h) built from /root/reference, from libstdc++'s
RNG stack the reference consumes, from numpy.polyfit and from the test.cpp
known answer; tests/golden/make_golden.py regenerates them.
"""
import json
import os

import numpy as np
import pytest

import oracle_lib

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def test_gripper_step_sequences_bit_exact():
    """luke::Gripper set_xyz_m_rad / set_xyz_m / step_to / reset (gripper.cpp:6-228):
    return codes and integer step counts exact, positions to the last bit."""
    g = load("gripper_sequences.json")
    cmds = np.array(g["cmds"], dtype=np.float64)
    ref = np.array(g["out"])
    out = oracle_lib.grip_step_sequence(cmds)
    assert out.shape == ref.shape
    int_cols = [0, 5, 6, 7, 12, 13, 14]
    np.testing.assert_array_equal(out[:, int_cols], ref[:, int_cols])
    np.testing.assert_array_equal(out, ref)


def test_gripper_sequences_cover_clamps():
    g = load("gripper_sequences.json")
    ref = np.array(g["out"])
    assert (ref[:, 0] == 0).any() and (ref[:, 0] == 1).any()   # both rejected and accepted moves
    x, z, th = ref[:, 1], ref[:, 3], ref[:, 4]
    assert np.nanmin(x) == pytest.approx(49e-3) and np.nanmax(x) >= 134e-3       # x clamps
    assert np.nanmin(z) == 0.0 and np.nanmax(z) == pytest.approx(165e-3)        # z clamps
    assert np.nanmax(np.abs(th)) == pytest.approx(np.deg2rad(40))               # angle clamp
    assert np.isnan(ref).any()                                                   # asin domain (gripper.cpp:50)


def test_sliding_window_reads():
    """SlidingWindow::add / read_element (slidingwindow.h:36-55): the oracle's ring (the
    device's GM_RING = 64 deep window) returns the same last-k readings as the reference
    for every k the golden trace holds (<= 7)."""
    w = load("sliding_window.json")
    rows = np.array(w["rows"])
    trace = oracle_lib.ring_trace(w["adds"], 7)
    np.testing.assert_array_equal(trace, rows[:, 1:8].astype(np.float32))


def test_change_sample_known_answer():
    """test.cpp:293-311: change_sample over [1..6] with prev_steps=3 -> [3,1,4,1,5,1,6]."""
    k = load("change_sample.json")
    recent_first = list(reversed(k["window_adds"]))
    out = oracle_lib.sample(1, recent_first, k["prev_steps"], k["readings_per_step"])
    np.testing.assert_array_equal(out, np.array(k["expected"], dtype=np.float32))


@pytest.mark.parametrize("seed", ["1", "5", "1234", "1000004", "2147483646"])
def test_rng_matches_libstdcxx(seed):
    """minstd_rand0 + generate_canonical as libstdc++ draws them: raw engine output,
    uniform_real_distribution<float>{0,1} (1 draw) and <double>(-a, a) (2 draws)."""
    r = load("rng.json")[seed]
    s = int(seed)
    assert oracle_lib.minstd_raw(s, 16) == [int(x) for x in r["raw"]]
    f = oracle_lib.canonical_floats(s, 16).astype(np.float32)
    np.testing.assert_array_equal(f, np.array(r["float"], dtype=np.float32))
    d = oracle_lib.canonical_doubles(s, 16) * (0.01 - -0.01) + -0.01
    np.testing.assert_array_equal(d, np.array(r["double_pm0.01"]))


@pytest.mark.parametrize("seed", ["1", "5", "1234", "1000004", "2147483646"])
def test_std_shuffle_matches_libstdcxx(seed):
    """std::shuffle(grid, minstd_rand0) as spawn_into_scene draws it (mjclass.cpp:2533-2536):
    the permutation and the engine position afterwards, against libstdc++ itself."""
    r = load("rng.json")[seed]
    for key in r:
        if not key.startswith("shuffle") or key.endswith("_next"):
            continue
        n = int(key[len("shuffle"):])
        perm, nxt = oracle_lib.std_shuffle(int(seed), n)
        assert perm == [int(x) for x in r[key]], key
        assert nxt == int(r[key + "_next"][0]), key


def test_box2d_overlap_known_answers():
    """luke::Box2d::overlapsWith (customtypes.h:83-131) by hand: SAT over this box's own
    edge normals; a positive separation smaller than the gap counts as *no* overlap
    (the containsOther flag), only a separation above the gap returns early."""
    ov = oracle_lib.box2d_overlaps
    sq = lambda cx, cy, rot=0.0: (cx, cy, 0.02, 0.02, rot)
    assert ov(sq(0, 0), sq(0.01, 0), 1e-3)            # half overlapping
    assert ov(sq(0, 0), sq(0, 0), 0.0)                # identical
    assert ov(sq(0, 0), sq(0.02, 0), 0.0)             # touching edges (max1 == min2)
    assert not ov(sq(0, 0), sq(0.021, 0), 5e-3)       # 1 mm apart, inside the 5 mm gap
    assert not ov(sq(0, 0), sq(0.03, 0), 5e-3)        # 10 mm apart, beyond the gap
    assert ov(sq(0, 0), sq(0.0, 0.015, np.pi / 4), 0.0)
    # only this box's axes are tested: a rotated box whose corner region misses
    # is still reported as overlapping when no own axis separates them
    assert ov(sq(0, 0), (0.0205, 0.0205, 0.02, 0.02, np.pi / 4), 0.0)
    assert not ov((0.0205, 0.0205, 0.02, 0.02, np.pi / 4), sq(0, 0), 0.0)


def test_gauge_polyfit_vs_numpy():
    """read_armadillo_gauge's cubic least-squares fit (myfunctions.cpp:2739) against
    numpy.polyfit on the same points, evaluated at 50 mm (in mm)."""
    p = load("polyfit.json")
    for c in p["cases"]:
        got = oracle_lib.polyfit_eval(c["X"], c["Y"], c["order"], c["x"])
        assert got == pytest.approx(c["reading_mm"], rel=1e-5, abs=1e-6)


def test_gauge_points_follow_joint_angles(model):
    """Cumulative segment angles -> joint points (myfunctions.cpp:2699-2740): a straight
    finger gives y = 0 and a zero reading; a uniform bend gives a monotone curve."""
    N = model.n_seg
    X, Y = oracle_lib.gauge_points(model, np.zeros(N))
    assert np.allclose(Y, 0) and np.all(np.diff(X) > 0)
    assert oracle_lib.gauge_reading(model, np.zeros(N)) == pytest.approx(0.0, abs=1e-9)
    X, Y = oracle_lib.gauge_points(model, np.full(N, 0.01))
    assert np.all(np.diff(Y) > 0)
    assert oracle_lib.gauge_reading(model, np.full(N, 0.01)) > 0


def test_engine_gauge_fit_equals_the_pinned_fit(model):
    """The engine's gauge evaluation (centred Vandermonde, shared by device and oracle)
    gives the reading of the numpy-pinned raw fit (or_polyfit_eval) on bent fingers."""
    rng = np.random.default_rng(3)
    N = model.n_seg
    for _ in range(50):
        q = rng.uniform(-0.05, 0.05, size=N)
        X, Y = oracle_lib.gauge_points(model, q)
        ref = oracle_lib.polyfit_eval(X, Y, 3, 50e-3)        # gm_host_model.cpp gauge_xpos
        got = oracle_lib.gauge_reading(model, q)
        assert got == pytest.approx(ref, rel=1e-5, abs=1e-6)
