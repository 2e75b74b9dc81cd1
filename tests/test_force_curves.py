"""The physics pinned to the reference's own MuJoCo output: the finger-gauge force curves of
its "measure constrict" and "measure tilt" programs (mysimulate.cpp:2720-2811), which the
reference ran with MuJoCo 2.1.5 and its real gripper MJCF and kept in
rl/juypter/thesis_plots/sim_vs_real_forces*.csv (-> tests/golden/force_curves.json,
tests/golden/make_force_curves.py).  They pin contact geometry, finger bending stiffness,
the revolute PD and the gauge chain (polyfit + SI calibration) together.

CPU (oracle): each program is replayed on the engine's model of the same scene
(tests/force_programs.py) and held to stated bands against every Sim column the thesis
notebook plots.  GPU: the device runs the same programs through the C ABI
(gm_set_motor_target / gm_get_sensor_si) and matches the oracle reading for reading.

Bands (measured values in DESIGN.md section 4):
- constrict, spheres 80 / 100 / 120 mm x finger variants EI1..3, both CSVs: contact onset
  within 1.0 mm, force-vs-travel slope within -6 % / +8 %, every reading within 0.10 N,
  the pre-contact reading within 0.04 N;
- constrict, the CSV's other Sim columns (spheres 70 / 90 / 110 mm x EI1..3, which the
  notebook does not plot): their onsets sit 7 mm past 35 + sqrt(r^2 - 6^2) (76.4-76.8 /
  86.0-86.5 / 96.6-96.9 mm against 69.5 / 79.6 / 89.7), i.e. they were made with a longer
  fingertip reach -- all nine fit one hook length, 42 mm: onset within 1.0 mm, slope
  within -6 % / +15 %, every reading within 0.20 N;
- tilt, 14 (Kp, EI) columns: force rises as y is stepped below x (the fingertips tilt
  inward, gripper.h:88-93), slope per mm of y within +-12 %, slope increasing with Kp as
  in the reference, and the y where the force reaches 0.5 N and 1 N within 0.75 mm of the
  reference's (the CSV does not say which sphere the run used; the 120 mm sphere of the
  constrict scene is used.  The notebook's offsets [-1, -0.3, -0.3] mm align these sim
  curves with the real ones, design_modelling_chapters.ipynb "tilt", not with each other);
- palm ("measure palm", mysimulate.cpp:2813-2853): no reference output exists (parity
  unpinned): property test on the oracle -- the palm reading is zero until the palm face
  meets the sphere's top, within 0.5 mm of the geometric onset, then rises monotonically --
  and the device reading for reading against the oracle.
"""
import json
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import force_programs as fp
import oracle_lib as ol
from conftest import gpu_available

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "force_curves.json")
ONSET_MM, SLOPE_BAND, MAX_ERR_N, BASE_N = 1.0, (0.94, 1.08), 0.10, 0.04
TILT_SLOPE_BAND = (0.88, 1.12)
TILT_CROSS_MM = 0.75
LONG_HOOK, LONG_SLOPE_BAND, LONG_MAX_ERR_N = 42e-3, (0.94, 1.15), 0.20


def golden():
    return json.load(open(GOLDEN))


def ref_col(tab, name):
    return np.array([np.nan if v is None else v for v in tab[name]], dtype=np.float64)


@pytest.fixture(scope="module")
def constrict_runs(gm):
    cases = [(d, v) for d in fp.SPHERES_MM for v in fp.VARIANTS]
    dts = {}
    for v in fp.VARIANTS:      # the timestep search does not depend on the sphere / clearance much,
        dts[v] = fp.auto_timestep(gm, ol, fp.model_params(gm, v, 120))   # but is run per variant

    def one(c):
        d, v = c
        model, cfg, objs = fp.scene(gm, ol, v, d, timestep=dts[v])
        return fp.constrict(fp.oracle_env(gm, ol, model, cfg, objs))
    with ThreadPoolExecutor(max_workers=min(9, os.cpu_count() or 1)) as ex:   # ctypes drops the GIL
        res = list(ex.map(one, cases))
    return dict(zip(cases, res)), dts


def test_constrict_matches_reference_mujoco_curves(constrict_runs):
    runs, dts = constrict_runs
    g = golden()
    report = []
    for (d, v), r in runs.items():
        x, F = r[:, 0], r[:, 1]
        # the three fingers are symmetric about the centred sphere
        np.testing.assert_allclose(r[:, 2], F, rtol=0, atol=2e-3)
        np.testing.assert_allclose(r[:, 3], F, rtol=0, atol=2e-3)
        o, s, b = fp.features(x, F)
        for tab in ("constrict_A", "constrict_B"):
            T = g[tab]
            Fr = ref_col(T, f"Sim {d} {v}")
            xr = ref_col(T, "XY pos")
            np.testing.assert_allclose(x[:len(xr)], xr, rtol=0, atol=1e-9)   # the program points, 130 .. 60 mm
            o2, s2, b2 = fp.features(xr, Fr)
            err = float(np.nanmax(np.abs(F[:len(Fr)] - Fr)))
            report.append((d, v, tab, o - o2, s / s2, err, b - b2))
            assert abs(o - o2) <= ONSET_MM, (d, v, tab, o, o2)
            assert SLOPE_BAND[0] <= s / s2 <= SLOPE_BAND[1], (d, v, tab, s, s2)
            assert err <= MAX_ERR_N, (d, v, tab, err)
            assert abs(b - b2) <= BASE_N, (d, v, tab, b, b2)
    print("\n".join(f"D{d} {v} {t}: onset {do:+.2f} mm, slope x{sr:.3f}, max err {e:.3f} N, base {db:+.3f} N"
                    for d, v, t, do, sr, e, db in report))
    print("timesteps (ms):", {k: round(1e3 * t, 3) for k, t in dts.items()})


def test_constrict_onset_tracks_sphere_radius(constrict_runs):
    """Contact begins when the 35 mm hook's inner end reaches the sphere 6 mm above its
    equator: onset = 35 mm + sqrt(r^2 - 6^2) (within the collision geometry's thickness),
    for every sphere and finger -- the relation the reference's curves follow (onsets
    74.6 / 84.9 / 94.8 mm)."""
    runs, _ = constrict_runs
    for (d, v), r in runs.items():
        o, _, _ = fp.features(r[:, 0], r[:, 1])
        geo = 35.0 + np.sqrt((0.5 * d) ** 2 - 6.0 ** 2)
        assert abs(o - geo) <= 1.0, (d, v, o, geo)


def test_constrict_70_90_110_columns_fit_one_longer_hook(gm):
    """The constrict CSV's Sim 70 / 90 / 110 x EI1..3 columns (not plotted by the notebook):
    with the 35 mm hook their onsets would be 69.5 / 79.6 / 89.7 mm, the reference's are 7 mm
    later; one hook length, 42 mm, puts every onset within 1 mm (35 -> 42 mm is the only
    change), the nine curves then within the stated bands."""
    g = golden()["constrict_A"]
    dts = {v: fp.auto_timestep(gm, ol, fp.model_params(gm, v, 120)) for v in fp.VARIANTS}
    cases = [(d, v) for d in (70, 90, 110) for v in fp.VARIANTS]

    def one(c):
        d, v = c
        model, cfg, objs = fp.scene(gm, ol, v, d, timestep=dts[v], hook_length=LONG_HOOK)
        return fp.constrict(fp.oracle_env(gm, ol, model, cfg, objs))
    with ThreadPoolExecutor(max_workers=min(9, os.cpu_count() or 1)) as ex:
        res = list(ex.map(one, cases))
    xr = ref_col(g, "XY pos")
    report = []
    for (d, v), r in zip(cases, res):
        x, F = r[:, 0], r[:, 1]
        Fr = ref_col(g, f"Sim {d} {v}")
        o, s, b = fp.features(x, F)
        o2, s2, b2 = fp.features(xr, Fr)
        err = float(np.nanmax(np.abs(F[:len(Fr)] - Fr)))
        report.append((d, v, o - o2, s / s2, err))
        # the 35 mm hook's geometric onset misses the reference by ~7 mm; the 42 mm one fits
        assert abs(35.0 + np.sqrt((0.5 * d) ** 2 - 36.0) - o2) > 6.0, (d, v, o2)
        assert abs(o - o2) <= ONSET_MM, (d, v, o, o2)
        assert LONG_SLOPE_BAND[0] <= s / s2 <= LONG_SLOPE_BAND[1], (d, v, s, s2)
        assert err <= LONG_MAX_ERR_N, (d, v, err)
        assert abs(b - b2) <= BASE_N, (d, v, b, b2)
    print("\n".join(f"D{d} {v}: onset {do:+.2f} mm, slope x{sr:.3f}, max err {e:.3f} N" for d, v, do, sr, e in report))


@pytest.fixture(scope="module")
def tilt_runs(gm):
    g = golden()["tilt"]
    cols = [h for h in g if h.startswith("Kp=")]
    assert len(cols) == 14
    dts = {v: fp.auto_timestep(gm, ol, fp.model_params(gm, v, 120)) for v in fp.VARIANTS}

    def one(h):
        kp, v = float(h.split()[0][3:]), h.split()[1]
        model, cfg, objs = fp.scene(gm, ol, v, 120, revolute_kp=kp, stepper=(1, 1.0 / 5000.0), timestep=dts[v])
        return fp.tilt(fp.oracle_env(gm, ol, model, cfg, objs))
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        res = list(ex.map(one, cols))
    return dict(zip(cols, res)), dts


def test_tilt_matches_reference_mujoco_slopes(tilt_runs):
    runs, _ = tilt_runs
    g = golden()["tilt"]
    xr = ref_col(g, "XY pos")
    slopes = {}
    for h, r in runs.items():
        y, F = r[:, 0], r[:, 1]
        nr = int(np.isfinite(xr).sum())                     # the CSV lists y = 100 .. 95.25 mm
        np.testing.assert_allclose(y[:nr], xr[:nr], rtol=0, atol=1e-9)
        # the fingertips press inward as y goes below x: the reading climbs past 1.5 N
        assert F[0] < 0.05 and F[-1] > 1.5, (h, F[0], F[-1])
        Fr = ref_col(g, h)
        _, s, _ = fp.features(y, F, base_from=100.0)
        _, s2, _ = fp.features(xr[:nr], Fr[:nr], base_from=100.0)
        slopes[h] = (s, s2)
        assert TILT_SLOPE_BAND[0] <= s / s2 <= TILT_SLOPE_BAND[1], (h, s, s2)
        # where the press reaches 0.5 N and 1 N: the onset of the tilt curve
        for lvl in (0.5, 1.0):
            c = fp.level_crossing(-y, F, lvl)
            c2 = fp.level_crossing(-xr[:nr], Fr[:nr], lvl)
            assert abs(c - c2) <= TILT_CROSS_MM, (h, lvl, -c, -c2)
    # a stiffer revolute PD gives a stiffer tilt, as in the reference
    for v in fp.VARIANTS:
        ks = sorted((float(h.split()[0][3:]), slopes[h]) for h in slopes if h.endswith(v))
        ours = [s for _, (s, _) in ks]
        theirs = [s for _, (_, s) in ks]
        assert ours == sorted(ours) and theirs == sorted(theirs), (v, ks)
    print("\n".join(f"{h}: slope {s:.4f} N/mm vs reference {s2:.4f} (x{s / s2:.3f})" for h, (s, s2) in slopes.items()))


def palm_scene(gm, d=100):
    """The "measure palm" scene: the sphere centred, the fingers open; fingertip clearance
    10 mm (MjEnv's default -- with the constrict scene's r + 6 mm the sphere's top would sit
    below the program's 60-85 mm palm range), the palm stepper at 1 step / 0.2 ms."""
    return fp.scene(gm, ol, "EI3", d, stepper=(1, 1.0 / 5000.0), clearance=10e-3, timestep=3.0e-3)


def palm_onset_mm(gm, model, cfg, objs, d, z0=60e-3):
    """Where the palm face meets the sphere's top: settle at the program's first point, then
    face - top from the settled joint positions (the base and the palm sag under gravity on
    their PD springs, 4.6 / 0.9 mm), the target z at which that gap closes."""
    import indep_physics as ip
    mv = ip.GmModel.from_buffer(model.buf)
    o = fp.oracle_env(gm, ol, model, cfg, objs)
    o.set_motor_target(130e-3, 130e-3, z0)
    for _ in range(100):
        o.action_step()
    q, _, _ = o.state()
    face = mv.body_pos[mv.body_base][2] - q[mv.dof_base] - ((mv.finger_length - 165e-3) + 0.004) - q[mv.dof_palm]
    top = q[mv.jnt_qposadr[mv.body_jnt[mv.body_obj]] + 2] + 0.5e-3 * d
    return (z0 + face - top) * 1e3


@pytest.mark.parametrize("d", [90, 100])
def test_palm_program_reads_the_press(gm, d):
    """Parity unpinned (no reference output): the palm reading stays at zero while the palm
    face is above the sphere, starts within 0.5 mm of where the face meets its top, and rises
    monotonically (the palm's axial force, +ve for compression -- the sphere is geom1 of the
    palm pair)."""
    model, cfg, objs = palm_scene(gm, d)
    r = fp.palm(fp.oracle_env(gm, ol, model, cfg, objs))
    z, P = r[:, 0], r[:, 1]
    on = palm_onset_mm(gm, model, cfg, objs, d)
    assert 60.0 < on < 84.0, on
    assert np.abs(P[z < on - 0.5]).max() < 0.02, P[z < on - 0.5]
    c = fp.level_crossing(z, P, 0.05)
    assert abs(c - on) <= 0.5, (c, on)
    after = P[z > on + 0.5]
    assert (np.diff(after) > -0.02).all() and after[-1] > 2.0, after
    print(f"D{d}: onset {c:.2f} mm (geometric {on:.2f}), {after[-1]:.2f} N at {z[-1]:.2f} mm, "
          f"slope {np.polyfit(z[z > on + 1.0], P[z > on + 1.0], 1)[0]:.2f} N/mm")


# ---------------------------------------------------------------- device vs oracle
GPU_CASES = [(120, "EI1"), (80, "EI3")]


@pytest.mark.gpu
@pytest.mark.parametrize("d,v", GPU_CASES)
def test_gpu_constrict_matches_oracle(gm, d, v):
    """The constrict program on one device env (set_motor_target / action_step /
    sensor_si through the C ABI) equals the oracle's reading for reading."""
    if not gpu_available():
        pytest.skip("no GPU")
    model, cfg, objs = fp.scene(gm, ol, v, d)
    dev = fp.DeviceEnv1(gm, model, gm.canonical_settings(noise=False, seed=1), objs)
    try:
        rd = fp.constrict(dev)
    finally:
        dev.close()
    ro = fp.constrict(fp.oracle_env(gm, ol, model, cfg, objs))
    np.testing.assert_array_equal(rd[:, 0], ro[:, 0])
    np.testing.assert_allclose(rd[:, 1:], ro[:, 1:], rtol=1e-4, atol=1e-5)
    assert rd[-1, 1] > 1.0                                  # the squeeze really loads the gauges


@pytest.mark.gpu
def test_gpu_tilt_matches_oracle(gm):
    if not gpu_available():
        pytest.skip("no GPU")
    model, cfg, objs = fp.scene(gm, ol, "EI2", 120, revolute_kp=12.64, stepper=(1, 1.0 / 5000.0))
    dev = fp.DeviceEnv1(gm, model, gm.canonical_settings(noise=False, seed=1), objs)
    try:
        rd = fp.tilt(dev)
    finally:
        dev.close()
    ro = fp.tilt(fp.oracle_env(gm, ol, model, cfg, objs))
    np.testing.assert_allclose(rd[:, 1:], ro[:, 1:], rtol=1e-4, atol=1e-5)
    assert rd[-1, 1] > 1.5


def test_set_motor_target_reports_limits(gm):
    """MjClass::set_motor_target returns Gripper::set_xyz_m's in-limits flag (gripper.h:152):
    a target past xy_max (134 mm) is clamped and reported."""
    model, cfg, objs = fp.scene(gm, ol, "EI1", 120, timestep=3.187e-3)
    o = fp.oracle_env(gm, ol, model, cfg, objs)
    assert o.set_motor_target(0.1, 0.1, 5e-3)
    assert not o.set_motor_target(0.2, 0.1, 5e-3)
    e, _, _, _ = o.target()
    assert e[0] == pytest.approx(0.134)


@pytest.mark.gpu
def test_gpu_palm_matches_oracle(gm):
    """The "measure palm" program on one device env equals the oracle reading for reading
    (parity unpinned against the reference: it kept no output of this program)."""
    if not gpu_available():
        pytest.skip("no GPU")
    model, cfg, objs = palm_scene(gm, 100)
    dev = fp.DeviceEnv1(gm, model, gm.canonical_settings(noise=False, seed=1), objs)
    try:
        rd = fp.palm(dev)
    finally:
        dev.close()
    ro = fp.palm(fp.oracle_env(gm, ol, model, cfg, objs))
    np.testing.assert_array_equal(rd[:, 0], ro[:, 0])
    np.testing.assert_allclose(rd[:, 1], ro[:, 1], rtol=1e-4, atol=1e-5)
    assert rd[-1, 1] > 5.0
