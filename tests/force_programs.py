"""The reference's force-measurement programs (mysimulate.cpp:2720-2811) as test drivers,
over anything with set_motor_target(x, y, z) / action_step() / sensor_si() -- the fp64
oracle (oracle_lib.OracleEnv) or one device env (DeviceEnv1 below) -- and the scene they
run in.

TEST INFRASTRUCTURE: used by tests/test_force_curves.py only.

Scene (what the reference's CSVs were made with; DESIGN.md section 4 "Force curves"):
- the gripper at N = 8 with one of the three finger variants the thesis notebook labels
  EI1..3 -- (t, w) = (0.9, 28), (1.0, 24), (1.0, 28) mm at the reference's default modulus
  193 GPa (MjEnv.py:125) -- a 90 degree fingertip hook and fingertip_clearance = r + 6 mm
  (the generator block that made the sized-sphere test set, MjEnv.py:2317-2321:
  finger_hook_angle_degrees = 90, fingertip_clearance "120e-3 / 2 + 6e-3" for the 120 mm
  sphere);
- one sphere of diameter D at the centre (reset_object + spawn_object(0)), 0.1 kg
  (its mass is absent; the squeeze is horizontal and symmetric);
- the timestep the model's own find_highest_stable_timestep picks (MjClass's default
  auto_set_timestep), S = ceil(0.2 s / dt) substeps per action_step.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

VARIANTS = {"EI1": (0.9e-3, 28e-3), "EI2": (1.0e-3, 24e-3), "EI3": (1.0e-3, 28e-3)}
SPHERES_MM = (80, 100, 120)
CLEARANCE_ABOVE_EQUATOR = 6e-3
SPHERE_MASS = 0.1


def model_params(gm, variant: str, diameter_mm: float, timestep: float = 1.0e-3):
    p = gm.ModelParams()
    gm.load_library().gm_default_model_params(C.byref(p))
    p.finger_thickness, p.finger_width = VARIANTS[variant]
    p.hook_angle_degrees = 90.0
    p.fingertip_clearance = 0.5e-3 * diameter_mm + CLEARANCE_ABOVE_EQUATOR
    p.timestep = timestep
    return p


def auto_timestep(gm, ol, p) -> float:
    """find_highest_stable_timestep on the oracle (mjclass.cpp:4745-4854, the reference's
    auto_set_timestep) for these model params: the final (factored) timestep."""
    m0 = gm.ModelBlob(p)
    cfg0 = gm.ConfigBlob(gm.canonical_settings(noise=False, seed=1), m0)
    cal, _ = ol.calibrate(m0, cfg0, gm.make_object_set("set1_synthetic", 1), 1)
    return float(cal.timestep)


def sphere(gm, diameter_mm: float):
    objs = (gm.Object * 1)()
    objs[0].type = 2                                    # GM_GEOM_SPHERE
    r = 0.5e-3 * diameter_mm
    objs[0].size[0] = objs[0].size[1] = objs[0].size[2] = r
    objs[0].mass = SPHERE_MASS
    objs[0].friction = 1.0
    return objs


def scene(gm, ol, variant: str, diameter_mm: float, revolute_kp=None, stepper=None, timestep=None, hook_length=None,
          clearance=None):
    """(model, cfg, objects) of one program run.  revolute_kp overrides the revolute PD gain
    (the tilt CSV's "Kp=..." columns); stepper = (num_steps, time_per_step) overrides
    j_.ctrl (the tilt program's own instruction: num_steps = 1, pulses_per_s = 5000)."""
    import indep_physics as ip
    p = model_params(gm, variant, diameter_mm)
    if hook_length is not None:
        p.hook_length = hook_length
    if clearance is not None:
        p.fingertip_clearance = clearance
    p.timestep = auto_timestep(gm, ol, p) if timestep is None else timestep
    model = gm.ModelBlob(p)
    if revolute_kp is not None or stepper is not None:
        mv = ip.GmModel.from_buffer(model.buf)
        if revolute_kp is not None:
            mv.kp_gripper[1] = revolute_kp
        if stepper is not None:
            mv.stepper_num_steps, mv.time_per_step = stepper
    cfg = gm.ConfigBlob(gm.canonical_settings(noise=False, seed=1), model)
    return model, cfg, sphere(gm, diameter_mm)


def constrict(env, x0_mm=130, x1_mm=58, step_mm=2, settle=10, per=7):
    """"measure constrict" (mysimulate.cpp:2720-2760): x = y = pos for pos = 130 .. 58 mm in
    2 mm steps, palm z 5 mm; 10 action steps at the start, then 7 per point; the three SI
    finger gauges after each point.  Returns [n_points, 4]: pos mm, gauge 1..3 N."""
    pos = [i * 1e-3 for i in range(x0_mm, x1_mm - 1, -step_mm)]
    env.set_motor_target(pos[0], pos[0], 5e-3)
    for _ in range(settle):
        env.action_step()
    out = []
    for x in pos:
        env.set_motor_target(x, x, 5e-3)
        for _ in range(per):
            env.action_step()
        g = env.sensor_si()
        out.append((x * 1e3, float(g[0]), float(g[1]), float(g[2])))
    return np.array(out)


def tilt(env, start_mm=100.0, span_mm=6.0, inc_mm=0.25, settle=100, per=5):
    """"measure tilt" (mysimulate.cpp:2762-2811): x held at 100 mm, y = 100 .. 94.25 mm in
    0.25 mm steps (the fingers tilt about the revolute joints), palm z 5 mm; 100 action
    steps at the start, then 5 per point.  Returns [n_points, 4]: y mm, gauge 1..3 N."""
    pos = []
    i = start_mm
    while i > start_mm - span_mm:
        pos.append(i * 1e-3)
        i -= inc_mm
    env.set_motor_target(pos[0], pos[0], 5e-3)
    for _ in range(settle):
        env.action_step()
    out = []
    for y in pos:
        env.set_motor_target(pos[0], y, 5e-3)
        for _ in range(per):
            env.action_step()
        g = env.sensor_si()
        out.append((y * 1e3, float(g[0]), float(g[1]), float(g[2])))
    return np.array(out)


def palm(env, start_mm=60.0, span_mm=25.0, inc_mm=0.25, settle=100, per=5, xy=130e-3):
    """"measure palm" (mysimulate.cpp:2813-2853): fingers fully open (x = y = 130 mm), the palm
    z target stepped 60 .. 84.75 mm in 0.25 mm steps onto the centred sphere; 100 action steps
    at the start, then 5 per point; the SI palm sensor after each point (its stepper at 1 step
    / 0.2 ms, as the program instructs).  Returns [n_points, 2]: z mm, palm N."""
    pos = []
    i = start_mm
    while i < start_mm + span_mm:
        pos.append(i * 1e-3)
        i += inc_mm
    env.set_motor_target(xy, xy, pos[0])
    for _ in range(settle):
        env.action_step()
    out = []
    for z in pos:
        env.set_motor_target(xy, xy, z)
        for _ in range(per):
            env.action_step()
        out.append((z * 1e3, float(env.sensor_si()[3])))
    return np.array(out)


def level_crossing(x, F, level):
    """First x where the curve reaches `level` (linear between the bracketing points)."""
    F = np.asarray(F, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64)
    i = int(np.argmax(F >= level))
    if F[i] < level:
        return float("nan")
    if i == 0:
        return float(x[0])
    return float(x[i - 1] + (level - F[i - 1]) * (x[i] - x[i - 1]) / (F[i] - F[i - 1]))


def features(x, F, contact_above=0.1, base_from=110.0):
    """(onset mm, slope N per mm of travel, pre-contact base N) of a force curve: the base
    is the median reading before contact (x >= base_from), the line is fitted to the
    points more than contact_above over it, the onset is where that line meets the base."""
    x = np.asarray(x, dtype=np.float64)
    F = np.asarray(F, dtype=np.float64)
    ok = np.isfinite(F)
    x, F = x[ok], F[ok]
    base = float(np.median(F[x >= base_from])) if (x >= base_from).any() else 0.0
    m = (F - base) > contact_above
    k = np.polyfit(x[m], F[m], 1)
    return float((base - k[1]) / k[0]), float(-k[0]), base


def oracle_env(gm, ol, model, cfg, objs):
    o = ol.OracleEnv(model, cfg, objs, 0)
    sp = gm.Spawn()
    sp.object_index, sp.x, sp.y, sp.zrot = 0, 0.0, 0.0, 0.0
    o.reset(sp)
    return o


class DeviceEnv1:
    """One device env (gmx.BatchedGripperEnv with n_envs = 1) behind the program interface."""

    def __init__(self, gm, model, cfg_settings, objs):
        self.env = gm.BatchedGripperEnv(1, object_set=None, objects=objs, settings=cfg_settings, seed=1,
                                        model_blob=model)
        sp = self.env.make_spawn(idx=0, x=0.0, y=0.0, rot=0.0)
        self.env.reset(spawn=sp)

    def set_motor_target(self, x, y, z):
        return bool(self.env.set_motor_target([x, y, z])[0])

    def action_step(self):
        self.env.action_step()

    def sensor_si(self):
        return self.env.sensor_si()[0]

    def close(self):
        self.env.close()
