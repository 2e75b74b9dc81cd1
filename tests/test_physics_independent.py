"""The physics oracle against references it does not share code or operation order with.

oracle/physics.c mirrors the device kernels lane for lane, so device == oracle shows the
HIP code does what the C code does, not that either does MuJoCo's mathematics.  These CPU
tests pin the oracle independently:

- kinematics, the joint-space inertia M and qfrc_bias against tests/indep_physics.py
  (natural-order FK, sum of J^T M_b J, per-body Newton-Euler with a complex-step J'),
  at 1e-12 of their scale, on reset states and on grasp states with random velocities;
- the narrowphase against closed-form answers: box-box face (aligned, rotated, clipped)
  and edge-edge, sphere-box (outside and inside), plane-cylinder rim points, plane-box
  corners, plane-sphere, and MPR on sphere-sphere, sphere-cylinder and cylinder-box
  (the cylinder object against the finger links: the MPR pair of the benched scenes);
- the oracle rebuilt with glibc sin / cos instead of gm_math.h's shared kernel: one
  substep from the same state agrees to rounding.
MuJoCo conventions: the contact normal points from geom1 to geom2 (geom1 = the lower
geom type), dist < 0 is penetration, the contact point is midway between the surfaces.
"""
import ctypes as C

import numpy as np
import pytest

import indep_physics as ip
import oracle_lib as ol

f64p = C.POINTER(C.c_double)


def _p(a):
    return np.ascontiguousarray(a, dtype=np.float64).ctypes.data_as(f64p)


@pytest.fixture(scope="module")
def world(gm):
    model = gm.ModelBlob()
    cfg = gm.ConfigBlob(gm.canonical_settings(noise=False, seed=3), model)
    objs = gm.make_object_set("set6_synthetic", 3)
    return gm, model, cfg, objs


def test_model_struct_layout(gm, world):
    _, model, _, _ = world
    from gmx._lib import struct_size
    assert C.sizeof(ip.GmModel) == struct_size(1)
    m = ip.model_view(model)
    assert (m.nbody, m.nv, m.nq) == (model.nbody, model.nv, model.nq)
    assert m.dof_obj == model.dof_obj and list(m.dof_pris) == model.dof_pris


def oracle_dynamics(L, h, model):
    nb, nv = model.nbody, model.nv
    bufs = [np.zeros(nb * 3), np.zeros(nb * 4), np.zeros(nv * nv), np.zeros(nv), np.zeros(nv)]
    L.or_dynamics(h, *[b.ctypes.data_as(f64p) for b in bufs])
    xpos, xquat, H, add, bias = bufs
    return xpos.reshape(nb, 3), xquat.reshape(nb, 4), H.reshape(nv, nv), add, bias


def dynamic_states(gm, model, cfg, objs, n_states=6, seed=11):
    """(qpos, qvel) pairs: a reset state, then grasp states of the scripted mix, each with
    random joint velocities added so Coriolis / centrifugal terms are large."""
    rng = np.random.default_rng(seed)
    o = ol.OracleEnv(model, cfg, objs, env_id=2)
    sp = gm.Spawn()
    sp.object_index, sp.x, sp.y, sp.zrot = 1, 0.004, -0.003, 0.3
    o.reset(sp)
    script = gm.GraspScript(cfg_settings(gm), 1, seed=5)
    out = []
    for k in range(48):
        if k % 8 == 0 and len(out) < n_states:
            q, v, _ = o.state()
            v = v + rng.normal(0.0, 0.5, size=v.shape)
            out.append((q.copy(), v))
        o.step(script.actions(k)[0])
    return o, out


def cfg_settings(gm):
    return gm.canonical_settings(noise=False, seed=3)


def test_kinematics_mass_matrix_and_bias_match_natural_order_newton_euler(world):
    gm, model, cfg, objs = world
    M = ip.Model(model)
    ip.set_object(M, objs[1])          # the live object of dynamic_states
    o, states = dynamic_states(gm, model, cfg, objs)
    assert len(states) >= 5
    for q, v in states:
        o.L.or_set_state(o.h, q.ctypes.data_as(f64p), v.ctypes.data_as(f64p))
        xpos, xquat, H, add, bias = oracle_dynamics(o.L, o.h, model)
        # forward kinematics
        xp_i, xq_i = ip.fk(M, q)
        np.testing.assert_allclose(xpos[1:], xp_i[1:], rtol=0, atol=1e-14)
        # quaternions up to sign
        s = np.sign(np.sum(xquat * xq_i, axis=1))[:, None]
        np.testing.assert_allclose(xquat[1:], (s * xq_i)[1:], rtol=0, atol=1e-14)
        # joint-space inertia: H~ minus its diagonal additions (armature, h (D + Kd), h^2 Kp)
        # is M; per entry within 1e-12 of sqrt(M_ii M_jj)
        Mo = H - np.diag(add) + np.diag(M.armature[M.jnt[M.dof_body]])
        Mi = ip.mass_matrix(M, q) + np.diag(M.armature[M.jnt[M.dof_body]])
        scale = np.sqrt(np.outer(np.diag(Mi), np.diag(Mi)))
        err = np.abs(Mo - Mi) / scale
        assert err.max() <= 1e-12, (err.max(), np.unravel_index(np.argmax(err), err.shape))
        np.testing.assert_allclose(Mo, Mo.T, rtol=0, atol=1e-15 * np.abs(Mo).max())
        # bias: Coriolis + centrifugal + gravity, within 1e-12 of the largest generalised
        # force magnitude in its dof's block (|M_d| |v|^2 + gravity scale)
        bi = ip.bias_force(M, q, v)
        sc = np.maximum(np.abs(bi), np.sqrt(np.diag(Mi)) * (1.0 + np.abs(v).max()) ** 2)
        berr = np.abs(bias - bi) / sc
        assert berr.max() <= 1e-12, (berr.max(), int(np.argmax(berr)))



def test_euler_implicit_damping_matches_dense_solve(world):
    """mj_Euler's implicit joint damping (MuJoCo 2.1.5, the default actuator order):
    qvel' = qvel + h (M + h D)^-1 (qfrc_smooth + qfrc_constraint).  The oracle's (and the
    device's, lane for lane) tree LDL^T of M + h D with the base as the border column is
    checked against a dense numpy solve built from the independent joint-space inertia
    (sum of J^T M_b J, tests/indep_physics.py) and the model's joint damping, on grasp
    states with contacts and random velocities.  At the solve's optimum qfrc_smooth +
    qfrc_constraint = M qacc (M with armature, the solve's matrix), so the right-hand side
    is formed from the solver's qacc; a capped solve carries the residual, see
    test_euler_damping_integrates_the_constraint_forces_on_capped_solves."""
    gm, model, cfg, objs = world
    M = ip.Model(model)
    ip.set_object(M, objs[1])
    damp = np.asarray(ip.arr(M.raw.jnt_damping), dtype=np.float64)[M.jnt[M.dof_body]]
    arm = M.armature[M.jnt[M.dof_body]]
    h = model.params.timestep
    o, states = dynamic_states(gm, model, cfg, objs)
    checked = 0
    for q, v in states:
        o.L.or_set_state(o.h, q.ctypes.data_as(f64p), v.ctypes.data_as(f64p))
        ncon, _, _, qacc = o.debug_substep()
        _, v1, _ = o.state()
        Mi = ip.mass_matrix(M, q) + np.diag(arm)
        qe = np.linalg.solve(Mi + h * np.diag(damp), Mi @ qacc)
        dv = (v1 - v) / h
        scale = np.abs(qe).max()
        assert np.abs(dv - qe).max() <= 1e-12 * scale, (np.abs(dv - qe).max(), scale)
        # the damping matters: the explicit update would be off by far more
        assert np.abs(qacc - qe).max() > 1e3 * np.abs(dv - qe).max()
        checked += ncon > 0
    assert checked >= 3


def test_euler_damping_integrates_the_constraint_forces_on_capped_solves(world):
    """MuJoCo's mj_Euler integrates qfrc_smooth + qfrc_constraint, qfrc_constraint = J^T efc of
    the solve's final forces.  At an optimum that is M qacc; a Newton solve capped before
    convergence (gm_model.newton_maxit = 1 forces it) leaves a residual, and the update must
    still be qvel' = qvel + h (M + h D)^-1 (qfrc_smooth + J^T efc).  Checked against a dense
    numpy solve with the independent joint-space inertia on grasp states, for the capped
    substeps (the correction is large there) and the converged ones."""
    gm, model, cfg, objs = world
    import ctypes as C
    capped_model = gm.ModelBlob(model.params)
    ip.GmModel.from_buffer(capped_model.buf).newton_maxit = 1
    ccfg = gm.ConfigBlob(gm.canonical_settings(noise=False, seed=3), capped_model)
    M = ip.Model(capped_model)
    ip.set_object(M, objs[1])
    damp = np.asarray(ip.arr(M.raw.jnt_damping), dtype=np.float64)[M.jnt[M.dof_body]]
    arm = M.armature[M.jnt[M.dof_body]]
    h = model.params.timestep
    _, states = dynamic_states(gm, model, cfg, objs)
    o = ol.OracleEnv(capped_model, ccfg, objs, env_id=2)
    sp = gm.Spawn()
    sp.object_index, sp.x, sp.y, sp.zrot = 1, 0.004, -0.003, 0.3
    o.reset(sp)
    o.L.or_want_forces(o.h, 1)
    seen = {True: 0, False: 0}
    fs, fc = np.zeros(model.nv), np.zeros(model.nv)
    for q, v in states:
        for _ in range(3):
            caps0 = int(gm.env_state_view(o.export_state())["newton_caps"])
            o.L.or_set_state(o.h, q.ctypes.data_as(f64p), v.ctypes.data_as(f64p))
            _, _, _, qacc = o.debug_substep()
            capped = int(gm.env_state_view(o.export_state())["newton_caps"]) > caps0
            _, v1, _ = o.state()
            o.L.or_last_forces(o.h, fs.ctypes.data_as(f64p), fc.ctypes.data_as(f64p))
            Mi = ip.mass_matrix(M, q) + np.diag(arm)
            qe = np.linalg.solve(Mi + h * np.diag(damp), fs + fc)
            dv = (v1 - v) / h
            scale = np.abs(qe).max()
            assert np.abs(dv - qe).max() <= 1e-9 * scale, (capped, np.abs(dv - qe).max(), scale)
            if capped:
                # the residual-free formula (M + h D)^-1 M qacc would be wrong here
                qe_opt = np.linalg.solve(Mi + h * np.diag(damp), Mi @ qacc)
                assert np.abs(qe_opt - qe).max() > 1e3 * np.abs(dv - qe).max()
            seen[capped] += 1
            q, v, _ = o.state()
    assert seen[True] >= 3 and seen[False] >= 1, seen

# ---------------------------------------------------------------- narrowphase
def collide(L, t1, s1, c1, R1, t2, s2, c2, R2, tol=1e-6, it=50):
    out = np.zeros(8 * 7)
    n = L.or_collide(int(t1), _p(np.resize(np.asarray(s1, float), 3)), _p(c1), _p(np.asarray(R1).ravel()), int(t2),
                     _p(np.resize(np.asarray(s2, float), 3)), _p(c2), _p(np.asarray(R2).ravel()), tol, it,
                     out.ctypes.data_as(f64p))
    r = out[:7 * n].reshape(n, 7)
    return r[:, 0], r[:, 1:4], r[:, 4:7]


def sorted_points(p):
    k = np.round(p, 9)
    return p[np.lexsort((k[:, 2], k[:, 1], k[:, 0]))]


I3 = np.eye(3)
BOX, CYL, SPH, PLANE = ip.GEOM_BOX, ip.GEOM_CYLINDER, ip.GEOM_SPHERE, ip.GEOM_PLANE


def test_box_box_face_contact_aligned():
    """A 4 cm cube resting 1 mm deep on a 10 x 10 x 2 cm slab: the four bottom corners,
    depth 1 mm, normal +z (slab -> cube), points midway through the overlap."""
    L = ol.lib()
    dist, pos, n = collide(L, BOX, [0.05, 0.05, 0.01], [0, 0, 0], I3, BOX, [0.02, 0.02, 0.02],
                           [0.003, -0.004, 0.01 + 0.02 - 0.001], I3)
    assert len(dist) == 4
    np.testing.assert_allclose(dist, -1e-3, rtol=0, atol=1e-15)
    np.testing.assert_allclose(n, np.tile([0, 0, 1.0], (4, 1)), atol=1e-15)
    exp = np.array([[0.003 + sx * 0.02, -0.004 + sy * 0.02, 0.0095] for sx in (-1, 1) for sy in (-1, 1)])
    np.testing.assert_allclose(sorted_points(pos), sorted_points(exp), rtol=0, atol=1e-15)


def test_box_box_face_contact_rotated_and_clipped():
    """(a) the cube turned 30 deg about z: the four rotated corners; (b) a bar overhanging
    a narrower block: the incident face clipped at the reference face's edges -- the
    manifold is the overlap rectangle's four corners."""
    L = ol.lib()
    Rz = ip.rotz(np.radians(30))
    c = np.array([0.0, 0.0, 0.01 + 0.02 - 0.002])
    dist, pos, n = collide(L, BOX, [0.05, 0.05, 0.01], [0, 0, 0], I3, BOX, [0.02, 0.02, 0.02], c, Rz)
    assert len(dist) == 4
    np.testing.assert_allclose(dist, -2e-3, atol=1e-15)
    np.testing.assert_allclose(n, np.tile([0, 0, 1.0], (4, 1)), atol=1e-15)
    exp = np.array([c[:2] + Rz[:2, :2] @ [sx * 0.02, sy * 0.02] for sx in (-1, 1) for sy in (-1, 1)])
    exp = np.column_stack([exp, np.full(4, 0.009)])
    np.testing.assert_allclose(sorted_points(pos), sorted_points(exp), atol=1e-15)
    # (b) block A 4 x 4 x 2 cm; bar B 6 x 2 x 2 cm on top, 0.5 mm deep
    dist, pos, n = collide(L, BOX, [0.02, 0.02, 0.01], [0, 0, 0], I3, BOX, [0.03, 0.01, 0.01],
                           [0, 0, 0.02 - 0.0005], I3)
    assert len(dist) == 4
    np.testing.assert_allclose(dist, -5e-4, atol=1e-15)
    np.testing.assert_allclose(n, np.tile([0, 0, 1.0], (4, 1)), atol=1e-15)
    exp = np.array([[sx * 0.02, sy * 0.01, 0.01 - 0.00025] for sx in (-1, 1) for sy in (-1, 1)])
    np.testing.assert_allclose(sorted_points(pos), sorted_points(exp), atol=1e-15)


def test_box_box_edge_edge():
    """Two cubes (half 2 cm) on crossed edges: A turned 45 deg about x (top edge along x at
    z = a sqrt 2), B turned 45 deg about y (bottom edge along y), 0.8 mm interpenetration:
    one contact midway between the edges, normal +z, depth 0.8 mm."""
    L = ol.lib()
    a, pen = 0.02, 0.8e-3
    zc = 2 * a * np.sqrt(2) - pen
    dist, pos, n = collide(L, BOX, [a, a, a], [0, 0, 0], ip.rotx(np.pi / 4), BOX, [a, a, a], [0, 0, zc],
                           ip.roty(np.pi / 4))
    assert len(dist) == 1
    np.testing.assert_allclose(dist, -pen, atol=1e-14)
    np.testing.assert_allclose(n[0], [0, 0, 1.0], atol=1e-14)
    np.testing.assert_allclose(pos[0], [0, 0, a * np.sqrt(2) - 0.5 * pen], atol=1e-14)


def test_sphere_box_outside_and_inside():
    """Sphere r = 1 cm pressed 2 mm into a box's top face (normal from the sphere into the
    box, -z; point midway between the sphere's surface and the face); then a sphere whose
    centre is inside the box, 3 mm below the nearest (+x) face."""
    L = ol.lib()
    hs = [0.05, 0.05, 0.02]
    c = np.array([0.01, -0.02, 0.02 + 0.01 - 0.002])
    dist, pos, n = collide(L, SPH, [0.01], c, I3, BOX, hs, [0, 0, 0], I3)
    assert len(dist) == 1
    np.testing.assert_allclose(dist, -2e-3, atol=1e-15)
    np.testing.assert_allclose(n[0], [0, 0, -1.0], atol=1e-15)
    np.testing.assert_allclose(pos[0], [0.01, -0.02, 0.019], atol=1e-15)
    # inside: centre 3 mm inside the +x face
    c = np.array([0.05 - 0.003, 0.01, 0.0])
    dist, pos, n = collide(L, SPH, [0.01], c, I3, BOX, hs, [0, 0, 0], I3)
    assert len(dist) == 1
    np.testing.assert_allclose(dist, -(0.003 + 0.01), atol=1e-15)
    np.testing.assert_allclose(n[0], [-1.0, 0, 0], atol=1e-15)
    # the face point and the sphere's far surface point, midway
    np.testing.assert_allclose(pos[0], [0.5 * (0.05 + (c[0] - 0.01)), 0.01, 0.0], atol=1e-15)


def test_plane_cylinder_plane_box_plane_sphere():
    """A cylinder (r 2 cm, half-height 3 cm) tilted 20 deg about x, its lowest rim point
    1.5 mm below the ground: that rim point (the only one below); a box tilted about z
    only, 1 mm into the ground: its four bottom corners; a sphere: one point."""
    L = ol.lib()
    r, hh, th, pen = 0.02, 0.03, np.radians(20), 1.5e-3
    Rx = ip.rotx(th)
    a = Rx[:, 2]
    w = -np.array([0, 0, 1.0]) + a[2] * a
    w /= np.linalg.norm(w)
    low = -hh * a + r * w                      # lowest rim point relative to the centre
    c = np.array([0.01, 0.02, -low[2] - pen])
    dist, pos, n = collide(L, PLANE, [10, 10, 0.1], [0, 0, 0], I3, CYL, [r, hh], c, Rx)
    assert len(dist) == 1
    np.testing.assert_allclose(dist, -pen, atol=1e-15)
    np.testing.assert_allclose(n[0], [0, 0, 1.0], atol=1e-15)
    p = c + low
    np.testing.assert_allclose(pos[0], p + [0, 0, 0.5 * pen], atol=1e-15)
    # box turned about z, 1 mm deep
    Rz = ip.rotz(0.7)
    hs = np.array([0.02, 0.01, 0.015])
    cb = np.array([0.0, 0.0, hs[2] - 1e-3])
    dist, pos, n = collide(L, PLANE, [10, 10, 0.1], [0, 0, 0], I3, BOX, hs, cb, Rz)
    assert len(dist) == 4
    np.testing.assert_allclose(dist, -1e-3, atol=1e-15)
    exp = np.array([cb + Rz @ [sx * hs[0], sy * hs[1], -hs[2]] for sx in (-1, 1) for sy in (-1, 1)])
    exp[:, 2] = -0.5e-3
    np.testing.assert_allclose(sorted_points(pos), sorted_points(exp), atol=1e-15)
    # sphere, 2 mm deep
    dist, pos, n = collide(L, PLANE, [10, 10, 0.1], [0, 0, 0], I3, SPH, [0.025], [0.1, 0.2, 0.023], I3)
    np.testing.assert_allclose(dist, [-2e-3], atol=1e-15)
    np.testing.assert_allclose(pos[0], [0.1, 0.2, -1e-3], atol=1e-15)


@pytest.mark.parametrize("direction", [[1, 0, 0], [0.3, -0.5, 0.8], [-0.2, 0.1, -0.9]])
def test_mpr_sphere_sphere_and_sphere_cylinder(direction):
    """MPR (libccd's, the convex fallback) on pairs with closed-form answers: two spheres
    (r 2 cm, 1.5 cm; centres 3 cm apart along `direction`): depth 5 mm, normal along the
    centre line, point midway through the overlap; a sphere against a cylinder's flat
    cap, 1 mm deep.  Within MPR's own tolerance (1e-6)."""
    L = ol.lib()
    u = np.asarray(direction, float)
    u /= np.linalg.norm(u)
    c1 = np.array([0.01, -0.02, 0.3])
    c2 = c1 + 0.03 * u
    # both spheres: the engine dispatches sphere-sphere to MPR
    dist, pos, n = collide(L, SPH, [0.02], c1, I3, SPH, [0.015], c2, I3)
    assert len(dist) == 1
    assert dist[0] == pytest.approx(-0.005, abs=1e-6)
    np.testing.assert_allclose(n[0], u, atol=1e-6 / 0.005)
    mid = c1 + u * (0.02 - 0.0025)
    np.testing.assert_allclose(pos[0], mid, atol=2e-6)
    # sphere (r 1 cm) on a cylinder's top cap (r 2 cm, half-height 3 cm), 1 mm deep
    cc = np.array([0.0, 0.0, 0.0])
    cs = np.array([0.004, -0.003, 0.03 + 0.01 - 0.001])
    dist, pos, n = collide(L, SPH, [0.01], cs, I3, CYL, [0.02, 0.03], cc, I3)
    assert len(dist) == 1
    assert dist[0] == pytest.approx(-0.001, abs=1e-6)
    np.testing.assert_allclose(n[0], [0, 0, -1.0], atol=2e-3)


@pytest.mark.parametrize("yaw", [0.0, 0.4])
def test_mpr_cylinder_box(yaw):
    """MPR on a cylinder (r 2 cm, half-height 3 cm) against a box (5 x 4 x 1 cm half
    sizes, top face at z = 1 cm, turned `yaw` about z): upright on its bottom cap 1 mm into
    the top face, then lying on its side (axis along x) 0.8 mm into it.  Depth to MPR's
    tolerance (1e-6); the normal points from geom1 (the cylinder, above) into the box, -z."""
    L = ol.lib()
    r, hh = 0.02, 0.03
    hs, Rb = [0.05, 0.04, 0.01], ip.rotz(yaw)
    for Rc, zc, pen in ((I3, 0.01 + hh - 1e-3, 1e-3), (ip.roty(np.pi / 2), 0.01 + r - 0.8e-3, 0.8e-3)):
        c = np.array([0.004, -0.006, zc])
        dist, pos, n = collide(L, CYL, [r, hh], c, Rc, BOX, hs, [0, 0, 0], Rb)
        assert len(dist) == 1
        assert dist[0] == pytest.approx(-pen, abs=1e-6)
        np.testing.assert_allclose(n[0], [0, 0, -1.0], atol=2e-3)
        # the point lies inside the overlap slab, under the cylinder's footprint
        assert 0.01 - pen - 1e-6 <= pos[0][2] <= 0.01 + 1e-6
        assert abs(pos[0][0] - c[0]) <= (hh if Rc is not I3 else r) + 1e-9
        assert abs(pos[0][1] - c[1]) <= r + 1e-9


def test_oracle_with_libm_trig_agrees(world):
    """The oracle rebuilt with glibc sin / cos (oracle/Makefile liboracle_libm.so) against
    the shared gm_math.h kernel: one substep from the same grasp state gives the same
    contacts and qacc to rounding, and one env-step the same observations -- the shared
    sine / cosine is a bit-for-bit convenience, not a source of agreement."""
    gm, model, cfg, objs = world
    Lm = ol.lib_libm()
    o, states = dynamic_states(gm, model, cfg, objs, n_states=1)
    n = int(ol.lib().or_state_size())
    st = np.zeros(n, dtype=np.uint8)
    o.L.or_export_state(o.h, st.ctypes.data_as(C.c_void_p))
    om = ol.OracleEnv.__new__(ol.OracleEnv)
    om.L, om.model, om.cfg, om.objects = Lm, model, cfg, objs
    om.h = Lm.or_create(model.ptr, cfg.ptr, C.cast(objs, C.c_void_p), len(objs), 2)
    om.n_obs, om.n_actions = cfg.n_obs, cfg.n_actions
    assert Lm.or_import_state(om.h, st.ctypes.data_as(C.c_void_p)) == 0
    from gmx._lib import GM_MAX_CON, GM_MAX_DOF, GM_MAX_EFC
    outs = []
    for L, h in ((o.L, o.h), (Lm, om.h)):
        ncon = np.zeros(1, np.int32)
        con = np.zeros(GM_MAX_CON * 16); efc = np.zeros(GM_MAX_EFC); qacc = np.zeros(GM_MAX_DOF); w = np.zeros(6)
        L.or_debug_substep(h, ncon.ctypes.data_as(C.POINTER(C.c_int32)), con.ctypes.data_as(f64p),
                           efc.ctypes.data_as(f64p), qacc.ctypes.data_as(f64p), w.ctypes.data_as(f64p))
        outs.append((int(ncon[0]), con.reshape(GM_MAX_CON, 16), qacc[:model.nv].copy()))
    (n0, c0, a0), (n1, c1, a1) = outs
    assert n0 == n1 and n0 > 0
    np.testing.assert_array_equal(c0[:n0, 13:15], c1[:n1, 13:15])
    np.testing.assert_allclose(c1[:n0, :13], c0[:n0, :13], rtol=0, atol=1e-13)
    qs = max(1.0, np.abs(a0).max())
    np.testing.assert_allclose(a1 / qs, a0 / qs, rtol=0, atol=1e-10)
    # one env-step from the same state on both builds
    assert o.L.or_import_state(o.h, st.ctypes.data_as(C.c_void_p)) == 0
    assert Lm.or_import_state(om.h, st.ctypes.data_as(C.c_void_p)) == 0
    a = np.array([0.3, -0.2, 0.1, 0.0], dtype=np.float32)[:cfg.n_actions]
    ob0, _, d0 = o.step(a)
    ob1, _, d1 = om.step(a)
    np.testing.assert_allclose(ob1, ob0, rtol=1e-6, atol=1e-6)
    assert d0 == d1
