"""Independent references for the physics the oracle restates (test infrastructure only).

The oracle (oracle/physics.c) follows the device kernels operation for operation -- the
same world-origin Plucker algebra, the same segmented scans, the same sin / cos -- so
device-vs-oracle agreement cannot catch an algorithmic error they share.  This module
computes the same quantities a different way, from the model arrays alone:

- forward kinematics body by body in natural (parent-first) order, MuJoCo's conventions
  (mj_kinematics): body frame = parent frame x (body_pos, body_quat), then the joint
  (slide: along the body-frame axis; hinge: about the body-frame axis through jnt_pos;
  free: world position + quaternion);
- the joint-space inertia as the sum over bodies of J^T M_b J with each body's
  centre-of-mass Jacobian (no composite inertias, no recursion);
- qfrc_bias (Coriolis, centrifugal, gravity) from each body's Newton-Euler equations,
  m (a_c - g) and I w' + w x I w, with the Jacobian's time derivative taken by the
  complex-step method along the motion q(t) (exact to rounding, no finite-difference
  truncation), instead of the oracle's recursive Newton-Euler;
- analytic answers for the narrowphase cases the colliders handle.

Everything is numpy, complex-capable where the complex step needs it.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from gmx._lib import GM_MAX_BODY, GM_MAX_DOF, GM_MAX_QPOS

GM_MAX_GEOM = 40
GM_MAX_PAIR = 80
GM_MAX_LOCK = 4
JNT_FREE, JNT_SLIDE, JNT_HINGE = 0, 2, 3
GEOM_PLANE, GEOM_SPHERE, GEOM_CYLINDER, GEOM_BOX = 0, 2, 5, 6

_i, _d = C.c_int32, C.c_double


class GmModel(C.Structure):
    """include/gripper_mi355x.h gm_model, field for field (checked against sizeof)."""
    _fields_ = [
        ("nbody", _i), ("njnt", _i), ("nq", _i), ("nv", _i), ("ngeom", _i), ("npair", _i), ("nlock", _i),
        ("n_seg", _i),
        ("body_parent", _i * GM_MAX_BODY), ("body_jnt", _i * GM_MAX_BODY), ("body_group", _i * GM_MAX_BODY),
        ("body_pos", _d * 3 * GM_MAX_BODY), ("body_quat", _d * 4 * GM_MAX_BODY), ("body_mass", _d * GM_MAX_BODY),
        ("body_ipos", _d * 3 * GM_MAX_BODY), ("body_inertia", _d * 3 * GM_MAX_BODY),
        ("jnt_type", _i * GM_MAX_BODY), ("jnt_body", _i * GM_MAX_BODY), ("jnt_qposadr", _i * GM_MAX_BODY),
        ("jnt_dofadr", _i * GM_MAX_BODY),
        ("jnt_pos", _d * 3 * GM_MAX_BODY), ("jnt_axis", _d * 3 * GM_MAX_BODY), ("jnt_stiffness", _d * GM_MAX_BODY),
        ("jnt_damping", _d * GM_MAX_BODY), ("jnt_armature", _d * GM_MAX_BODY),
        ("dof_parent", _i * GM_MAX_DOF), ("dof_body", _i * GM_MAX_DOF), ("dof_group", _i * GM_MAX_DOF),
        ("dof_slot", _i * GM_MAX_DOF),
        ("geom_type", _i * GM_MAX_GEOM), ("geom_body", _i * GM_MAX_GEOM), ("geom_class", _i * GM_MAX_GEOM),
        ("geom_pos", _d * 3 * GM_MAX_GEOM), ("geom_quat", _d * 4 * GM_MAX_GEOM), ("geom_size", _d * 3 * GM_MAX_GEOM),
        ("geom_friction", _d * GM_MAX_GEOM), ("geom_rbound", _d * GM_MAX_GEOM),
        ("pair_a", _i * GM_MAX_PAIR), ("pair_b", _i * GM_MAX_PAIR),
        ("lock_dof", _i * GM_MAX_LOCK), ("lock_kind", _i * GM_MAX_LOCK),
        ("qpos0", _d * GM_MAX_QPOS),
        ("body_invweight0", _d * 2 * GM_MAX_BODY), ("dof_invweight0", _d * GM_MAX_DOF),
        ("dof_base", _i), ("dof_palm", _i), ("dof_obj", _i),
        ("dof_pris", _i * 3), ("dof_rev", _i * 3), ("dof_seg", _i * 3),
        ("body_base", _i), ("body_finger", _i * 3), ("body_palm", _i), ("body_obj", _i), ("geom_obj", _i),
        ("geom_ground", _i),
        ("timestep", _d), ("gravity", _d * 3), ("solref", _d * 2), ("solimp", _d * 5),
        ("pgs_iterations", _i), ("mpr_tolerance", _d), ("mpr_iterations", _i),
        ("finger_length", _d), ("finger_width", _d), ("finger_thickness", _d), ("finger_E", _d), ("finger_EI", _d),
        ("segment_length", _d), ("hook_length", _d), ("hook_angle_degrees", _d), ("fingertip_clearance", _d),
        ("yield_stress", _d), ("fixed_first_segment", _i),
        ("kp_gripper", _d * 3), ("kd_gripper", _d * 3), ("kp_base", _d * 3), ("kd_base", _d * 3),
        ("time_per_step", _d), ("stepper_num_steps", _i),
        ("gauge_xpos", _d), ("gauge_order", _i),
        ("body_tip", _i * 3), ("tip_dir", _d * 3 * 3),
        ("mujoco_actuators", _i), ("newton_maxit", _i),
    ]


def model_view(model_blob) -> GmModel:
    """The compiled model (gmx.ModelBlob) as a ctypes struct (a copy)."""
    m = GmModel()
    C.memmove(C.byref(m), model_blob.buf, C.sizeof(GmModel))
    return m


def arr(x, *shape):
    return np.ctypeslib.as_array(x).reshape(shape).astype(np.float64) if shape else np.ctypeslib.as_array(x)


# ---------------------------------------------------------------- rotations (complex-safe)
def quat2mat(q):
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def quatmul(a, b):
    return np.array([a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
                     a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
                     a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
                     a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]])


def qnormalise(q):
    return q / np.sqrt(np.sum(q * q))


class Model:
    """The model arrays the references need, as numpy."""

    def __init__(self, model_blob):
        m = model_view(model_blob)
        self.raw = m
        self.nbody, self.nv, self.nq = m.nbody, m.nv, m.nq
        nb = m.nbody
        self.parent = arr(m.body_parent)[:nb].copy()
        self.jnt = arr(m.body_jnt)[:nb].copy()
        self.pos = arr(m.body_pos, GM_MAX_BODY, 3)[:nb]
        self.quat = arr(m.body_quat, GM_MAX_BODY, 4)[:nb]
        self.mass = arr(m.body_mass).astype(np.float64)[:nb]
        self.ipos = arr(m.body_ipos, GM_MAX_BODY, 3)[:nb]
        self.inertia = arr(m.body_inertia, GM_MAX_BODY, 3)[:nb]
        self.jtype = arr(m.jnt_type).copy()
        self.jqadr = arr(m.jnt_qposadr).copy()
        self.jdadr = arr(m.jnt_dofadr).copy()
        self.jpos = arr(m.jnt_pos, GM_MAX_BODY, 3)
        self.jaxis = arr(m.jnt_axis, GM_MAX_BODY, 3)
        self.armature = arr(m.jnt_armature).astype(np.float64)
        self.dof_body = arr(m.dof_body)[:m.nv].copy()
        self.gravity = np.array(m.gravity[:])


def set_object(M: Model, obj):
    """The live object's mass and principal inertia from its shape (uniform solids:
    box m (b^2 + c^2) / 12 over full edge lengths; cylinder m r^2 / 2 about its axis and
    m (3 r^2 + h^2) / 12 across; sphere 2 m r^2 / 5)."""
    b = M.raw.body_obj
    m, t, sz = float(obj.mass), int(obj.type), [float(x) for x in obj.size]
    if t == GEOM_BOX:
        a, bb, c = 2 * sz[0], 2 * sz[1], 2 * sz[2]
        I = [m * (bb * bb + c * c) / 12, m * (a * a + c * c) / 12, m * (a * a + bb * bb) / 12]
    elif t == GEOM_CYLINDER:
        r, h = sz[0], 2 * sz[1]
        I = [m * (3 * r * r + h * h) / 12] * 2 + [m * r * r / 2]
    else:
        I = [2 * m * sz[0] ** 2 / 5] * 3
    M.mass[b] = m
    M.inertia[b] = I


def fk(M: Model, qpos):
    """mj_kinematics in natural order: world positions / orientations of every body (the
    dtype of qpos -- complex for the complex step)."""
    dt = np.result_type(qpos, np.float64)
    xpos = np.zeros((M.nbody, 3), dtype=dt)
    xquat = np.zeros((M.nbody, 4), dtype=dt)
    xquat[0, 0] = 1
    for b in range(1, M.nbody):
        p = M.parent[b]
        Rp = quat2mat(xquat[p])
        pb = xpos[p] + Rp @ M.pos[b]
        qb = quatmul(xquat[p], M.quat[b])
        j = M.jnt[b]
        if j >= 0:
            qa = M.jqadr[j]
            t = M.jtype[j]
            if t == JNT_FREE:
                pb = qpos[qa:qa + 3].astype(dt)
                qb = qpos[qa + 3:qa + 7].astype(dt)
            elif t == JNT_SLIDE:
                pb = pb + quat2mat(qb) @ M.jaxis[j] * qpos[qa]
            elif t == JNT_HINGE:
                anchor = pb + quat2mat(qb) @ M.jpos[j]
                h = 0.5 * qpos[qa]
                qb = quatmul(qb, np.concatenate([[np.cos(h)], M.jaxis[j] * np.sin(h)]))
                pb = anchor - quat2mat(qb) @ M.jpos[j]
        xpos[b] = pb
        xquat[b] = qnormalise(qb)
    return xpos, xquat


def jacobians(M: Model, qpos):
    """Centre-of-mass Jacobians (translation Jp [nbody, 3, nv], rotation Jr) and the
    world inertia tensors, from the natural-order kinematics: a hinge dof contributes
    axis x (c - anchor) / axis, a slide its axis, the free joint world translation and
    body-frame rotation (MuJoCo's free-joint velocity convention)."""
    xpos, xquat = fk(M, qpos)
    dt = xpos.dtype
    nb, nv = M.nbody, M.nv
    R = [quat2mat(xquat[b]) for b in range(nb)]
    com = np.array([xpos[b] + R[b] @ M.ipos[b] for b in range(nb)], dtype=dt)
    Jp = np.zeros((nb, 3, nv), dtype=dt)
    Jr = np.zeros((nb, 3, nv), dtype=dt)
    for b in range(1, nb):
        a = b
        while a > 0:
            j = M.jnt[a]
            if j >= 0:
                d0, t = M.jdadr[j], M.jtype[j]
                if t == JNT_FREE:
                    for k in range(3):
                        Jp[b, k, d0 + k] = 1.0
                        w = R[a][:, k]
                        Jr[b, :, d0 + 3 + k] = w
                        Jp[b, :, d0 + 3 + k] = np.cross(w, com[b] - xpos[a])
                else:
                    ax = R[a] @ M.jaxis[j]
                    if t == JNT_SLIDE:
                        Jp[b, :, d0] = ax
                    else:
                        anchor = xpos[a] + R[a] @ M.jpos[j]
                        Jr[b, :, d0] = ax
                        Jp[b, :, d0] = np.cross(ax, com[b] - anchor)
            a = M.parent[a]
    Iw = np.array([R[b] @ np.diag(M.inertia[b]) @ R[b].T for b in range(nb)], dtype=dt)
    return Jp, Jr, Iw, xpos, xquat


def mass_matrix(M: Model, qpos):
    """sum_b m_b Jp^T Jp + Jr^T I_w Jr (without armature)."""
    Jp, Jr, Iw, _, _ = jacobians(M, qpos)
    Mq = np.zeros((M.nv, M.nv))
    for b in range(1, M.nbody):
        Mq += M.mass[b] * Jp[b].T @ Jp[b] + Jr[b].T @ Iw[b] @ Jr[b]
    return Mq


def _qpos_along(M: Model, qpos, qvel, t):
    """q(t) along the motion with velocity qvel (hinge / slide linear in t; the free joint
    translates in world and rotates about its body-frame angular velocity)."""
    q = qpos.astype(np.complex128 if np.iscomplexobj(t) else np.float64)
    for b in range(1, M.nbody):
        j = M.jnt[b]
        if j < 0:
            continue
        qa, d0 = M.jqadr[j], M.jdadr[j]
        if M.jtype[j] == JNT_FREE:
            q[qa:qa + 3] = qpos[qa:qa + 3] + t * qvel[d0:d0 + 3]
            w = qvel[d0 + 3:d0 + 6]
            wn = np.linalg.norm(w)
            if wn > 0:
                h = 0.5 * wn * t
                dq = np.concatenate([[np.cos(h)], w / wn * np.sin(h)])
                q[qa + 3:qa + 7] = quatmul(qpos[qa + 3:qa + 7], dq)
        else:
            q[qa] = qpos[qa] + t * qvel[d0]
    return q


def bias_force(M: Model, qpos, qvel, h=1e-30):
    """qfrc_bias = sum_b Jp^T m (Jp' qd - g) + Jr^T (I_w Jr' qd + w x I_w w): each body's
    Newton-Euler equations at zero joint acceleration, J' = dJ/dt by the complex step."""
    qpos = np.asarray(qpos, dtype=np.float64)
    qvel = np.asarray(qvel, dtype=np.float64)
    Jp, Jr, Iw, _, _ = jacobians(M, qpos)
    Jpc, Jrc, _, _, _ = jacobians(M, _qpos_along(M, qpos, qvel, 1j * h))
    dJp = Jpc.imag / h
    dJr = Jrc.imag / h
    bias = np.zeros(M.nv)
    for b in range(1, M.nbody):
        ac = dJp[b] @ qvel - M.gravity
        w = Jr[b] @ qvel
        al = dJr[b] @ qvel
        tau = Iw[b] @ al + np.cross(w, Iw[b] @ w)
        bias += Jp[b].T @ (M.mass[b] * ac) + Jr[b].T @ tau
    return bias


# ---------------------------------------------------------------- collider helpers
def rotz(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1.0]])


def rotx(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[1.0, 0, 0], [0, c, -s], [0, s, c]])


def roty(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1.0, 0], [-s, 0, c]])
