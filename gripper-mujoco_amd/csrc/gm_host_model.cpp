// gm_host_model.cpp -- host-side model compiler, settings defaults and derived
// configuration for the MI355X gripper env-step path.
//
// The reference loads a generated MJCF (mj_loadXML, mjclass.cpp:377-409) whose
// source lives in the empty `description` submodule.  Here the same gripper is
// compiled directly from the numerics the reference reads out of that MJCF
// (read_gripper_dimensions, myfunctions.cpp:836-953) and the constants it
// hard-codes (JointSettings, myfunctions.cpp:166-296).  Values the MJCF alone
// holds (masses, damping, collision thickness, solref/solimp) are invented and
// listed in DESIGN.md section "Model spec".
#include "gripper_mi355x.h"

#include <algorithm>
#include <cmath>
#include <vector>
#include <cstring>
#include <cstdint>
#include <string>

namespace {

constexpr double kPi = 3.14159265358979323846;
constexpr double kSteelDensity = 7850.0;

void quat_from_mat(const double R[9], double q[4]) {
  // R row-major; columns are the body axes in the parent frame.
  double tr = R[0] + R[4] + R[8];
  if (tr > 0) {
    double s = std::sqrt(tr + 1.0) * 2;
    q[0] = 0.25 * s;
    q[1] = (R[7] - R[5]) / s;
    q[2] = (R[2] - R[6]) / s;
    q[3] = (R[3] - R[1]) / s;
  } else if (R[0] > R[4] && R[0] > R[8]) {
    double s = std::sqrt(1.0 + R[0] - R[4] - R[8]) * 2;
    q[0] = (R[7] - R[5]) / s;
    q[1] = 0.25 * s;
    q[2] = (R[1] + R[3]) / s;
    q[3] = (R[2] + R[6]) / s;
  } else if (R[4] > R[8]) {
    double s = std::sqrt(1.0 + R[4] - R[0] - R[8]) * 2;
    q[0] = (R[2] - R[6]) / s;
    q[1] = (R[1] + R[3]) / s;
    q[2] = 0.25 * s;
    q[3] = (R[5] + R[7]) / s;
  } else {
    double s = std::sqrt(1.0 + R[8] - R[0] - R[4]) * 2;
    q[0] = (R[3] - R[1]) / s;
    q[1] = (R[2] + R[6]) / s;
    q[2] = (R[5] + R[7]) / s;
    q[3] = 0.25 * s;
  }
  double n = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  for (int i = 0; i < 4; i++) q[i] /= n;
}

void set3(double* d, double a, double b, double c) { d[0] = a; d[1] = b; d[2] = c; }
void set4(double* d, double a, double b, double c, double e) { d[0] = a; d[1] = b; d[2] = c; d[3] = e; }

struct Builder {
  gm_model* m;
  int add_body(int parent, int group, const double pos[3], const double quat[4],
               double mass, const double ipos[3], const double inertia[3]) {
    int b = m->nbody++;
    m->body_parent[b] = parent;
    m->body_group[b] = group;
    m->body_jnt[b] = -1;
    for (int i = 0; i < 3; i++) m->body_pos[b][i] = pos[i];
    for (int i = 0; i < 4; i++) m->body_quat[b][i] = quat[i];
    m->body_mass[b] = mass;
    for (int i = 0; i < 3; i++) m->body_ipos[b][i] = ipos[i];
    for (int i = 0; i < 3; i++) m->body_inertia[b][i] = inertia[i];
    return b;
  }
  int add_joint(int body, int type, const double axis[3], double stiffness, double damping,
                double armature, int parent_dof) {
    int j = m->njnt++;
    m->body_jnt[body] = j;
    m->jnt_type[j] = type;
    m->jnt_body[j] = body;
    m->jnt_qposadr[j] = m->nq;
    m->jnt_dofadr[j] = m->nv;
    set3(m->jnt_pos[j], 0, 0, 0);
    for (int i = 0; i < 3; i++) m->jnt_axis[j][i] = axis[i];
    m->jnt_stiffness[j] = stiffness;
    m->jnt_damping[j] = damping;
    m->jnt_armature[j] = armature;
    int ndof = (type == GM_JNT_FREE) ? 6 : 1;
    m->nq += (type == GM_JNT_FREE) ? 7 : 1;
    for (int k = 0; k < ndof; k++) {
      int d = m->nv++;
      m->dof_parent[d] = (k == 0) ? parent_dof : d - 1;
      m->dof_body[d] = body;
      m->dof_group[d] = m->body_group[body];
    }
    return m->jnt_dofadr[j];
  }
  int add_geom(int body, int type, int cls, const double pos[3], const double quat[4],
               const double size[3], double friction) {
    int g = m->ngeom++;
    m->geom_type[g] = type;
    m->geom_body[g] = body;
    m->geom_class[g] = cls;
    for (int i = 0; i < 3; i++) m->geom_pos[g][i] = pos[i];
    for (int i = 0; i < 4; i++) m->geom_quat[g][i] = quat[i];
    for (int i = 0; i < 3; i++) m->geom_size[g][i] = size[i];
    m->geom_friction[g] = friction;
    double rb = 0;
    if (type == GM_GEOM_BOX) rb = std::sqrt(size[0] * size[0] + size[1] * size[1] + size[2] * size[2]);
    else if (type == GM_GEOM_SPHERE) rb = size[0];
    else if (type == GM_GEOM_CYLINDER) rb = std::sqrt(size[0] * size[0] + size[1] * size[1]);
    else if (type == GM_GEOM_CAPSULE) rb = size[0] + size[1];
    m->geom_rbound[g] = rb;
    return g;
  }
};

void box_inertia(double mass, double hx, double hy, double hz, double out[3]) {
  out[0] = mass * (4 * hy * hy + 4 * hz * hz) / 12.0;
  out[1] = mass * (4 * hx * hx + 4 * hz * hz) / 12.0;
  out[2] = mass * (4 * hx * hx + 4 * hy * hy) / 12.0;
}

}  // namespace

void gm_derive_model_constants(gm_model* m);
void gm_derive_invweights(gm_model* m);

// mj_setConst's body_invweight0 / dof_invweight0 at qpos0 (the inputs of mj_diagApprox):
// forward kinematics, the joint-space inertia M (composite rigid bodies, + armature), the
// centre-of-mass Jacobian of every body, A = J M^-1 J^T; a body's translational /
// rotational weight is the mean of A's translational / rotational diagonal, a slide or
// hinge dof's the diagonal of M^-1, a free joint's the mean of its three translational /
// rotational diagonal entries.  Dense and sequential: a one-time host computation.
void gm_derive_invweights(gm_model* m) {
  const int nb = m->nbody, nv = m->nv;
  std::vector<double> xpos(3 * nb, 0.0), xq(4 * nb, 0.0), R(9 * nb, 0.0), xi(3 * nb, 0.0);
  std::vector<double> cdof(6 * nv, 0.0), cin(10 * nb, 0.0);
  auto qmul = [](const double* a, const double* b, double* r) {
    const double t0 = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
    const double t1 = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
    const double t2 = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
    const double t3 = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
    r[0] = t0; r[1] = t1; r[2] = t2; r[3] = t3;
  };
  auto q2m = [](const double* q, double* M) {
    const double w = q[0], x = q[1], y = q[2], z = q[3];
    M[0] = 1 - 2 * (y * y + z * z); M[1] = 2 * (x * y - w * z); M[2] = 2 * (x * z + w * y);
    M[3] = 2 * (x * y + w * z); M[4] = 1 - 2 * (x * x + z * z); M[5] = 2 * (y * z - w * x);
    M[6] = 2 * (x * z - w * y); M[7] = 2 * (y * z + w * x); M[8] = 1 - 2 * (x * x + y * y);
  };
  auto cross = [](const double* a, const double* b, double* r) {
    const double t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
    r[0] = t0; r[1] = t1; r[2] = t2;
  };
  xq[0] = 1;
  q2m(&xq[0], &R[0]);
  for (int b = 1; b < nb; b++) {
    const int p = m->body_parent[b];
    for (int i = 0; i < 3; i++)
      xpos[3 * b + i] = xpos[3 * p + i] + R[9 * p + 3 * i] * m->body_pos[b][0] + R[9 * p + 3 * i + 1] * m->body_pos[b][1] +
                        R[9 * p + 3 * i + 2] * m->body_pos[b][2];
    qmul(&xq[4 * p], m->body_quat[b], &xq[4 * b]);
    const int j = m->body_jnt[b];
    if (j >= 0) {
      const int qa = m->jnt_qposadr[j];
      if (m->jnt_type[j] == GM_JNT_SLIDE) {
        double Rb[9];
        q2m(&xq[4 * b], Rb);
        for (int i = 0; i < 3; i++)
          xpos[3 * b + i] += (Rb[3 * i] * m->jnt_axis[j][0] + Rb[3 * i + 1] * m->jnt_axis[j][1] + Rb[3 * i + 2] * m->jnt_axis[j][2]) * m->qpos0[qa];
      } else if (m->jnt_type[j] == GM_JNT_HINGE) {
        const double s = std::sin(0.5 * m->qpos0[qa]), c = std::cos(0.5 * m->qpos0[qa]);
        const double ql[4] = {c, m->jnt_axis[j][0] * s, m->jnt_axis[j][1] * s, m->jnt_axis[j][2] * s};
        double t[4];
        qmul(&xq[4 * b], ql, t);
        for (int k = 0; k < 4; k++) xq[4 * b + k] = t[k];
      } else if (m->jnt_type[j] == GM_JNT_FREE) {
        for (int k = 0; k < 3; k++) xpos[3 * b + k] = m->qpos0[qa + k];
        for (int k = 0; k < 4; k++) xq[4 * b + k] = m->qpos0[qa + 3 + k];
      }
    }
    double n = 0;
    for (int k = 0; k < 4; k++) n += xq[4 * b + k] * xq[4 * b + k];
    n = std::sqrt(n);
    if (n < 1e-15) { xq[4 * b] = 1; xq[4 * b + 1] = xq[4 * b + 2] = xq[4 * b + 3] = 0; }
    else for (int k = 0; k < 4; k++) xq[4 * b + k] /= n;
    q2m(&xq[4 * b], &R[9 * b]);
    for (int i = 0; i < 3; i++)
      xi[3 * b + i] = xpos[3 * b + i] + R[9 * b + 3 * i] * m->body_ipos[b][0] + R[9 * b + 3 * i + 1] * m->body_ipos[b][1] +
                      R[9 * b + 3 * i + 2] * m->body_ipos[b][2];
    // spatial inertia about the world origin
    const double* Rb = &R[9 * b];
    const double* I = m->body_inertia[b];
    const double mass = m->body_mass[b];
    const double* c = &xi[3 * b];
    double Iw[9];
    for (int i = 0; i < 3; i++)
      for (int k = 0; k < 3; k++)
        Iw[3 * i + k] = Rb[3 * i] * I[0] * Rb[3 * k] + Rb[3 * i + 1] * I[1] * Rb[3 * k + 1] + Rb[3 * i + 2] * I[2] * Rb[3 * k + 2];
    const double cc = c[0] * c[0] + c[1] * c[1] + c[2] * c[2];
    double* ci = &cin[10 * b];
    ci[0] = Iw[0] + mass * (cc - c[0] * c[0]); ci[1] = Iw[4] + mass * (cc - c[1] * c[1]); ci[2] = Iw[8] + mass * (cc - c[2] * c[2]);
    ci[3] = Iw[1] - mass * c[0] * c[1]; ci[4] = Iw[2] - mass * c[0] * c[2]; ci[5] = Iw[5] - mass * c[1] * c[2];
    ci[6] = mass * c[0]; ci[7] = mass * c[1]; ci[8] = mass * c[2]; ci[9] = mass;
  }
  for (int d = 0; d < nv; d++) {
    const int b = m->dof_body[d], j = m->body_jnt[b];
    double* cd = &cdof[6 * d];
    const double* Rb = &R[9 * b];
    if (m->jnt_type[j] == GM_JNT_FREE) {
      const int k = d - m->jnt_dofadr[j];
      for (int t = 0; t < 6; t++) cd[t] = 0;
      if (k < 3) cd[3 + k] = 1;
      else { const double w[3] = {Rb[k - 3], Rb[3 + k - 3], Rb[6 + k - 3]}; cd[0] = w[0]; cd[1] = w[1]; cd[2] = w[2]; cross(&xpos[3 * b], w, cd + 3); }
    } else {
      double wa[3];
      for (int i = 0; i < 3; i++) wa[i] = Rb[3 * i] * m->jnt_axis[j][0] + Rb[3 * i + 1] * m->jnt_axis[j][1] + Rb[3 * i + 2] * m->jnt_axis[j][2];
      if (m->jnt_type[j] == GM_JNT_SLIDE) { cd[0] = cd[1] = cd[2] = 0; cd[3] = wa[0]; cd[4] = wa[1]; cd[5] = wa[2]; }
      else { cd[0] = wa[0]; cd[1] = wa[1]; cd[2] = wa[2]; cross(&xpos[3 * b], wa, cd + 3); }
    }
  }
  // composite inertias and M (CRB), + armature
  std::vector<double> Ic(cin);
  for (int b = nb - 1; b > 0; b--) {
    const int p = m->body_parent[b];
    if (p > 0) for (int k = 0; k < 10; k++) Ic[10 * p + k] += Ic[10 * b + k];
  }
  auto imul = [](const double* ci, const double* v, double* r) {
    const double* w = v; const double* u = v + 3;
    const double hxu[3] = {ci[7] * u[2] - ci[8] * u[1], ci[8] * u[0] - ci[6] * u[2], ci[6] * u[1] - ci[7] * u[0]};
    const double hxw[3] = {ci[7] * w[2] - ci[8] * w[1], ci[8] * w[0] - ci[6] * w[2], ci[6] * w[1] - ci[7] * w[0]};
    r[0] = ci[0] * w[0] + ci[3] * w[1] + ci[4] * w[2] + hxu[0];
    r[1] = ci[3] * w[0] + ci[1] * w[1] + ci[5] * w[2] + hxu[1];
    r[2] = ci[4] * w[0] + ci[5] * w[1] + ci[2] * w[2] + hxu[2];
    r[3] = ci[9] * u[0] - hxw[0]; r[4] = ci[9] * u[1] - hxw[1]; r[5] = ci[9] * u[2] - hxw[2];
  };
  std::vector<double> M(nv * nv, 0.0);
  for (int j = 0; j < nv; j++) {
    double F[6];
    imul(&Ic[10 * m->dof_body[j]], &cdof[6 * j], F);
    for (int i = j; i >= 0; i = m->dof_parent[i]) {
      double v = 0;
      for (int t = 0; t < 6; t++) v += cdof[6 * i + t] * F[t];
      M[j * nv + i] = v; M[i * nv + j] = v;
    }
    M[j * nv + j] += m->jnt_armature[m->body_jnt[m->dof_body[j]]];
  }
  // Cholesky of M
  std::vector<double> L(M);
  for (int k = 0; k < nv; k++) {
    double s = L[k * nv + k];
    for (int t = 0; t < k; t++) s -= L[k * nv + t] * L[k * nv + t];
    L[k * nv + k] = std::sqrt(s > 0 ? s : 1e-300);
    for (int i = k + 1; i < nv; i++) {
      double t2 = L[i * nv + k];
      for (int t = 0; t < k; t++) t2 -= L[i * nv + t] * L[k * nv + t];
      L[i * nv + k] = t2 / L[k * nv + k];
    }
  }
  auto solveM = [&](std::vector<double>& x) {
    for (int i = 0; i < nv; i++) { double s = x[i]; for (int t = 0; t < i; t++) s -= L[i * nv + t] * x[t]; x[i] = s / L[i * nv + i]; }
    for (int i = nv - 1; i >= 0; i--) { double s = x[i]; for (int t = i + 1; t < nv; t++) s -= L[t * nv + i] * x[t]; x[i] = s / L[i * nv + i]; }
  };
  auto is_anc = [&](int dof, int b) {
    for (int x = b; x > 0; x = m->body_parent[x]) if (m->dof_body[dof] == x) return true;
    return false;
  };
  for (int b = 0; b < GM_MAX_BODY; b++) m->body_invweight0[b][0] = m->body_invweight0[b][1] = 0.0;
  for (int b = 1; b < nb; b++) {
    // 6 x nv Jacobian of the centre of mass: rows 0-2 translation, 3-5 rotation
    std::vector<std::vector<double>> Jr(6, std::vector<double>(nv, 0.0));
    for (int d = 0; d < nv; d++) {
      if (!is_anc(d, b)) continue;
      const double* cd = &cdof[6 * d];
      double wxp[3];
      cross(cd, &xi[3 * b], wxp);
      for (int k = 0; k < 3; k++) { Jr[k][d] = cd[3 + k] + wxp[k]; Jr[3 + k][d] = cd[k]; }
    }
    double diag[6];
    for (int r = 0; r < 6; r++) {
      std::vector<double> x(Jr[r]);
      solveM(x);
      double v = 0;
      for (int d = 0; d < nv; d++) v += Jr[r][d] * x[d];
      diag[r] = v;
    }
    m->body_invweight0[b][0] = (diag[0] + diag[1] + diag[2]) / 3.0;
    m->body_invweight0[b][1] = (diag[3] + diag[4] + diag[5]) / 3.0;
  }
  for (int d = 0; d < GM_MAX_DOF; d++) m->dof_invweight0[d] = 0.0;
  std::vector<double> minv(nv);
  for (int d = 0; d < nv; d++) {
    std::vector<double> e(nv, 0.0);
    e[d] = 1.0;
    solveM(e);
    minv[d] = e[d];
  }
  for (int j = 0; j < m->njnt; j++) {
    const int d0 = m->jnt_dofadr[j];
    if (m->jnt_type[j] == GM_JNT_FREE) {
      const double t = (minv[d0] + minv[d0 + 1] + minv[d0 + 2]) / 3.0;
      const double r = (minv[d0 + 3] + minv[d0 + 4] + minv[d0 + 5]) / 3.0;
      for (int k = 0; k < 3; k++) { m->dof_invweight0[d0 + k] = t; m->dof_invweight0[d0 + 3 + k] = r; }
    } else {
      m->dof_invweight0[d0] = minv[d0];
    }
  }
}
// Everything the reference derives from the MJCF's gripper numerics rather than reading
// it (JointSettings::Dim / ctrl / gauge, myfunctions.cpp:207-296, 535): shared by the
// builder and the MJCF loader (gm_mjcf.cpp) so both produce the same model bit for bit.
void gm_derive_model_constants(gm_model* m) {
  const double I = m->finger_width * std::pow(m->finger_thickness, 3) / 12.0;
  m->finger_EI = m->finger_E * I;
  m->yield_stress = 215e6;
  const int Ntotal = m->n_seg + m->fixed_first_segment;
  m->segment_length = m->finger_length / double(Ntotal);   // myfunctions.cpp:535
  const double EI = m->finger_EI;
  set3(m->kp_gripper, EI * 541.3 + 49.65, EI * 44.92 - 0.846, 1000);
  set3(m->kd_gripper, 1, 1, 1);
  set3(m->kp_base, 500, 500, 2000);
  set3(m->kd_base, 80, 80, 100);
  m->stepper_num_steps = 10;
  m->time_per_step = 10 / 2000.0;
  m->gauge_xpos = 50e-3;
  m->gauge_order = 3;
}

extern "C" {

void gm_default_model_params(gm_model_params* p) {
  p->n_seg = 8;
  p->finger_length = 235e-3;
  p->finger_width = 28e-3;
  p->finger_thickness = 0.86e-3;
  p->finger_E = 193e9;
  p->hook_length = 35e-3;
  p->hook_angle_degrees = 75.0;
  p->fingertip_clearance = 10e-3;
  p->segment_inertia_scaling = 50.0;
  p->timestep = 3.187e-3;
  p->pgs_iterations = 24;
  p->collision_half_thickness = 1.5e-3;
  // with MuJoCo 2.1.5's actuator order (below) the segment damping law 0.16 N^-0.85
  // reproduces the reference's stable timesteps at inertia x50 within 7 % (DESIGN.md
  // section 2, tests/test_calibration.py); the revolute motor's reflected inertia 0.01 kg m^2
  // keeps its explicit kd = 1 stable (h kd / a < 2 up to the search's 20 ms ceiling)
  p->segment_damping = 0.16;
  p->segment_damping_power = 0.85;
  p->segment_armature = 0.0;
  p->segment_armature_power = 0.0;
  p->mujoco_actuators = 1;
  p->pad_params = 0;
  p->actuator_armature[0] = 0.0;     // prismatic (finger_f_prismatic_joint)
  p->actuator_armature[1] = 0.01;    // revolute (finger_f_revolute_joint)
  p->actuator_armature[2] = 0.0;     // palm
  p->actuator_armature[3] = 0.0;     // base Z
}

int gm_build_model(const gm_model_params* p, gm_model* m) {
  if (!p || !m) return GM_E_ARG;
  if (p->n_seg < 1 || p->n_seg > GM_MAX_SEG) return GM_E_RANGE;
  std::memset(m, 0, sizeof(*m));
  Builder B{m};
  const int N = p->n_seg;
  m->n_seg = N;

  // ---- dimensions (JointSettings::Dim, myfunctions.cpp:207-242) ----
  m->finger_length = p->finger_length;
  m->finger_width = p->finger_width;
  m->finger_thickness = p->finger_thickness;
  m->finger_E = p->finger_E;
  m->hook_length = p->hook_length;
  m->hook_angle_degrees = p->hook_angle_degrees;
  m->fingertip_clearance = p->fingertip_clearance;
  m->fixed_first_segment = 1;   // links 2..N+1 carry the N joints (myfunctions.cpp:650-660)
  m->mujoco_actuators = p->mujoco_actuators ? 1 : 0;
  gm_derive_model_constants(m);
  const double Ls = m->segment_length;
  const double EI = m->finger_EI;

  // ---- options ----
  m->timestep = p->timestep;
  set3(m->gravity, 0, 0, -9.81);
  m->solref[0] = 0.02; m->solref[1] = 1.0;
  m->solimp[0] = 0.9; m->solimp[1] = 0.95; m->solimp[2] = 0.001; m->solimp[3] = 0.5; m->solimp[4] = 2.0;
  m->pgs_iterations = p->pgs_iterations;
  m->mpr_tolerance = 1e-6;
  m->mpr_iterations = 50;

  const double id4[4] = {1, 0, 0, 0};
  const double zero3[3] = {0, 0, 0};

  // ---- world (body 0) + ground plane ----
  {
    double in[3] = {0, 0, 0};
    B.add_body(-1, GM_GRP_WORLD, zero3, id4, 0, zero3, in);
  }
  // ground plane geom id 0 (ObjectHandler::gnd_geom_name "ground_geom")
  {
    double sz[3] = {10, 10, 0.1};
    m->geom_ground = B.add_geom(0, GM_GEOM_PLANE, GM_CLS_GROUND, zero3, id4, sz, 1.0);
  }

  // ---- gripper base: slide "world_to_base" along -z (target base z +ve = down) ----
  // the lowest point of the fixed hook sits at fingertip_clearance above the ground
  const double z_root = p->fingertip_clearance + p->finger_length +
                        p->hook_length * std::cos(p->hook_angle_degrees * kPi / 180.0) +
                        std::max(p->collision_half_thickness, 0.5 * p->finger_thickness);
  {
    double pos[3] = {0, 0, z_root};
    double in[3];
    box_inertia(0.5, 0.05, 0.05, 0.02, in);
    double ipos[3] = {0, 0, 0.03};
    m->body_base = B.add_body(0, GM_GRP_BASE, pos, id4, 0.5, ipos, in);
    double ax[3] = {0, 0, -1};
    m->dof_base = B.add_joint(m->body_base, GM_JNT_SLIDE, ax, 0, 0, p->actuator_armature[3], -1);
  }

  const double ht = std::max(p->collision_half_thickness, 0.5 * p->finger_thickness);
  const double hw = 0.5 * p->finger_width;
  const double mseg = kSteelDensity * Ls * p->finger_width * p->finger_thickness;
  const double mhook = kSteelDensity * p->hook_length * p->finger_width * p->finger_thickness;
  const double th_h = p->hook_angle_degrees * kPi / 180.0;

  // segment stiffness, set_finger_stiffness_using_model (myfunctions.cpp:1019-1031)
  auto seg_stiffness = [&](int n) {
    if (n == 1) return ((2 * EI) / p->finger_length) * ((N * N) / (double)(N - (1.0 / 3.0)));
    return (N * EI) / p->finger_length;
  };

  // segment hinge damping (the MJCF's value is absent): segment_damping N^-power N m s / rad
  // (default 0.16 N^-0.85).  With the springs explicit and the damping implicit (MuJoCo
  // 2.1.5 Euler), this makes find_highest_stable_timestep reproduce the reference's own
  // measured stable timesteps (rl/juypter/thesis_plots/mujoco_timesteps.csv, the inertia
  // x50 columns) within a few percent for N = 5..10 (tests/test_calibration.py, DESIGN.md
  // section 2).
  const double seg_damping = p->segment_damping * std::pow((double)N, -p->segment_damping_power);
  const double seg_armature = p->segment_armature * std::pow((double)N, -p->segment_armature_power);

  int first_finger_geom = m->ngeom;
  for (int f = 0; f < 3; f++) {
    const double a = f * 2.0 * kPi / 3.0;   // angles[] in myfunctions.cpp:3640
    const double r[3] = {-std::sin(a), -std::cos(a), 0.0};
    // intermediate carriage: prismatic "finger_f_prismatic_joint" along r (q = radius x)
    double in_int[3] = {2e-5, 2e-5, 2e-5};
    int bint = B.add_body(m->body_base, GM_GRP_FINGER0 + f, zero3, id4, 0.05, zero3, in_int);
    m->dof_pris[f] = B.add_joint(bint, GM_JNT_SLIDE, r, 0, 5.0, p->actuator_armature[0], m->dof_base);
    // finger body frame: x down the finger, y radially outward, z = x cross y
    double xb[3] = {0, 0, -1};
    double yb[3] = {r[0], r[1], r[2]};
    // tip load direction (apply_segment_force rotates its pull into the finger's rest
    // frame so it bends the finger, myfunctions.cpp:1700-1722): here the bending
    // direction is the finger frame's +y, radially outward, at every keyframe pose
    for (int k = 0; k < 3; k++) m->tip_dir[f][k] = r[k];
    double zb[3] = {xb[1] * yb[2] - xb[2] * yb[1], xb[2] * yb[0] - xb[0] * yb[2],
                    xb[0] * yb[1] - xb[1] * yb[0]};
    double R[9] = {xb[0], yb[0], zb[0], xb[1], yb[1], zb[1], xb[2], yb[2], zb[2]};
    double qf[4];
    quat_from_mat(R, qf);
    double in_seg[3];
    box_inertia(mseg, 0.5 * Ls, 0.5 * p->finger_thickness, hw, in_seg);
    for (int i = 0; i < 3; i++) in_seg[i] *= p->segment_inertia_scaling;
    double ipos_seg[3] = {0.5 * Ls, 0, 0};
    // finger_f body (carries fixed segment link 1): revolute "finger_f_revolute_joint",
    // about +z: +q tilts the tip outward, so th = asin((y - x) / 35 mm) < 0 (the y motor
    // inside the x motor) tilts it inward -- luke::Gripper's own fingertip geometry
    // (calc_fingertip_radius = x - hyp sin(rest - th), gripper.h:88-93) and the reference's
    // MuJoCo "measure tilt" run (mysimulate.cpp:2762-2811: y stepped below x = 100 mm presses
    // the fingertips into the sphere, rl/juypter/thesis_plots/sim_vs_real_forces_tilt.csv;
    // tests/test_force_curves.py).  (The analytic get_fingerend_and_palm_xyz,
    // myfunctions.cpp:3653, uses the opposite sign; it stays as the reference wrote it.)
    int bf = B.add_body(bint, GM_GRP_FINGER0 + f, zero3, qf, mseg, ipos_seg, in_seg);
    m->body_finger[f] = bf;
    double axr[3] = {0, 0, 1};
    m->dof_rev[f] = B.add_joint(bf, GM_JNT_HINGE, axr, 0, 0.0, p->actuator_armature[1], m->dof_pris[f]);
    double gpos[3] = {0.5 * Ls, 0, 0};
    double gsz[3] = {0.5 * Ls, ht, hw};
    B.add_geom(bf, GM_GEOM_BOX, GM_CLS_FINGER1 + f, gpos, id4, gsz, 1.0);
    // segment links 2..N+1, hinge about the plate width axis, +q bends outward
    int parent = bf;
    int parent_dof = m->dof_rev[f];
    for (int k = 1; k <= N; k++) {
      double pos[3] = {Ls, 0, 0};
      double mass = mseg;
      double ipos[3] = {0.5 * Ls, 0, 0};
      double in[3] = {in_seg[0], in_seg[1], in_seg[2]};
      bool last = (k == N);
      if (last) {
        // fixed hook (fixed_hook_segment): lump its mass into the last link
        double hc[3] = {Ls + 0.5 * p->hook_length * std::cos(th_h),
                        -0.5 * p->hook_length * std::sin(th_h), 0};
        double mt = mseg + mhook;
        double c[3] = {(mseg * 0.5 * Ls + mhook * hc[0]) / mt, (mhook * hc[1]) / mt, 0};
        // diagonal of the combined tensor (parallel axis), products of inertia dropped
        double d1[3] = {0.5 * Ls - c[0], 0 - c[1], 0};
        double d2[3] = {hc[0] - c[0], hc[1] - c[1], 0};
        double ih[3];
        box_inertia(mhook, 0.5 * p->hook_length, 0.5 * p->finger_thickness, hw, ih);
        for (int i = 0; i < 3; i++) ih[i] *= p->segment_inertia_scaling;
        in[0] = in_seg[0] + ih[0] + mseg * (d1[1] * d1[1]) + mhook * (d2[1] * d2[1]);
        in[1] = in_seg[1] + ih[1] + mseg * (d1[0] * d1[0]) + mhook * (d2[0] * d2[0]);
        in[2] = in_seg[2] + ih[2] + mseg * (d1[0] * d1[0] + d1[1] * d1[1]) +
                mhook * (d2[0] * d2[0] + d2[1] * d2[1]);
        mass = mt;
        set3(ipos, c[0], c[1], c[2]);
      }
      int bs = B.add_body(parent, GM_GRP_FINGER0 + f, pos, id4, mass, ipos, in);
      double axs[3] = {0, 0, 1};
      int d = B.add_joint(bs, GM_JNT_HINGE, axs, seg_stiffness(k), seg_damping, seg_armature, parent_dof);
      if (k == 1) m->dof_seg[f] = d;
      B.add_geom(bs, GM_GEOM_BOX, GM_CLS_FINGER1 + f, gpos, id4, gsz, 1.0);
      if (last) m->body_tip[f] = bs;
      if (last) {
        double hpos[3] = {Ls + 0.5 * p->hook_length * std::cos(th_h),
                          -0.5 * p->hook_length * std::sin(th_h), 0};
        double hq[4] = {std::cos(-0.5 * th_h), 0, 0, std::sin(-0.5 * th_h)};
        double hsz[3] = {0.5 * p->hook_length, ht, hw};
        B.add_geom(bs, GM_GEOM_BOX, GM_CLS_FINGER1 + f, hpos, hq, hsz, 1.0);
      }
      parent = bs;
      parent_dof = d;
    }
  }
  int last_finger_geom = m->ngeom;

  // ---- palm: slide "palm_prismatic_joint" along -z; palm z=0 is 165 mm above the
  //      finger end (fingerend_to_palm_Z, myfunctions.cpp:3636) ----
  //      palm body frame: x along the gripper axis pointing up (away from the palm face),
  //      y = world y, z = x cross y, so palm_local[0] is the axial force ("+ve for
  //      compression", mjclass.cpp:1010; the palm sensor reads it, mjclass.cpp:826) --
  //      not a horizontal component.  MuJoCo orders a pair by geom type, so a sphere or
  //      cylinder object is geom1 of the palm pair and the pair's force is the one on the
  //      palm (up: +ve); a box object (same type, higher index) is geom2 and reads -ve.
  {
    double in[3];
    box_inertia(0.1, 0.004, 0.03, 0.03, in);
    const double Rp[9] = {0, 0, -1, 0, 1, 0, 1, 0, 0};
    double qp[4];
    quat_from_mat(Rp, qp);
    m->body_palm = B.add_body(m->body_base, GM_GRP_PALM, zero3, qp, 0.1, zero3, in);
    double ax[3] = {-1, 0, 0};   // world -z
    m->dof_palm = B.add_joint(m->body_palm, GM_JNT_SLIDE, ax, 0, 10.0, p->actuator_armature[2], m->dof_base);
    double gpos[3] = {-(p->finger_length - 165e-3), 0, 0};
    double gsz[3] = {0.004, 0.03, 0.03};
    B.add_geom(m->body_palm, GM_GEOM_BOX, GM_CLS_PALM, gpos, id4, gsz, 1.0);
  }
  int palm_geom = m->ngeom - 1;

  // ---- object: free joint, one geom; the per-env object set overrides it ----
  {
    double in[3];
    box_inertia(0.2, 0.02, 0.02, 0.03, in);
    m->body_obj = B.add_body(0, GM_GRP_OBJECT, zero3, id4, 0.2, zero3, in);
    m->dof_obj = B.add_joint(m->body_obj, GM_JNT_FREE, zero3, 0, 0, 0, -1);
    double sz[3] = {0.02, 0.02, 0.03};
    m->geom_obj = B.add_geom(m->body_obj, GM_GEOM_BOX, GM_CLS_OBJECT, zero3, id4, sz, 1.0);
  }

  // ---- dof compact slots: object dofs 0..5, base, then chain slot ----
  for (int d = 0; d < m->nv; d++) {
    int g = m->dof_group[d];
    if (g == GM_GRP_OBJECT) m->dof_slot[d] = d - m->dof_obj;
    else if (g == GM_GRP_BASE) m->dof_slot[d] = 0;
    else if (g == GM_GRP_PALM) m->dof_slot[d] = 0;
    else m->dof_slot[d] = d - m->dof_pris[g];
  }

  // ---- collision pairs: object pairs first (kept first under GM_MAX_CON) ----
  m->npair = 0;
  auto add_pair = [&](int a, int b) {
    if (m->npair < GM_MAX_PAIR) { m->pair_a[m->npair] = a; m->pair_b[m->npair] = b; }
    m->npair++;
  };
  add_pair(m->geom_ground, m->geom_obj);
  for (int g = first_finger_geom; g < last_finger_geom; g++) add_pair(g, m->geom_obj);
  add_pair(palm_geom, m->geom_obj);
  for (int g = first_finger_geom; g < last_finger_geom; g++) add_pair(m->geom_ground, g);
  add_pair(m->geom_ground, palm_geom);
  if (m->npair > GM_MAX_PAIR) return GM_E_RANGE;

  // ---- motor locks: prismatic x3, palm (revolute locks disabled, myfunctions.cpp:479) ----
  m->nlock = 4;
  for (int f = 0; f < 3; f++) { m->lock_dof[f] = m->dof_pris[f]; m->lock_kind[f] = 0; }
  m->lock_dof[3] = m->dof_palm; m->lock_kind[3] = 2;

  // ---- keyframe "initial pose": gripper at home (gripper.h:51-52) ----
  const double xy_home = 134e-3 - 1.0 * (4 * 1e-3 / 1.0);
  const double z_home = 0 + 1.0 * (4.8768 * 1e-3 / 1.0);
  for (int i = 0; i < GM_MAX_QPOS; i++) m->qpos0[i] = 0;
  for (int f = 0; f < 3; f++) m->qpos0[m->jnt_qposadr[m->body_jnt[m->body_finger[f]] - 1]] = xy_home;
  m->qpos0[m->jnt_qposadr[m->body_jnt[m->body_palm]]] = z_home;
  {
    int qa = m->jnt_qposadr[m->body_jnt[m->body_obj]];
    m->qpos0[qa + 0] = 1.0; m->qpos0[qa + 1] = 1.0; m->qpos0[qa + 2] = 0.03;
    m->qpos0[qa + 3] = 1.0;
  }
  if (m->nbody > GM_MAX_BODY || m->nv > GM_MAX_DOF || m->nq > GM_MAX_QPOS || m->ngeom > GM_MAX_GEOM)
    return GM_E_RANGE;
  gm_derive_invweights(m);
  return GM_OK;
}

int64_t gm_struct_size(int which) {
  switch (which) {
    case 0: return (int64_t)sizeof(gm_settings);
    case 1: return (int64_t)sizeof(gm_model);
    case 2: return (int64_t)sizeof(gm_config);
    case 3: return (int64_t)sizeof(gm_object);
    case 4: return (int64_t)sizeof(gm_spawn);
    case 5: return (int64_t)sizeof(gm_model_params);
    case 6: return (int64_t)sizeof(gm_spawn_params);
    case 7: return (int64_t)sizeof(gm_calibration);
    default: return -1;
  }
}

// MjType::SpawnParams member initialisers (mjclass.h:916-931)
void gm_default_spawn_params(gm_spawn_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->index = -1;
  p->x = 0.0; p->y = 0.0; p->zrot = 0.0;
  p->xrange = 0.0; p->yrange = 0.0; p->rotrange = 0.0;
  p->xmin = -100; p->xmax = 100; p->ymin = -100; p->ymax = 100;
  p->smallest_gap = 1e-3;
  p->xy_increment = 2e-3;
  p->rot_increment = M_PI / 30.0;
}

void gm_model_info(const gm_model* m, int32_t* o) {
  o[0] = m->nq; o[1] = m->nv; o[2] = m->nbody; o[3] = m->ngeom; o[4] = m->npair; o[5] = m->n_seg;
  o[6] = m->dof_base; o[7] = m->dof_palm; o[8] = m->dof_obj;
  for (int f = 0; f < 3; f++) { o[9 + f] = m->dof_pris[f]; o[12 + f] = m->dof_rev[f]; o[15 + f] = m->dof_seg[f]; }
  o[18] = m->nlock;
  int nM = 0;   // tree-sparse mass-matrix nonzeros (lower triangle): sum of dof depths
  for (int d = 0; d < m->nv; d++)
    for (int a = d; a >= 0; a = m->dof_parent[a]) nM++;
  o[19] = nM;
}

void gm_config_info(const gm_config* c, int32_t* o) {
  o[0] = c->n_obs; o[1] = c->n_actions; o[2] = c->sim_steps_per_action; o[3] = c->sensor_fcn; o[4] = c->state_fcn;
}

void gm_default_settings(gm_settings* s) {
#define GM_XX(n, t, v) s->n = (t)(v);
#define GM_SS(n, u, nm, r)                                                        \
  s->n.in_use = u; s->n.normalise = nm; s->n.read_rate = r;                       \
  s->n.use_normalisation = 1; s->n.use_noise = 1; s->n.raw_value_offset = 0;      \
  s->n.noise_mag = 0; s->n.noise_mu = 0; s->n.noise_std = -1; s->n.noise_overriden = 0; \
  s->n.prev_steps = 1; s->n.readings_per_step = 1; s->n.total_readings = 1;
#define GM_AA(n, u, v, sg) s->n.in_use = u; s->n.continous = 0; s->n.value = v; s->n.sign = sg;
#define GM_BR(n, r, d, t) s->n.reward = r; s->n.done = d; s->n.trigger = t;
#define GM_LR(n, r, d, t, a, b, o) s->n.reward = r; s->n.done = d; s->n.trigger = t; \
  s->n.min = a; s->n.max = b; s->n.overshoot = o;
#include "gm_settings.def"
}

static int n_samples(int fcn, const gm_sensor& s) {
  if (fcn == GM_SAMPLE_RAW) return s.total_readings - 1;
  return 2 * s.prev_steps + 1;
}

// ---- calibrate_simulated_sensors without the simulation ----
// The reference normalises the bending gauges by the reading its simulation settles at
// under the saturation tip load (mjclass.cpp:4643-4676, validate_curve_under_force
// 4023-4105: every fingertip pulled outward for 50 s, then read_armadillo_gauge of finger
// 0).  That settled state is the static equilibrium of finger 0's joint chain, solved
// here directly in the finger's plane (x down the finger, y outward): revolute motor
// (PD spring kp about the joint's axis at the finger root), the fixed first segment, N segment hinges
// (stiffness c_k about +z); loads = the tip pull at the last link's centre of mass and
// gravity on every link.  The gauge then fits the settled joint points as
// read_armadillo_gauge does.  gm_calibrate runs the actual simulation (device) and the
// two agree to a fraction of a percent (tests/test_calibration.py).
static double cubic_fit_eval(const double* X, const double* Y, int P, double x) {
  // least-squares cubic through (X, Y) (arma::polyfit, myfunctions.cpp:2739) on the
  // centred / scaled abscissa, solved by modified Gram-Schmidt
  double lo = X[0], hi = X[0];
  for (int i = 1; i < P; i++) { lo = std::min(lo, X[i]); hi = std::max(hi, X[i]); }
  const double mid = 0.5 * (lo + hi), half = std::max(0.5 * (hi - lo), 1e-12);
  double Q[4][GM_MAX_SEG + 2], R[4][4] = {{0}};
  for (int i = 0; i < P; i++) {
    const double t = (X[i] - mid) / half;
    Q[0][i] = 1; Q[1][i] = t; Q[2][i] = t * t; Q[3][i] = t * t * t;
  }
  for (int k = 0; k < 4; k++) {
    for (int j = 0; j < k; j++) {
      double d = 0;
      for (int i = 0; i < P; i++) d += Q[j][i] * Q[k][i];
      R[j][k] = d;
      for (int i = 0; i < P; i++) Q[k][i] -= d * Q[j][i];
    }
    double n = 0;
    for (int i = 0; i < P; i++) n += Q[k][i] * Q[k][i];
    n = std::sqrt(n);
    R[k][k] = n;
    for (int i = 0; i < P; i++) Q[k][i] /= n;
  }
  double b[4], a[4];
  for (int k = 0; k < 4; k++) { b[k] = 0; for (int i = 0; i < P; i++) b[k] += Q[k][i] * Y[i]; }
  for (int k = 3; k >= 0; k--) { double v = b[k]; for (int j = k + 1; j < 4; j++) v -= R[k][j] * a[j]; a[k] = v / R[k][k]; }
  const double t = (x - mid) / half;
  return ((a[3] * t + a[2]) * t + a[1]) * t + a[0];
}

static double static_gauge_reading(const gm_model* m, double P) {
  const int N = m->n_seg;
  const double Ls = m->segment_length;
  const int b0 = m->body_finger[0];            // fixed first segment; segments b0+1 .. b0+N
  const double g = -m->gravity[2];              // finger x axis points down: gravity is +x
  double q[GM_MAX_SEG + 1] = {0};               // q[0]: revolute (about az z), q[1..N]: segments
  const double az = m->jnt_axis[m->body_jnt[b0]][2];   // the revolute's axis (+-1 along z)
  double stiff[GM_MAX_SEG + 1];
  stiff[0] = m->kp_gripper[1];
  for (int k = 1; k <= N; k++) stiff[k] = m->jnt_stiffness[m->body_jnt[b0 + k]];
  for (int it = 0; it < 2000; it++) {
    double px[GM_MAX_SEG + 2], py[GM_MAX_SEG + 2], phi[GM_MAX_SEG + 2];
    double cx[GM_MAX_SEG + 2], cy[GM_MAX_SEG + 2], mass[GM_MAX_SEG + 2];
    px[0] = 0; py[0] = 0; phi[0] = az * q[0];
    for (int k = 0; k <= N; k++) {
      if (k > 0) {
        px[k] = px[k - 1] + Ls * std::cos(phi[k - 1]);
        py[k] = py[k - 1] + Ls * std::sin(phi[k - 1]);
        phi[k] = phi[k - 1] + q[k];
      }
      const double* ip = m->body_ipos[b0 + k];
      cx[k] = px[k] + std::cos(phi[k]) * ip[0] - std::sin(phi[k]) * ip[1];
      cy[k] = py[k] + std::sin(phi[k]) * ip[0] + std::cos(phi[k]) * ip[1];
      mass[k] = m->body_mass[b0 + k];
    }
    double change = 0;
    for (int j = 0; j <= N; j++) {
      // torque about +z at joint j from the loads on links j .. N (the revolute carries all)
      double tau = (cx[N] - px[j]) * P;                      // tip pull (0, P)
      for (int k = j; k <= N; k++) tau += -(cy[k] - py[j]) * mass[k] * g;   // gravity (m g, 0)
      const double qn = (j == 0) ? az * tau / stiff[0] : tau / stiff[j];
      change = std::max(change, std::fabs(qn - q[j]));
      q[j] = qn;
    }
    if (change < 1e-15) break;
  }
  double X[GM_MAX_SEG + 2], Y[GM_MAX_SEG + 2];
  X[0] = m->fixed_first_segment ? Ls : 0.0;
  Y[0] = 0;
  double cum = 0;
  for (int i = 0; i < N; i++) {
    cum += q[i + 1];
    X[i + 1] = X[i] + Ls * std::cos(cum);
    Y[i + 1] = Y[i] + Ls * std::sin(cum);
  }
  return 1000.0 * cubic_fit_eval(X, Y, N + 1, m->gauge_xpos);
}

int gm_configure(const gm_settings* in, const gm_model* m, gm_config* c) {
  if (!in || !m || !c) return GM_E_ARG;
  std::memset(c, 0, sizeof(*c));
  c->s = *in;
  gm_settings& s = c->s;

  // ---- action options (mjclass.cpp:109-141) ----
  for (int i = 0; i < GM_ACTION_CODE_COUNT; i++) c->action_options[i] = -1;
  int i = 0, kind = 0;
#define GM_AA(n, u, v, sg)                                                        \
  s.n.continous = s.continous_actions;                                            \
  if (s.n.in_use) {                                                               \
    if (s.n.continous) { c->action_options[i++] = 3 * kind + 2; }                 \
    else { c->action_options[i++] = 3 * kind + 0; c->action_options[i++] = 3 * kind + 1; } \
  }                                                                               \
  kind++;
#include "gm_settings.def"
  if (s.use_termination_action) c->action_options[i++] = GM_ACTION_TERMINATION;
  c->n_actions = i;

  // ---- sampling functions (mjclass.cpp:144-211) ----
  if (s.sensor_sample_mode < 0 || s.sensor_sample_mode > 6) return GM_E_RANGE;
  if (s.state_sample_mode < 0 || s.state_sample_mode > 6) return GM_E_RANGE;
  c->sensor_fcn = s.sensor_sample_mode;
  c->state_fcn = s.state_sample_mode;
  c->sensor_fcn_state_override = 0;
  if (s.state_sample_mode == GM_SAMPLE_SCALED_CHANGE_SQ) {
    // quirk: writes sampleFcnPtr, stateFcnPtr keeps its previous value (mjclass.cpp:204-206)
    c->sensor_fcn = GM_SAMPLE_SCALED_CHANGE_SQ;
    c->state_fcn = GM_SAMPLE_SIGN;   // previous default; see DESIGN.md quirks
    c->sensor_fcn_state_override = 1;
  }

  // ---- timestep / sim steps (auto timestep search is out of scope: model dt is the
  //      pinned "found" value; mjclass.cpp:241-308) ----
  c->timestep = m->timestep;
  s.mujoco_timestep = m->timestep;
  if (s.auto_sim_steps) s.sim_steps_per_action = (int32_t)std::ceil(s.time_for_action / c->timestep);
  if (s.sim_steps_per_action < 1) return GM_E_RANGE;
  c->sim_steps_per_action = s.sim_steps_per_action;

  // ---- gauge calibration (mjclass.cpp:273-291): normalise = the gauge reading the
  //      saturation tip load settles at (static_gauge_reading above) ----
  if (s.auto_calibrate_gauges) {
    // calc_yield_point_load (myfunctions.cpp:3587-3595) in the reference's float steps
    const double Ifing = m->finger_width * std::pow(m->finger_thickness, 3) / 12.0;
    const float M_max = (m->yield_stress * Ifing) / (0.5 * m->finger_thickness);
    const float yield = M_max / m->finger_length;
    const float P = s.saturation_yield_factor * yield;
    s.bending_gauge.normalise = (float)static_gauge_reading(m, P);
    c->sim_gauge_raw_to_N_factor = P / s.bending_gauge.normalise;
    s.wrist_sensor_Z.raw_value_offset = 0.0f;   // userdata[2] is never written
  } else {
    c->sim_gauge_raw_to_N_factor = 1.0;
  }

  // ---- sensor reading counts (mjclass.cpp:5236-5265) ----
  double time_per_step = c->timestep * s.sim_steps_per_action;
#define GM_SS(n, u, nm, r) s.n.prev_steps = s.sensor_n_prev_steps;
#include "gm_settings.def"
  gm_sensor* state_sensors[5] = {&s.motor_state_sensor, &s.base_state_sensor_XY,
                                 &s.base_state_sensor_Z, &s.base_state_sensor_yaw,
                                 &s.cartesian_contacts_XYZ};
  for (auto* ss : state_sensors) {
    ss->prev_steps = s.state_n_prev_steps;
    ss->readings_per_step = 1;
    ss->total_readings = 1 + ss->readings_per_step * ss->prev_steps;
  }
  gm_sensor* other[5] = {&s.bending_gauge, &s.axial_gauge, &s.palm_sensor,
                         &s.wrist_sensor_XY, &s.wrist_sensor_Z};
  for (auto* ss : other) {
    double rs = time_per_step * ss->read_rate;
    ss->readings_per_step = (int32_t)std::floor(rs);
    ss->total_readings = 1 + ss->readings_per_step * ss->prev_steps;
    if (ss->total_readings > GM_RING || ss->total_readings < 1) return GM_E_RANGE;
  }
  for (auto* ss : state_sensors)
    if (ss->total_readings > GM_RING) return GM_E_RANGE;

  // ---- observation size (get_observation order, mjclass.cpp:1721-1936) ----
  int n = 0;
  if (s.bending_gauge.in_use) n += 3 * n_samples(c->sensor_fcn, s.bending_gauge);
  if (s.axial_gauge.in_use) n += 3 * n_samples(c->sensor_fcn, s.axial_gauge);
  if (s.palm_sensor.in_use) n += n_samples(c->sensor_fcn, s.palm_sensor);
  if (s.wrist_sensor_XY.in_use) n += 2 * n_samples(c->sensor_fcn, s.wrist_sensor_XY);
  if (s.wrist_sensor_Z.in_use) n += n_samples(c->sensor_fcn, s.wrist_sensor_XY);  // quirk 1806
  if (s.motor_state_sensor.in_use) n += 3 * n_samples(c->state_fcn, s.motor_state_sensor);
  if (s.base_state_sensor_XY.in_use) n += 2 * n_samples(c->state_fcn, s.base_state_sensor_XY);
  if (s.base_state_sensor_Z.in_use) n += n_samples(c->state_fcn, s.base_state_sensor_Z);
  if (s.base_state_sensor_yaw.in_use) n += n_samples(c->state_fcn, s.base_state_sensor_yaw);
  if (s.cartesian_contacts_XYZ.in_use) n += 12 * (2 * s.cartesian_contacts_XYZ.prev_steps + 1);
  c->n_obs = n;

  // ---- noise parameters that do not need the RNG (apply_noise_params, 5293-5346) ----
#define GM_SS(nm, u, no, r)                                                        \
  if (!s.nm.noise_overriden) {                                                    \
    s.nm.noise_mag = (float)s.sensor_noise_mag;                                   \
    s.nm.noise_std = (float)s.sensor_noise_std;                                   \
    s.nm.noise_mu = (float)s.sensor_noise_mu;                                     \
  }
#include "gm_settings.def"
  for (auto* ss : state_sensors) {
    if (!ss->noise_overriden) {
      ss->noise_mag = (float)s.state_noise_mag;
      ss->noise_mu = (float)s.state_noise_mu;
      ss->noise_std = (float)s.state_noise_std;
    }
  }

  // ---- base limits (myfunctions.cpp:245-261, 2286-2307) ----
  double bmin[6] = {-500e-3, -500e-3, -30e-3, -0.5, -0.5, -kPi / 2};
  double bmax[6] = {500e-3, 500e-3, 30e-3, 0.5, 0.5, kPi / 2};
  for (int k = 0; k < 6; k++) { c->base_min[k] = bmin[k]; c->base_max[k] = bmax[k]; }
  return GM_OK;
}

// luke::set_base_XYZ_limits / set_base_yaw_limit -> update_base_limits
// (myfunctions.cpp:2286-2333): symmetric limits written into target_.base_min/max, which
// the base action clamps and the base state normalisation read.
int gm_config_set_base_limits(gm_config* c, double x, double y, double z, double yaw) {
  if (!c) return GM_E_ARG;
  if (x < 0 || y < 0 || z < 0) return GM_E_RANGE;
  c->base_min[0] = -x; c->base_max[0] = x;
  c->base_min[1] = -y; c->base_max[1] = y;
  c->base_min[2] = -z; c->base_max[2] = z;
  if (yaw >= 0) { c->base_min[5] = -yaw; c->base_max[5] = yaw; }
  return GM_OK;
}

// ---- synthetic object sets (the reference's MJCF object sets are unavailable) ----
static uint64_t splitmix(uint64_t& x) {
  uint64_t z = (x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static double unif(uint64_t& x, double a, double b) {
  return a + (b - a) * ((splitmix(x) >> 11) * (1.0 / 9007199254740992.0));
}

int gm_make_object_set(const char* name, uint64_t seed, gm_object* out, int max_objects) {
  if (!name || !out) return GM_E_ARG;
  std::string nm(name);
  int n = 0;
  auto add = [&](int type, double a, double b, double c, double mass) {
    if (n >= max_objects) return;
    out[n].type = type;
    out[n].size[0] = a; out[n].size[1] = b; out[n].size[2] = c;
    out[n].mass = mass;
    out[n].friction = 1.0;
    n++;
  };
  if (nm == "cylinder") {                       // configs[1]: one cylinder r=20 mm h=60 mm
    add(GM_GEOM_CYLINDER, 0.020, 0.030, 0, 0.2);
  } else if (nm == "set1_synthetic") {          // configs[0] stand-in
    add(GM_GEOM_BOX, 0.020, 0.020, 0.030, 0.2);
    add(GM_GEOM_CYLINDER, 0.020, 0.030, 0, 0.2);
    add(GM_GEOM_SPHERE, 0.025, 0, 0, 0.2);
  } else if (nm == "set6_synthetic") {          // configs[2]: 20 mixed objects
    uint64_t x = seed ^ 0x5E76ull;
    for (int k = 0; k < 20; k++) {
      int t = k % 3;
      double mass = unif(x, 0.05, 0.4);
      if (t == 0) add(GM_GEOM_BOX, unif(x, 0.010, 0.030), unif(x, 0.010, 0.030), unif(x, 0.010, 0.030), mass);
      else if (t == 1) add(GM_GEOM_CYLINDER, unif(x, 0.010, 0.030), unif(x, 0.010, 0.030), 0, mass);
      else add(GM_GEOM_SPHERE, unif(x, 0.010, 0.030), 0, 0, mass);
    }
  } else {
    return GM_E_ARG;
  }
  return n;
}

}  // extern "C"
