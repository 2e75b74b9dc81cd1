/* oracle.c -- fp64 CPU restatement of the reference MjClass env-step hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Serial, one env per or_env, written
 * for readability against the reference sources it restates.  The physics is a
 * restatement of MuJoCo 2.1.5's published pipeline (mj_step1 / mj_step2, an
 * un-vendored dependency pinned by reference buildsettings.mk:32) with the
 * deliberate, documented deviations listed in DESIGN.md ("Engine spec"):
 * the Euler step keeps MuJoCo's explicit joint springs and implicit joint damping but
 * folds the PD motor gains in implicitly; the constraint problem (pyramidal cones, the
 * diagApprox regulariser) is solved to its unique optimum by MuJoCo's Newton method.
 * The physics substep (physics.c) follows the device kernels' association order
 * operation for operation, so the two agree bit for bit from the same state.
 */
#define _POSIX_C_SOURCE 200809L
#include "oracle.h"
#include "../gripper-mujoco_amd/csrc/gm_state.h"
#include "../gripper-mujoco_amd/csrc/gm_math.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#include <time.h>
#include <pthread.h>
#include <stdio.h>

#define NB GM_MAX_BODY
#define NV GM_MAX_DOF
#define NQ GM_MAX_QPOS
#define NG GM_MAX_GEOM
#define NC GM_MAX_CON
#define NE (GM_MAX_EFC + 2 * GM_MAX_LOCK)   /* + the weld-lock variant's extra rows */
#define PI_D 3.14159265358979323846

/* =====================================================================
 * RNG: std::default_random_engine == minstd_rand0 in libstdc++
 * (mjclass.cpp:4, 219-224); generate_canonical as libstdc++ implements it.
 * ===================================================================== */
static uint32_t lcg_next(uint32_t* s) {
  uint64_t x = (uint64_t)(*s) * 16807ull % 2147483647ull;
  *s = (uint32_t)x;
  return *s;
}
static uint32_t lcg_seed(uint64_t seed) {
  uint32_t s = (uint32_t)(seed % 2147483647ull);
  return s == 0 ? 1u : s;
}
/* generate_canonical<float, 24>: one draw, computed in float */
static float canon_f(uint32_t* s) {
  const float r = 2147483646.0f;   /* max - min + 1, rounded to float */
  float sum = (float)(lcg_next(s) - 1u) * 1.0f;
  float ret = sum / r;
  if (ret >= 1.0f) ret = nextafterf(1.0f, 0.0f);
  return ret;
}
/* generate_canonical<double, 53>: two draws */
static double canon_d(uint32_t* s) {
  const double r = 2147483646.0;
  double sum = 0.0, tmp = 1.0;
  for (int k = 0; k < 2; k++) { sum += (double)(lcg_next(s) - 1u) * tmp; tmp *= r; }
  double ret = sum / tmp;
  if (ret >= 1.0) ret = nextafter(1.0, 0.0);
  return ret;
}
double or_minstd_next_canonical_float(uint32_t* s) { return canon_f(s); }
double or_minstd_next_canonical_double(uint32_t* s) { return canon_d(s); }
/* uniform_real_distribution<float>(0,1) used by MjClass::uniform_dist (mjclass.h:1567) */
static float unif01(uint32_t* s) { return canon_f(s) * (1.0f - 0.0f) + 0.0f; }

/* =====================================================================
 * luke::Gripper (gripper.h / gripper.cpp), restated in fp64
 * ===================================================================== */
typedef struct { double x, y, z, th; int32_t sx, sy, sz; } grip_t;
static const double G_leadscrew = 35e-3, G_finger_length = 235e-3, G_hook_length = 35.0e-3;
static const double G_xy_min = 49e-3, G_xy_max = 134e-3, G_z_min = 0e-3, G_z_max = 165e-3;
static const double G_limit_tol = 1e-4;
#define G_TO_RAD (PI_D / 180.0)
#define G_TO_DEG (180.0 / PI_D)
static double g_xy_step_m(void) { return 4.0 / (1.0 * 400 * 1e3); }
static double g_z_step_m(void) { return 4.8768 / (1 * 400 * 1e3); }
static double g_xy_home(void) { return G_xy_max - 1.0 * (4 * 1e-3 / 1.0); }
static double g_z_home(void) { return G_z_min + 1.0 * (4.8768 * 1e-3 / 1); }
static double g_hyp(void) { return sqrt(pow(G_finger_length, 2) + pow(G_hook_length, 2)); }
static double g_rest(void) { return atan(G_hook_length / G_finger_length); }
static double g_th_min(void) { return -40 * G_TO_RAD; }
static double g_th_max(void) { return 40 * G_TO_RAD; }
static const double G_fingertip_radius_min = -1;

static double g_calc_y(const grip_t* g, double th) { return g->x + 1 * G_leadscrew * sin(th); }
static double g_calc_th(double x, double y) { return asin((y - x) / G_leadscrew) * 1; }
static int32_t g_x_step(const grip_t* g) { return (int32_t)round((G_xy_max - g->x) / g_xy_step_m()); }
static int32_t g_y_step(const grip_t* g) { return (int32_t)round((G_xy_max - g->y) / g_xy_step_m()); }
static int32_t g_z_step(const grip_t* g) { return (int32_t)round(g->z / g_z_step_m()); }
static double g_th_rad(const grip_t* g) { return g_calc_th(g->x, g->y); }
static double g_th_deg(const grip_t* g) { return G_TO_DEG * g_th_rad(g); }

/* Gripper::update_xy, gripper.cpp:6-90 */
static int g_update_xy(grip_t* g) {
  int wl = 1;
  if (g->x > G_xy_max + G_limit_tol) { g->x = G_xy_max; wl = 0; }
  if (g->x < G_xy_min - G_limit_tol) { g->x = G_xy_min; wl = 0; }
  if (g->y > G_xy_max + G_limit_tol) { g->y = G_xy_max; wl = 0; }
  if (g->y < G_xy_min - G_limit_tol) { g->y = G_xy_min; wl = 0; }
  double new_th = g_calc_th(g->x, g->y);
  if (new_th > g_th_max()) { new_th = g_th_max(); g->y = g_calc_y(g, g_th_max()); wl = 0; }
  if (new_th < g_th_min()) { new_th = g_th_min(); g->y = g_calc_y(g, g_th_min()); wl = 0; }
  g->th = new_th;
  double th_lim = (asin((G_fingertip_radius_min - g->x) / g_hyp()) + g_rest()) * 1;
  if (g->th < th_lim) { g->y = g_calc_y(g, th_lim); g->th = th_lim; wl = 0; }
  g->sx = g_x_step(g);
  g->sy = g_y_step(g);
  return wl;
}
/* Gripper::update_z, gripper.cpp:92-118 */
static int g_update_z(grip_t* g) {
  int wl = 1;
  if (g->z > G_z_max + G_limit_tol) { g->z = G_z_max; wl = 0; }
  if (g->z < G_z_min - G_limit_tol) { g->z = G_z_min; wl = 0; }
  g->sz = g_z_step(g);
  return wl;
}
static int g_update(grip_t* g) { int a = g_update_xy(g); int b = g_update_z(g); return a * b; }
static void g_reset(grip_t* g) { g->x = g_xy_home(); g->y = g_xy_home(); g->z = g_z_home(); g_update(g); }
/* set_th_rad / set_xyz_m_rad / set_xyz_m / set_xyz_step (gripper.h:113-166) */
static int g_set_th_rad(grip_t* g, double th) { g->y = g_calc_y(g, th); return g_update_xy(g); }
static int g_set_xyz_m_rad(grip_t* g, double x, double th, double z) {
  g->x = x; int in_lim = g_set_th_rad(g, th); g->z = z;
  return g_update_z(g) ? in_lim : 0;
}
static int g_set_xyz_m(grip_t* g, double x, double y, double z) {
  g->x = x; g->y = y; g->z = z; return g_update(g);
}
static int g_set_xyz_step(grip_t* g, int xs, int ys, int zs) {
  g->x = G_xy_max - g_xy_step_m() * xs; g->y = G_xy_max - g_xy_step_m() * ys;
  int in_lim = g_update_xy(g);
  g->z = g_z_step_m() * zs;
  return g_update_z(g) ? in_lim : 0;
}
/* Gripper::step_to, gripper.cpp:158-213 */
static int g_step_to(grip_t* g, const grip_t* t, int num) {
  int fin = 1;
  int xg = t->sx - g->sx, yg = t->sy - g->sy, zg = t->sz - g->sz;
  if (xg < 0) { if (-xg > num) { xg = -num; fin = 0; } } else if (xg > num) { xg = num; fin = 0; }
  if (yg < 0) { if (-yg > num) { yg = -num; fin = 0; } } else if (yg > num) { yg = num; fin = 0; }
  if (zg < 0) { if (-zg > num) { zg = -num; fin = 0; } } else if (zg > num) { zg = num; fin = 0; }
  g_set_xyz_step(g, g->sx + xg, g->sy + yg, g->sz + zg);
  return fin;
}

/* golden driver: op 0 set_xyz_m_rad, 1 set_xyz_m (both relative to end), 2 next.step_to(end, a),
 * 3 reset -- the ops of oracle/ref_golden_driver.cpp, fixtures by tests/golden/make_golden.py */
int or_grip_step_sequence(const double* cmds, int n, double* out) {
  grip_t end, next;
  g_reset(&end); g_reset(&next);
  for (int i = 0; i < n; i++) {
    int op = (int)cmds[4 * i];
    double a = cmds[4 * i + 1], b = cmds[4 * i + 2], c = cmds[4 * i + 3];
    int ret = 0;
    if (op == 0) ret = g_set_xyz_m_rad(&end, end.x + a, end.th + b, end.z + c);
    else if (op == 1) ret = g_set_xyz_m(&end, end.x + a, end.y + b, end.z + c);
    else if (op == 2) ret = g_step_to(&next, &end, (int)a);
    else if (op == 3) { g_reset(&end); g_reset(&next); ret = 1; }
    double* o = out + 15 * i;
    o[0] = ret;
    o[1] = end.x; o[2] = end.y; o[3] = end.z; o[4] = end.th; o[5] = end.sx; o[6] = end.sy; o[7] = end.sz;
    o[8] = next.x; o[9] = next.y; o[10] = next.z; o[11] = next.th; o[12] = next.sx; o[13] = next.sy; o[14] = next.sz;
  }
  return n;
}

/* =====================================================================
 * small vector helpers
 * ===================================================================== */
static double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static void cross3(double* r, const double* a, const double* b) {
  double t0 = a[1] * b[2] - a[2] * b[1], t1 = a[2] * b[0] - a[0] * b[2], t2 = a[0] * b[1] - a[1] * b[0];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static double norm3(const double* a) { return sqrt(dot3(a, a)); }
static void sub3(double* r, const double* a, const double* b) { r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2]; }
static void add3(double* r, const double* a, const double* b) { r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2]; }
static void scl3(double* r, const double* a, double s) { r[0] = a[0] * s; r[1] = a[1] * s; r[2] = a[2] * s; }
static void copy3(double* r, const double* a) { r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; }
static void mulmv3(double* r, const double* M, const double* v) {   /* r = M v, M row-major */
  double t0 = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
  double t1 = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
  double t2 = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static void mulmtv3(double* r, const double* M, const double* v) {  /* r = M^T v */
  double t0 = M[0] * v[0] + M[3] * v[1] + M[6] * v[2];
  double t1 = M[1] * v[0] + M[4] * v[1] + M[7] * v[2];
  double t2 = M[2] * v[0] + M[5] * v[1] + M[8] * v[2];
  r[0] = t0; r[1] = t1; r[2] = t2;
}
static void mulmm3(double* r, const double* A, const double* B) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
  memcpy(r, t, sizeof(t));
}
static void quat2mat(double* R, const double* q) {
  double w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z);     R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y);     R[7] = 2 * (y * z + w * x);     R[8] = 1 - 2 * (x * x + y * y);
}
static void quatmul(double* r, const double* a, const double* b) {
  double t[4];
  t[0] = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  t[1] = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  t[2] = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  t[3] = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  memcpy(r, t, sizeof(t));
}
static void quatnorm(double* q) {
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < 1e-15) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  for (int i = 0; i < 4; i++) q[i] /= n;
}
/* mju_makeFrame-style tangent basis from a unit normal (engine spec) */
static void make_frame(double* F, const double* n) {
  double a[3] = {0, 0, 0};
  if (fabs(n[0]) < 0.5) a[0] = 1; else a[1] = 1;
  double d = dot3(a, n);
  double t1[3] = {a[0] - d * n[0], a[1] - d * n[1], a[2] - d * n[2]};
  double l = norm3(t1);
  scl3(t1, t1, 1.0 / l);
  double t2[3];
  cross3(t2, n, t1);
  copy3(F, n); copy3(F + 3, t1); copy3(F + 6, t2);
}

/* =====================================================================
 * env state
 * ===================================================================== */
typedef struct { float v[GM_RING]; int i; } ring_t;
static void ring_reset(ring_t* r) { for (int k = 0; k < GM_RING; k++) r->v[k] = 0; r->i = -1; }
/* SlidingWindow::add / read_element (slidingwindow.h:36-55) on a ring of GM_RING */
static void ring_add(ring_t* r, float x) { r->i += 1; if (r->i > GM_RING - 1) r->i = 0; r->v[r->i] = x; }
static float ring_read(const ring_t* r, int n) {
  int idx = r->i - n;
  while (idx < 0) idx += GM_RING;
  return r->v[idx];
}
static float ring_latest(const ring_t* r) { return r->i == -1 ? r->v[0] : r->v[r->i]; }

typedef struct { int value; int last_value; int active_sum; int row; int abs; } bev_t;
typedef struct { float value; float last_value; int active_sum; int row; int abs; } lev_t;

typedef struct {
  double dist, pos[3], frame[9], mu;
  double force[3];            /* contact-frame force (normal, t1, t2) after the solve */
  int g1, g2;
} con_t;

/* sensor slots in settings order (SS macro order) */
enum { S_MOTOR = 0, S_BASEZ, S_BASEXY, S_YAW, S_BEND, S_AXIAL, S_PALM, S_WRISTXY, S_WRISTZ, S_CART, S_N };

/* the device's lane topology (gm_capi.hip build_topo) */
typedef struct {
  int CL;
  int body_f0[3], dof_f0[3];
  int body_grp[NB], body_cpos[NB];
  int lane_body[64];
  int kl_type[64], kl_qadr[64], kl_grp[64], kl_cpos[64];
  double kl_pos[64][3], kl_quat[64][4], kl_axis[64][3];
  int dof_grp[NV], dof_p[NV], dof_target[NV];
  double dof_arm[NV], dof_dsum[NV], dof_ksum[NV], dof_stiff[NV], dof_damp[NV], dof_kp[NV], dof_kd[NV];
  int geom_grp[NG];
  int lane_opair[64][2], lane_gpair[64][2];   /* the lane body's geoms' pairs with the object / ground */
} otopo;

#define GM_TRIF ((GM_CHAIN + 1) * (GM_CHAIN + 2) / 2)

struct or_env {
  gm_model m;
  gm_config c;
  gm_object objs[GM_MAX_OBJSET];
  int nobj;
  int64_t env_id;
  otopo T;
  /* physics state */
  double qpos[NQ], qvel[NV], time;
  double qacc_warm[NV];            /* mjData qacc_warmstart: the last substep's solution */
  double obj_invw[2];              /* the live object's body_invweight0 (translation, rotation) */
  /* kinematics / dynamics scratch (mjData) */
  double xpos[NB][3], xmat[NB][9], xquat[NB][4];
  double cinert[NB][10], cdof[NV][6], Ic[NB][10], cfrc[NB][6];
  double Hf[3][GM_TRIF], Hp[3], Ho[21], Hbb;   /* H~ tree blocks (TRI: finger p = 0 base .. CL) */
  double frc[NV], qacc[NV];
  /* a capped Newton solve's residual H~ qacc - (qfrc_smooth + J^T efc) (mj_Euler integrates
   * qfrc_smooth + qfrc_constraint, which only equals H~ qacc at the optimum) */
  double res[NV];
  int res_valid;
  double last_smooth[NV], last_constraint[NV];   /* the last substep's forces (want_forces) */
  int want_forces;
  int ncon, ncon_total, overflow;
  con_t con[NC];
  int pair_off[GM_MAX_PAIR], pair_cnt[GM_MAX_PAIR];
  int nefc, nl;
  double efc_f[NE], efc_D[NE], efc_aref[NE];
  int efc_type[NE];  /* 0 equality, 1 pyramid edge */
  int lock_row_dof[3 * GM_MAX_LOCK];
  double lock_row_a[3 * GM_MAX_LOCK];   /* the row's Jacobian on its dof (1 for a joint lock) */
  int weld_locks;                       /* motor locks as MuJoCo weld rows (test variant) */
  int solver_pgs;                  /* 0: Newton (the engine); > 0: dense PGS cross-check, this many sweeps */
  int stat_it, stat_ls;            /* Newton iterations / line-search evaluations of the last substep */
  long stat_it_sum, stat_ls_sum, stat_solves, stat_it_max, stat_ncon_max, stat_nefc_sum;
  double qpos_pre[NQ];
  /* target (myfunctions.cpp:470, customtypes.h:574-694) */
  grip_t end, next;
  double base[6];
  double last_step_time;
  int lock_active[GM_MAX_LOCK];
  double lock_q[GM_MAX_LOCK];
  int old_x, old_y, old_z;         /* function-static in update_constraints (2221-2223) */
  double eq_q[NQ];                 /* calibrate_reset equilibrium (gripper + base) */
  /* sensors */
  double last_read[S_N];
  float rand_mu[S_N][3];
  ring_t w_gauge[3], w_axial[3], w_palm, w_wx, w_wy, w_wz, w_motor[3], w_base[3], w_yaw, w_cart[12];
  ring_t si_gauge[3], si_palm, si_wz, si_axial[3];
  uint32_t rng;
  /* env tracking (MjType::Env, mjclass.h:782-913) */
  bev_t bev[GM_N_BINARY];
  lev_t lev[GM_N_LINEAR];
  float cumulative_reward;
  int num_action_steps;
  int termination_signal_sent;
  int term_pending_steps;
  int last_done;                   /* the last is_done() / reward() results (GmEnvState::done / reward) */
  int episode;                     /* resets so far (GmEnvState::episode) */
  float last_reward;
  float grp_peak_lateral;
  int obj_index;
  double start_qpos[7];
  /* calibration (curve_validation tip load, mjWARN_BADQACC) */
  double tip_force;
  int badqacc;
  int newton_caps;                 /* solves that hit GM_NEWTON_MAXIT / _MAXLS (GmEnvState::newton_caps) */
};

size_t or_sizeof(void) { return sizeof(or_env); }

/* =====================================================================
 * model helpers: per-env object slot (objects are culled to one live slot)
 * ===================================================================== */
static double object_rest_z(const gm_object* o) {
  if (o->type == GM_GEOM_BOX) return o->size[2];
  if (o->type == GM_GEOM_CYLINDER) return o->size[1];
  return o->size[0];
}
static void apply_object(gm_model* m, const gm_object* o) {
  int g = m->geom_obj, b = m->body_obj;
  m->geom_type[g] = o->type;
  for (int i = 0; i < 3; i++) m->geom_size[g][i] = o->size[i];
  m->geom_friction[g] = o->friction;
  double mass = o->mass, I0, I1, I2;
  if (o->type == GM_GEOM_BOX) {
    double a = 2 * o->size[0], bb = 2 * o->size[1], c = 2 * o->size[2];
    I0 = mass * (bb * bb + c * c) / 12; I1 = mass * (a * a + c * c) / 12; I2 = mass * (a * a + bb * bb) / 12;
    m->geom_rbound[g] = sqrt(o->size[0] * o->size[0] + o->size[1] * o->size[1] + o->size[2] * o->size[2]);
  } else if (o->type == GM_GEOM_CYLINDER) {
    double r = o->size[0], h = 2 * o->size[1];
    I0 = I1 = mass * (3 * r * r + h * h) / 12; I2 = mass * r * r / 2;
    m->geom_rbound[g] = sqrt(o->size[0] * o->size[0] + o->size[1] * o->size[1]);
  } else {
    double r = o->size[0];
    I0 = I1 = I2 = 2 * mass * r * r / 5;
    m->geom_rbound[g] = r;
  }
  m->body_mass[b] = mass;
  m->body_inertia[b][0] = I0; m->body_inertia[b][1] = I1; m->body_inertia[b][2] = I2;}
/* body_invweight0 of the live object (mj_setConst at qpos0: a free body's translational
 * J M^-1 J^T diagonal mean 1/m, rotational the mean of 1/I) */
static void object_invweight(or_env* e) {
  const gm_model* m = &e->m;
  const int b = m->body_obj;
  e->obj_invw[0] = 1.0 / m->body_mass[b];
  e->obj_invw[1] = ((1.0 / m->body_inertia[b][0] + 1.0 / m->body_inertia[b][1]) + 1.0 / m->body_inertia[b][2]) / 3.0;
}

#include "physics.c"

/* =====================================================================
 * after_step: update_all -> update_stepper / update_constraints, antiroll
 * myfunctions.cpp:2110-2284, objecthandler.cpp:1034-1059
 * ===================================================================== */
static int prismatic_moving(const or_env* e) { return g_x_step(&e->end) != g_x_step(&e->next); }
static int revolute_moving(const or_env* e) { return !(fabs(g_th_deg(&e->end) - g_th_deg(&e->next)) < 5e-1); }
static int z_moving(const or_env* e) { return g_z_step(&e->end) != g_z_step(&e->next); }

static void set_lock(or_env* e, int kind, int active) {
  for (int k = 0; k < e->m.nlock; k++) {
    if (e->m.lock_kind[k] != kind) continue;
    e->lock_active[k] = active;
    /* set_constraint reads xpos/xmat of mj_step1 (pre-integration) */
    if (active) e->lock_q[k] = e->qpos_pre[e->m.lock_dof[k]];
  }
}
static void update_constraints(or_env* e) {
  int nx = prismatic_moving(e), ny = revolute_moving(e), nz = z_moving(e);
  if (nx != e->old_x) { set_lock(e, 0, !nx); e->old_x = nx; }
  if (ny != e->old_y) { /* revolute locks disabled (myfunctions.cpp:479, 2261) */ e->old_y = ny; }
  if (nz != e->old_z) { set_lock(e, 2, !nz); e->old_z = nz; }
}
static void update_all(or_env* e) {
  if (e->time > e->last_step_time + e->m.time_per_step) {
    update_constraints(e);
    e->last_step_time = e->time;
    g_step_to(&e->next, &e->end, e->m.stepper_num_steps);
  }
  /* apply_antiroll on the live object */
  const double* v = &e->qvel[e->m.dof_obj];
  double mag = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
  if (mag < 1e-6) for (int k = 0; k < 6; k++) e->qvel[e->m.dof_obj + k] = 0;
}

/* =====================================================================
 * sensors
 * ===================================================================== */
/* read_armadillo_gauge (myfunctions.cpp:2699-2795): cubic least squares through the
 * N+1 joint points, evaluated at gauge.xpos, in mm.  Least squares by Householder
 * QR on the Vandermonde matrix, as arma::polyfit -> LAPACK does. */
/* least-squares polynomial of `order` through (X, Y), evaluated at x, in mm */
float or_polyfit_eval(const double* X, const double* Y, int P, int order, double x) {
  double A[GM_MAX_SEG + 1][4], b[GM_MAX_SEG + 1];
  int nc = order + 1;
  for (int i = 0; i < P; i++) {
    for (int k = 0; k < nc; k++) A[i][k] = pow(X[i], order - k);
    b[i] = Y[i];
  }
  for (int k = 0; k < nc; k++) {
    double nrm = 0;
    for (int i = k; i < P; i++) nrm += A[i][k] * A[i][k];
    nrm = sqrt(nrm);
    double alpha = A[k][k] > 0 ? -nrm : nrm;
    double v[GM_MAX_SEG + 1];
    for (int i = 0; i < P; i++) v[i] = 0;
    for (int i = k; i < P; i++) v[i] = A[i][k];
    v[k] -= alpha;
    double vv = 0;
    for (int i = k; i < P; i++) vv += v[i] * v[i];
    if (vv < 1e-300) continue;
    for (int j = k; j < nc; j++) {
      double s = 0;
      for (int i = k; i < P; i++) s += v[i] * A[i][j];
      s = 2 * s / vv;
      for (int i = k; i < P; i++) A[i][j] -= s * v[i];
    }
    double s = 0;
    for (int i = k; i < P; i++) s += v[i] * b[i];
    s = 2 * s / vv;
    for (int i = k; i < P; i++) b[i] -= s * v[i];
  }
  double coeff[4];
  for (int k = nc - 1; k >= 0; k--) {
    double s = b[k];
    for (int j = k + 1; j < nc; j++) s -= A[k][j] * coeff[j];
    coeff[k] = s / A[k][k];
  }
  float y = 0.0f;
  for (int i = 0; i <= order; i++) y += (float)(coeff[i] * pow(x, order - i));
  return y * 1000;
}

/* The engine's evaluation of the same cubic fit (the device's gauge_reading, operation
 * for operation): Householder QR on the Vandermonde matrix of the abscissa centred on
 * and scaled by half the finger length (better conditioned than the raw one; the same
 * least-squares solution, pinned to numpy.polyfit through or_polyfit_eval in
 * tests/test_oracle_golden.py). */
float or_gauge_reading(const gm_model* m, const double* q) {
  int N = m->n_seg, P = N + 1;
  double X[GM_MAX_SEG + 1], Yv[GM_MAX_SEG + 1];
  or_gauge_points(m, q, X, Yv);
  const double half = 0.5 * m->finger_length;
  const double ihalf = 1.0 / half;
  double A[GM_MAX_SEG + 1][4], b[GM_MAX_SEG + 1];
  for (int i = 0; i < P; i++) {
    const double t = (X[i] - half) * ihalf;
    A[i][0] = t * t * t; A[i][1] = t * t; A[i][2] = t; A[i][3] = 1.0;
    b[i] = Yv[i];
  }
  for (int k = 0; k < 4; k++) {
    double nrm = 0;
    for (int i = k; i < P; i++) nrm += A[i][k] * A[i][k];
    nrm = sqrt(nrm);
    const double alpha = A[k][k] > 0 ? -nrm : nrm;
    double v[GM_MAX_SEG + 1];
    for (int i = 0; i < P; i++) v[i] = (i >= k) ? A[i][k] : 0.0;
    v[k] -= alpha;
    double vv = 0;
    for (int i = k; i < P; i++) vv += v[i] * v[i];
    if (vv < 1e-300) continue;
    const double ivv = 2.0 / vv;
    for (int j = k; j < 4; j++) {
      double sacc = 0;
      for (int i = k; i < P; i++) sacc += v[i] * A[i][j];
      sacc *= ivv;
      for (int i = k; i < P; i++) A[i][j] -= sacc * v[i];
    }
    double sacc = 0;
    for (int i = k; i < P; i++) sacc += v[i] * b[i];
    sacc *= ivv;
    for (int i = k; i < P; i++) b[i] -= sacc * v[i];
  }
  double coeff[4];
  for (int k = 3; k >= 0; k--) {
    double sacc = b[k];
    for (int j = k + 1; j < 4; j++) sacc -= A[k][j] * coeff[j];
    coeff[k] = sacc / A[k][k];
  }
  const double tg = (m->gauge_xpos - half) * ihalf;
  const double y = ((coeff[0] * tg + coeff[1]) * tg + coeff[2]) * tg + coeff[3];
  return (float)y * 1000;
}

/* finger joint points (myfunctions.cpp:2699-2740): cumulative segment angles */
void or_gauge_points(const gm_model* m, const double* q, double* X, double* Y) {
  int N = m->n_seg;
  X[0] = m->fixed_first_segment ? m->segment_length : 0;
  Y[0] = 0;
  double cum = 0;
  for (int i = 0; i < N; i++) {
    cum = (i == 0) ? q[0] : cum + q[i];
    double sn, cs;
    gm_sincos(cum, &sn, &cs);
    X[i + 1] = X[i] + m->segment_length * cs;
    Y[i + 1] = Y[i] + m->segment_length * sn;
  }
}

/* SlidingWindow trace: after each add, read_element(0 .. n_reads-1) */
void or_ring_trace(const float* adds, int n_adds, int n_reads, float* out) {
  ring_t r;
  ring_reset(&r);
  for (int k = 0; k < n_adds; k++) {
    ring_add(&r, adds[k]);
    for (int n = 0; n < n_reads; n++) out[k * n_reads + n] = ring_read(&r, n);
  }
}

/* Sensor::apply_normalisation (mjclass.h:155-174) */
static float s_normalise(const gm_sensor* s, float v) {
  if (!s->use_normalisation) return v;
  if (s->normalise <= 0) return v < 0 ? -1.0f : 1.0f;
  else if (v > s->normalise) return 1.0f;
  if (v < -s->normalise) return -1.0f;
  return v / s->normalise;
}
/* Sensor::apply_noise (mjclass.h:176-223) */
static float s_noise(or_env* e, const gm_sensor* s, int slot, float value, int i) {
  if (!s->use_noise) return value;
  const float two_pi = (float)(2.0 * PI_D);
  const float eps = FLT_EPSILON;
  float mu = e->rand_mu[slot][i - 1];
  if (s->noise_std < eps) {
    float noise = mu + s->noise_mag * (2 * unif01(&e->rng) - 1);
    value += noise;
  } else {
    float u1, u2;
    do { u1 = unif01(&e->rng); } while (u1 <= eps);
    u2 = unif01(&e->rng);
    float mag = (float)(s->noise_std * sqrt(-2.0 * (double)logf(u1)));
    float z0 = mag * cosf(two_pi * u2) + mu;
    value += z0;
  }
  if (value > 1) value = 1;
  else if (value < -1) value = -1;
  return value;
}
/* Sensor::ready_to_read (mjclass.h:225-241) */
static int s_ready(or_env* e, const gm_sensor* s, int slot) {
  double tbr = (double)(1 / s->read_rate);
  if (e->time > e->last_read[slot] + tbr) { e->last_read[slot] = e->time; return 1; }
  return 0;
}

/* ObjectHandler::extract_forces_faster (objecthandler.cpp:737-992) over the contacts
 * and forces of the last substep; body frames from that substep's mj_step1 kinematics */
typedef struct {
  double obj_glob[6][6];     /* sum, f1, f2, f3, palm, gnd (global, [f; t]) */
  double obj_loc[4][3];      /* f1, f2, f3, palm (local) */
  double all_glob[4][6];
  double all_loc[4][3];
  double gnd_glob[3][6];
  double gnd_loc[3][3];
} forces_t;
static void extract_forces(const or_env* e, forces_t* F) {
  const gm_model* m = &e->m;
  memset(F, 0, sizeof(*F));
  for (int i = 0; i < e->ncon; i++) {
    const con_t* C = &e->con[i];
    int c1 = m->geom_class[C->g1], c2 = m->geom_class[C->g2];
    int w_obj = (c1 == GM_CLS_OBJECT || c2 == GM_CLS_OBJECT);
    int w_f[3];
    for (int f = 0; f < 3; f++) w_f[f] = (c1 == GM_CLS_FINGER1 + f || c2 == GM_CLS_FINGER1 + f);
    int w_palm = (c1 == GM_CLS_PALM || c2 == GM_CLS_PALM);
    int w_gnd = (c1 == GM_CLS_GROUND || c2 == GM_CLS_GROUND);
    if (!(w_obj || w_f[0] || w_f[1] || w_f[2] || w_palm || w_gnd)) continue;
    /* global = frame^T * local; torques are zero for condim 3 */
    double g[6] = {0, 0, 0, 0, 0, 0};
    for (int k = 0; k < 3; k++)
      for (int r = 0; r < 3; r++) g[k] += C->frame[3 * r + k] * C->force[r];
    if (w_obj) {
      for (int k = 0; k < 6; k++) F->obj_glob[0][k] += g[k];
      for (int f = 0; f < 3; f++) if (w_f[f]) for (int k = 0; k < 6; k++) F->obj_glob[1 + f][k] += g[k];
      if (w_palm) for (int k = 0; k < 6; k++) F->obj_glob[4][k] += g[k];
      if (w_gnd) for (int k = 0; k < 6; k++) F->obj_glob[5][k] += g[k];
    }
    for (int f = 0; f < 3; f++) {
      if (w_f[f]) {
        for (int k = 0; k < 6; k++) F->all_glob[f][k] += g[k];
        if (w_gnd) for (int k = 0; k < 6; k++) F->gnd_glob[f][k] += g[k];
      }
    }
    if (w_palm) for (int k = 0; k < 6; k++) F->all_glob[3][k] += g[k];
  }
  for (int f = 0; f < 4; f++) {
    const double* R = e->xmat[f < 3 ? m->body_finger[f] : m->body_palm];
    mulmtv3(F->obj_loc[f], R, F->obj_glob[1 + f]);
    mulmtv3(F->all_loc[f], R, F->all_glob[f]);
    if (f < 3) mulmtv3(F->gnd_loc[f], R, F->gnd_glob[f]);
  }
}

/* MjClass::monitor_sensors (mjclass.cpp:741-898) */
static void monitor_sensors(or_env* e) {
  gm_settings* s = &e->c.s;
  int have_forces = 0;
  forces_t F;
  if (s_ready(e, &s->bending_gauge, S_BEND)) {
    float g[3];
    for (int f = 0; f < 3; f++) g[f] = or_gauge_reading(&e->m, &e->qpos[e->m.dof_seg[f]]);
    for (int f = 0; f < 3; f++) ring_add(&e->si_gauge[f], (float)(g[f] * e->c.sim_gauge_raw_to_N_factor));
    for (int f = 0; f < 3; f++) g[f] = s_normalise(&s->bending_gauge, g[f]);
    for (int f = 0; f < 3; f++) g[f] = s_noise(e, &s->bending_gauge, S_BEND, g[f], f + 1);
    for (int f = 0; f < 3; f++) ring_add(&e->w_gauge[f], g[f]);
  }
  if (s_ready(e, &s->axial_gauge, S_AXIAL)) {
    if (!have_forces) { extract_forces(e, &F); have_forces = 1; }
    float a[3];
    for (int f = 0; f < 3; f++) a[f] = (float)F.all_loc[f][0];
    for (int f = 0; f < 3; f++) ring_add(&e->si_axial[f], a[f]);
    for (int f = 0; f < 3; f++) a[f] = s_normalise(&s->axial_gauge, a[f]);
    for (int f = 0; f < 3; f++) a[f] = s_noise(e, &s->axial_gauge, S_AXIAL, a[f], f + 1);
    for (int f = 0; f < 3; f++) ring_add(&e->w_axial[f], a[f]);
  }
  if (s_ready(e, &s->palm_sensor, S_PALM)) {
    if (!have_forces) { extract_forces(e, &F); have_forces = 1; }
    float p = (float)F.all_loc[3][0];
    p *= s->palm_scale_factor;
    ring_add(&e->si_palm, p);
    p = s_normalise(&s->palm_sensor, p);
    p = s_noise(e, &s->palm_sensor, S_PALM, p, 1);
    ring_add(&e->w_palm, p);
  }
  if (s_ready(e, &s->wrist_sensor_Z, S_WRISTZ)) {
    float z = 0.0f;   /* data->userdata[2] is never written */
    z -= s->wrist_sensor_Z.raw_value_offset;
    ring_add(&e->si_wz, z);
    z = s_normalise(&s->wrist_sensor_Z, z);
    z = s_noise(e, &s->wrist_sensor_Z, S_WRISTZ, z, 1);
    ring_add(&e->w_wz, z);
  }
}

/* normalise_between (mjclass.cpp:4896-4904) */
static float normalise_between(float val, float mn, float mx) {
  if (val > mx) return 1.0f;
  else if (val < mn) return -1.0f;
  return 2 * (val - mn) / (mx - mn) - 1;
}

/* luke::get_fingerend_and_palm_xyz (myfunctions.cpp:3622-3688) */
static void fingerend_palm_xyz(const or_env* e, const double* fsi, double out[4][3]) {
  const gm_model* m = &e->m;
  double bx = e->base[0], by = e->base[1], bz = e->base[2], yaw = e->base[5];
  double fx = e->end.x, fth = g_th_rad(&e->end), pz = e->end.z;
  const double PI23 = PI_D * (2.0 / 3.0);
  double ang[3] = {0.0, PI23, 2 * PI23};
  double unt = m->fingertip_clearance - bz;
  double lift = m->finger_length * (1 - cos(fth));
  double tilted = unt + lift;
  for (int i = 0; i < 3; i++) {
    double tilt_x = fx - m->finger_length * sin(fth);
    double defl = fsi[i] * pow(m->finger_length, 3) / (3 * m->finger_EI);
    double fin_x = tilt_x + defl * cos(fth);
    out[i][0] = -fin_x * sin(ang[i] + yaw) + bx;
    out[i][1] = -fin_x * cos(ang[i] + yaw) + by;
    out[i][2] = tilted - defl * sin(fth);
  }
  out[3][0] = bx; out[3][1] = by; out[3][2] = unt + 165e-3 - pz;
}

/* MjClass::sense_gripper_state (mjclass.cpp:900-964) */
static void sense_gripper_state(or_env* e) {
  gm_settings* s = &e->c.s;
  const double* bmn = e->c.base_min;
  const double* bmx = e->c.base_max;
  double gx = normalise_between((float)e->end.x, (float)G_xy_min, (float)G_xy_max);
  double gy = normalise_between((float)e->end.y, (float)G_xy_min, (float)G_xy_max);
  double gz = normalise_between((float)e->end.z, (float)G_z_min, (float)G_z_max);
  double bx = normalise_between((float)e->base[0], (float)bmn[0], (float)bmx[0]);
  double by = normalise_between((float)e->base[1], (float)bmn[1], (float)bmx[1]);
  double bz = normalise_between((float)e->base[2], (float)bmn[2], (float)bmx[2]);
  double byaw = normalise_between((float)e->base[5], (float)bmn[5], (float)bmx[5]);
  gx = s_noise(e, &s->motor_state_sensor, S_MOTOR, (float)gx, 1);
  gy = s_noise(e, &s->motor_state_sensor, S_MOTOR, (float)gy, 2);
  gz = s_noise(e, &s->motor_state_sensor, S_MOTOR, (float)gz, 3);
  bx = s_noise(e, &s->base_state_sensor_XY, S_BASEXY, (float)bx, 1);
  by = s_noise(e, &s->base_state_sensor_XY, S_BASEXY, (float)by, 2);
  bz = s_noise(e, &s->base_state_sensor_Z, S_BASEZ, (float)bz, 1);
  byaw = s_noise(e, &s->base_state_sensor_yaw, S_YAW, (float)byaw, 1);
  ring_add(&e->w_motor[0], (float)gx);
  ring_add(&e->w_motor[1], (float)gy);
  ring_add(&e->w_motor[2], (float)gz);
  ring_add(&e->w_base[0], (float)bx);
  ring_add(&e->w_base[1], (float)by);
  ring_add(&e->w_base[2], (float)bz);
  ring_add(&e->w_yaw, (float)byaw);
  /* MAT cartesian contact points */
  double fsi[3] = {ring_latest(&e->si_gauge[0]), ring_latest(&e->si_gauge[1]), ring_latest(&e->si_gauge[2])};
  double psi = ring_latest(&e->si_palm);
  double xyz[4][3];
  fingerend_palm_xyz(e, fsi, xyz);
  const double ft = 0.2;
  for (int f = 0; f < 3; f++)
    for (int k = 0; k < 3; k++) ring_add(&e->w_cart[3 * f + k], (float)((fabs(fsi[f]) > ft) ? xyz[f][k] : 0.0));
  for (int k = 0; k < 3; k++) ring_add(&e->w_cart[9 + k], (float)((psi > ft) ? xyz[3][k] : 0.0));
}

static double mag3(const double* v) { return sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]); }

/* update_events (mjclass.cpp:5437-5469) */
static void update_events(or_env* e) {
  const gm_settings* s = &e->c.s;
  for (int k = 0; k < GM_N_BINARY; k++) {
    bev_t* b = &e->bev[k];
    b->row = b->row * b->value + b->value;
    b->abs += b->value;
    b->last_value = b->value;
    b->active_sum = b->row != 0;
    b->value = 0;
  }
  const gm_linear_reward* lr[GM_N_LINEAR] = {
#define GM_LR(n, r, d, t, a, b, o) &s->n,
#include "../include/gm_settings.def"
  };
  for (int k = 0; k < GM_N_LINEAR; k++) {
    lev_t* l = &e->lev[k];
    int active = 0;
    if (l->value > lr[k]->min && (l->value < lr[k]->overshoot || lr[k]->overshoot < 0)) active = 1;
    l->row = l->row * active + active;
    l->abs += active;
    l->last_value = l->value;
    l->active_sum = active;
    l->value = 0.0f;
  }
}

/* MjClass::update_env (mjclass.cpp:966-1346) for the single live object */
static void update_env(or_env* e) {
  const gm_settings* s = &e->c.s;
  const gm_model* m = &e->m;
  const double ftol = 1e-5;
  forces_t F;
  extract_forces(e, &F);
  int qa = m->jnt_qposadr[m->body_jnt[m->body_obj]];
  double ox = e->qpos[qa], oy = e->qpos[qa + 1], oz = e->qpos[qa + 2];
  double relx = e->base[0] - ox, rely = e->base[1] - oy;
  float dist_from_gripper = (float)sqrt(pow(relx, 2) + pow(rely, 2));
  float f1m = (float)mag3(F.obj_loc[0]), f2m = (float)mag3(F.obj_loc[1]), f3m = (float)mag3(F.obj_loc[2]);
  float pm = (float)mag3(F.obj_loc[3]);
  float gm = (float)mag3(F.obj_glob[5]);
  float palm_axial = (float)F.obj_loc[3][0];
  float lift_height = (float)(oz - e->start_qpos[2]);
  float avg_finger = (float)(0.33333 * (f1m + f2m + f3m));
  double mn = F.obj_loc[0][1];
  if (F.obj_loc[1][1] < mn) mn = F.obj_loc[1][1];
  if (F.obj_loc[2][1] < mn) mn = F.obj_loc[2][1];
  float peak_lat = (float)(-1 * mn);
  float ov_avg = 0, ov_palm = 0, ov_lift = 0;
  if (avg_finger > ov_avg) ov_avg = avg_finger;
  if (palm_axial > ov_palm) ov_palm = palm_axial;
  if (peak_lat > e->grp_peak_lateral) e->grp_peak_lateral = peak_lat;
  if (lift_height > ov_lift) ov_lift = lift_height;
  float gripper_z_height = (float)(-1 * e->base[2]);
  double ga = F.gnd_loc[0][0];
  if (F.gnd_loc[1][0] < ga) ga = F.gnd_loc[1][0];
  if (F.gnd_loc[2][0] < ga) ga = F.gnd_loc[2][0];
  float grp_peak_axial = (float)(-1 * ga);
  float g1 = ring_latest(&e->si_gauge[0]), g2 = ring_latest(&e->si_gauge[1]), g3 = ring_latest(&e->si_gauge[2]);
  float last_palm = ring_latest(&e->si_palm), last_wrist = ring_latest(&e->si_wz);
  float max_gauge = g1 > g2 ? g1 : g2;
  max_gauge = max_gauge > g3 ? max_gauge : g3;
  float avg_gauge = (float)((1.0 / 3.0) * (g1 + g2 + g3));

  bev_t* B = e->bev;
  B[GM_EV_step_num].value = 1;
  double closest = dist_from_gripper;
  /* quirk: Obj::peak_finger_axial_force is never assigned (stays 0) (mjclass.cpp:1156) */
  int o_lifted = 0, o_oob = 0, o_l2h = 0, o_th = 0, o_stable = 0, o_sh = 0;
  if (gm < ftol && 0.0f < ftol) { B[GM_EV_lifted].value = 1; o_lifted = 1; }
  if (ox > s->oob_distance || ox < -s->oob_distance || oy > s->oob_distance || oy < -s->oob_distance) {
    B[GM_EV_oob].value = 1; o_oob = 1;
  }
  if (ov_lift > s->lift_height - ftol && o_lifted && !o_oob) { B[GM_EV_lifted_to_height].value = 1; o_l2h = 1; }
  if (o_l2h && gripper_z_height > s->gripper_target_height - ftol) { B[GM_EV_target_height].value = 1; o_th = 1; }
  if (f1m > ftol || f2m > ftol || f3m > ftol || pm > ftol) B[GM_EV_object_contact].value = 1;
  if (f1m > s->stable_finger_force && f2m > s->stable_finger_force && f3m > s->stable_finger_force &&
      f1m < s->stable_finger_force_lim && f2m < s->stable_finger_force_lim && f3m < s->stable_finger_force_lim &&
      pm > s->stable_palm_force && pm < s->stable_palm_force_lim && B[GM_EV_lifted].value) {
    B[GM_EV_object_stable].value = 1; o_stable = 1;
  }
  if (o_stable && o_th) { B[GM_EV_stable_height].value = 1; o_sh = 1; }
  (void)o_sh;
  if (e->termination_signal_sent) {
    if (s->lifted_termination.done) {
      if (o_l2h) B[GM_EV_lifted_termination].value = 1;
      else B[GM_EV_failed_termination].value = 1;
    } else {
      if (B[GM_EV_stable_height].value) B[GM_EV_stable_termination].value = 1;
      else B[GM_EV_failed_termination].value = 1;
    }
  }
  if (dist_from_gripper < s->XY_distance_threshold) B[GM_EV_within_XY_distance].value = 1;
  if (dist_from_gripper < closest) closest = dist_from_gripper;
  {
    int v = (!B[GM_EV_dropped].row * !B[GM_EV_lifted].value * B[GM_EV_lifted].row) ? 1
            : (B[GM_EV_lifted].value ? 0 : (B[GM_EV_dropped].row ? B[GM_EV_dropped].row + 1 : 0));
    B[GM_EV_dropped].value = v != 0;
  }
  lev_t* Lv = e->lev;
  Lv[GM_LEV_exceed_axial].value = grp_peak_axial;
  Lv[GM_LEV_exceed_lateral].value = e->grp_peak_lateral;
  Lv[GM_LEV_palm_force].value = ov_palm * B[GM_EV_lifted].value;
  Lv[GM_LEV_exceed_palm].value = ov_palm;
  Lv[GM_LEV_finger_force].value = ov_avg;
  Lv[GM_LEV_finger1_force].value = f1m;
  Lv[GM_LEV_finger2_force].value = f2m;
  Lv[GM_LEV_finger3_force].value = f3m;
  Lv[GM_LEV_ground_force].value = gm;
  Lv[GM_LEV_good_bend_sensor].value = avg_gauge;
  Lv[GM_LEV_exceed_bend_sensor].value = max_gauge;
  Lv[GM_LEV_dangerous_bend_sensor].value = max_gauge;
  Lv[GM_LEV_good_palm_sensor].value = last_palm;
  Lv[GM_LEV_exceed_palm_sensor].value = last_palm;
  Lv[GM_LEV_dangerous_palm_sensor].value = last_palm;
  Lv[GM_LEV_exceed_wrist_sensor].value = last_wrist;
  Lv[GM_LEV_dangerous_wrist_sensor].value = last_wrist;
  Lv[GM_LEV_action_penalty_lin].value /= (float)(e->c.n_actions - s->use_termination_action);
  Lv[GM_LEV_action_penalty_sq].value /= (float)(e->c.n_actions - s->use_termination_action);
  Lv[GM_LEV_object_XY_distance].value = (float)(-closest);
  /* successful_grasp metric (mjclass.cpp:1305-1322) */
  const gm_binary_reward* br[GM_N_BINARY] = {
#define GM_BR(n, r, d, t) &s->n,
#include "../include/gm_settings.def"
  };
  for (int k = 0; k < GM_N_BINARY; k++)
    if (B[k].value && br[k]->reward >= (1.0 - 1e-5) && br[k]->done && B[k].row + 1 >= br[k]->trigger)
      B[GM_EV_successful_grasp].value = 1;
  update_events(e);
}

/* sample functions (mjclass.h:278-453) on a ring */
static int sample_ring(int mode, const ring_t* w, int prev_steps, int rps, int total, float* out) {
  if (mode == GM_SAMPLE_RAW) {
    int n = total - 1;
    for (int j = n - 1, k = 0; j >= 0; j--, k++) out[k] = ring_read(w, j);
    return n;
  }
  out[0] = ring_read(w, total - 1);
  for (int i = 0; i < prev_steps; i++) {
    int first = total - 1 - i * rps;
    out[2 * i + 2] = ring_read(w, first - rps);
    float a = out[2 * i], b = out[2 * i + 2];
    if (mode == GM_SAMPLE_CHANGE) out[2 * i + 1] = b - a;
    else if (mode == GM_SAMPLE_AVERAGE) {
      float acc = 0;
      for (int j = 0; j < rps + 1; j++) acc += ring_read(w, first - j);
      out[2 * i + 1] = acc / (rps + 1);
    } else if (mode == GM_SAMPLE_MEDIAN) {
      float v[GM_RING + 1];
      int nv = rps + 1;
      for (int j = 0; j < nv; j++) v[j] = ring_read(w, first - j);
      for (int x = 1; x < nv; x++) { float t = v[x]; int y = x - 1; while (y >= 0 && v[y] > t) { v[y + 1] = v[y]; y--; } v[y + 1] = t; }
      int hn = nv / 2;
      float med = v[hn];
      if (!(nv & 1)) med = (v[hn - 1] + med) / 2.0f;
      out[2 * i + 1] = med;
    } else if (mode == GM_SAMPLE_SIGN) {
      float ch = b - a;
      out[2 * i + 1] = ch > 1e-6f ? 1.0f : (ch < -1e-6f ? -1.0f : 0.0f);
    } else if (mode == GM_SAMPLE_SCALED_CHANGE) {
      float sc = (b - a) / 0.07f;
      if (sc > 1.0f) sc = 1.0f; else if (sc < -1.0f) sc = -1.0f;
      out[2 * i + 1] = sc;
    } else {
      float ch = fabsf(b - a);
      float f = 1.0f / (0.10f * 0.10f);
      float sc = (b - a) * ch * f;
      if (sc > 1.0f) sc = 1.0f; else if (sc < -1.0f) sc = -1.0f;
      out[2 * i + 1] = sc;
    }
  }
  return 2 * prev_steps + 1;
}
int or_sample(int mode, const float* recent_first, int n_avail, int prev_steps, int rps, float* out) {
  ring_t w;
  ring_reset(&w);
  for (int k = n_avail - 1; k >= 0; k--) ring_add(&w, recent_first[k]);
  return sample_ring(mode, &w, prev_steps, rps, 1 + rps * prev_steps, out);
}
static int sample_sensor(int mode, const ring_t* w, const gm_sensor* s, float* out) {
  return sample_ring(mode, w, s->prev_steps, s->readings_per_step, s->total_readings, out);
}

/* MjClass::get_observation (mjclass.cpp:1707-1959) */
int or_get_obs(or_env* e, float* out) {
  const gm_settings* s = &e->c.s;
  int sf = e->c.sensor_fcn, tf = e->c.state_fcn, n = 0;
  if (s->bending_gauge.in_use) for (int f = 0; f < 3; f++) n += sample_sensor(sf, &e->w_gauge[f], &s->bending_gauge, out + n);
  if (s->axial_gauge.in_use) for (int f = 0; f < 3; f++) n += sample_sensor(sf, &e->w_axial[f], &s->axial_gauge, out + n);
  if (s->palm_sensor.in_use) n += sample_sensor(sf, &e->w_palm, &s->palm_sensor, out + n);
  if (s->wrist_sensor_XY.in_use) {
    n += sample_sensor(sf, &e->w_wx, &s->wrist_sensor_XY, out + n);
    n += sample_sensor(sf, &e->w_wy, &s->wrist_sensor_XY, out + n);
  }
  if (s->wrist_sensor_Z.in_use) n += sample_sensor(sf, &e->w_wz, &s->wrist_sensor_XY, out + n);  /* quirk 1806 */
  if (s->motor_state_sensor.in_use) for (int k = 0; k < 3; k++) n += sample_sensor(tf, &e->w_motor[k], &s->motor_state_sensor, out + n);
  if (s->base_state_sensor_XY.in_use) for (int k = 0; k < 2; k++) n += sample_sensor(tf, &e->w_base[k], &s->base_state_sensor_XY, out + n);
  if (s->base_state_sensor_Z.in_use) n += sample_sensor(tf, &e->w_base[2], &s->base_state_sensor_Z, out + n);
  if (s->base_state_sensor_yaw.in_use) n += sample_sensor(tf, &e->w_yaw, &s->base_state_sensor_yaw, out + n);
  if (s->cartesian_contacts_XYZ.in_use)
    for (int k = 0; k < 12; k++) n += sample_sensor(GM_SAMPLE_CHANGE, &e->w_cart[k], &s->cartesian_contacts_XYZ, out + n);
  return n;
}

/* MjClass::is_done (mjclass.cpp:1632-1698) */
static int is_done_eval(or_env* e) {
  const gm_settings* s = &e->c.s;
  int k = 0;
#define GM_BR(n, r, d, t) if (s->n.done && e->bev[k].row >= s->n.done) return 1; k++;
#include "../include/gm_settings.def"
  k = 0;
#define GM_LR(n, r, d, t, a, b, o) if (s->n.done && e->lev[k].row >= s->n.done) return 1; k++;
#include "../include/gm_settings.def"
  if (s->cap_reward && s->quit_if_cap_exceeded) {
    if (e->cumulative_reward - 1e-5 < s->reward_cap_lower_bound) return 1;
    if (e->cumulative_reward + 1e-5 > s->reward_cap_upper_bound) return 1;
  }
  return 0;
}

/* linear_reward (mjclass.cpp:4866-4894) */
static float linear_reward(float val, float mn, float mx, float overshoot) {
  if (val < mn) return 0.0f;
  if (val > mx) {
    if (overshoot < mx) return 1.0f;
    if (val > overshoot) return 0.0f;
    mn = 0; mx = overshoot - mx; val = overshoot - val;
  }
  return (val - mn) / (mx - mn);
}
/* MjClass::reward + calc_rewards (mjclass.cpp:3000-3049, 5471-5528) */
/* is_done (mjclass.cpp:1632-1698); the result is kept as GmEnvState::done */
int or_is_done(or_env* e) { return e->last_done = is_done_eval(e); }
float or_reward(or_env* e) {
  const gm_settings* s = &e->c.s;
  float r = 0;
  int k = 0;
#define GM_BR(n, rr, d, t) if (e->bev[k].row >= s->n.trigger) r += s->n.reward; k++;
#include "../include/gm_settings.def"
  k = 0;
#define GM_LR(n, rr, d, t, a, b, o)                                                   \
  if (e->lev[k].row >= s->n.trigger) {                                               \
    float fr = linear_reward(e->lev[k].last_value, s->n.min, s->n.max, s->n.overshoot); \
    r += s->n.reward * fr;                                                           \
  }                                                                                  \
  k++;
#include "../include/gm_settings.def"
  e->cumulative_reward += r;
  if (e->cumulative_reward < s->reward_cap_lower_bound && s->cap_reward) {
    r += s->reward_cap_lower_bound - e->cumulative_reward;
    e->cumulative_reward = s->reward_cap_lower_bound;
  }
  if (e->cumulative_reward > s->reward_cap_upper_bound && s->cap_reward) {
    r += s->reward_cap_upper_bound - e->cumulative_reward;
    e->cumulative_reward = s->reward_cap_upper_bound;
  }
  e->last_reward = r;
  return r;
}

/* =====================================================================
 * actions: MjClass::set_action (mjclass.cpp:1528-1630) + luke::move_* (2422-2536)
 * ===================================================================== */
static int move_base_target_m(or_env* e, double x, double y, double z) {
  double* b = e->base;
  const double* mn = e->c.base_min;
  const double* mx = e->c.base_max;
  b[0] += x; b[1] += y; b[2] += z;
  int wl = 1;
  for (int k = 0; k < 3; k++) {
    if (b[k] > mx[k]) { b[k] = mx[k]; wl = 0; }
    if (b[k] < mn[k]) { b[k] = mn[k]; wl = 0; }
  }
  return wl;
}
static int move_base_target_rad(or_env* e, double r, double p, double y) {
  (void)r; (void)p;
  e->base[5] += y;
  int wl = 1;
  if (e->base[5] > e->c.base_max[5]) { e->base[5] = e->c.base_max[5]; wl = 0; }
  if (e->base[5] < e->c.base_min[5]) { e->base[5] = e->c.base_min[5]; wl = 0; }
  return wl;
}
/* ActionSetting::call_action_function (mjclass.h:546-571) with the name-derived
 * function and argument (update_action_function, mjclass.h:488-544) */
static int call_action(or_env* e, int kind, double v) {
  const gm_action* acts[GM_N_ACTION_KINDS] = {
#define GM_AA(n, u, vv, sg) &e->c.s.n,
#include "../include/gm_settings.def"
  };
  v *= acts[kind]->sign;
  double a[3] = {0, 0, 0};
  switch (kind) {
    case GM_ACT_gripper_X: a[0] = v; return g_set_xyz_m(&e->end, e->end.x + a[0], e->end.y, e->end.z);
    case GM_ACT_gripper_Y: a[1] = v; return g_set_xyz_m(&e->end, e->end.x, e->end.y + a[1], e->end.z);
    case GM_ACT_gripper_prismatic_X: return g_set_xyz_m_rad(&e->end, e->end.x + v, e->end.th, e->end.z);
    case GM_ACT_gripper_revolute_Y: return g_set_xyz_m_rad(&e->end, e->end.x, e->end.th + v, e->end.z);
    case GM_ACT_gripper_Z: return g_set_xyz_m(&e->end, e->end.x, e->end.y, e->end.z + v);
    case GM_ACT_base_X: return move_base_target_m(e, v, 0, 0);
    case GM_ACT_base_Y: return move_base_target_m(e, 0, v, 0);
    case GM_ACT_base_Z: return move_base_target_m(e, 0, 0, v);
    case GM_ACT_base_roll: return move_base_target_rad(e, v, 0, 0);
    case GM_ACT_base_pitch: return move_base_target_rad(e, 0, v, 0);
    default: return move_base_target_rad(e, 0, 0, v);
  }
}
/* luke::get_fingertip_z_height (myfunctions.cpp:3608-3620) */
static float fingertip_z_height(const or_env* e) {
  float straight = (float)(-e->c.base_min[2] - e->base[2]);
  float tip_lift = (float)(e->m.finger_length * (1 - cos(g_th_rad(&e->end))));
  float h = straight + tip_lift;
  return (float)(h + e->c.base_min[2]);
}
static void lift_base_to_height(or_env* e, double z) {
  e->base[2] = -z;
  if (e->base[2] > e->c.base_max[2]) e->base[2] = e->c.base_max[2];
  if (e->base[2] < e->c.base_min[2]) e->base[2] = e->c.base_min[2];
}
static void full_substep(or_env* e);
static void set_action(or_env* e, int action, float frac) {
  const gm_settings* s = &e->c.s;
  int wl = 1;
  e->termination_signal_sent = 0;
  if (action < 0 || action >= e->c.n_actions) return;
  int code = e->c.action_options[action];
  if (code == GM_ACTION_TERMINATION) {
    float value = s->continous_actions ? frac : 1.0f;
    if (value > s->termination_threshold) {
      e->termination_signal_sent = 1;
      if (s->lift_on_termination) {
        lift_base_to_height(e, e->c.base_max[2]);
        for (int i = 0; i < e->c.sim_steps_per_action * 2; i++) full_substep(e);
      }
    }
    wl = 1;
  } else {
    int kind = code / 3, sub = code % 3;
    const gm_action* acts[GM_N_ACTION_KINDS] = {
#define GM_AA(n, u, vv, sg) &s->n,
#include "../include/gm_settings.def"
    };
    if (sub == 0) wl = call_action(e, kind, acts[kind]->value);
    else if (sub == 1) wl = call_action(e, kind, -1 * acts[kind]->value);
    else {
      wl = call_action(e, kind, acts[kind]->value * frac);
      e->lev[GM_LEV_action_penalty_lin].value += fabsf(frac);
      e->lev[GM_LEV_action_penalty_sq].value += (frac * frac);
    }
  }
  if (fingertip_z_height(e) < s->fingertip_min_mm * 1e-3) wl = 0;
  e->bev[GM_EV_exceed_limits].value = e->bev[GM_EV_exceed_limits].value || !wl;
}
void or_set_action(or_env* e, const float* a) {
  for (int i = 0; i < e->c.n_actions; i++) {
    float f = a[i];
    if (f < -1.0f) f = -1.0f; else if (f > 1.0f) f = 1.0f;
    set_action(e, i, f);
  }
}
void or_set_discrete_action(or_env* e, int32_t a) { set_action(e, a, 0); }

/* the rollout drivers' fractions for the env's current state (the device's driver_fraction,
 * gm_kernels.hip; test infrastructure): 0 scripted grasp mix, 1 uniform random (the counter
 * hash), 3 grasp-lift-hold program (gm_state.h gm_program_fraction), 4 the program in 1
 * episode of 4 and the scripted mix otherwise; gid = the env's global id */
void or_driver_actions(const or_env* e, int mode, uint64_t seed, float jitter, int64_t gid, float* out) {
  const gm_model* m = &e->m;
  const gm_settings* st = &e->c.s;
  const gm_action* acts[GM_N_ACTION_KINDS] = {
#define GM_AA(n, u, vv, sg) &st->n,
#include "gm_settings.def"
  };
  gm_program_in in;
  in.x = e->end.x; in.y = e->end.y; in.z = e->end.z;
  in.base_z = e->base[2];
  in.q_base = e->qpos[m->jnt_qposadr[m->body_jnt[m->body_base]]];
  in.q_palm = e->qpos[m->jnt_qposadr[m->body_jnt[m->body_palm]]];
  in.obj_z = e->qpos[m->jnt_qposadr[m->body_jnt[m->body_obj]] + 2];
  in.obj_top = gm_program_obj_top(m->geom_type[m->geom_obj], m->geom_size[m->geom_obj]);
  in.z_root = m->body_pos[m->body_base][2];
  in.palm_drop = (m->finger_length - 165e-3) + 0.004;
  {
    const float g0 = ring_latest(&e->si_gauge[0]), g1 = ring_latest(&e->si_gauge[1]), g2 = ring_latest(&e->si_gauge[2]);
    in.g_max = fmaxf(g0, fmaxf(g1, g2));
  }
  in.palm = ring_latest(&e->si_palm);
  const int prog = mode == 3 || (mode == 4 && gm_program_episode(seed, gid, e->episode));
  for (int i = 0; i < e->c.n_actions; i++) {
    const int code = e->c.action_options[i];
    const int kind = (code >= 0 && code < GM_ACTION_TERMINATION) ? code / 3 : -1;
    float v;
    if (prog) v = kind < 0 ? 0.0f : gm_program_fraction(&in, kind, acts[kind]->value, acts[kind]->sign);
    else if (mode == 0 || mode == 4) v = gm_script_fraction(seed, gid, e->episode, e->num_action_steps, i, kind, jitter);
    else v = gm_random_fraction(seed, gid, e->episode, e->num_action_steps, i);
    out[i] = v < -1.0f ? -1.0f : (v > 1.0f ? 1.0f : v);
  }
}

/* MjClass::step (mjclass.cpp:504-530): physics + update_all + monitor_sensors */
static void full_substep(or_env* e) {
  physics_substep(e);
  update_all(e);
  monitor_sensors(e);
}
/* MjClass::action_step (mjclass.cpp:1483-1508) */
void or_step(or_env* e) {
  for (int i = 0; i < e->c.sim_steps_per_action; i++) full_substep(e);
  sense_gripper_state(e);
  update_env(e);
  e->num_action_steps += 1;
}

/* =====================================================================
 * reset (mjclass.cpp:434-486, myfunctions.cpp:544-570, 1441-1519) and spawn
 * ===================================================================== */
static void keyframe_state(or_env* e) {
  for (int i = 0; i < NQ; i++) e->qpos[i] = e->m.qpos0[i];
  for (int i = 0; i < NV; i++) e->qvel[i] = 0;
  for (int i = 0; i < NV; i++) e->qacc_warm[i] = 0;
  e->time = 0;
  e->last_step_time = 0;
}
static int is_motor_or_base_dof(const gm_model* m, int d) {
  if (d == m->dof_base || d == m->dof_palm) return 1;
  for (int f = 0; f < 3; f++) if (d == m->dof_pris[f] || d == m->dof_rev[f]) return 1;
  return 0;
}
/* first-call settle of calibrate_reset (400 substeps, no sensors) */
/* calibrate_reset's function-static first_call (myfunctions.cpp:1447), as a switch: with
 * the cache on, the first env created settles and every later env with the same segment
 * count takes that equilibrium (or_set_settle_cache; gm_set_settle_cache on the device) */
static pthread_mutex_t g_settle_mu = PTHREAD_MUTEX_INITIALIZER;
static int g_settle_cache_on = 0, g_settle_valid = 0, g_settle_nseg = -1;
static double g_settle_eq[NQ];
void or_set_settle_cache(int on) {
  pthread_mutex_lock(&g_settle_mu);
  g_settle_cache_on = on != 0;
  g_settle_valid = 0;
  pthread_mutex_unlock(&g_settle_mu);
}
static void settle_uncached(or_env* e);
static void settle(or_env* e) {
  pthread_mutex_lock(&g_settle_mu);
  if (g_settle_cache_on && g_settle_valid && g_settle_nseg == e->m.n_seg) {
    for (int i = 0; i < NQ; i++) e->eq_q[i] = g_settle_eq[i];
    /* the settle's side effects on the env (targets home, locks off, keyframe) */
    g_reset(&e->end); g_reset(&e->next);
    for (int k = 0; k < 6; k++) e->base[k] = 0;
    for (int k = 0; k < GM_MAX_LOCK; k++) { e->lock_active[k] = 0; e->lock_q[k] = 0; }
    e->old_x = e->old_y = e->old_z = 1;
    keyframe_state(e);
    pthread_mutex_unlock(&g_settle_mu);
    return;
  }
  pthread_mutex_unlock(&g_settle_mu);
  settle_uncached(e);
  pthread_mutex_lock(&g_settle_mu);
  /* a changed joint count re-settles and keeps the new settle (myfunctions.cpp:1453-1468) */
  if (g_settle_cache_on && (!g_settle_valid || g_settle_nseg != e->m.n_seg)) {
    for (int i = 0; i < NQ; i++) g_settle_eq[i] = e->eq_q[i];
    g_settle_valid = 1;
    g_settle_nseg = e->m.n_seg;
  }
  pthread_mutex_unlock(&g_settle_mu);
}
static void settle_uncached(or_env* e) {
  g_reset(&e->end); g_reset(&e->next);
  for (int k = 0; k < 6; k++) e->base[k] = 0;
  for (int k = 0; k < GM_MAX_LOCK; k++) { e->lock_active[k] = 0; e->lock_q[k] = 0; }
  e->old_x = e->old_y = e->old_z = 1;
  keyframe_state(e);
  for (int i = 0; i < 400; i++) { physics_substep(e); update_all(e); }
  for (int i = 0; i < NQ; i++) e->eq_q[i] = e->qpos[i];
}

static void sensors_reset(or_env* e) {
  for (int f = 0; f < 3; f++) {
    ring_reset(&e->w_gauge[f]); ring_reset(&e->w_axial[f]); ring_reset(&e->w_motor[f]);
    ring_reset(&e->w_base[f]); ring_reset(&e->si_gauge[f]); ring_reset(&e->si_axial[f]);
  }
  ring_reset(&e->w_palm); ring_reset(&e->w_wx); ring_reset(&e->w_wy); ring_reset(&e->w_wz);
  ring_reset(&e->w_yaw); ring_reset(&e->si_palm); ring_reset(&e->si_wz);
  for (int k = 0; k < 12; k++) ring_reset(&e->w_cart[k]);
  for (int k = 0; k < S_N; k++) e->last_read[k] = 0;
}

/* Settings::apply_noise_params RNG draws (mjclass.cpp:5293-5346) */
static void randomise_mu(or_env* e) {
  gm_settings* s = &e->c.s;
  gm_sensor* ss[S_N] = {&s->motor_state_sensor, &s->base_state_sensor_Z, &s->base_state_sensor_XY,
                        &s->base_state_sensor_yaw, &s->bending_gauge, &s->axial_gauge, &s->palm_sensor,
                        &s->wrist_sensor_XY, &s->wrist_sensor_Z, &s->cartesian_contacts_XYZ};
  for (int k = 0; k < S_N; k++)
    for (int i = 0; i < 3; i++) e->rand_mu[k][i] = ss[k]->noise_mu * (2 * unif01(&e->rng) - 1);
  int order[5] = {S_MOTOR, S_BASEXY, S_BASEZ, S_YAW, S_CART};
  for (int k = 0; k < 5; k++)
    for (int i = 0; i < 3; i++) e->rand_mu[order[k]][i] = ss[order[k]]->noise_mu * (2 * unif01(&e->rng) - 1);
}

/* spawn_object (mjclass.cpp:2352-2420, objecthandler.cpp:403-428) */
void or_spawn(or_env* e, const gm_spawn* sp) {
  int oi = sp ? sp->object_index : 0;
  if (oi < 0 || oi >= e->nobj) oi = 0;
  e->obj_index = oi;
  apply_object(&e->m, &e->objs[oi]);
  object_invweight(e);
  int qa = e->m.jnt_qposadr[e->m.body_jnt[e->m.body_obj]];
  double zr = sp ? sp->zrot : 0.0;
  /* quaternion exactly as the reference composes it: QPos (x,y,z,qx,qy,qz,qw) with
   * qx written to qpos[3] (MuJoCo's w slot) -- net effect: rotation pi+zrot about z */
  double x2, w2;
  gm_sincos(-zr / 2.0, &x2, &w2);
  const double q4[4] = {x2, 0, 0, w2};
  const double nq = sqrt(q4[0] * q4[0] + q4[1] * q4[1] + q4[2] * q4[2] + q4[3] * q4[3]);
  e->qpos[qa + 0] = sp ? sp->x : 0.0;
  e->qpos[qa + 1] = sp ? sp->y : 0.0;
  e->qpos[qa + 2] = object_rest_z(&e->objs[oi]) + 1e-6;
  for (int k = 0; k < 4; k++) e->qpos[qa + 3 + k] = q4[k] / nq;
  for (int k = 0; k < 6; k++) e->qvel[e->m.dof_obj + k] = 0;
  for (int k = 0; k < 7; k++) e->start_qpos[k] = e->qpos[qa + k];
}

/* =====================================================================
 * MjClass::spawn_into_scene(SpawnParams) (mjclass.cpp:2475-2654)
 * ===================================================================== */
/* std::uniform_int_distribution<unsigned long>{a, b}(minstd_rand0) as libstdc++
 * implements it (bits/uniform_int_dist.h): engine range 2^31 - 3 takes the
 * downscaling two-division rejection path */
static uint64_t uid_minstd(uint32_t* st, uint64_t a, uint64_t b) {
  const uint64_t urngrange = 2147483646ull - 1ull, urange = b - a;
  uint64_t ret;
  if (urngrange > urange) {
    const uint64_t uerange = urange + 1, scaling = urngrange / uerange, past = uerange * scaling;
    do ret = (uint64_t)lcg_next(st) - 1ull; while (ret >= past);
    ret /= scaling;
  } else {
    ret = (uint64_t)lcg_next(st) - 1ull;
  }
  return ret + a;
}
/* std::shuffle with minstd_rand0 as libstdc++ implements it (bits/stl_algo.h):
 * positions drawn in pairs (__gen_two_uniform_ints) when the engine range allows,
 * one leading {0,1} draw for an even count */
static void shuffle_minstd(int* v, int n, uint32_t* st) {
  if (n <= 0) return;
  const uint64_t urngrange = 2147483645ull, urange = (uint64_t)n;
  int t;
  if (urngrange / urange >= urange) {
    int i = 1;
    if (urange % 2 == 0) { int j = (int)uid_minstd(st, 0, 1); t = v[i]; v[i] = v[j]; v[j] = t; i++; }
    while (i != n) {
      uint64_t r = (uint64_t)i + 1, x = uid_minstd(st, 0, r * (r + 1) - 1);
      int p1 = (int)(x / (r + 1)), p2 = (int)(x % (r + 1));
      t = v[i]; v[i] = v[p1]; v[p1] = t; i++;
      t = v[i]; v[i] = v[p2]; v[p2] = t; i++;
    }
  } else {
    for (int i = 1; i < n; i++) { int j = (int)uid_minstd(st, 0, (uint64_t)i); t = v[i]; v[i] = v[j]; v[j] = t; }
  }
}
/* luke::Box2d (customtypes.h:35-172) */
typedef struct { double x[4], y[4]; } box2_t;
static void box_init_centre(box2_t* b, double cx, double cy, double w, double h) {
  double hw = w / 2.0, hh = h / 2.0;
  b->x[0] = cx - hw; b->y[0] = cy - hh; b->x[1] = cx + hw; b->y[1] = cy - hh;
  b->x[2] = cx + hw; b->y[2] = cy + hh; b->x[3] = cx - hw; b->y[3] = cy + hh;
}
static void box_rotate(box2_t* b, double th) {
  double cx = (b->x[0] + b->x[1] + b->x[2] + b->x[3]) / 4.0, cy = (b->y[0] + b->y[1] + b->y[2] + b->y[3]) / 4.0;
  for (int i = 0; i < 4; i++) {
    double nx = cx + (b->x[i] - cx) * cos(th) - (b->y[i] - cy) * sin(th);
    double ny = cy + (b->x[i] - cx) * sin(th) + (b->y[i] - cy) * cos(th);
    b->x[i] = nx; b->y[i] = ny;
  }
}
static int box_inbounds(const box2_t* b, double xmin, double ymin, double xmax, double ymax) {
  for (int i = 0; i < 4; i++) if (b->x[i] < xmin || b->x[i] > xmax || b->y[i] < ymin || b->y[i] > ymax) return 0;
  return 1;
}
static int box_overlaps(const box2_t* a, const box2_t* o, double gap) {
  int contains = 1;
  for (int i = 0; i < 4; i++) {
    int j = (i + 1) % 4;
    double px = -(a->y[j] - a->y[i]), py = a->x[j] - a->x[i];
    double len = sqrt(px * px + py * py);
    px /= len; py /= len;
    double min1 = a->x[0] * px + a->y[0] * py, max1 = min1, min2 = o->x[0] * px + o->y[0] * py, max2 = min2;
    for (int k = 1; k < 4; k++) {
      double p1 = a->x[k] * px + a->y[k] * py, p2 = o->x[k] * px + o->y[k] * py;
      if (p1 < min1) min1 = p1;
      if (p1 > max1) max1 = p1;
      if (p2 < min2) min2 = p2;
      if (p2 > max2) max2 = p2;
    }
    if (max1 + gap < min2 || max2 + gap < min1) return 0;
    if (max1 < min2 || max2 < min1) contains = 0;
  }
  return contains;
}
/* "Task object i" bounding box (objecthandler.cpp:91-110): full geom extents */
static void object_bbox(const gm_object* o, double* xyz) {
  if (o->type == GM_GEOM_BOX) { xyz[0] = 2 * o->size[0]; xyz[1] = 2 * o->size[1]; xyz[2] = 2 * o->size[2]; }
  else if (o->type == GM_GEOM_CYLINDER) { xyz[0] = xyz[1] = 2 * o->size[0]; xyz[2] = 2 * o->size[1]; }
  else { xyz[0] = xyz[1] = xyz[2] = 2 * o->size[0]; }
}
int or_spawn_into_scene(or_env* e, const gm_spawn_params* p) {
  int num_x = (int)(((2 * p->xrange) / p->xy_increment) + 1);
  int num_y = (int)(((2 * p->yrange) / p->xy_increment) + 1);
  int num_r = (int)(((2 * p->rotrange) / p->rot_increment) + 1);
  int nxy = num_x * num_y;
  if (num_x < 1 || num_y < 1 || num_r < 1 || nxy > GM_SPAWN_MAX_XY || num_r > GM_SPAWN_MAX_ROT) return 0;
  int pxy[GM_SPAWN_MAX_XY], prot[GM_SPAWN_MAX_ROT];
  for (int i = 0; i < nxy; i++) pxy[i] = i;
  for (int i = 0; i < num_r; i++) prot[i] = i;
  if (nxy > 1) shuffle_minstd(pxy, nxy, &e->rng);
  if (num_r > 1) shuffle_minstd(prot, num_r, &e->rng);
  int oi = p->index;
  if (oi < 0 || oi >= e->nobj) oi = 0;
  double bb[3];
  object_bbox(&e->objs[oi], bb);
  /* Env::reset (mjclass.h:895-904) + get_finger_hook_locations (myfunctions.cpp:3717-3761) */
  box2_t tips[3];
  const double PI_23 = PI_D * (2.0 / 3.0);
  const double angles[3] = {0.0, PI_23, 2 * PI_23};
  double hook_th = e->m.hook_angle_degrees * (PI_D / 180.000);
  for (int i = 0; i < 3; i++) {
    double hook_x = 0.5 * e->m.hook_length * sin(hook_th);
    double x = -(e->end.x - hook_x) * sin(angles[i]) + e->base[0];
    double y = -(e->end.x - hook_x) * cos(angles[i]) + e->base[1];
    box_init_centre(&tips[i], x, y, e->m.finger_width, e->m.hook_length);
    box_rotate(&tips[i], -angles[i]);
  }
  int total = nxy > num_r ? nxy : num_r, ixy = -1, ir = -1;
  for (int i = 0; i < total; i++) {
    ixy += 1; ir += 1;
    if (ixy >= nxy) ixy = 0;
    if (ir >= num_r) ir = 0;
    int kx = pxy[ixy] / num_y, ky = pxy[ixy] % num_y;
    double px = num_x > 1 ? -p->xrange + kx * p->xy_increment + p->x : p->x;
    double py = num_y > 1 ? -p->yrange + ky * p->xy_increment + p->y : p->y;
    double pr = num_r > 1 ? -p->rotrange + prot[ir] * p->rot_increment + p->zrot : p->zrot;
    box2_t ob;
    box_init_centre(&ob, px, py, bb[0], bb[1]);
    box_rotate(&ob, pr);
    if (!box_inbounds(&ob, p->xmin, p->ymin, p->xmax, p->ymax)) continue;
    int good = 1;
    for (int f = 0; f < 3 && good; f++) if (box_overlaps(&ob, &tips[f], p->smallest_gap)) good = 0;
    if (!good) continue;
    gm_spawn sp = {p->index, px, py, pr};
    or_spawn(e, &sp);
    return 1;
  }
  return 0;
}
/* golden-vector hooks: libstdc++ std::shuffle / Box2d restatements */
uint32_t or_std_shuffle(uint32_t seed, int n, int32_t* out) {
  uint32_t st = lcg_seed(seed);
  for (int i = 0; i < n; i++) out[i] = i;
  shuffle_minstd(out, n, &st);
  return lcg_next(&st);   /* the engine's next draw: pins how many draws the shuffle used */
}
int or_box2d_overlaps(const double* a5, const double* b5, double gap) {
  /* boxes as (cx, cy, w, h, rot): initCentre then rotate */
  box2_t a, b;
  box_init_centre(&a, a5[0], a5[1], a5[2], a5[3]); box_rotate(&a, a5[4]);
  box_init_centre(&b, b5[0], b5[1], b5[2], b5[3]); box_rotate(&b, b5[4]);
  return box_overlaps(&a, &b, gap);
}

void or_reset(or_env* e, const gm_spawn* sp) {
  const gm_model* m0 = &e->m;
  /* luke::reset: targets home, locks off, keyframe, object parked */
  g_reset(&e->end); g_reset(&e->next);
  for (int k = 0; k < 6; k++) e->base[k] = 0;
  keyframe_state(e);
  /* calibrate_reset: equilibrium gripper + base joints */
  for (int d = 0; d < m0->nv; d++) if (is_motor_or_base_dof(m0, d)) e->qpos[d] = e->eq_q[d];
  /* set_all_constraints(true): locks read the stale keyframe kinematics */
  for (int k = 0; k < m0->nlock; k++) { e->lock_active[k] = 1; e->lock_q[k] = m0->qpos0[m0->lock_dof[k]]; }
  sensors_reset(e);
  memset(e->bev, 0, sizeof(e->bev));
  memset(e->lev, 0, sizeof(e->lev));
  e->cumulative_reward = 0;
  e->num_action_steps = 0;
  e->termination_signal_sent = 0;
  e->grp_peak_lateral = 0;
  e->last_done = 0;
  e->last_reward = 0;
  e->episode += 1;
  /* configure_settings: noise mean draws */
  randomise_mu(e);
  /* random_base_Z_movement (mjclass.cpp:1423-1434) */
  {
    double size = e->c.s.base_position_noise;
    double u = canon_d(&e->rng);
    double z = u * (size - (-size)) + (-size);
    e->base[2] = z;
    if (e->base[2] > e->c.base_max[2]) e->base[2] = e->c.base_max[2];
    if (e->base[2] < e->c.base_min[2]) e->base[2] = e->c.base_min[2];
    e->qpos[m0->dof_base] = e->base[2] + e->eq_q[m0->dof_base];
  }
  or_spawn(e, sp);
}

/* =====================================================================
 * automatic calibration (MjClass::configure_settings, mjclass.cpp:241-308), sequential
 * as the reference runs it: find_highest_stable_timestep (4745-4854), then
 * calibrate_simulated_sensors (4643-4676) with validate_curve_under_force (4023-4105).
 * Noise off (base_position_noise = 0); forward declarations of the env entry points.
 * ===================================================================== */
or_env* or_create(const gm_model* m, const gm_config* c, const gm_object* objects, int n_objects,
                  int64_t env_id);
static float yield_point_load(const gm_model* m) {      /* myfunctions.cpp:3587-3595 */
  double I = (m->finger_width * pow(m->finger_thickness, 3)) / 12.0;
  float M_max = (m->yield_stress * I) / (0.5 * m->finger_thickness);
  float F_max = M_max / m->finger_length;
  return F_max;
}
/* n substeps of MjClass::step (before_step / resolve_segment_forces / step / after_step /
 * monitor_sensors); stops at the first BADQACC like the reference's break */
static __thread int cal_ran;   /* substeps the last cal_steps made (the unstable one included) */
static int cal_steps(or_env* e, int n) {
  /* a run starts from the reset's mj_forward pose */
  memcpy(e->qpos_pre, e->qpos, sizeof(e->qpos));
  e->badqacc = 0;
  cal_ran = 0;
  for (int i = 0; i < n; i++) {
    cal_ran = i + 1;
    if (e->tip_force != 0.0) {
      /* apply_segment_force locks the prismatic motors every step (set_constraint,
       * myfunctions.cpp:1679-1685), anchored at the last mj_step1 pose */
      for (int k = 0; k < e->m.nlock; k++)
        if (e->m.lock_kind[k] == 0) { e->lock_active[k] = 1; e->lock_q[k] = e->qpos_pre[e->m.lock_dof[k]]; }
    }
    physics_substep(e);
    update_all(e);
    if (e->badqacc) return 1;
  }
  return 0;
}
int or_calibrate(const gm_model* m, const gm_config* c, const gm_object* objects, int n_objects, int what,
                 gm_calibration* out, double* trace_dt, uint8_t* trace_unstable, int max_trace) {
  memset(out, 0, sizeof(*out));
  gm_config cc = *c;
  cc.s.base_position_noise = 0;
  or_env* e = or_create(m, &cc, objects, n_objects, 0);
  if (!e) return -1;
  gm_spawn sp = {0, 0.0, 0.0, 0.0};
  double timestep = m->timestep;
  if (what & GM_CAL_TIMESTEP) {
    float coarse_increment = 0.5e-3f, fine_increment = 50e-6f, start_value = 1.0e-3f;
    float test_time = 1.0f, max_allowable_timestep = 20.0e-3f, tune_param = 1.0f;
    float next_timestep = start_value;
    int unstable = 0, coarse_pass = 1, ntr = 0;
    while (1) {
      int num_steps = (test_time / next_timestep) + 1;
      or_reset(e, &sp);
      e->m.timestep = next_timestep;
      unstable = cal_steps(e, num_steps);
      if (ntr < max_trace) {
        if (trace_dt) trace_dt[ntr] = next_timestep;
        if (trace_unstable) trace_unstable[ntr] = (uint8_t)unstable;
      }
      ntr++;
      if (unstable) {
        if (coarse_pass) coarse_pass = 0;
        next_timestep -= fine_increment;
        unstable = 0;
      } else {
        if (coarse_pass) next_timestep += coarse_increment;
        else break;
      }
      if (next_timestep < fine_increment) { or_destroy(e); return -2; }
      if (next_timestep > max_allowable_timestep) { next_timestep = max_allowable_timestep; coarse_pass = 0; }
    }
    float factor;
    if (next_timestep <= 3.0e-3) factor = tune_param * 0.8;
    else if (next_timestep < 5.0e-3) factor = tune_param * 0.75;
    else if (next_timestep < 10.0e-3) factor = tune_param * 0.65;
    else factor = tune_param * 0.65;
    float final_timestep = next_timestep * factor;
    final_timestep = (float)((int)(final_timestep * 1e6) * 1e-6);
    out->search_timestep = next_timestep;
    out->n_tested = ntr;
    timestep = final_timestep;
  }
  out->timestep = timestep;
  if (what & GM_CAL_GAUGES) {
    float yield = yield_point_load(m);
    float bend_gauge_normalise = cc.s.saturation_yield_factor * yield;
    double ts = timestep;                                 /* s_.mujoco_timestep (double) */
    or_reset(e, &sp);
    e->m.timestep = ts;
    e->tip_force = 0;
    float settle_time = 0.3;
    int steps_for_settle = settle_time / ts;
    cal_steps(e, steps_for_settle);
    float time_to_settle = 50;
    int steps_to_make = time_to_settle / ts;
    int repeats_done = 1;
    const int ref_retry = (what & GM_CAL_REFERENCE_RETRY) != 0;
    int left = steps_to_make;
    double tip = bend_gauge_normalise;
    while (1) {
      e->tip_force = tip;
      if (cal_steps(e, ref_retry ? left : steps_to_make)) {
        ts *= 0.8;
        e->tip_force = 0;
        or_reset(e, &sp);
        e->m.timestep = ts;
        repeats_done += 1;
        if (repeats_done > 5) { or_destroy(e); return -3; }
        if (ref_retry) {
          /* validate_curve_under_force (mjclass.cpp:4073-4090): reset() wiped the segment
           * forces and `continue` resumes the step loop after the unstable step, unloaded */
          tip = 0.0;
          left -= cal_ran;
          if (left <= 0) break;
        }
        continue;
      }
      break;
    }
    e->tip_force = 0;
    int qa = e->m.dof_seg[0];    /* read_armadillo_gauge(data, 0): finger 0's segment joints */
    float normalise = or_gauge_reading(&e->m, &e->qpos[qa]);
    out->yield_load = yield;
    out->bend_gauge_normalise = bend_gauge_normalise;
    out->bending_normalise = normalise;
    out->sim_gauge_raw_to_N_factor = bend_gauge_normalise / normalise;
    out->wrist_Z_offset = 0.0f;
    out->gauge_retries = repeats_done - 1;
    out->timestep = ts;
  }
  out->sim_steps_per_action = (int32_t)ceil(cc.s.time_for_action / out->timestep);
  or_destroy(e);
  return 0;
}

/* test hook: the constraint solver of envs created from now on (0 Newton, > 0 PGS sweeps) */
static int g_solver_pgs = 0;
void or_set_default_solver(int pgs_sweeps) { g_solver_pgs = pgs_sweeps; }
/* test variant: the reference's motor locks as 6-row weld equalities between the slide's
 * two bodies (myfunctions.cpp:1177-1279) instead of the engine's 1-row joint locks */
static int g_weld_locks = 0;
void or_set_default_weld_locks(int on) { g_weld_locks = on; }
void or_set_solver(or_env* e, int pgs_sweeps) { e->solver_pgs = pgs_sweeps; }
/* solver statistics since creation: solves, Newton iterations, line-search evaluations,
 * max iterations, max contacts generated, constraint rows */
void or_get_stats(const or_env* e, int64_t* out) {
  out[0] = e->stat_solves; out[1] = e->stat_it_sum; out[2] = e->stat_ls_sum; out[3] = e->stat_it_max;
  out[4] = e->stat_ncon_max; out[5] = e->stat_nefc_sum;
}

or_env* or_create(const gm_model* m, const gm_config* c, const gm_object* objects, int n_objects,
                  int64_t env_id) {
  or_env* e = (or_env*)calloc(1, sizeof(or_env));
  if (!e) return NULL;
  e->m = *m;
  e->c = *c;
  e->nobj = n_objects > GM_MAX_OBJSET ? GM_MAX_OBJSET : n_objects;
  for (int i = 0; i < e->nobj; i++) e->objs[i] = objects[i];
  e->env_id = env_id;
  e->solver_pgs = g_solver_pgs;
  e->weld_locks = g_weld_locks;
  e->rng = lcg_seed((uint64_t)c->s.random_seed + (uint64_t)env_id * 1000003ull);
  /* settle with the first object parked at the keyframe pose */
  if (topo_init(e) != 0) { free(e); return NULL; }
  if (e->nobj > 0) { apply_object(&e->m, &e->objs[0]); object_invweight(e); }
  settle(e);
  e->old_x = e->old_y = e->old_z = 0;
  return e;
}
void or_destroy(or_env* e) { free(e); }

void or_get_state(const or_env* e, double* qpos, double* qvel, double* time) {
  if (qpos) for (int i = 0; i < e->m.nq; i++) qpos[i] = e->qpos[i];
  if (qvel) for (int i = 0; i < e->m.nv; i++) qvel[i] = e->qvel[i];
  if (time) *time = e->time;
}
void or_set_state(or_env* e, const double* qpos, const double* qvel) {
  if (qpos) for (int i = 0; i < e->m.nq; i++) e->qpos[i] = qpos[i];
  if (qvel) for (int i = 0; i < e->m.nv; i++) e->qvel[i] = qvel[i];
}
void or_get_target(const or_env* e, double* end_xyzth, int32_t* es, int32_t* ns, double* base_xyz) {
  if (end_xyzth) { end_xyzth[0] = e->end.x; end_xyzth[1] = e->end.y; end_xyzth[2] = e->end.z; end_xyzth[3] = e->end.th; }
  if (es) { es[0] = e->end.sx; es[1] = e->end.sy; es[2] = e->end.sz; }
  if (ns) { ns[0] = e->next.sx; ns[1] = e->next.sy; ns[2] = e->next.sz; }
  if (base_xyz) { base_xyz[0] = e->base[0]; base_xyz[1] = e->base[1]; base_xyz[2] = e->base[2]; }
}
void or_get_event_rows(const or_env* e, int32_t* rows, int32_t* absc, float* lastv) {
  for (int k = 0; k < GM_N_BINARY; k++) {
    if (rows) rows[k] = e->bev[k].row;
    if (absc) absc[k] = e->bev[k].abs;
    if (lastv) lastv[k] = (float)e->bev[k].last_value;
  }
  for (int k = 0; k < GM_N_LINEAR; k++) {
    if (rows) rows[GM_N_BINARY + k] = e->lev[k].row;
    if (absc) absc[GM_N_BINARY + k] = e->lev[k].abs;
    if (lastv) lastv[GM_N_BINARY + k] = e->lev[k].last_value;
  }
}
/* MjClass::set_motor_target (mjclass.cpp:1359-1364) -> luke::set_gripper_target_m
 * (myfunctions.cpp:2347-2355) -> Gripper::set_xyz_m (gripper.h:152-154) */
int or_set_motor_target(or_env* e, double x, double y, double z) {
  e->end.x = x; e->end.y = y; e->end.z = z;
  return g_update(&e->end);
}
/* sim_sensors_SI_.read_finger1_gauge() ... read_wrist_Z_sensor() (mjclass.h SensorData) */
void or_get_sensor_si(const or_env* e, float* out) {
  for (int f = 0; f < 3; f++) out[f] = ring_latest(&e->si_gauge[f]);
  out[3] = ring_latest(&e->si_palm);
  out[4] = ring_latest(&e->si_wz);
}
int or_overflow(const or_env* e) { return e->overflow; }
void or_get_eq(const or_env* e, double* eq) { for (int i = 0; i < e->m.nq; i++) eq[i] = e->eq_q[i]; }

/* mj_rnePostConstraint's cfrc_ext for the live object (myfunctions.cpp:1905), as
 * ObjectHandler::get_object_net_force_faster reads it (objecthandler.cpp:543-565): every
 * contact's world force (frame^T * contact-frame force) acts on geom2 and its reaction on
 * geom1; torques about the object's centre of mass (its c-frame origin: the object is the
 * root of its own tree).  out = [force; torque] (the reference's swapped order). */
void or_object_net_wrench(const or_env* e, double* out) {
  const gm_model* m = &e->m;
  const double* com = e->xpos[m->body_obj];   /* free object: centre of mass at the body origin */
  for (int k = 0; k < 6; k++) out[k] = 0;
  for (int i = 0; i < e->ncon; i++) {
    const con_t* C = &e->con[i];
    double sgn = 0;
    if (C->g2 == m->geom_obj) sgn = 1;
    else if (C->g1 == m->geom_obj) sgn = -1;
    else continue;
    double g[3] = {0, 0, 0};
    for (int k = 0; k < 3; k++)
      for (int r = 0; r < 3; r++) g[k] += C->frame[3 * r + k] * C->force[r];
    double rr[3], t[3];
    sub3(rr, C->pos, com);
    cross3(t, rr, g);
    for (int k = 0; k < 3; k++) { out[k] += sgn * g[k]; out[3 + k] += sgn * t[k]; }
  }
}

/* the last substep's qfrc_smooth and qfrc_constraint = J^T efc (dense, test hook); only
 * recorded while or_want_forces(e, 1) is on */
void or_want_forces(or_env* e, int on) { e->want_forces = on != 0; }
void or_last_forces(const or_env* e, double* smooth, double* constraint) {
  for (int d = 0; d < e->m.nv; d++) { smooth[d] = e->last_smooth[d]; constraint[d] = e->last_constraint[d]; }
}
void or_debug_substep(or_env* e, int32_t* ncon, double* contact, double* efc_force, double* qacc,
                      double* obj_wrench) {
  full_substep(e);
  if (ncon) *ncon = e->ncon;
  if (contact) {
    for (int c = 0; c < NC; c++) {
      double* o = contact + 16 * c;
      for (int k = 0; k < 16; k++) o[k] = 0;
      if (c >= e->ncon) continue;
      const con_t* C = &e->con[c];
      o[0] = C->dist;
      for (int k = 0; k < 3; k++) o[1 + k] = C->pos[k];
      for (int k = 0; k < 9; k++) o[4 + k] = C->frame[k];
      o[13] = C->g1; o[14] = C->g2; o[15] = C->mu;
    }
  }
  if (efc_force) for (int r = 0; r < GM_MAX_EFC; r++) efc_force[r] = r < e->nefc ? e->efc_f[r] : 0.0;
  if (qacc) for (int d = 0; d < e->m.nv; d++) qacc[d] = e->qacc[d];
  if (obj_wrench) or_object_net_wrench(e, obj_wrench);
}

/* ---- hooks for the independent physics checks (tests/test_physics_independent.py) ----
 * or_dynamics: the engine's kinematics, joint-space inertia and bias at the env's current
 * state -- body poses, the dense smooth matrix H~ (M + armature + h (D + Kd) + h^2 Kp, from
 * the tree blocks), its diagonal additions, and qfrc_bias (RNE: Coriolis, centrifugal,
 * gravity); the test compares them with a natural-order Jacobian formulation. */
void or_dynamics(or_env* e, double* xpos, double* xquat, double* H, double* add, double* bias) {
  const gm_model* m = &e->m;
  fk(e);
  crb_rne(e);
  mass_and_forces(e);
  const int nv = m->nv;
  if (xpos) for (int b = 0; b < m->nbody; b++) for (int k = 0; k < 3; k++) xpos[3 * b + k] = e->xpos[b][k];
  if (xquat) for (int b = 0; b < m->nbody; b++) for (int k = 0; k < 4; k++) xquat[4 * b + k] = e->xquat[b][k];
  if (H) {
    static double Hd[NV][NV];
    dense_H(e, Hd);
    for (int i = 0; i < nv; i++) for (int j = 0; j < nv; j++) H[i * nv + j] = Hd[i][j];
  }
  for (int d = 0; d < nv; d++) {
    const double h = m->timestep;
    double a = e->T.dof_arm[d] + h * e->T.dof_dsum[d];
    a += h * h * e->T.dof_ksum[d];
    if (add) add[d] = a;
    if (bias) bias[d] = dot6(e->cdof[d], e->cfrc[m->dof_body[d]]);
  }
}
/* or_collide: the engine's narrowphase for one canonical pair (geom1 type <= geom2 type),
 * geoms given by type, size, centre and row-major rotation; up to 8 contacts as
 * [dist, pos[3], normal[3]] (normal from geom1 to geom2); returns the count. */
int or_collide(int type1, const double* size1, const double* c1, const double* R1, int type2, const double* size2,
               const double* c2, const double* R2, double mpr_tol, int mpr_it, double* out) {
  geomv_t A, B;
  A.type = type1; B.type = type2;
  for (int k = 0; k < 3; k++) { A.size[k] = size1[k]; A.c[k] = c1[k]; B.size[k] = size2[k]; B.c[k] = c2[k]; }
  for (int k = 0; k < 9; k++) { A.R[k] = R1[k]; B.R[k] = R2[k]; }
  A.rbound = B.rbound = 1e9; A.friction = B.friction = 1.0;
  hit_t hs[8];
  int n = 0;
  hit_t h;
  if (A.type == GM_GEOM_PLANE) {
    if (B.type == GM_GEOM_SPHERE) { if (plane_sphere(&A, &B, &h)) hs[n++] = h; }
    else if (B.type == GM_GEOM_BOX) {
      for (int i = 0; i < 8 && n < 4; i++) if (plane_box_point(&A, &B, i, &h)) hs[n++] = h;
    } else if (B.type == GM_GEOM_CYLINDER) {
      cylframe_t cf;
      cyl_frame(&A, &B, &cf);
      for (int i = 0; i < 8 && n < 4; i++) if (plane_cyl_point(&A, &B, &cf, i, &h)) hs[n++] = h;
    }
  } else if (A.type == GM_GEOM_SPHERE && B.type == GM_GEOM_BOX) {
    if (sphere_box(&A, &B, &h)) hs[n++] = h;
  } else if (A.type == GM_GEOM_BOX && B.type == GM_GEOM_BOX) {
    bbox_t S;
    bb_setup(&A, &B, &S);
    if (S.kind == 1) {
      for (int i = 0; i < BB_NCAND && n < 8; i++) {
        double P[3], depth;
        if (bb_face_cand(&S, i, P, &depth)) { bb_face_hit(&S, P, depth, &h); hs[n++] = h; }
      }
    } else if (S.kind == 2) {
      if (bb_edge_hit(&S, &h)) hs[n++] = h;
    }
  } else {
    if (mpr(&A, &B, mpr_tol, mpr_it, &h) && h.dist < 0) hs[n++] = h;
  }
  for (int i = 0; i < n; i++) {
    out[7 * i] = hs[i].dist;
    for (int k = 0; k < 3; k++) { out[7 * i + 1 + k] = hs[i].pos[k]; out[7 * i + 4 + k] = hs[i].n[k]; }
  }
  return n;
}

/* =====================================================================
 * fp64 state hand-off with the device (GmEnvState, gripper-mujoco_amd/csrc/gm_state.h):
 * the parity tests snapshot the device state at any point of an episode and run the
 * oracle from exactly that state.  Stream ids / slots are the device's (gm_state.h).
 * ===================================================================== */
static ring_t* ring_of(or_env* e, int st) {
  if (st < 3) return &e->w_gauge[st];
  if (st < 6) return &e->w_axial[st - 3];
  switch (st) {
    case ST_PALM: return &e->w_palm;
    case ST_WX: return &e->w_wx;
    case ST_WY: return &e->w_wy;
    case ST_WZ: return &e->w_wz;
    case ST_YAW: return &e->w_yaw;
    case ST_SI_PALM: return &e->si_palm;
    case ST_SI_WZ: return &e->si_wz;
    default: break;
  }
  if (st >= ST_MOTOR && st < ST_MOTOR + 3) return &e->w_motor[st - ST_MOTOR];
  if (st >= ST_BASE && st < ST_BASE + 3) return &e->w_base[st - ST_BASE];
  if (st >= ST_CART && st < ST_CART + 12) return &e->w_cart[st - ST_CART];
  if (st >= ST_SI_GAUGE && st < ST_SI_GAUGE + 3) return &e->si_gauge[st - ST_SI_GAUGE];
  return &e->si_axial[st - ST_SI_AXIAL];
}
static void grip_in(grip_t* g, const GmGrip* s) {
  g->x = s->x; g->y = s->y; g->z = s->z; g->th = s->th; g->sx = s->sx; g->sy = s->sy; g->sz = s->sz;
}
static void grip_out(GmGrip* s, const grip_t* g) {
  s->x = g->x; s->y = g->y; s->z = g->z; s->th = g->th; s->sx = g->sx; s->sy = g->sy; s->sz = g->sz; s->pad = 0;
}
size_t or_state_size(void) { return sizeof(GmEnvState); }

int or_import_state(or_env* e, const void* state) {
  const GmEnvState* s = (const GmEnvState*)state;
  const gm_model* m = &e->m;
  if (s->extra_substeps != 0) return -1;   /* a pending termination lift: not a step boundary */
  if (s->obj_index < 0 || s->obj_index >= e->nobj) return -2;
  e->obj_index = s->obj_index;
  apply_object(&e->m, &e->objs[s->obj_index]);
  object_invweight(e);
  e->time = s->time;
  e->last_step_time = s->last_step_time;
  grip_in(&e->end, &s->end);
  grip_in(&e->next, &s->next);
  for (int k = 0; k < 6; k++) e->base[k] = s->base[k];
  for (int k = 0; k < S_N; k++) e->last_read[k] = s->last_read[k];
  for (int i = 0; i < NQ; i++) e->qpos[i] = i < m->nq ? s->qpos[i] : 0.0;
  for (int i = 0; i < NV; i++) e->qvel[i] = i < m->nv ? s->qvel[i] : 0.0;
  for (int i = 0; i < NV; i++) e->qacc_warm[i] = i < m->nv ? s->qacc_warm[i] : 0.0;
  e->obj_invw[0] = s->obj_invw[0]; e->obj_invw[1] = s->obj_invw[1];
  for (int k = 0; k < GM_MAX_LOCK; k++) { e->lock_q[k] = s->lock_q[k]; e->lock_active[k] = s->lock_active[k]; }
  for (int k = 0; k < 7; k++) e->start_qpos[k] = s->start_qpos[k];
  for (int k = 0; k < S_N; k++)
    for (int i = 0; i < 3; i++) e->rand_mu[k][i] = s->rand_mu[k][i];
  for (int st = 0; st < GM_NSTREAM; st++) {
    ring_t* r = ring_of(e, st);
    for (int k = 0; k < GM_RING; k++) r->v[k] = s->ring[st][k];
    r->i = s->ring_i[st];
  }
  for (int k = 0; k < GM_N_BINARY; k++) {
    e->bev[k].value = s->bev_value[k]; e->bev[k].last_value = s->bev_last[k];
    e->bev[k].row = s->bev_row[k]; e->bev[k].abs = s->bev_abs[k]; e->bev[k].active_sum = s->bev_row[k] != 0;
  }
  for (int k = 0; k < GM_N_LINEAR; k++) {
    e->lev[k].value = s->lev_value[k]; e->lev[k].last_value = s->lev_last[k];
    e->lev[k].row = s->lev_row[k]; e->lev[k].abs = s->lev_abs[k]; e->lev[k].active_sum = s->lev_row[k] != 0;
  }
  e->cumulative_reward = s->cumulative_reward;
  e->grp_peak_lateral = s->grp_peak_lateral;
  e->old_x = s->old_x; e->old_y = s->old_y; e->old_z = s->old_z;
  e->num_action_steps = s->num_action_steps;
  e->termination_signal_sent = s->termination_signal_sent;
  e->overflow = s->overflow;
  e->rng = s->rng;
  e->tip_force = s->tip_force;
  e->badqacc = s->badqacc;
  e->newton_caps = s->newton_caps;
  e->last_done = s->done;
  e->last_reward = s->reward;
  e->episode = s->episode;
  return 0;
}

void or_export_state(const or_env* e, void* state) {
  GmEnvState* s = (GmEnvState*)state;
  const gm_model* m = &e->m;
  memset(s, 0, sizeof(*s));
  s->time = e->time;
  s->last_step_time = e->last_step_time;
  grip_out(&s->end, &e->end);
  grip_out(&s->next, &e->next);
  for (int k = 0; k < 6; k++) s->base[k] = e->base[k];
  for (int k = 0; k < S_N; k++) s->last_read[k] = e->last_read[k];
  for (int i = 0; i < m->nq; i++) s->qpos[i] = e->qpos[i];
  for (int i = 0; i < m->nv; i++) s->qvel[i] = e->qvel[i];
  for (int i = 0; i < m->nv; i++) s->qacc_warm[i] = e->qacc_warm[i];
  s->obj_invw[0] = e->obj_invw[0]; s->obj_invw[1] = e->obj_invw[1];
  for (int k = 0; k < GM_MAX_LOCK; k++) { s->lock_q[k] = e->lock_q[k]; s->lock_active[k] = e->lock_active[k]; }
  for (int k = 0; k < 7; k++) s->start_qpos[k] = e->start_qpos[k];
  {
    const int g = m->geom_obj, b = m->body_obj;
    const gm_object* o = &e->objs[e->obj_index];
    for (int k = 0; k < 3; k++) { s->obj_size[k] = m->geom_size[g][k]; s->obj_inertia[k] = m->body_inertia[b][k]; }
    s->obj_mass = m->body_mass[b];
    s->obj_friction = m->geom_friction[g];
    s->obj_rbound = m->geom_rbound[g];
    s->obj_rest_z = object_rest_z(o);
    s->obj_type = m->geom_type[g];
  }
  s->dt = m->timestep;
  s->tip_force = e->tip_force;
  for (int k = 0; k < S_N; k++)
    for (int i = 0; i < 3; i++) s->rand_mu[k][i] = e->rand_mu[k][i];
  for (int st = 0; st < GM_NSTREAM; st++) {
    const ring_t* r = ring_of((or_env*)e, st);
    for (int k = 0; k < GM_RING; k++) s->ring[st][k] = r->v[k];
    s->ring_i[st] = r->i;
  }
  for (int k = 0; k < GM_N_BINARY; k++) {
    s->bev_value[k] = e->bev[k].value; s->bev_last[k] = e->bev[k].last_value;
    s->bev_row[k] = e->bev[k].row; s->bev_abs[k] = e->bev[k].abs;
  }
  for (int k = 0; k < GM_N_LINEAR; k++) {
    s->lev_value[k] = e->lev[k].value; s->lev_last[k] = e->lev[k].last_value;
    s->lev_row[k] = e->lev[k].row; s->lev_abs[k] = e->lev[k].abs;
  }
  s->cumulative_reward = e->cumulative_reward;
  s->grp_peak_lateral = e->grp_peak_lateral;
  s->old_x = e->old_x; s->old_y = e->old_y; s->old_z = e->old_z;
  s->num_action_steps = e->num_action_steps;
  s->termination_signal_sent = e->termination_signal_sent;
  s->obj_index = e->obj_index;
  s->overflow = e->overflow;
  s->rng = e->rng;
  s->badqacc = e->badqacc;
  s->newton_caps = e->newton_caps;
  s->done = e->last_done;
  s->reward = e->last_reward;
  s->episode = e->episode;
}

/* One env-step for n envs from device-format states (threaded, one oracle env per
 * thread): import, set_action (continuous row or discrete code), action_step,
 * get_observation, is_done, reward -- MjEnv.step's order -- then export.  states is
 * updated in place; obs [n x n_obs], reward [n], done [n] (any may be NULL). */
typedef struct {
  const or_env* proto;
  int n, tid, n_threads, n_obs, n_act;
  unsigned char* states;
  const float* cont;
  const int32_t* disc;
  float* obs; float* rew; uint8_t* done;
  int err;
} batch_job;
static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  or_env* e = (or_env*)malloc(sizeof(or_env));
  float ob[512];
  for (int k = j->tid; k < j->n; k += j->n_threads) {
    *e = *j->proto;
    GmEnvState* st = (GmEnvState*)(j->states + (size_t)k * sizeof(GmEnvState));
    if (or_import_state(e, st) != 0) { j->err = k + 1; continue; }
    if (j->cont) or_set_action(e, j->cont + (size_t)k * j->n_act);
    else if (j->disc) or_set_discrete_action(e, j->disc[k]);
    or_step(e);
    int no = or_get_obs(e, ob);
    int d = or_is_done(e);
    float r = or_reward(e);
    if (j->obs) for (int i = 0; i < no && i < j->n_obs; i++) j->obs[(size_t)k * j->n_obs + i] = ob[i];
    if (j->rew) j->rew[k] = r;
    if (j->done) j->done[k] = (uint8_t)d;
    or_export_state(e, st);
  }
  free(e);
  return NULL;
}
int or_batch_step(const gm_model* m, const gm_config* c, const gm_object* objects, int n_objects, int n,
                  void* states, const float* cont_actions, const int32_t* disc_actions, float* obs,
                  float* reward, uint8_t* done, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  or_env* proto = or_create(m, c, objects, n_objects, 0);
  if (!proto) return -1;
  batch_job jobs[256];
  pthread_t th[256];
  for (int t = 0; t < n_threads; t++) {
    jobs[t] = (batch_job){proto, n, t, n_threads, c->n_obs, c->n_actions, (unsigned char*)states,
                          cont_actions, disc_actions, obs, reward, done, 0};
    if (n_threads == 1) batch_worker(&jobs[0]);
    else pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
  }
  int err = 0;
  for (int t = 0; t < n_threads; t++) {
    if (n_threads > 1) pthread_join(th[t], NULL);
    if (jobs[t].err) err = jobs[t].err;
  }
  or_destroy(proto);
  return err ? -1000 - err : 0;
}

/* One physics substep (with update_all + monitor_sensors, like gm_debug_substep) for n
 * envs from device-format states, with the substep diagnostics; threaded as above.
 * contact [n x GM_MAX_CON x 16], efc_force [n x GM_MAX_EFC], qacc [n x GM_MAX_DOF],
 * obj_wrench [n x 6], nefc [n]. */
typedef struct {
  const or_env* proto;
  int n, tid, n_threads;
  unsigned char* states;
  int32_t* ncon; int32_t* nefc; double* contact; double* efc; double* qacc; double* wrench;
  int err;
} sub_job;
static void* sub_worker(void* arg) {
  sub_job* j = (sub_job*)arg;
  or_env* e = (or_env*)malloc(sizeof(or_env));
  for (int k = j->tid; k < j->n; k += j->n_threads) {
    *e = *j->proto;
    GmEnvState* st = (GmEnvState*)(j->states + (size_t)k * sizeof(GmEnvState));
    if (or_import_state(e, st) != 0) { j->err = k + 1; continue; }
    double qacc[NV];
    or_debug_substep(e, j->ncon ? &j->ncon[k] : NULL, j->contact ? j->contact + (size_t)k * NC * 16 : NULL,
                     j->efc ? j->efc + (size_t)k * GM_MAX_EFC : NULL, qacc, j->wrench ? j->wrench + (size_t)k * 6 : NULL);
    if (j->qacc) for (int d = 0; d < NV; d++) j->qacc[(size_t)k * NV + d] = d < e->m.nv ? qacc[d] : 0.0;
    if (j->nefc) j->nefc[k] = e->nefc;
    or_export_state(e, st);
  }
  free(e);
  return NULL;
}
int or_batch_substep(const gm_model* m, const gm_config* c, const gm_object* objects, int n_objects, int n,
                     void* states, int32_t* ncon, int32_t* nefc, double* contact, double* efc_force, double* qacc,
                     double* obj_wrench, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  or_env* proto = or_create(m, c, objects, n_objects, 0);
  if (!proto) return -1;
  sub_job jobs[256];
  pthread_t th[256];
  for (int t = 0; t < n_threads; t++) {
    jobs[t] = (sub_job){proto, n, t, n_threads, (unsigned char*)states, ncon, nefc, contact, efc_force, qacc,
                        obj_wrench, 0};
    if (n_threads == 1) sub_worker(&jobs[0]);
    else pthread_create(&th[t], NULL, sub_worker, &jobs[t]);
  }
  int err = 0;
  for (int t = 0; t < n_threads; t++) {
    if (n_threads > 1) pthread_join(th[t], NULL);
    if (jobs[t].err) err = jobs[t].err;
  }
  or_destroy(proto);
  return err ? -1000 - err : 0;
}

/* CPU throughput baseline: n_envs independent envs x n_steps env-steps, spread over
 * n_threads POSIX threads (envs share nothing, like the reference's one-env-per-process
 * model).  The workload is the benchmark's: MjEnv.reset -> _spawn_object with the same
 * counter-based object / pose draws as the device (gm_spawn_int; spawn_into_scene with
 * +-10 mm / +-pi/2, 3 tries, then the fallback pose), actions from the benchmark mix
 * (mode 1: or_driver_actions mode 4, the grasp program in 1 episode of 4 and the scripted
 * grasp mix otherwise) or uniform random (mode 0), a reset at done or at
 * max_episode_steps (MjEnv.py:616-637).  Returns env-steps per wall second. */
typedef struct {
  const or_env* proto;
  const gm_config* c;
  int n_objects, n_envs, n_steps, tid, n_threads, mode, max_steps;
  uint64_t seed;
  long done_steps, episodes;
} bench_job;

static void bench_reset(or_env* e, uint64_t seed, int64_t gid, int n_objects) {
  const int ep = e->episode + 1;
  gm_spawn sp;
  sp.object_index = gm_spawn_int(seed, gid, ep, 0, 0, n_objects - 1);
  sp.x = gm_spawn_int(seed, gid, ep, 1, -10, 10) * 1e-3;
  sp.y = gm_spawn_int(seed, gid, ep, 2, -10, 10) * 1e-3;
  const int noise = gm_spawn_int(seed, gid, ep, 3, -5, 5), opt = gm_spawn_int(seed, gid, ep, 4, 0, 2);
  sp.zrot = (60 * opt + noise) * (PI_D / 180.0);
  or_reset(e, &sp);
  gm_spawn_params sc;
  memset(&sc, 0, sizeof(sc));
  sc.index = sp.object_index;
  sc.xrange = sc.yrange = 10e-3; sc.rotrange = PI_D / 2.0;
  sc.xmin = sc.ymin = -100; sc.xmax = sc.ymax = 100;
  sc.smallest_gap = 1e-3; sc.xy_increment = 2e-3; sc.rot_increment = PI_D / 30.0;
  for (int tr = 0; tr < 3; tr++) if (or_spawn_into_scene(e, &sc)) break;
}

static void* bench_worker(void* arg) {
  bench_job* j = (bench_job*)arg;
  or_env* e = (or_env*)malloc(sizeof(or_env));
  for (int k = j->tid; k < j->n_envs; k += j->n_threads) {
    *e = *j->proto;
    e->env_id = k;
    e->rng = lcg_seed((uint64_t)j->c->s.random_seed + (uint64_t)k * 1000003ull);
    e->episode = 0;
    bench_reset(e, j->seed, k, j->n_objects);
    uint64_t x = j->seed + (uint64_t)k * 0x9E3779B97F4A7C15ull;
    for (int t = 0; t < j->n_steps; t++) {
      float a[GM_ACTION_CODE_COUNT];
      if (j->mode == 1) {
        or_driver_actions(e, 4, j->seed, 0.2f, k, a);   /* the benchmark mix (device mode 4) */
      } else {
        for (int i = 0; i < e->c.n_actions && i < GM_ACTION_CODE_COUNT; i++) {
          x = x * 6364136223846793005ull + 1442695040888963407ull;
          a[i] = (float)((double)(x >> 11) / 9007199254740992.0 * 2 - 1);
        }
      }
      or_set_action(e, a);
      or_step(e);
      float obs[256];
      or_get_obs(e, obs);
      int d = or_is_done(e);
      or_reward(e);
      j->done_steps++;
      if (d || (j->max_steps > 0 && e->num_action_steps >= j->max_steps)) {
        j->episodes++;
        bench_reset(e, j->seed, k, j->n_objects);
      }
    }
  }
  free(e);
  return NULL;
}

double or_bench(const gm_model* m, const gm_config* c, const gm_object* objects, int n_objects,
                int n_envs, int n_steps, uint64_t seed, int n_threads, int mode, int max_episode_steps) {
  if (n_threads < 1) n_threads = 1;
  if (n_threads > 256) n_threads = 256;
  or_env* proto = or_create(m, c, objects, n_objects, 0);
  if (!proto) return -1;
  bench_job jobs[256];
  pthread_t th[256];
  struct timespec t0, t1;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int t = 0; t < n_threads; t++) {
    jobs[t] = (bench_job){proto, c, n_objects, n_envs, n_steps, t, n_threads, mode, max_episode_steps, seed, 0, 0};
    if (n_threads == 1) bench_worker(&jobs[0]);
    else pthread_create(&th[t], NULL, bench_worker, &jobs[t]);
  }
  long done_steps = 0;
  for (int t = 0; t < n_threads; t++) {
    if (n_threads > 1) pthread_join(th[t], NULL);
    done_steps += jobs[t].done_steps;
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  or_destroy(proto);
  double dt = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
  return dt > 0 ? done_steps / dt : 0;
}
