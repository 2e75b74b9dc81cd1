/* physics.c -- the engine's physics substep, fp64, restated for the CPU oracle.
 *
 * TEST INFRASTRUCTURE ONLY (included by oracle.c; see oracle.h).  This is the engine
 * specification of DESIGN.md section 2 -- MuJoCo 2.1.5's mj_step1 / mj_step2 pipeline
 * restated (kinematics, composite rigid bodies, RNE bias, the Euler step with implicit
 * damping, collision, soft constraints, MuJoCo's Newton solver) -- written so that
 * every floating-point operation happens in the same order as in the device kernels
 * (gripper-mujoco_amd/csrc/gm_kernels.hip): where the device composes a finger chain by a
 * Hillis-Steele scan across a 16-lane DPP row, or sums a wave by an xor butterfly, this
 * file emulates that scan / butterfly lane by lane, so one substep from the same state
 * gives the same bits on both sides.  The algorithms are the reference's (MuJoCo's)
 * mathematics; only the association order is the device's.  The dense PGS of
 * ref_pgs_solve is kept as an independent cross-check of the Newton solution (the
 * regularised dual has a unique optimum).
 */

/* ---------------------------------------------------------------- topology
 * The canonical gripper tree as the device lays it out (gm_capi.hip build_topo): finger f
 * chain position p (1..CL) on scan lane 16 f + p, base on lane 48, palm 49, object 50. */
static int topo_init(or_env* e) {   /* 0, or -1: a contact pair the solver cannot take */
  const gm_model* m = &e->m;
  otopo* T = &e->T;
  memset(T, 0, sizeof(*T));
  T->CL = m->n_seg + 2;
  for (int f = 0; f < 3; f++) { T->dof_f0[f] = m->dof_pris[f]; T->body_f0[f] = m->dof_body[m->dof_pris[f]]; }
  for (int b = 0; b < NB; b++) { T->body_grp[b] = -1; T->body_cpos[b] = 0; }
  for (int b = 0; b < m->nbody; b++) {
    T->body_grp[b] = m->body_group[b];
    if (m->body_group[b] >= 0 && m->body_group[b] < 3) T->body_cpos[b] = b - T->body_f0[m->body_group[b]] + 1;
    else if (m->body_group[b] == GM_GRP_PALM) T->body_cpos[b] = 1;
  }
  for (int l = 0; l < 64; l++) T->lane_body[l] = -1;
  for (int f = 0; f < 3; f++)
    for (int p = 1; p <= T->CL; p++) T->lane_body[16 * f + p] = T->body_f0[f] + p - 1;
  T->lane_body[48] = m->body_base;
  T->lane_body[49] = m->body_palm;
  T->lane_body[50] = m->body_obj;
  for (int l = 0; l < 64; l++) {
    const int b = T->lane_body[l];
    T->kl_type[l] = -1; T->kl_qadr[l] = 0;
    T->kl_grp[l] = b >= 0 ? T->body_grp[b] : -1;
    const int chain = T->kl_grp[l] >= 0 && T->kl_grp[l] <= 3;
    T->kl_cpos[l] = chain ? T->body_cpos[b] : 0;
    for (int k = 0; k < 3; k++) { T->kl_pos[l][k] = 0; T->kl_axis[l][k] = 0; }
    T->kl_quat[l][0] = 1; T->kl_quat[l][1] = T->kl_quat[l][2] = T->kl_quat[l][3] = 0;
    if (b > 0) {
      for (int k = 0; k < 3; k++) T->kl_pos[l][k] = m->body_pos[b][k];
      for (int k = 0; k < 4; k++) T->kl_quat[l][k] = m->body_quat[b][k];
      const int j = m->body_jnt[b];
      if (j >= 0) {
        T->kl_type[l] = m->jnt_type[j];
        T->kl_qadr[l] = m->jnt_qposadr[j];
        for (int k = 0; k < 3; k++) T->kl_axis[l][k] = m->jnt_axis[j][k];
      }
    }
  }
  for (int d = 0; d < m->nv; d++) {
    const int b = m->dof_body[d], j = m->body_jnt[b];
    double kp = 0, kd = 0;
    int tgt = 0;
    for (int f = 0; f < 3; f++) {
      if (d == m->dof_pris[f]) { kp = m->kp_gripper[0]; kd = m->kd_gripper[0]; tgt = 1; }
      if (d == m->dof_rev[f]) { kp = m->kp_gripper[1]; kd = m->kd_gripper[1]; tgt = 2; }
    }
    if (d == m->dof_palm) { kp = m->kp_gripper[2]; kd = m->kd_gripper[2]; tgt = 3; }
    if (d == m->dof_base) { kp = m->kp_base[2]; kd = m->kd_base[2]; tgt = 4; }
    const int fr = m->jnt_type[j] == GM_JNT_FREE;
    T->dof_grp[d] = m->body_group[b];
    T->dof_p[d] = (m->body_group[b] == GM_GRP_OBJECT) ? d - m->dof_obj : T->body_cpos[b];
    T->dof_arm[d] = m->jnt_armature[j];
    /* MuJoCo's actuator order (mujoco_actuators): the solve's matrix is M + armature */
    T->dof_dsum[d] = m->mujoco_actuators ? 0.0 : m->jnt_damping[j] + kd;
    T->dof_ksum[d] = (fr || m->mujoco_actuators) ? 0.0 : kp;
    T->dof_stiff[d] = fr ? 0.0 : m->jnt_stiffness[j];
    T->dof_damp[d] = m->jnt_damping[j];
    T->dof_kp[d] = kp; T->dof_kd[d] = kd; T->dof_target[d] = tgt;
  }
  for (int g = 0; g < m->ngeom; g++) {
    const int b = m->geom_body[g];
    T->geom_grp[g] = (b == 0) ? -1 : T->body_grp[b];
    if (T->geom_grp[g] == GM_GRP_BASE) T->geom_grp[g] = -1;
  }
  /* per scan lane: the pairs of the lane's body's geoms with the object / the ground */
  for (int l = 0; l < 64; l++)
    for (int s = 0; s < 2; s++) { T->lane_opair[l][s] = -1; T->lane_gpair[l][s] = -1; }
  for (int pr = 0; pr < m->npair; pr++) {
    const int a = m->pair_a[pr], bgeom = m->pair_b[pr];
    const int with_obj = (a == m->geom_obj || bgeom == m->geom_obj);
    const int with_gnd = (a == m->geom_ground || bgeom == m->geom_ground);
    int g = -1;
    if (with_obj && !with_gnd) g = (a == m->geom_obj) ? bgeom : a;
    else if (with_gnd && !with_obj) g = (a == m->geom_ground) ? bgeom : a;
    if (g < 0) continue;
    const int b = m->geom_body[g];
    int assigned = 0;
    for (int l = 0; l < 64; l++) {
      if (T->lane_body[l] != b || l == 50) continue;
      int* slot = with_obj ? T->lane_opair[l] : T->lane_gpair[l];
      if (slot[0] < 0) slot[0] = pr; else slot[1] = pr;
      assigned = 1;
    }
    /* gm_capi.hip build_topo rejects the same: the Hessian composites reach a contact only
     * through its gripper body's scan lane */
    if (!assigned) return -1;
  }
  return 0;
}

/* ---------------------------------------------------------------- small helpers */
#define TRI(p, q) ((p) * ((p) + 1) / 2 + (q))
static void quatnorm_d(double* q) {   /* device quatnorm: multiply by the reciprocal */
  double n = sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  if (n < 1e-15) { q[0] = 1; q[1] = q[2] = q[3] = 0; return; }
  const double in = 1.0 / n;
  for (int i = 0; i < 4; i++) q[i] *= in;
}
/* DPP row shift inside a 16-lane row; bound_ctrl: 0 shifted in at the row edge */
static double rshr(const double* row16, int pos, int off) { return pos - off >= 0 ? row16[pos - off] : 0.0; }
static double rshl(const double* row16, int pos, int off) { return pos + off <= 15 ? row16[pos + off] : 0.0; }
/* xor butterfly over 64 lanes (every lane ends with the same sum) */
static double butterfly64(const double* v_in) {
  double v[64], w[64];
  memcpy(v, v_in, sizeof(v));
  for (int s = 32; s >= 1; s >>= 1) {
    for (int i = 0; i < 64; i++) w[i] = v[i] + v[i ^ s];
    memcpy(v, w, sizeof(v));
  }
  return v[0];
}

/* =====================================================================
 * kinematics (mj_kinematics + mj_comPos restated; the device's gm_kernels.hip kinematics)
 * ===================================================================== */
static void fk(or_env* e) {
  const gm_model* m = &e->m;
  const otopo* T = &e->T;
  const int CL = T->CL;
  double lp[64][3], lq[64][4];
  /* A: local transform of every scan lane's body */
  for (int l = 0; l < 64; l++) {
    for (int k = 0; k < 3; k++) lp[l][k] = T->kl_pos[l][k];
    for (int k = 0; k < 4; k++) lq[l][k] = T->kl_quat[l][k];
    const int type = T->kl_type[l];
    if (type >= 0) {
      const double qv = e->qpos[T->kl_qadr[l]];
      const double* ax = T->kl_axis[l];
      if (type == GM_JNT_SLIDE) {
        double R[9], wa[3];
        quat2mat(R, lq[l]);
        mulmv3(wa, R, ax);
        lp[l][0] += wa[0] * qv; lp[l][1] += wa[1] * qv; lp[l][2] += wa[2] * qv;
      } else if (type == GM_JNT_HINGE) {
        double sn, cs;
        gm_sincos(0.5 * qv, &sn, &cs);
        const double ql[4] = {cs, ax[0] * sn, ax[1] * sn, ax[2] * sn};
        quatmul(lq[l], lq[l], ql);
      }
    }
  }
  /* B: segmented Hillis-Steele scan per 16-lane row, root-side operand on the left */
  double bpos[3], bq[4], bR[9];
  for (int k = 0; k < 3; k++) bpos[k] = lp[48][k];
  for (int k = 0; k < 4; k++) bq[k] = lq[48][k];
  quatnorm_d(bq);
  quat2mat(bR, bq);
  for (int off = 1; off < CL; off <<= 1) {
    double op[64][3], oq[64][4];
    memcpy(op, lp, sizeof(op));
    memcpy(oq, lq, sizeof(oq));
    for (int l = 0; l < 64; l++) {
      const int pos = l & 15, row = l & ~15;
      double np[3], nq[4];
      for (int k = 0; k < 3; k++) np[k] = pos - off >= 0 ? op[row + pos - off][k] : 0.0;
      for (int k = 0; k < 4; k++) nq[k] = pos - off >= 0 ? oq[row + pos - off][k] : 0.0;
      if (T->kl_cpos[l] > off) {
        double R[9], t[3], q[4];
        quat2mat(R, nq);
        mulmv3(t, R, op[l]);
        quatmul(q, nq, oq[l]);
        lp[l][0] = np[0] + t[0]; lp[l][1] = np[1] + t[1]; lp[l][2] = np[2] + t[2];
        for (int k = 0; k < 4; k++) lq[l][k] = q[k];
      }
    }
  }
  for (int l = 0; l < 64; l++) {
    const int b = T->lane_body[l];
    const int grp = T->kl_grp[l];
    if (grp >= 0 && grp <= 3) {
      double t[3], q[4];
      mulmv3(t, bR, lp[l]);
      quatmul(q, bq, lq[l]);
      quatnorm_d(q);
      e->xpos[b][0] = bpos[0] + t[0]; e->xpos[b][1] = bpos[1] + t[1]; e->xpos[b][2] = bpos[2] + t[2];
      for (int k = 0; k < 4; k++) e->xquat[b][k] = q[k];
    } else if (b == m->body_base) {
      for (int k = 0; k < 3; k++) e->xpos[b][k] = bpos[k];
      for (int k = 0; k < 4; k++) e->xquat[b][k] = bq[k];
    } else if (b == m->body_obj) {
      const int qa = m->dof_obj;
      double q[4] = {e->qpos[qa + 3], e->qpos[qa + 4], e->qpos[qa + 5], e->qpos[qa + 6]};
      quatnorm_d(q);
      e->xpos[b][0] = e->qpos[qa]; e->xpos[b][1] = e->qpos[qa + 1]; e->xpos[b][2] = e->qpos[qa + 2];
      for (int k = 0; k < 4; k++) e->xquat[b][k] = q[k];
    }
  }
  for (int k = 0; k < 3; k++) e->xpos[0][k] = 0;
  e->xquat[0][0] = 1; e->xquat[0][1] = e->xquat[0][2] = e->xquat[0][3] = 0;
  for (int b = 0; b < m->nbody; b++) quat2mat(e->xmat[b], e->xquat[b]);
  /* C1: spatial inertia about the world origin, one lane per body */
  for (int b = 1; b < m->nbody; b++) {
    const double* R = e->xmat[b];
    double c[3];
    mulmv3(c, R, m->body_ipos[b]);
    c[0] += e->xpos[b][0]; c[1] += e->xpos[b][1]; c[2] += e->xpos[b][2];
    double I[3] = {m->body_inertia[b][0], m->body_inertia[b][1], m->body_inertia[b][2]};
    double mass = m->body_mass[b];
    double Iw[9];
    for (int i = 0; i < 3; i++)
      for (int k = 0; k < 3; k++)
        Iw[3 * i + k] = R[3 * i] * I[0] * R[3 * k] + R[3 * i + 1] * I[1] * R[3 * k + 1] + R[3 * i + 2] * I[2] * R[3 * k + 2];
    const double cc = dot3(c, c);
    double* ci = e->cinert[b];
    ci[0] = Iw[0] + mass * (cc - c[0] * c[0]);
    ci[1] = Iw[4] + mass * (cc - c[1] * c[1]);
    ci[2] = Iw[8] + mass * (cc - c[2] * c[2]);
    ci[3] = Iw[1] - mass * c[0] * c[1];
    ci[4] = Iw[2] - mass * c[0] * c[2];
    ci[5] = Iw[5] - mass * c[1] * c[2];
    ci[6] = mass * c[0]; ci[7] = mass * c[1]; ci[8] = mass * c[2];
    ci[9] = mass;
  }
  /* C2: motion subspaces, one lane per dof */
  for (int d = 0; d < m->nv; d++) {
    const int b = m->dof_body[d], j = m->body_jnt[b];
    double* cd = e->cdof[d];
    const double* xp = e->xpos[b];
    if (m->jnt_type[j] == GM_JNT_FREE) {
      const int k = d - m->jnt_dofadr[j];
      if (k < 3) {
        cd[0] = cd[1] = cd[2] = 0; cd[3] = cd[4] = cd[5] = 0; cd[3 + k] = 1;
      } else {
        const double* Rb = e->xmat[b];
        const double w[3] = {Rb[k - 3], Rb[3 + k - 3], Rb[6 + k - 3]};
        cd[0] = w[0]; cd[1] = w[1]; cd[2] = w[2];
        cross3(cd + 3, xp, w);
      }
    } else {
      double wa[3];
      mulmv3(wa, e->xmat[b], m->jnt_axis[j]);
      if (m->jnt_type[j] == GM_JNT_SLIDE) {
        cd[0] = cd[1] = cd[2] = 0; cd[3] = wa[0]; cd[4] = wa[1]; cd[5] = wa[2];
      } else {
        cd[0] = wa[0]; cd[1] = wa[1]; cd[2] = wa[2];
        cross3(cd + 3, xp, wa);
      }
    }
  }
}

/* spatial algebra (Plucker [angular; linear] about the world origin) */
static void inert_mul(double* r, const double* ci, const double* v) {
  const double* w = v; const double* u = v + 3;
  double Iw0 = ci[0] * w[0] + ci[3] * w[1] + ci[4] * w[2];
  double Iw1 = ci[3] * w[0] + ci[1] * w[1] + ci[5] * w[2];
  double Iw2 = ci[4] * w[0] + ci[5] * w[1] + ci[2] * w[2];
  double hxu[3], hxw[3];
  cross3(hxu, ci + 6, u);
  cross3(hxw, ci + 6, w);
  r[0] = Iw0 + hxu[0]; r[1] = Iw1 + hxu[1]; r[2] = Iw2 + hxu[2];
  r[3] = ci[9] * u[0] - hxw[0]; r[4] = ci[9] * u[1] - hxw[1]; r[5] = ci[9] * u[2] - hxw[2];
}
static void cross_motion(double* r, const double* v, const double* mv) {
  double a[3], b[3], c[3];
  cross3(a, v, mv); cross3(b, v, mv + 3); cross3(c, v + 3, mv);
  r[0] = a[0]; r[1] = a[1]; r[2] = a[2];
  r[3] = b[0] + c[0]; r[4] = b[1] + c[1]; r[5] = b[2] + c[2];
}
static void cross_force(double* r, const double* v, const double* f) {
  double a[3], b[3], c[3];
  cross3(a, v, f); cross3(b, v + 3, f + 3); cross3(c, v, f + 3);
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
  r[3] = c[0]; r[4] = c[1]; r[5] = c[2];
}
static double dot6(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3] + a[4] * b[4] + a[5] * b[5];
}
static void body_force(const double* ci, const double* cvel, const double* cacc, double* out) {
  double t1[6], t2[6], f[6];
  inert_mul(f, ci, cacc);
  inert_mul(t1, ci, cvel);
  cross_force(t2, cvel, t1);
  for (int k = 0; k < 6; k++) out[k] = f[k] + t2[k];
}

/* =====================================================================
 * mj_crb + mj_rne bias (the device's crb_rne: segmented prefix / suffix scans)
 * ===================================================================== */
static void crb_rne(or_env* e) {
  const gm_model* m = &e->m;
  const otopo* T = &e->T;
  const int CL = T->CL;
  const int db = m->dof_base;
  const double qdb = e->qvel[db];
  double cvb[6], cab[6];
  for (int k = 0; k < 6; k++) { cvb[k] = e->cdof[db][k] * qdb; cab[k] = 0; }
  cab[3] = -m->gravity[0]; cab[4] = -m->gravity[1]; cab[5] = -m->gravity[2];
  double cd[64][6], qd[64], v[64][6];
  for (int l = 0; l < 64; l++) {
    const int grp = T->kl_grp[l];
    const int chain = grp >= 0 && grp <= 3;
    const int p = T->kl_cpos[l];
    const int d = chain ? (grp < 3 ? T->dof_f0[grp] + p - 1 : m->dof_palm) : db;
    qd[l] = chain ? e->qvel[d] : 0.0;
    for (int k = 0; k < 6; k++) { cd[l][k] = chain ? e->cdof[d][k] : 0.0; v[l][k] = cd[l][k] * qd[l]; }
  }
  /* velocities: inclusive prefix, then the base */
  double cv[64][6], cvp[64][6];
  memcpy(cv, v, sizeof(cv));
  for (int off = 1; off < CL; off <<= 1) {
    double o[64][6];
    memcpy(o, cv, sizeof(o));
    for (int l = 0; l < 64; l++) {
      const int pos = l & 15, row = l & ~15;
      for (int k = 0; k < 6; k++) cv[l][k] = o[l][k] + (pos - off >= 0 ? o[row + pos - off][k] : 0.0);
    }
  }
  for (int l = 0; l < 64; l++) {
    const int pos = l & 15, row = l & ~15;
    const int p = T->kl_cpos[l];
    for (int k = 0; k < 6; k++) {
      const double nb = pos - 1 >= 0 ? cv[row + pos - 1][k] : 0.0;
      cvp[l][k] = cvb[k] + (p > 1 ? nb : 0.0);
    }
  }
  for (int l = 0; l < 64; l++) for (int k = 0; k < 6; k++) cv[l][k] += cvb[k];
  /* bias accelerations: prefix of (cvel_parent x cdof) qd, then gravity */
  double ca[64][6];
  for (int l = 0; l < 64; l++) {
    cross_motion(ca[l], cvp[l], cd[l]);
    for (int k = 0; k < 6; k++) ca[l][k] *= qd[l];
  }
  for (int off = 1; off < CL; off <<= 1) {
    double o[64][6];
    memcpy(o, ca, sizeof(o));
    for (int l = 0; l < 64; l++) {
      const int pos = l & 15, row = l & ~15;
      for (int k = 0; k < 6; k++) ca[l][k] = o[l][k] + (pos - off >= 0 ? o[row + pos - off][k] : 0.0);
    }
  }
  for (int l = 0; l < 64; l++) for (int k = 0; k < 6; k++) ca[l][k] += cab[k];
  /* body forces and composite inertias: suffix sums */
  double f[64][6], ci[64][10];
  for (int l = 0; l < 64; l++) {
    const int grp = T->kl_grp[l];
    const int chain = grp >= 0 && grp <= 3;
    const int b = T->lane_body[l];
    for (int k = 0; k < 10; k++) ci[l][k] = chain ? e->cinert[b][k] : 0.0;
    double t1[6], t2[6];
    inert_mul(f[l], ci[l], ca[l]);
    inert_mul(t1, ci[l], cv[l]);
    cross_force(t2, cv[l], t1);
    for (int k = 0; k < 6; k++) f[l][k] += t2[k];
  }
  for (int off = 1; off < CL; off <<= 1) {
    double of[64][6], oi[64][10];
    memcpy(of, f, sizeof(of));
    memcpy(oi, ci, sizeof(oi));
    for (int l = 0; l < 64; l++) {
      const int pos = l & 15, row = l & ~15;
      for (int k = 0; k < 6; k++) f[l][k] = of[l][k] + (pos + off <= 15 ? of[row + pos + off][k] : 0.0);
      for (int k = 0; k < 10; k++) ci[l][k] = oi[l][k] + (pos + off <= 15 ? oi[row + pos + off][k] : 0.0);
    }
  }
  double chain_f[4][6], chain_I[4][10];
  for (int l = 0; l < 64; l++) {
    const int grp = T->kl_grp[l];
    if (!(grp >= 0 && grp <= 3)) continue;
    const int b = T->lane_body[l];
    for (int k = 0; k < 6; k++) e->cfrc[b][k] = f[l][k];
    for (int k = 0; k < 10; k++) e->Ic[b][k] = ci[l][k];
    if (T->kl_cpos[l] == 1) {
      for (int k = 0; k < 6; k++) chain_f[grp][k] = f[l][k];
      for (int k = 0; k < 10; k++) chain_I[grp][k] = ci[l][k];
    }
  }
  /* the object: free joint on one body */
  {
    const int b = m->body_obj, d0 = m->dof_obj;
    double cvel[6], cacc[6];
    for (int k = 0; k < 6; k++) { cvel[k] = 0; cacc[k] = 0; }
    cacc[3] = -m->gravity[0]; cacc[4] = -m->gravity[1]; cacc[5] = -m->gravity[2];
    for (int k = 0; k < 3; k++) {
      const double qv = e->qvel[d0 + k];
      for (int t = 0; t < 6; t++) cvel[t] += e->cdof[d0 + k][t] * qv;
    }
    double cdd[3][6];
    for (int k = 0; k < 3; k++) cross_motion(cdd[k], cvel, e->cdof[d0 + 3 + k]);
    for (int k = 0; k < 3; k++) {
      const double qv = e->qvel[d0 + 3 + k];
      for (int t = 0; t < 6; t++) cvel[t] += e->cdof[d0 + 3 + k][t] * qv;
    }
    for (int k = 0; k < 3; k++) {
      const double qv = e->qvel[d0 + 3 + k];
      for (int t = 0; t < 6; t++) cacc[t] += cdd[k][t] * qv;
    }
    body_force(e->cinert[b], cvel, cacc, e->cfrc[b]);
    for (int k = 0; k < 10; k++) e->Ic[b][k] = e->cinert[b][k];
  }
  /* the base: its own force / inertia plus the four chain roots */
  {
    const int bb = m->body_base;
    body_force(e->cinert[bb], cvb, cab, e->cfrc[bb]);
    double ic[10], fb[6];
    for (int k = 0; k < 10; k++) ic[k] = e->cinert[bb][k];
    for (int k = 0; k < 6; k++) fb[k] = e->cfrc[bb][k];
    for (int c = 0; c < 4; c++) {
      for (int k = 0; k < 10; k++) ic[k] += chain_I[c][k];
      for (int k = 0; k < 6; k++) fb[k] += chain_f[c][k];
    }
    for (int k = 0; k < 10; k++) e->Ic[bb][k] = ic[k];
    for (int k = 0; k < 6; k++) e->cfrc[bb][k] = fb[k];
  }
}

/* =====================================================================
 * smooth dynamics: H~ = M + armature + h (D + Kd) + h^2 Kp on the tree blocks (TRI
 * storage: finger f rows p = 0 (base) .. CL, palm 0..1, object 0..5) and the smooth
 * force frc = passive + PD actuation - bias (the device's mass_and_forces)
 * ===================================================================== */
static void mass_and_forces(or_env* e) {
  const gm_model* m = &e->m;
  const otopo* T = &e->T;
  const double h = m->timestep;
  for (int d = 0; d < m->nv; d++) {
    const int b = m->dof_body[d];
    const int c = T->dof_grp[d];
    const int p = T->dof_p[d];
    double add = T->dof_arm[d] + h * T->dof_dsum[d];
    add += h * h * T->dof_ksum[d];
    const double* cd = e->cdof[d];
    double F[6];
    inert_mul(F, e->Ic[b], cd);
    if (c == GM_GRP_BASE) {
      e->Hbb = dot6(cd, F) + add;
    } else {
      const int objd = c == GM_GRP_OBJECT;
      const int d0 = objd ? m->dof_obj : (c < 3) ? T->dof_f0[c] : m->dof_palm;
      double* Hrow = objd ? &e->Ho[TRI(p, 0)] : (c < 3) ? &e->Hf[c][TRI(p, 0)] : &e->Hp[TRI(p, 0)];
      for (int q = 0; q <= p; q++) {
        const int dq = objd ? d0 + q : (q == 0) ? m->dof_base : d0 + q - 1;
        double v = dot6(e->cdof[dq], F);
        if (q == p) v += add;
        Hrow[q] = v;
      }
    }
    const double bias = dot6(cd, e->cfrc[b]);
    const double qp = e->qpos[d], qv = e->qvel[d];
    double pas = 0;
    pas -= T->dof_stiff[d] * qp;
    pas -= T->dof_damp[d] * qv;
    const int tgt = T->dof_target[d];
    double act = 0;
    if (tgt != 0) {
      const double target = tgt == 1 ? e->next.x : tgt == 2 ? e->next.th : tgt == 3 ? e->next.z : e->base[2];
      act = -((qp - target) * T->dof_kp[d] + qv * T->dof_kd[d]);
    }
    double frc = pas + act - bias;
    if (e->tip_force != 0.0 && (c < 3 || c == GM_GRP_BASE)) {
      /* calibration tip load (resolve_segment_forces -> apply_segment_force,
       * myfunctions.cpp:1642-1727): each finger's tip link pulled at its centre of mass
       * along the finger's rest bending direction; J^T F for the dofs above that link */
      for (int f = 0; f < 3; f++) {
        if (c < 3 && f != c) continue;
        const int bt = m->body_tip[f];
        double pc[3], wxp[3];
        mulmv3(pc, e->xmat[bt], m->body_ipos[bt]);
        pc[0] += e->xpos[bt][0]; pc[1] += e->xpos[bt][1]; pc[2] += e->xpos[bt][2];
        const double Fv[3] = {e->tip_force * m->tip_dir[f][0], e->tip_force * m->tip_dir[f][1],
                              e->tip_force * m->tip_dir[f][2]};
        cross3(wxp, cd, pc);
        const double col[3] = {cd[3] + wxp[0], cd[4] + wxp[1], cd[5] + wxp[2]};
        frc += dot3(col, Fv);
      }
    }
    e->frc[d] = frc;
  }
}

/* =====================================================================
 * collision (mj_collision restated; the device's lane-per-candidate-pair collision):
 * geom poses from the body poses, bounding-sphere broadphase, narrowphase per type pair,
 * contacts in candidate-pair order (generation order inside a pair)
 * ===================================================================== */
typedef struct { int type; double size[3], c[3], R[9], rbound, friction; } geomv_t;
typedef struct { double dist, pos[3], n[3]; } hit_t;

static void geom_pose(const or_env* e, int b, const double* gpos, const double* gquat, double* c, double* Rw) {
  double R[9];
  if (b == 0) { R[0] = 1; R[1] = 0; R[2] = 0; R[3] = 0; R[4] = 1; R[5] = 0; R[6] = 0; R[7] = 0; R[8] = 1; }
  else quat2mat(R, e->xquat[b]);
  double t[3], Rg[9];
  mulmv3(t, R, gpos);
  const double bp0 = b == 0 ? 0.0 : e->xpos[b][0], bp1 = b == 0 ? 0.0 : e->xpos[b][1], bp2 = b == 0 ? 0.0 : e->xpos[b][2];
  c[0] = bp0 + t[0]; c[1] = bp1 + t[1]; c[2] = bp2 + t[2];
  quat2mat(Rg, gquat);
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) Rw[3 * i + k] = R[3 * i] * Rg[k] + R[3 * i + 1] * Rg[3 + k] + R[3 * i + 2] * Rg[6 + k];
}
static void load_geom(const or_env* e, int g, geomv_t* G) {
  const gm_model* m = &e->m;
  G->type = m->geom_type[g];
  for (int k = 0; k < 3; k++) G->size[k] = m->geom_size[g][k];
  G->rbound = m->geom_rbound[g];
  G->friction = m->geom_friction[g];
  geom_pose(e, m->geom_body[g], m->geom_pos[g], m->geom_quat[g], G->c, G->R);
}

static int plane_box_point(const geomv_t* P, const geomv_t* B, int i, hit_t* h) {
  const double nz[3] = {P->R[2], P->R[5], P->R[8]};
  const double s[3] = {(i & 1) ? B->size[0] : -B->size[0], (i & 2) ? B->size[1] : -B->size[1],
                       (i & 4) ? B->size[2] : -B->size[2]};
  double v[3];
  mulmv3(v, B->R, s);
  v[0] += B->c[0]; v[1] += B->c[1]; v[2] += B->c[2];
  const double dv[3] = {v[0] - P->c[0], v[1] - P->c[1], v[2] - P->c[2]};
  const double d = dot3(dv, nz);
  if (!(d < 0)) return 0;
  h->dist = d;
  for (int k = 0; k < 3; k++) { h->pos[k] = v[k] - 0.5 * d * nz[k]; h->n[k] = nz[k]; }
  return 1;
}
typedef struct { double nz[3], a[3], w[3], axw[3]; } cylframe_t;
static void cyl_frame(const geomv_t* P, const geomv_t* Cy, cylframe_t* F) {
  F->nz[0] = P->R[2]; F->nz[1] = P->R[5]; F->nz[2] = P->R[8];
  F->a[0] = Cy->R[2]; F->a[1] = Cy->R[5]; F->a[2] = Cy->R[8];
  const double na = dot3(F->nz, F->a);
  double w[3] = {-F->nz[0] + na * F->a[0], -F->nz[1] + na * F->a[1], -F->nz[2] + na * F->a[2]};
  const double lw = sqrt(dot3(w, w));
  if (lw < 1e-6) { w[0] = Cy->R[0]; w[1] = Cy->R[3]; w[2] = Cy->R[6]; }
  else { w[0] = w[0] / lw; w[1] = w[1] / lw; w[2] = w[2] / lw; }
  F->w[0] = w[0]; F->w[1] = w[1]; F->w[2] = w[2];
  cross3(F->axw, F->a, F->w);
}
static int plane_cyl_point(const geomv_t* P, const geomv_t* Cy, const cylframe_t* F, int i, hit_t* h) {
  const double* nz = F->nz;
  const double* a = F->a;
  const double r = Cy->size[0], hh = Cy->size[1];
  const int s = i >> 2, k = i & 3;
  const double sg = s == 0 ? 1.0 : -1.0;
  double dir[3];
  if (k == 0) { dir[0] = F->w[0]; dir[1] = F->w[1]; dir[2] = F->w[2]; }
  else if (k == 1) { dir[0] = F->axw[0]; dir[1] = F->axw[1]; dir[2] = F->axw[2]; }
  else if (k == 2) { dir[0] = -F->w[0]; dir[1] = -F->w[1]; dir[2] = -F->w[2]; }
  else { dir[0] = -F->axw[0]; dir[1] = -F->axw[1]; dir[2] = -F->axw[2]; }
  double v[3];
  for (int t = 0; t < 3; t++) v[t] = Cy->c[t] + sg * hh * a[t] + r * dir[t];
  const double dv[3] = {v[0] - P->c[0], v[1] - P->c[1], v[2] - P->c[2]};
  const double d = dot3(dv, nz);
  if (!(d < 0)) return 0;
  h->dist = d;
  for (int t = 0; t < 3; t++) { h->pos[t] = v[t] - 0.5 * d * nz[t]; h->n[t] = nz[t]; }
  return 1;
}
static int plane_sphere(const geomv_t* P, const geomv_t* Sp, hit_t* h) {
  const double nz[3] = {P->R[2], P->R[5], P->R[8]};
  const double r = Sp->size[0];
  const double dv[3] = {Sp->c[0] - P->c[0], Sp->c[1] - P->c[1], Sp->c[2] - P->c[2]};
  const double dist = dot3(dv, nz) - r;
  if (!(dist < 0)) return 0;
  h->dist = dist;
  for (int k = 0; k < 3; k++) { h->pos[k] = Sp->c[k] - nz[k] * (r + 0.5 * dist); h->n[k] = nz[k]; }
  return 1;
}
static int sphere_box(const geomv_t* Sp, const geomv_t* B, hit_t* h) {
  const double* R = B->R;
  const double* hs = B->size;
  const double r = Sp->size[0];
  const double dv[3] = {Sp->c[0] - B->c[0], Sp->c[1] - B->c[1], Sp->c[2] - B->c[2]};
  double cl[3];
  mulmtv3(cl, R, dv);
  double q[3];
  int inside = 1;
  for (int k = 0; k < 3; k++) {
    q[k] = cl[k];
    if (q[k] > hs[k]) { q[k] = hs[k]; inside = 0; }
    if (q[k] < -hs[k]) { q[k] = -hs[k]; inside = 0; }
  }
  double nl[3], dist, ql[3];
  if (!inside) {
    const double df[3] = {cl[0] - q[0], cl[1] - q[1], cl[2] - q[2]};
    const double l = sqrt(dot3(df, df));
    if (l < 1e-12) return 0;
    dist = l - r;
    if (!(dist < 0)) return 0;
    nl[0] = -df[0] / l; nl[1] = -df[1] / l; nl[2] = -df[2] / l;
    ql[0] = q[0]; ql[1] = q[1]; ql[2] = q[2];
  } else {
    int kmin = 0;
    double best = hs[0] - fabs(cl[0]);
    for (int k = 1; k < 3; k++) { const double v = hs[k] - fabs(cl[k]); if (v < best) { best = v; kmin = k; } }
    const double clk = cl[kmin], hsk = hs[kmin];
    const double sg = clk >= 0 ? 1.0 : -1.0;
    dist = -(best + r);
    for (int k = 0; k < 3; k++) {
      nl[k] = (k == kmin) ? -sg : 0.0;
      ql[k] = (k == kmin) ? sg * hsk : cl[k];
    }
  }
  double n[3], qw[3];
  mulmv3(n, R, nl);
  mulmv3(qw, R, ql);
  h->dist = dist;
  for (int k = 0; k < 3; k++) {
    qw[k] += B->c[k];
    const double sp = Sp->c[k] + n[k] * r;
    h->pos[k] = 0.5 * (qw[k] + sp);
    h->n[k] = n[k];
  }
  return 1;
}

/* ---- MPR (Minkowski portal refinement, libccd's algorithm as MuJoCo's mjc_Convex
 *      uses it for box-cylinder / cylinder-cylinder) ---- */
typedef struct { double v[3], p1[3], p2[3]; } sv_t;
static void support_geom(const geomv_t* G, const double* d, double* out) {
  double dl[3];
  mulmtv3(dl, G->R, d);
  double pl[3] = {0, 0, 0};
  /* a direction (numerically) perpendicular to a face or to the cylinder axis has the whole
   * face / rim line as its support set: the face centre is taken (GM_SUPPORT_TIE) */
  if (G->type == GM_GEOM_BOX) {
    for (int k = 0; k < 3; k++) pl[k] = fabs(dl[k]) < GM_SUPPORT_TIE ? 0.0 : (dl[k] >= 0 ? G->size[k] : -G->size[k]);
  } else if (G->type == GM_GEOM_CYLINDER) {
    const double rr = sqrt(dl[0] * dl[0] + dl[1] * dl[1]);
    if (rr > 1e-12) { pl[0] = G->size[0] * dl[0] / rr; pl[1] = G->size[0] * dl[1] / rr; }
    pl[2] = fabs(dl[2]) < GM_SUPPORT_TIE ? 0.0 : (dl[2] >= 0 ? G->size[1] : -G->size[1]);
  } else if (G->type == GM_GEOM_SPHERE) {
    const double l = sqrt(dot3(dl, dl));
    if (l > 1e-12) { pl[0] = dl[0] * G->size[0] / l; pl[1] = dl[1] * G->size[0] / l; pl[2] = dl[2] * G->size[0] / l; }
  }
  mulmv3(out, G->R, pl);
  out[0] += G->c[0]; out[1] += G->c[1]; out[2] += G->c[2];
}
static void mpr_support(const geomv_t* A, const geomv_t* B, const double* d, sv_t* sv) {
  const double nd[3] = {-d[0], -d[1], -d[2]};
  support_geom(A, d, sv->p1);
  support_geom(B, nd, sv->p2);
  sv->v[0] = sv->p1[0] - sv->p2[0]; sv->v[1] = sv->p1[1] - sv->p2[1]; sv->v[2] = sv->p1[2] - sv->p2[2];
}
static int fzero(double x) { return fabs(x) < 1e-12; }
static void normalize3(double* d) {
  const double l = sqrt(dot3(d, d));
  if (l > 0) { const double il = 1.0 / l; d[0] *= il; d[1] *= il; d[2] *= il; }
}
static void portal_dir(const sv_t* P1, const sv_t* P2, const sv_t* P3, double* dir) {
  const double a[3] = {P2->v[0] - P1->v[0], P2->v[1] - P1->v[1], P2->v[2] - P1->v[2]};
  const double b[3] = {P3->v[0] - P1->v[0], P3->v[1] - P1->v[1], P3->v[2] - P1->v[2]};
  cross3(dir, a, b);
  normalize3(dir);
}
static void expand_portal(const sv_t* P0, sv_t* P1, sv_t* P2, sv_t* P3, const sv_t* v4) {
  double v4v0[3];
  cross3(v4v0, v4->v, P0->v);
  const int s1 = dot3(P1->v, v4v0) > 0;
  const int s2 = dot3(P2->v, v4v0) > 0;
  const int s3 = dot3(P3->v, v4v0) > 0;
  const int t1 = s1 ? s2 : !s3, t2 = !s1 && s3, t3 = s1 && !s2;
  if (t1) *P1 = *v4;
  if (t2) *P2 = *v4;
  if (t3) *P3 = *v4;
}
static int reach_tol(const sv_t* P1, const sv_t* P2, const sv_t* P3, const sv_t* v4, const double* dir, double tol) {
  const double dv1 = dot3(P1->v, dir), dv2 = dot3(P2->v, dir), dv3 = dot3(P3->v, dir), dv4 = dot3(v4->v, dir);
  const double d1 = dv4 - dv1, d2 = dv4 - dv2, d3 = dv4 - dv3;
  const double dd = fmin(fmin(d1, d2), d3);
  return dd < tol || fabs(dd - tol) < 1e-12;
}
static void tri_closest_origin(const double* a, const double* b, const double* c, double* out) {
  const double ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  const double ac[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  const double ap[3] = {-a[0], -a[1], -a[2]};
  const double d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0 && d2 <= 0) { copy3(out, a); return; }
  const double bp[3] = {-b[0], -b[1], -b[2]};
  const double d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0 && d4 <= d3) { copy3(out, b); return; }
  const double vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) { const double v = d1 / (d1 - d3); for (int k = 0; k < 3; k++) out[k] = a[k] + v * ab[k]; return; }
  const double cp[3] = {-c[0], -c[1], -c[2]};
  const double d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0 && d5 <= d6) { copy3(out, c); return; }
  const double vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) { const double w = d2 / (d2 - d6); for (int k = 0; k < 3; k++) out[k] = a[k] + w * ac[k]; return; }
  const double va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    const double w = (d4 - d3) / ((d4 - d3) + (d5 - d6));
    for (int k = 0; k < 3; k++) out[k] = b[k] + w * (c[k] - b[k]);
    return;
  }
  const double den = 1.0 / (va + vb + vc);
  const double v = vb * den, w = vc * den;
  for (int k = 0; k < 3; k++) out[k] = a[k] + ab[k] * v + ac[k] * w;
}
static void mpr_pos(const sv_t* P0, const sv_t* P1, const sv_t* P2, const sv_t* P3, double* pos) {
  double dir[3];
  portal_dir(P1, P2, P3, dir);
  double t[3];
  cross3(t, P1->v, P2->v); double b0 = dot3(t, P3->v);
  cross3(t, P3->v, P2->v); double b1 = dot3(t, P0->v);
  cross3(t, P0->v, P1->v); double b2 = dot3(t, P3->v);
  cross3(t, P2->v, P1->v); double b3 = dot3(t, P0->v);
  double sum = b0 + b1 + b2 + b3;
  if (sum <= 0) {
    b0 = 0;
    cross3(t, P2->v, P3->v); b1 = dot3(t, dir);
    cross3(t, P3->v, P1->v); b2 = dot3(t, dir);
    cross3(t, P1->v, P2->v); b3 = dot3(t, dir);
    sum = b1 + b2 + b3;
  }
  const double inv = 1.0 / sum;
  double p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
  for (int k = 0; k < 3; k++) {
    p1[k] += b0 * P0->p1[k]; p2[k] += b0 * P0->p2[k];
    p1[k] += b1 * P1->p1[k]; p2[k] += b1 * P1->p2[k];
    p1[k] += b2 * P2->p1[k]; p2[k] += b2 * P2->p2[k];
    p1[k] += b3 * P3->p1[k]; p2[k] += b3 * P3->p2[k];
  }
  for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p1[k] + p2[k]) * inv;
}
static int mpr(const geomv_t* A, const geomv_t* B, double tol, int maxit, hit_t* h) {
  sv_t P0, P1, P2, P3;
  for (int k = 0; k < 3; k++) { P0.v[k] = A->c[k] - B->c[k]; P0.p1[k] = A->c[k]; P0.p2[k] = B->c[k]; }
  if (fzero(P0.v[0]) && fzero(P0.v[1]) && fzero(P0.v[2])) P0.v[0] += 1e-5;
  double d[3] = {-P0.v[0], -P0.v[1], -P0.v[2]};
  normalize3(d);
  mpr_support(A, B, d, &P1);
  if (dot3(P1.v, d) <= 0) return 0;
  cross3(d, P0.v, P1.v);
  if (fzero(sqrt(dot3(d, d)))) {
    const double l1 = sqrt(dot3(P1.v, P1.v));
    if (fzero(l1)) return 0;
    h->dist = -l1;
    const double il = 1.0 / l1;
    for (int k = 0; k < 3; k++) { h->n[k] = P1.v[k] * il; h->pos[k] = 0.5 * (P1.p1[k] + P1.p2[k]); }
    return 1;
  }
  normalize3(d);
  mpr_support(A, B, d, &P2);
  if (dot3(P2.v, d) <= 0) return 0;
  double va[3], vb[3];
  for (int k = 0; k < 3; k++) { va[k] = P1.v[k] - P0.v[k]; vb[k] = P2.v[k] - P0.v[k]; }
  cross3(d, va, vb);
  normalize3(d);
  if (dot3(d, P0.v) > 0) {
    const sv_t t = P1;
    P1 = P2; P2 = t;
    d[0] = -d[0]; d[1] = -d[1]; d[2] = -d[2];
  }
  int it = 0;
  for (;;) {
    mpr_support(A, B, d, &P3);
    if (dot3(P3.v, d) <= 0) return 0;
    cross3(va, P1.v, P3.v);
    const int c2 = dot3(va, P0.v) < -1e-12;
    cross3(va, P3.v, P2.v);
    const int c1 = !c2 && dot3(va, P0.v) < -1e-12;
    if (c2) P2 = P3;
    if (c1) P1 = P3;
    if (!(c1 || c2)) break;
    for (int k = 0; k < 3; k++) { va[k] = P1.v[k] - P0.v[k]; vb[k] = P2.v[k] - P0.v[k]; }
    cross3(d, va, vb);
    normalize3(d);
    if (++it > maxit) return 0;
  }
  it = 0;
  for (;;) {
    portal_dir(&P1, &P2, &P3, d);
    if (dot3(d, P1.v) >= -1e-12) break;
    sv_t v4;
    mpr_support(A, B, d, &v4);
    const double dv4 = dot3(v4.v, d);
    if (!(fzero(dv4) || dv4 > 0)) return 0;
    if (reach_tol(&P1, &P2, &P3, &v4, d, tol)) return 0;
    expand_portal(&P0, &P1, &P2, &P3, &v4);
    if (++it > maxit) return 0;
  }
  it = 0;
  for (;;) {
    portal_dir(&P1, &P2, &P3, d);
    sv_t v4;
    mpr_support(A, B, d, &v4);
    if (reach_tol(&P1, &P2, &P3, &v4, d, tol) || it > maxit) {
      double cp[3];
      tri_closest_origin(P1.v, P2.v, P3.v, cp);
      const double depth = sqrt(dot3(cp, cp));
      if (fzero(depth)) return 0;
      h->dist = -depth;
      const double id = 1.0 / depth;
      h->n[0] = cp[0] * id; h->n[1] = cp[1] * id; h->n[2] = cp[2] * id;
      mpr_pos(&P0, &P1, &P2, &P3, h->pos);
      return depth > 0;
    }
    expand_portal(&P0, &P1, &P2, &P3, &v4);
    it++;
  }
}

/* ---- box-box: MuJoCo's dedicated multi-contact collider (mjc_BoxBox) restated as a
 * separating-axis test over the 15 axes plus a face-clipped contact manifold:
 *  - separated on any axis -> no contact;
 *  - the axis of least penetration picks the case; a face axis wins ties, and an
 *    edge-edge axis is used only when it is clearly (5 %) shallower than the best face;
 *  - face case: the reference face is the axis owner's face towards the other box, the
 *    incident face the other box's face most anti-parallel to it; the manifold is the
 *    vertex set of the two faces' overlap polygon (incident vertices inside the
 *    reference rectangle, reference corners inside the incident quad, edge-edge
 *    crossings), each kept when it lies below the reference face; contact position half
 *    way between the two surfaces (up to 8 points, candidate order);
 *  - edge case: one contact at the midpoint of the two edges' closest points.
 * The normal points from geom1 to geom2. ---- */
#define BB_NCAND 24
typedef struct {
  int kind;                /* 0 none, 1 face, 2 edge */
  double n[3];             /* reference outward normal (face) / axis A -> B (edge) */
  double pen;
  double sgn;              /* +1: the reference box is geom1, -1: geom2 (face case) */
  double crf[3], ru[3], rv[3], hu, hv;      /* reference face centre, in-plane axes, half sizes */
  double V[4][3];                           /* incident face vertices (cyclic) */
  double cinc[3], ninc[3];                  /* incident face centre / outward normal */
  double pu[4], pv[4];                      /* incident vertices in reference face coordinates */
  double ea[3], eb[3], da[3], db[3];        /* edge case: edge centres / directions */
} bbox_t;

static void bb_setup(const geomv_t* A, const geomv_t* B, bbox_t* S) {
  S->kind = 0;
  const double d[3] = {B->c[0] - A->c[0], B->c[1] - A->c[1], B->c[2] - A->c[2]};
  double a[3][3], b[3][3];
  for (int i = 0; i < 3; i++)
    for (int k = 0; k < 3; k++) { a[i][k] = A->R[3 * k + i]; b[i][k] = B->R[3 * k + i]; }   /* box axes = R columns */
  double Cm[3][3], Ca[3][3];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) { Cm[i][j] = dot3(a[i], b[j]); Ca[i][j] = fabs(Cm[i][j]); }
  double best = 0;
  int code = -1;
  /* face axes of A, then of B */
  for (int i = 0; i < 3; i++) {
    const double rb = B->size[0] * Ca[i][0] + B->size[1] * Ca[i][1] + B->size[2] * Ca[i][2];
    const double pen = (A->size[i] + rb) - fabs(dot3(d, a[i]));
    if (pen < 0) return;
    if (code < 0 || pen < best) { best = pen; code = i; }
  }
  for (int j = 0; j < 3; j++) {
    const double ra = A->size[0] * Ca[0][j] + A->size[1] * Ca[1][j] + A->size[2] * Ca[2][j];
    const double pen = (ra + B->size[j]) - fabs(dot3(d, b[j]));
    if (pen < 0) return;
    if (pen < best) { best = pen; code = 3 + j; }
  }
  /* edge-edge axes a_i x b_j */
  double ebest = 0, eL[3] = {0, 0, 0};
  int ecode = -1;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double L[3];
      cross3(L, a[i], b[j]);
      const double len = sqrt(dot3(L, L));
      if (len < 1e-6) continue;
      const double il = 1.0 / len;
      L[0] *= il; L[1] *= il; L[2] *= il;
      const double ra = A->size[0] * fabs(dot3(a[0], L)) + A->size[1] * fabs(dot3(a[1], L)) + A->size[2] * fabs(dot3(a[2], L));
      const double rb = B->size[0] * fabs(dot3(b[0], L)) + B->size[1] * fabs(dot3(b[1], L)) + B->size[2] * fabs(dot3(b[2], L));
      const double pen = (ra + rb) - fabs(dot3(d, L));
      if (pen < 0) return;
      if (ecode < 0 || pen < ebest) { ebest = pen; ecode = 3 * i + j; eL[0] = L[0]; eL[1] = L[1]; eL[2] = L[2]; }
    }
  if (ecode >= 0 && ebest < 0.95 * best) {
    /* edge-edge: supporting edges of A towards +L and of B towards -L */
    const int i = ecode / 3, j = ecode % 3;
    double L[3] = {eL[0], eL[1], eL[2]};
    if (dot3(d, L) < 0) { L[0] = -L[0]; L[1] = -L[1]; L[2] = -L[2]; }
    S->kind = 2;
    S->pen = ebest;
    copy3(S->n, L);
    for (int k = 0; k < 3; k++) { S->ea[k] = A->c[k]; S->eb[k] = B->c[k]; S->da[k] = a[i][k]; S->db[k] = b[j][k]; }
    for (int k = 0; k < 3; k++) {
      if (k != i) {
        const double s = dot3(a[k], L) >= 0 ? A->size[k] : -A->size[k];
        for (int t = 0; t < 3; t++) S->ea[t] += s * a[k][t];
      }
      if (k != j) {
        const double s = dot3(b[k], L) >= 0 ? -B->size[k] : B->size[k];
        for (int t = 0; t < 3; t++) S->eb[t] += s * b[k][t];
      }
    }
    return;
  }
  /* face case */
  const int ref_is_a = code < 3;
  const geomv_t* Rf = ref_is_a ? A : B;
  const geomv_t* In = ref_is_a ? B : A;
  const int ri = ref_is_a ? code : code - 3;
  const double (*ra)[3] = ref_is_a ? a : b;
  const double (*ia)[3] = ref_is_a ? b : a;
  const double dd[3] = {In->c[0] - Rf->c[0], In->c[1] - Rf->c[1], In->c[2] - Rf->c[2]};
  const double s0 = dot3(dd, ra[ri]) >= 0 ? 1.0 : -1.0;
  S->kind = 1;
  S->pen = best;
  S->sgn = ref_is_a ? 1.0 : -1.0;
  for (int k = 0; k < 3; k++) S->n[k] = s0 * ra[ri][k];
  const int ui = (ri + 1) % 3, vi = (ri + 2) % 3;
  for (int k = 0; k < 3; k++) {
    S->crf[k] = Rf->c[k] + Rf->size[ri] * S->n[k];
    S->ru[k] = ra[ui][k]; S->rv[k] = ra[vi][k];
  }
  S->hu = Rf->size[ui]; S->hv = Rf->size[vi];
  /* incident face: the other box's face most anti-parallel to n */
  int jm = 0;
  double bm = fabs(dot3(S->n, ia[0]));
  for (int j = 1; j < 3; j++) { const double v = fabs(dot3(S->n, ia[j])); if (v > bm) { bm = v; jm = j; } }
  const double sj = dot3(S->n, ia[jm]) >= 0 ? -1.0 : 1.0;   /* outward normal of the incident face: sj * ia[jm] */
  for (int k = 0; k < 3; k++) { S->ninc[k] = sj * ia[jm][k]; S->cinc[k] = In->c[k] + In->size[jm] * S->ninc[k]; }
  const int e1 = (jm + 1) % 3, e2 = (jm + 2) % 3;
  const double h1 = In->size[e1], h2 = In->size[e2];
  const double su[4] = {-1, 1, 1, -1}, sv[4] = {-1, -1, 1, 1};
  for (int q = 0; q < 4; q++) {
    for (int k = 0; k < 3; k++) S->V[q][k] = S->cinc[k] + (su[q] * h1) * ia[e1][k] + (sv[q] * h2) * ia[e2][k];
    const double r[3] = {S->V[q][0] - S->crf[0], S->V[q][1] - S->crf[1], S->V[q][2] - S->crf[2]};
    S->pu[q] = dot3(r, S->ru);
    S->pv[q] = dot3(r, S->rv);
  }
}
/* face case candidate i (0-3 incident vertices, 4-7 reference corners, 8-23 crossings of
 * incident edge (i-8)/4 with reference edge (i-8)%4); returns 1 with the point on the
 * incident face and its depth below the reference face when it is a manifold vertex */
static int bb_face_cand(const bbox_t* S, int i, double* P, double* depth) {
  if (i < 4) {
    if (!(fabs(S->pu[i]) <= S->hu && fabs(S->pv[i]) <= S->hv)) return 0;
    copy3(P, S->V[i]);
  } else if (i < 8) {
    const int m = i - 4;
    const double cu = (m == 1 || m == 2) ? S->hu : -S->hu, cv = (m >= 2) ? S->hv : -S->hv;
    /* inside the incident quad (cyclic vertices, either orientation, boundary included) */
    double sgn_min = 0, sgn_max = 0;
    for (int q = 0; q < 4; q++) {
      const int q1 = (q + 1) & 3;
      const double ex = S->pu[q1] - S->pu[q], ey = S->pv[q1] - S->pv[q];
      const double cr = ex * (cv - S->pv[q]) - ey * (cu - S->pu[q]);
      if (q == 0) { sgn_min = cr; sgn_max = cr; }
      else { sgn_min = fmin(sgn_min, cr); sgn_max = fmax(sgn_max, cr); }
    }
    if (!(sgn_min >= 0 || sgn_max <= 0)) return 0;
    double Q[3];
    for (int k = 0; k < 3; k++) Q[k] = S->crf[k] + cu * S->ru[k] + cv * S->rv[k];
    const double den = dot3(S->ninc, S->n);
    if (fabs(den) < 1e-12) return 0;
    const double r[3] = {S->cinc[0] - Q[0], S->cinc[1] - Q[1], S->cinc[2] - Q[2]};
    const double t = dot3(S->ninc, r) / den;
    for (int k = 0; k < 3; k++) P[k] = Q[k] + t * S->n[k];
  } else {
    const int q = (i - 8) >> 2, m = (i - 8) & 3;
    const int q1 = (q + 1) & 3;
    const double du = S->pu[q1] - S->pu[q], dv = S->pv[q1] - S->pv[q];
    double t;
    if (m < 2) {                     /* reference edges u = -hu, +hu */
      if (fabs(du) < 1e-15) return 0;
      const double bound = m == 0 ? -S->hu : S->hu;
      t = (bound - S->pu[q]) / du;
      if (!(t > 0 && t < 1)) return 0;
      const double vt = S->pv[q] + t * dv;
      if (!(fabs(vt) < S->hv)) return 0;
    } else {                         /* reference edges v = -hv, +hv */
      if (fabs(dv) < 1e-15) return 0;
      const double bound = m == 2 ? -S->hv : S->hv;
      t = (bound - S->pv[q]) / dv;
      if (!(t > 0 && t < 1)) return 0;
      const double ut = S->pu[q] + t * du;
      if (!(fabs(ut) < S->hu)) return 0;
    }
    for (int k = 0; k < 3; k++) P[k] = S->V[q][k] + t * (S->V[q1][k] - S->V[q][k]);
  }
  const double r[3] = {S->crf[0] - P[0], S->crf[1] - P[1], S->crf[2] - P[2]};
  *depth = dot3(S->n, r);
  return *depth > 0;
}
static void bb_face_hit(const bbox_t* S, const double* P, double depth, hit_t* h) {
  h->dist = -depth;
  for (int k = 0; k < 3; k++) { h->pos[k] = P[k] + (0.5 * depth) * S->n[k]; h->n[k] = S->sgn * S->n[k]; }
}
static int bb_edge_hit(const bbox_t* S, hit_t* h) {
  /* closest points of the lines ea + s da and eb + t db */
  const double w[3] = {S->ea[0] - S->eb[0], S->ea[1] - S->eb[1], S->ea[2] - S->eb[2]};
  const double b = dot3(S->da, S->db), dd = dot3(S->da, w), e = dot3(S->db, w);
  const double den = 1.0 - b * b;
  if (!(den > 1e-12)) return 0;
  const double s = (b * e - dd) / den, t = (e - b * dd) / den;
  h->dist = -S->pen;
  for (int k = 0; k < 3; k++) {
    const double pa = S->ea[k] + s * S->da[k], pb = S->eb[k] + t * S->db[k];
    h->pos[k] = 0.5 * (pa + pb);
    h->n[k] = S->n[k];
  }
  return 1;
}

static int add_contact(or_env* e, int g1, int g2, const hit_t* h, double mu) {
  if (e->ncon >= NC) { e->overflow = 1; e->ncon_total++; return 0; }
  con_t* c = &e->con[e->ncon++];
  e->ncon_total++;
  c->dist = h->dist;
  copy3(c->pos, h->pos);
  copy3(c->frame, h->n);
  c->mu = mu;
  c->g1 = g1; c->g2 = g2;
  return 1;
}

static void collision(or_env* e) {
  const gm_model* m = &e->m;
  e->ncon = 0;
  e->ncon_total = 0;
  e->overflow = 0;
  for (int pr = 0; pr < m->npair; pr++) {
    const int a = m->pair_a[pr], b = m->pair_b[pr];
    const int ta = m->geom_type[a], tb = m->geom_type[b];
    int g1 = a, g2 = b;
    if (ta > tb || (ta == tb && a > b)) { g1 = b; g2 = a; }
    e->pair_off[pr] = e->ncon_total;
    e->pair_cnt[pr] = 0;
    geomv_t A, B;
    load_geom(e, g1, &A);
    load_geom(e, g2, &B);
    int pass;
    if (A.type == GM_GEOM_PLANE) {
      const double nz[3] = {A.R[2], A.R[5], A.R[8]};
      const double dv[3] = {B.c[0] - A.c[0], B.c[1] - A.c[1], B.c[2] - A.c[2]};
      pass = !(dot3(dv, nz) > B.rbound);
    } else {
      const double dv[3] = {B.c[0] - A.c[0], B.c[1] - A.c[1], B.c[2] - A.c[2]};
      const double rr = A.rbound + B.rbound;
      pass = !(dot3(dv, dv) > rr * rr);
    }
    if (!pass) continue;
    const double mu = fmax(A.friction, B.friction);
    hit_t h;
    int n0 = e->ncon_total;
    if (A.type == GM_GEOM_PLANE) {
      if (B.type == GM_GEOM_SPHERE) { if (plane_sphere(&A, &B, &h)) add_contact(e, g1, g2, &h, mu); }
      else if (B.type == GM_GEOM_BOX) {
        int cnt = 0;
        for (int i = 0; i < 8 && cnt < 4; i++) if (plane_box_point(&A, &B, i, &h)) { add_contact(e, g1, g2, &h, mu); cnt++; }
      } else if (B.type == GM_GEOM_CYLINDER) {
        cylframe_t cf;
        cyl_frame(&A, &B, &cf);
        int cnt = 0;
        for (int i = 0; i < 8 && cnt < 4; i++) if (plane_cyl_point(&A, &B, &cf, i, &h)) { add_contact(e, g1, g2, &h, mu); cnt++; }
      }
    } else if (A.type == GM_GEOM_SPHERE && B.type == GM_GEOM_BOX) {
      if (sphere_box(&A, &B, &h)) add_contact(e, g1, g2, &h, mu);
    } else if (A.type == GM_GEOM_BOX && B.type == GM_GEOM_BOX) {
      bbox_t S;
      bb_setup(&A, &B, &S);
      if (S.kind == 1) {
        int cnt = 0;
        for (int i = 0; i < BB_NCAND && cnt < 8; i++) {
          double P[3], depth;
          if (bb_face_cand(&S, i, P, &depth)) { bb_face_hit(&S, P, depth, &h); add_contact(e, g1, g2, &h, mu); cnt++; }
        }
      } else if (S.kind == 2) {
        if (bb_edge_hit(&S, &h)) add_contact(e, g1, g2, &h, mu);
      }
    } else {
      if (mpr(&A, &B, m->mpr_tolerance, m->mpr_iterations, &h) && h.dist < 0) add_contact(e, g1, g2, &h, mu);
    }
    e->pair_cnt[pr] = e->ncon_total - n0;
  }
  if (e->ncon_total > NC) e->overflow = 1;
  /* contact frames (mju_makeFrame-style tangents from the normal) */
  for (int c = 0; c < e->ncon; c++) {
    double n[3] = {e->con[c].frame[0], e->con[c].frame[1], e->con[c].frame[2]};
    make_frame(e->con[c].frame, n);
  }
}

/* =====================================================================
 * constraints: MuJoCo's soft constraints (mj_makeConstraint / mj_makeImpedance) with the
 * regulariser from MuJoCo's diagonal approximation (mj_diagApprox: body / dof invweight0
 * at qpos0; pyramid edge = tran + mu^2 tran), solved by MuJoCo's Newton method
 * (mj_solNewton: primal, qacc space, exact line search) -- the unique optimum of the
 * regularised problem, the same one PGS iterates towards (ref_pgs_solve).
 * Rows: active motor locks (1-dof joint equalities, in lock order), then 4 pyramid edges
 * per contact (n + mu t1, n - mu t1, n + mu t2, n - mu t2).
 * ===================================================================== */
static double impedance(const gm_model* m, double r) {
  const double dmin = m->solimp[0], dmax = m->solimp[1], width = m->solimp[2], mid = m->solimp[3], pw = m->solimp[4];
  if (dmin == dmax || width <= 1e-15) return dmin;
  const double x = fabs(r) / width;
  if (x >= 1) return dmax;
  if (x <= 0) return dmin;
  double y;
  if (pw == 1) y = x;
  else if (pw == 2) y = (x <= mid) ? x * x / mid : 1 - (1 - x) * (1 - x) / (1 - mid);
  else if (x <= mid) y = pow(x, pw) / pow(mid, pw - 1);
  else y = 1 - pow(1 - x, pw) / pow(1 - mid, pw - 1);
  return dmin + y * (dmax - dmin);
}
static double body_invw(const or_env* e, int b) {
  return b == e->m.body_obj ? e->obj_invw[0] : e->m.body_invweight0[b][0];
}
/* spatial velocity [angular; linear at the world origin] of every body for the dof
 * vector v (the device's body_vel: chain prefix scans + the base; the object's free joint) */
static void body_vel(or_env* e, const double* v, double V[NB][6]) {
  const gm_model* m = &e->m;
  const otopo* T = &e->T;
  const int CL = T->CL, db = m->dof_base;
  const double vb = v[db];
  double cvb[6];
  for (int k = 0; k < 6; k++) cvb[k] = e->cdof[db][k] * vb;
  double s[64][6];
  for (int l = 0; l < 64; l++) {
    const int grp = T->kl_grp[l];
    const int chain = grp >= 0 && grp <= 3;
    const int p = T->kl_cpos[l];
    const int d = chain ? (grp < 3 ? T->dof_f0[grp] + p - 1 : m->dof_palm) : db;
    const double vd = chain ? v[d] : 0.0;
    for (int k = 0; k < 6; k++) s[l][k] = (chain ? e->cdof[d][k] : 0.0) * vd;
  }
  for (int off = 1; off < CL; off <<= 1) {
    double o[64][6];
    memcpy(o, s, sizeof(o));
    for (int l = 0; l < 64; l++) {
      const int pos = l & 15, row = l & ~15;
      for (int k = 0; k < 6; k++) s[l][k] = o[l][k] + (pos - off >= 0 ? o[row + pos - off][k] : 0.0);
    }
  }
  for (int b = 0; b < NB; b++) for (int k = 0; k < 6; k++) V[b][k] = 0.0;
  for (int l = 0; l < 64; l++) {
    const int grp = T->kl_grp[l];
    if (!(grp >= 0 && grp <= 3)) continue;
    const int b = T->lane_body[l];
    for (int k = 0; k < 6; k++) V[b][k] = s[l][k] + cvb[k];
  }
  for (int k = 0; k < 6; k++) V[m->body_base][k] = cvb[k];
  {
    const int b = m->body_obj, d0 = m->dof_obj;
    double acc[6] = {0, 0, 0, 0, 0, 0};
    for (int k = 0; k < 6; k++)
      for (int t = 0; t < 6; t++) acc[t] += e->cdof[d0 + k][t] * v[d0 + k];
    for (int t = 0; t < 6; t++) V[b][t] = acc[t];
  }
}
/* velocity of body b's point p (zero for the world) */
static void point_vel(const double V[NB][6], int b, const double* p, double* out) {
  double t[3];
  cross3(t, V[b], p);
  out[0] = V[b][3] + t[0]; out[1] = V[b][4] + t[1]; out[2] = V[b][5] + t[2];
}
/* J v for the 4 pyramid edges of contact c */
static void contact_jv(const or_env* e, int c, const double V[NB][6], double* jv) {
  const con_t* C = &e->con[c];
  const int b1 = e->m.geom_body[C->g1], b2 = e->m.geom_body[C->g2];
  double v1[3], v2[3];
  point_vel(V, b1, C->pos, v1);
  point_vel(V, b2, C->pos, v2);
  const double dv[3] = {v2[0] - v1[0], v2[1] - v1[1], v2[2] - v1[2]};
  const double cn = dot3(C->frame, dv), c1 = dot3(C->frame + 3, dv), c2 = dot3(C->frame + 6, dv);
  const double m1 = C->mu * c1, m2 = C->mu * c2;
  jv[0] = cn + m1; jv[1] = cn - m1; jv[2] = cn + m2; jv[3] = cn - m2;
}
static void edge_dir(const con_t* C, int ed, double* u) {
  const double* t = C->frame + 3 * (1 + (ed >> 1));
  const double mt[3] = {C->mu * t[0], C->mu * t[1], C->mu * t[2]};
  if (ed & 1) { u[0] = C->frame[0] - mt[0]; u[1] = C->frame[1] - mt[1]; u[2] = C->frame[2] - mt[2]; }
  else { u[0] = C->frame[0] + mt[0]; u[1] = C->frame[1] + mt[1]; u[2] = C->frame[2] + mt[2]; }
}
/* K = S Q S^T with S = [skew(p); I]: 21 entries [A xx yy zz xy xz yz | B row-major | Q xx yy zz xy xz yz] */
static void spatial_K(const double* Q, const double* p, double* K) {
  const double Qm[3][3] = {{Q[0], Q[3], Q[4]}, {Q[3], Q[1], Q[5]}, {Q[4], Q[5], Q[2]}};
  double Bm[3][3];
  for (int j = 0; j < 3; j++) {
    double c[3];
    cross3(c, p, Qm[j]);   /* column j of Q (symmetric: row j) */
    Bm[0][j] = c[0]; Bm[1][j] = c[1]; Bm[2][j] = c[2];
  }
  double Am[3][3];
  for (int i = 0; i < 3; i++) cross3(Am[i], p, Bm[i]);
  K[0] = Am[0][0]; K[1] = Am[1][1]; K[2] = Am[2][2]; K[3] = Am[0][1]; K[4] = Am[0][2]; K[5] = Am[1][2];
  for (int i = 0; i < 3; i++) for (int j = 0; j < 3; j++) K[6 + 3 * i + j] = Bm[i][j];
  for (int k = 0; k < 6; k++) K[15 + k] = Q[k];
}
/* K v for a spatial motion v = [w; l] */
static void symK_mul(const double* K, const double* v, double* y) {
  const double *A = K, *B = K + 6, *Q = K + 15;
  const double w0 = v[0], w1 = v[1], w2 = v[2], l0 = v[3], l1 = v[4], l2 = v[5];
  y[0] = A[0] * w0 + A[3] * w1 + A[4] * w2 + B[0] * l0 + B[1] * l1 + B[2] * l2;
  y[1] = A[3] * w0 + A[1] * w1 + A[5] * w2 + B[3] * l0 + B[4] * l1 + B[5] * l2;
  y[2] = A[4] * w0 + A[5] * w1 + A[2] * w2 + B[6] * l0 + B[7] * l1 + B[8] * l2;
  y[3] = B[0] * w0 + B[3] * w1 + B[6] * w2 + Q[0] * l0 + Q[3] * l1 + Q[4] * l2;
  y[4] = B[1] * w0 + B[4] * w1 + B[7] * w2 + Q[3] * l0 + Q[1] * l1 + Q[5] * l2;
  y[5] = B[2] * w0 + B[5] * w1 + B[8] * w2 + Q[4] * l0 + Q[5] * l1 + Q[2] * l2;
}

/* H~ v on the tree blocks (the device's smooth_matvec) */
static void smooth_matvec(const or_env* e, const double* v, double* out) {
  const gm_model* m = &e->m;
  const otopo* T = &e->T;
  const int CL = T->CL;
  for (int f = 0; f < 3; f++)
    for (int p = 1; p <= CL; p++) {
      const double* H = e->Hf[f];
      double acc = H[TRI(p, 0)] * v[m->dof_base];
      for (int j = 1; j <= CL; j++) {
        const double hv = (j <= p) ? H[TRI(p, j)] : H[TRI(j, p)];
        acc = acc + hv * v[T->dof_f0[f] + j - 1];
      }
      out[T->dof_f0[f] + p - 1] = acc;
    }
  {
    double acc = e->Hbb * v[m->dof_base];
    for (int f = 0; f < 3; f++)
      for (int p = 1; p <= CL; p++) acc = acc + e->Hf[f][TRI(p, 0)] * v[T->dof_f0[f] + p - 1];
    acc = acc + e->Hp[TRI(1, 0)] * v[m->dof_palm];
    out[m->dof_base] = acc;
  }
  out[m->dof_palm] = e->Hp[TRI(1, 0)] * v[m->dof_base] + e->Hp[TRI(1, 1)] * v[m->dof_palm];
  for (int k = 0; k < 6; k++) {
    double acc = 0;
    for (int l = 0; l < 6; l++) {
      const double hv = (l <= k) ? e->Ho[TRI(k, l)] : e->Ho[TRI(l, k)];
      acc = acc + hv * v[m->dof_obj + l];
    }
    out[m->dof_obj + k] = acc;
  }
}

/* --- the Newton system: H = H~ + J_a^T D_a J_a, rhs = frc + J_a^T (D_a aref_a), factored
 * as the device does (finger chain blocks on DPP rows with the border [base, object 0..5]
 * carried as extra columns, leaf-first LDL^T, Schur complements into the border, border
 * LDL^T, palm as a one-dof chain) --- */
typedef struct {
  double h[3][16][GM_CHAIN + 1];   /* finger f, chain position p (1..CL): lower row + multiplier slots */
  double hb[3][16][7];             /* border columns [base, obj0..5] */
  double ub[3][16][7];             /* unscaled border row at elimination (Schur) */
  double invd[3][16];
  double ph, phb[7], pub[7], pinvd;   /* palm */
  double bb[7][7], binvd[7];          /* border lower rows + multiplier slots */
  double rhs_f[3][16], rhs_p, rhs_b[7];
} nsys_t;

static void newton_assemble(or_env* e, const int* act, nsys_t* S) {
  const gm_model* m = &e->m;
  const otopo* T = &e->T;
  const int CL = T->CL;
  /* per-contact K_c and spatial force Fs_c from the active edges */
  static __thread double Kc[NC][21], Fs[NC][6];
  for (int c = 0; c < e->ncon; c++) {
    const con_t* C = &e->con[c];
    double Q[6] = {0, 0, 0, 0, 0, 0}, F[3] = {0, 0, 0};
    for (int ed = 0; ed < 4; ed++) {
      double u[3];
      edge_dir(C, ed, u);
      const double w = act[e->nl + 4 * c + ed] ? e->efc_D[e->nl + 4 * c + ed] : 0.0;
      const double du[3] = {w * u[0], w * u[1], w * u[2]};
      Q[0] += du[0] * u[0]; Q[1] += du[1] * u[1]; Q[2] += du[2] * u[2];
      Q[3] += du[0] * u[1]; Q[4] += du[0] * u[2]; Q[5] += du[1] * u[2];
      const double g = w * e->efc_aref[e->nl + 4 * c + ed];
      F[0] += g * u[0]; F[1] += g * u[1]; F[2] += g * u[2];
    }
    spatial_K(Q, C->pos, Kc[c]);
    cross3(Fs[c], C->pos, F);
    Fs[c][3] = F[0]; Fs[c][4] = F[1]; Fs[c][5] = F[2];
  }
  /* per scan lane: sums over the lane's body's contacts with the object (o) / ground (g) */
  double Ko[64][21], Kg[64][21], Fo[64][6], Fg[64][6];
  int any_g = 0;
  for (int l = 0; l < 64; l++) {
    for (int k = 0; k < 21; k++) { Ko[l][k] = 0; Kg[l][k] = 0; }
    for (int k = 0; k < 6; k++) { Fo[l][k] = 0; Fg[l][k] = 0; }
    const int b = T->lane_body[l];
    for (int s = 0; s < 2; s++) {
      for (int og = 0; og < 2; og++) {
        const int pr = og == 0 ? T->lane_opair[l][s] : T->lane_gpair[l][s];
        if (pr < 0) continue;
        const int c0 = e->pair_off[pr];
        int c1 = c0 + e->pair_cnt[pr];
        if (c1 > e->ncon) c1 = e->ncon;
        for (int c = c0; c < c1; c++) {
          const double sg = (m->geom_body[e->con[c].g2] == b) ? 1.0 : -1.0;
          double* K = og == 0 ? Ko[l] : Kg[l];
          double* F = og == 0 ? Fo[l] : Fg[l];
          for (int k = 0; k < 21; k++) K[k] += Kc[c][k];
          for (int k = 0; k < 6; k++) F[k] += sg * Fs[c][k];
          if (og == 1) any_g = 1;
        }
      }
    }
  }
  /* suffix scans along the chains */
  for (int off = 1; off < CL; off <<= 1) {
    double oKo[64][21], oFo[64][6];
    memcpy(oKo, Ko, sizeof(oKo)); memcpy(oFo, Fo, sizeof(oFo));
    for (int l = 0; l < 64; l++) {
      const int pos = l & 15, row = l & ~15;
      for (int k = 0; k < 21; k++) Ko[l][k] = oKo[l][k] + (pos + off <= 15 ? oKo[row + pos + off][k] : 0.0);
      for (int k = 0; k < 6; k++) Fo[l][k] = oFo[l][k] + (pos + off <= 15 ? oFo[row + pos + off][k] : 0.0);
    }
    if (any_g) {
      double oKg[64][21], oFg[64][6];
      memcpy(oKg, Kg, sizeof(oKg)); memcpy(oFg, Fg, sizeof(oFg));
      for (int l = 0; l < 64; l++) {
        const int pos = l & 15, row = l & ~15;
        for (int k = 0; k < 21; k++) Kg[l][k] = oKg[l][k] + (pos + off <= 15 ? oKg[row + pos + off][k] : 0.0);
        for (int k = 0; k < 6; k++) Fg[l][k] = oFg[l][k] + (pos + off <= 15 ? oFg[row + pos + off][k] : 0.0);
      }
    }
  }
  /* base composites: the four chain roots (fingers at position 1, palm) in order */
  double KBo[21], KBg[21], FBo[6], FBg[6];
  for (int k = 0; k < 21; k++) { KBo[k] = 0; KBg[k] = 0; }
  for (int k = 0; k < 6; k++) { FBo[k] = 0; FBg[k] = 0; }
  for (int c = 0; c < 4; c++) {
    const int l = c < 3 ? 16 * c + 1 : 49;
    for (int k = 0; k < 21; k++) { KBo[k] += Ko[l][k]; KBg[k] += Kg[l][k]; }
    for (int k = 0; k < 6; k++) { FBo[k] += Fo[l][k]; FBg[k] += Fg[l][k]; }
  }
  /* the object: every gripper-object contact (the base composite) + the ground-object pair */
  double Kgo[21], Fgo[6];
  for (int k = 0; k < 21; k++) Kgo[k] = 0;
  for (int k = 0; k < 6; k++) Fgo[k] = 0;
  for (int pr = 0; pr < m->npair; pr++) {
    const int a = m->pair_a[pr], b = m->pair_b[pr];
    if (!((a == m->geom_obj && b == m->geom_ground) || (b == m->geom_obj && a == m->geom_ground))) continue;
    const int c0 = e->pair_off[pr];
    int c1 = c0 + e->pair_cnt[pr];
    if (c1 > e->ncon) c1 = e->ncon;
    for (int c = c0; c < c1; c++) {
      const double sg = (m->geom_body[e->con[c].g2] == m->body_obj) ? 1.0 : -1.0;
      for (int k = 0; k < 21; k++) Kgo[k] += Kc[c][k];
      for (int k = 0; k < 6; k++) Fgo[k] += sg * Fs[c][k];
    }
  }
  double Koo[21], Fobj[6];
  for (int k = 0; k < 21; k++) Koo[k] = KBo[k] + Kgo[k];
  for (int k = 0; k < 6; k++) Fobj[k] = Fgo[k] - FBo[k];
  /* lock rows per dof */
  double lockD[NV], lockR[NV];
  int lockon[NV];
  for (int d = 0; d < NV; d++) { lockon[d] = 0; lockD[d] = 0; lockR[d] = 0; }
  for (int r = 0; r < e->nl; r++) {
    const int d = e->lock_row_dof[r];
    const double a = e->lock_row_a[r];
    if (a == 1.0 && !lockon[d]) { lockD[d] = e->efc_D[r]; lockR[d] = e->efc_D[r] * e->efc_aref[r]; }
    else { lockD[d] += (e->efc_D[r] * a) * a; lockR[d] += (e->efc_D[r] * a) * e->efc_aref[r]; }
    lockon[d] = 1;
  }
  const double* cdb = e->cdof[m->dof_base];
  /* finger chain rows */
  for (int f = 0; f < 3; f++)
    for (int p = 1; p <= CL; p++) {
      const int l = 16 * f + p, d = T->dof_f0[f] + p - 1;
      double Kt[21], Ft[6];
      for (int k = 0; k < 21; k++) Kt[k] = any_g ? Ko[l][k] + Kg[l][k] : Ko[l][k];
      for (int k = 0; k < 6; k++) Ft[k] = any_g ? Fo[l][k] + Fg[l][k] : Fo[l][k];
      const double* cd = e->cdof[d];
      double y[6], yo[6];
      symK_mul(Kt, cd, y);
      symK_mul(Ko[l], cd, yo);
      for (int j = 1; j <= CL; j++) S->h[f][p][j] = 0.0;
      for (int j = 1; j <= p; j++) S->h[f][p][j] = e->Hf[f][TRI(p, j)] + dot6(e->cdof[T->dof_f0[f] + j - 1], y);
      S->hb[f][p][0] = e->Hf[f][TRI(p, 0)] + dot6(cdb, y);
      for (int k = 0; k < 6; k++) S->hb[f][p][1 + k] = -dot6(e->cdof[m->dof_obj + k], yo);
      double r = e->frc[d] + dot6(cd, Ft);
      if (lockon[d]) { S->h[f][p][p] += lockD[d]; r += lockR[d]; }
      S->rhs_f[f][p] = r;
    }
  /* palm */
  {
    const int l = 49, d = m->dof_palm;
    double Kt[21], Ft[6];
    for (int k = 0; k < 21; k++) Kt[k] = any_g ? Ko[l][k] + Kg[l][k] : Ko[l][k];
    for (int k = 0; k < 6; k++) Ft[k] = any_g ? Fo[l][k] + Fg[l][k] : Fo[l][k];
    const double* cd = e->cdof[d];
    double y[6], yo[6];
    symK_mul(Kt, cd, y);
    symK_mul(Ko[l], cd, yo);
    S->ph = e->Hp[TRI(1, 1)] + dot6(cd, y);
    S->phb[0] = e->Hp[TRI(1, 0)] + dot6(cdb, y);
    for (int k = 0; k < 6; k++) S->phb[1 + k] = -dot6(e->cdof[m->dof_obj + k], yo);
    double r = e->frc[d] + dot6(cd, Ft);
    if (lockon[d]) { S->ph += lockD[d]; r += lockR[d]; }
    S->rhs_p = r;
  }
  /* border rows [base, obj0..5] (lower triangles) */
  {
    double KBt[21], FBt[6];
    for (int k = 0; k < 21; k++) KBt[k] = any_g ? KBo[k] + KBg[k] : KBo[k];
    for (int k = 0; k < 6; k++) FBt[k] = any_g ? FBo[k] + FBg[k] : FBo[k];
    double y[6], yob[6];
    symK_mul(KBt, cdb, y);
    symK_mul(KBo, cdb, yob);
    for (int i = 0; i < 7; i++) for (int j = 0; j < 7; j++) S->bb[i][j] = 0.0;
    S->bb[0][0] = e->Hbb + dot6(cdb, y);
    S->rhs_b[0] = e->frc[m->dof_base] + dot6(cdb, FBt);
    for (int k = 0; k < 6; k++) {
      const double* cok = e->cdof[m->dof_obj + k];
      double yk[6];
      symK_mul(Koo, cok, yk);
      S->bb[1 + k][0] = -dot6(cok, yob);
      for (int l2 = 0; l2 <= k; l2++) S->bb[1 + k][1 + l2] = e->Ho[TRI(k, l2)] + dot6(e->cdof[m->dof_obj + l2], yk);
      S->rhs_b[1 + k] = e->frc[m->dof_obj + k] + dot6(cok, Fobj);
    }
  }
}

/* LDL^T of the assembled system (in place) and the solve x = H^-1 rhs; x in dof order.
 * Lane-for-lane the device's arithmetic, including its branch-free row updates applied to
 * every lane of a DPP row (h <- (h - hk aa) sc with aa = 0, sc = 1 on lanes that take no
 * part in a pivot) and the masked solve updates. */
static void newton_factor_solve(or_env* e, nsys_t* S, double* x) {
  const gm_model* m = &e->m;
  const otopo* T = &e->T;
  const int CL = T->CL;
  double sch[3][16][28], sch_p[28];
  /* finger chains: pivots CL .. 1 */
  for (int f = 0; f < 3; f++) {
    for (int k = CL; k >= 1; k--) {
      const double hkk = S->h[f][k][k];
      const double ihk = 1.0 / hkk;
      double hk[GM_CHAIN + 1], hkb[7];
      for (int j = 1; j < k; j++) hk[j] = S->h[f][k][j];
      for (int b = 0; b < 7; b++) hkb[b] = S->hb[f][k][b];
      for (int p = 1; p <= CL; p++) {
        const int upd = p < k, piv = p == k;
        double Hpk = 0.0;
        for (int j = 1; j < k; j++) Hpk = (p == j) ? hk[j] : Hpk;
        const double a = Hpk * ihk;
        const double aa = upd ? a : 0.0;
        const double sc = piv ? ihk : 1.0;
        if (piv) for (int b = 0; b < 7; b++) S->ub[f][p][b] = S->hb[f][p][b];
        for (int j = 1; j < k; j++) S->h[f][p][j] = (S->h[f][p][j] - hk[j] * aa) * sc;
        for (int b = 0; b < 7; b++) S->hb[f][p][b] = (S->hb[f][p][b] - hkb[b] * aa) * sc;
        S->h[f][p][k] = upd ? a : S->h[f][p][k];
        if (piv) S->invd[f][p] = ihk;
      }
    }
    for (int k = 1; k <= CL; k++) {
      int e2 = 0;
      for (int i = 0; i < 7; i++)
        for (int j = 0; j <= i; j++) sch[f][k][e2++] = S->hb[f][k][i] * S->ub[f][k][j];
    }
  }
  /* palm: one pivot */
  {
    const double ih = 1.0 / S->ph;
    for (int b = 0; b < 7; b++) { S->pub[b] = S->phb[b]; S->phb[b] = S->phb[b] * ih; }
    S->pinvd = ih;
    int e2 = 0;
    for (int i = 0; i < 7; i++)
      for (int j = 0; j <= i; j++) sch_p[e2++] = S->phb[i] * S->pub[j];
  }
  /* Schur complements into the border, in elimination order */
  {
    int e2 = 0;
    for (int i = 0; i < 7; i++)
      for (int j = 0; j <= i; j++) {
        double v = S->bb[i][j];
        for (int f = 0; f < 3; f++)
          for (int k = CL; k >= 1; k--) v = v - sch[f][k][e2];
        v = v - sch_p[e2];
        S->bb[i][j] = v;
        e2++;
      }
  }
  /* border: pivots 6 .. 0 */
  for (int k = 6; k >= 0; k--) {
    const double ihk = 1.0 / S->bb[k][k];
    double bk[7];
    for (int j = 0; j < k; j++) bk[j] = S->bb[k][j];
    for (int i = 0; i < 7; i++) {
      const int upd = i < k, piv = i == k;
      double Bik = 0.0;
      for (int j = 0; j < k; j++) Bik = (i == j) ? bk[j] : Bik;
      const double a = Bik * ihk;
      const double aa = upd ? a : 0.0;
      const double sc = piv ? ihk : 1.0;
      for (int j = 0; j < k; j++) S->bb[i][j] = (S->bb[i][j] - bk[j] * aa) * sc;
      S->bb[i][k] = upd ? a : S->bb[i][k];
      if (piv) S->binvd[i] = ihk;
    }
  }
  /* forward: chains (leaf first), border sums, border */
  double y[3][16], yp, yb[7];
  for (int f = 0; f < 3; f++) {
    for (int p = 1; p <= CL; p++) y[f][p] = S->rhs_f[f][p];
    for (int k = CL; k >= 1; k--) {
      const double yk = y[f][k];
      for (int p = 1; p <= CL; p++) {
        const double Lc = (p < k) ? S->h[f][p][k] : 0.0;
        y[f][p] = y[f][p] - Lc * yk;
      }
    }
  }
  yp = S->rhs_p;
  for (int i = 0; i < 7; i++) {
    double v = S->rhs_b[i];
    for (int f = 0; f < 3; f++)
      for (int k = CL; k >= 1; k--) v = v - S->hb[f][k][i] * y[f][k];
    v = v - S->phb[i] * yp;
    yb[i] = v;
  }
  for (int k = 6; k >= 0; k--) {
    const double yk = yb[k];
    for (int i = 0; i < 7; i++) {
      const double Lc = (i < k) ? S->bb[i][k] : 0.0;
      yb[i] = yb[i] - Lc * yk;
    }
  }
  for (int f = 0; f < 3; f++) for (int p = 1; p <= CL; p++) y[f][p] = y[f][p] * S->invd[f][p];
  yp = yp * S->pinvd;
  for (int i = 0; i < 7; i++) yb[i] = yb[i] * S->binvd[i];
  /* backward: border (root first), then the chains root -> leaf */
  for (int j = 0; j < 6; j++) {
    const double xj = yb[j];
    for (int i = 0; i < 7; i++) {
      const double Lr = (j < i) ? S->bb[i][j] : 0.0;
      yb[i] = yb[i] - Lr * xj;
    }
  }
  for (int f = 0; f < 3; f++) {
    for (int p = 1; p <= CL; p++)
      for (int b = 0; b < 7; b++) y[f][p] = y[f][p] - S->hb[f][p][b] * yb[b];
    for (int j = 1; j < CL; j++) {
      const double xj = y[f][j];
      for (int p = 1; p <= CL; p++) {
        const double Lr = (j < p) ? S->h[f][p][j] : 0.0;
        y[f][p] = y[f][p] - Lr * xj;
      }
    }
    for (int p = 1; p <= CL; p++) x[T->dof_f0[f] + p - 1] = y[f][p];
  }
  for (int b = 0; b < 7; b++) yp = yp - S->phb[b] * yb[b];
  x[m->dof_palm] = yp;
  x[m->dof_base] = yb[0];
  for (int k = 0; k < 6; k++) x[m->dof_obj + k] = yb[1 + k];
}

/* constraint rows of this substep: impedance, regulariser, reference acceleration */
static void constraint_setup(or_env* e) {
  const gm_model* m = &e->m;
  const double h = m->timestep;
  double tc = m->solref[0];
  if (tc < 2 * h) tc = 2 * h;
  const double dr = m->solref[1], dmax = m->solimp[1];
  const double K = 1.0 / (dmax * dmax * tc * tc * dr * dr);
  const double Bd = 2.0 / (dmax * tc);
  int n = 0;
  for (int k = 0; k < m->nlock; k++) {
    if (!e->lock_active[k]) continue;
    const int d = m->lock_dof[k];
    const double pos = e->qpos[d] - e->lock_q[k];
    const double vel = e->qvel[d];
    if (e->weld_locks) {
      /* a weld between the slide's child and parent bodies: of its 6 rows only the
       * translational ones along the slide axis have a nonzero Jacobian (the joint fixes
       * every other relative motion); per world axis r the row is a_r qdot_d with its
       * own violation a_r pos, impedance, and the weld regulariser (mj_diagApprox:
       * translational body_invweight0 of both bodies) */
      const int b = m->dof_body[d], pb = m->body_parent[b];
      const double tran = body_invw(e, b) + body_invw(e, pb);
      for (int r = 0; r < 3; r++) {
        const double a = e->cdof[d][3 + r];
        if (fabs(a) < 1e-12) continue;
        const double pr = a * pos, vr = a * vel;
        const double imp = impedance(m, pr);
        double R = ((1 - imp) / imp) * tran;
        if (R < 1e-15) R = 1e-15;
        e->efc_D[n] = 1.0 / R;
        e->efc_aref[n] = -Bd * vr - K * imp * pr;
        e->efc_type[n] = 0;
        e->lock_row_dof[n] = d;
        e->lock_row_a[n] = a;
        n++;
      }
      continue;
    }
    /* the reference's weld (myfunctions.cpp:1177-1279) on a slide: of its 6 rows only the
     * translational ones have a nonzero Jacobian (a_r, the slide axis' world component r;
     * the joint fixes every other relative motion), each with its own violation a_r pos,
     * impedance and the weld regulariser (mj_diagApprox for mjEQ_WELD: the two bodies'
     * translational body_invweight0).  Their sum on the dof is one row with
     * D = sum_r D_r a_r^2 and D aref = sum_r D_r a_r aref_r, the same cost exactly. */
    const int b = m->dof_body[d], pb = m->body_parent[b];
    const double tran = body_invw(e, b) + body_invw(e, pb);
    double De = 0.0, Dar = 0.0;
    for (int r = 0; r < 3; r++) {
      const double a = e->cdof[d][3 + r];
      if (a == 0.0) continue;
      const double pr = a * pos, vr = a * vel;
      const double imp = impedance(m, pr);
      double R = ((1 - imp) / imp) * tran;
      if (R < 1e-15) R = 1e-15;
      const double Da = (1.0 / R) * a;
      De = De + Da * a;
      Dar = Dar + Da * (-Bd * vr - K * imp * pr);
    }
    e->efc_D[n] = De;
    e->efc_aref[n] = Dar / De;
    e->efc_type[n] = 0;
    e->lock_row_dof[n] = d;
    e->lock_row_a[n] = 1.0;
    n++;
  }
  e->nl = n;
  double V[NB][6];
  body_vel(e, e->qvel, V);
  for (int c = 0; c < e->ncon; c++) {
    const con_t* C = &e->con[c];
    const int b1 = m->geom_body[C->g1], b2 = m->geom_body[C->g2];
    const double tran = body_invw(e, b1) + body_invw(e, b2);
    const double diag = tran + (C->mu * C->mu) * tran;
    const double imp = impedance(m, C->dist);
    double R = ((1 - imp) / imp) * diag;
    if (R < 1e-15) R = 1e-15;
    const double D = 1.0 / R;
    double vel[4];
    contact_jv(e, c, V, vel);
    for (int ed = 0; ed < 4; ed++) {
      e->efc_D[n] = D;
      e->efc_aref[n] = -Bd * vel[ed] - K * imp * C->dist;
      e->efc_type[n] = 1;
      n++;
    }
  }
  e->nefc = n;
}
/* J v - aref for every row */
static void rows_jar(or_env* e, const double* v, double* jar) {
  double V[NB][6];
  body_vel(e, v, V);
  for (int r = 0; r < e->nl; r++)
    jar[r] = (e->lock_row_a[r] == 1.0 ? v[e->lock_row_dof[r]] : e->lock_row_a[r] * v[e->lock_row_dof[r]]) - e->efc_aref[r];
  for (int c = 0; c < e->ncon; c++) {
    double jv[4];
    contact_jv(e, c, V, jv);
    for (int ed = 0; ed < 4; ed++) jar[e->nl + 4 * c + ed] = jv[ed] - e->efc_aref[e->nl + 4 * c + ed];
  }
}
/* J^T f over every constraint row, dense (body_vel per unit vector); test paths and the
 * capped-solve residual only */
static void jt_force(or_env* e, const double* f, double* out) {
  const gm_model* m = &e->m;
  const int nv = m->nv;
  for (int i = 0; i < nv; i++) {
    double ev[NV];
    for (int k = 0; k < NV; k++) ev[k] = (k == i) ? 1.0 : 0.0;
    double V[NB][6];
    body_vel(e, ev, V);
    double acc = 0.0;
    for (int r = 0; r < e->nl; r++)
      if (e->lock_row_dof[r] == i) acc += e->lock_row_a[r] * f[r];
    for (int c = 0; c < e->ncon; c++) {
      double jv[4];
      contact_jv(e, c, V, jv);
      for (int ed = 0; ed < 4; ed++) acc += jv[ed] * f[e->nl + 4 * c + ed];
    }
    out[i] = acc;
  }
}
/* per-lane partial of a row sum (contact c's 4 edges on lane c, lock row r on lane r),
 * then the 64-lane butterfly: the device's row reduction */
static double row_reduce(const or_env* e, const double* t) {
  double v[64];
  for (int l = 0; l < 64; l++) {
    double a = 0.0;
    if (l < e->ncon) {
      const double* tc = t + e->nl + 4 * l;
      a = ((tc[0] + tc[1]) + tc[2]) + tc[3];
    }
    if (l < e->nl) a = a + t[l];
    v[l] = a;
  }
  return butterfly64(v);
}
static double dof_reduce(const or_env* e, const double* t) {
  double v[64];
  for (int l = 0; l < 64; l++) v[l] = l < e->m.nv ? t[l] : 0.0;
  return butterfly64(v);
}
static int row_active(const or_env* e, int r, double jar) { return r < e->nl ? 1 : (jar < 0); }

/* mj_solNewton restated: from the warm start (the previous substep's qacc), repeat: the
 * Newton point x of the quadratic model on the current active set (one LDL^T of
 * H~ + J_a^T D_a J_a), accept it when the active set at x is the same (then x is the
 * exact optimum), otherwise an exact line search along x - q (bracketed Newton on the
 * piecewise-quadratic cost, stopping on the piece it lands in). */
#ifdef OR_NEWTON_STATS
/* developer probe (tools/newton_active_set_probe.py): per extra Newton point, how many
 * constraint rows entered / left the active set since the previous point -- the work an
 * incremental (rank-1 update) factorisation would do instead of a refactor */
long long or_nstat[40];
void or_newton_stats(long long* out) { for (int i = 0; i < 40; i++) out[i] = or_nstat[i]; }
#define OR_NSTAT(k, v) __atomic_fetch_add(&or_nstat[k], (v), __ATOMIC_RELAXED)
#endif
static void newton_solve(or_env* e) {
  const gm_model* m = &e->m;
  const int nv = m->nv, nefc = e->nefc;
  double* q = e->qacc;
  double Ma[NV], Mv[NV], xv[NV], d[NV], tmp[NV];
  double jq[NE], jx[NE], dj[NE], tg[NE], th[NE];
  int act[NE], actx[NE];
  for (int i = 0; i < nv; i++) q[i] = e->qacc_warm[i];
  rows_jar(e, q, jq);
  int it = 0, capped = 1, ls_cap = 0;
  e->stat_ls = 0;
  const int maxit = (m->newton_maxit > 0 && m->newton_maxit < GM_NEWTON_MAXIT) ? m->newton_maxit : GM_NEWTON_MAXIT;
  for (it = 0; it < maxit; it++) {
    for (int r = 0; r < nefc; r++) act[r] = row_active(e, r, jq[r]);
#ifdef OR_NEWTON_STATS
    {
      static __thread int pact[NE];
      if (it > 0) {
        int ent = 0, lv = 0;
        for (int r = 0; r < nefc; r++) if (act[r] != pact[r]) { if (act[r]) ent++; else lv++; }
        OR_NSTAT(ent + lv < 30 ? ent + lv : 30, 1); OR_NSTAT(31, ent); OR_NSTAT(32, lv);
      }
      OR_NSTAT(33, 1);
      for (int r = 0; r < nefc; r++) pact[r] = act[r];
    }
#endif
    nsys_t S;
    newton_assemble(e, act, &S);
    newton_factor_solve(e, &S, xv);
    rows_jar(e, xv, jx);
    int same = 1;
    for (int r = 0; r < nefc; r++) { actx[r] = row_active(e, r, jx[r]); same = same && (actx[r] == act[r]); }
    if (same) {
      for (int i = 0; i < nv; i++) q[i] = xv[i];
      for (int r = 0; r < nefc; r++) jq[r] = jx[r];
      it++;
      capped = 0;
      break;
    }
    /* exact line search along d = x - q.  H~ q is formed here, when first needed: the
     * search is only reached at iteration 0 with q still the warm start, later
     * iterations update it incrementally (the device does the same) */
    if (it == 0) smooth_matvec(e, q, Ma);
    for (int i = 0; i < nv; i++) d[i] = xv[i] - q[i];
    smooth_matvec(e, d, Mv);
    for (int i = 0; i < nv; i++) tmp[i] = d[i] * (Ma[i] - e->frc[i]);
    const double g0 = dof_reduce(e, tmp);
    for (int i = 0; i < nv; i++) tmp[i] = d[i] * Mv[i];
    const double h0 = dof_reduce(e, tmp);
    for (int r = 0; r < nefc; r++) dj[r] = jx[r] - jq[r];
    double alpha = 1.0, lo = 0.0, hi = 0.0;
    int hi_set = 0, newton = 0, have_prev = 0;
    int prev[NE];
    int ls = 0;
    for (; ls < GM_NEWTON_MAXLS; ls++) {
      e->stat_ls++;
      int pat[NE], same_piece = 1;
      for (int r = 0; r < nefc; r++) {
        const double j = jq[r] + alpha * dj[r];
        pat[r] = row_active(e, r, j);
        same_piece = same_piece && have_prev && (pat[r] == prev[r]);
        tg[r] = pat[r] ? (e->efc_D[r] * j) * dj[r] : 0.0;
        th[r] = pat[r] ? (e->efc_D[r] * dj[r]) * dj[r] : 0.0;
      }
      if (nefc == 0) same_piece = have_prev;
      if (newton && same_piece) break;
      const double g = (g0 + alpha * h0) + row_reduce(e, tg);
      const double hh = h0 + row_reduce(e, th);
      if (g == 0.0) break;
      if (g < 0) lo = alpha; else { hi = alpha; hi_set = 1; }
      if (!(hh > 0)) break;
      double an = alpha - g / hh;
      newton = 1;
      if (!(an > lo) || (hi_set && !(an < hi))) { an = hi_set ? 0.5 * (lo + hi) : 2.0 * alpha; newton = 0; }
      for (int r = 0; r < nefc; r++) prev[r] = pat[r];
      have_prev = 1;
      alpha = an;
    }
    if (ls == GM_NEWTON_MAXLS) ls_cap = 1;
    for (int i = 0; i < nv; i++) { q[i] = q[i] + alpha * d[i]; Ma[i] = Ma[i] + alpha * Mv[i]; }
    for (int r = 0; r < nefc; r++) jq[r] = jq[r] + alpha * dj[r];
  }
  e->stat_it = it;
#ifdef OR_NEWTON_STATS
  OR_NSTAT(34, 1); OR_NSTAT(35, nefc);
#endif
  /* a solve that ran out of iterations, or a line search out of evaluations, is counted
   * (GmEnvState::newton_caps; the device counts the same) */
  if (capped || ls_cap) e->newton_caps += 1;
  /* constraint forces at the solution, contact-frame forces (mj_contactForce, pyramid) */
  for (int r = 0; r < nefc; r++) {
    const double j = jq[r];
    e->efc_f[r] = row_active(e, r, j) ? -(e->efc_D[r] * j) : 0.0;
  }
  for (int c = 0; c < e->ncon; c++) {
    const double* fe = &e->efc_f[e->nl + 4 * c];
    con_t* C = &e->con[c];
    C->force[0] = ((fe[0] + fe[1]) + fe[2]) + fe[3];
    C->force[1] = C->mu * (fe[0] - fe[1]);
    C->force[2] = C->mu * (fe[2] - fe[3]);
  }
  for (int i = 0; i < nv; i++) e->qacc_warm[i] = q[i];
  /* a capped solve: qacc is no optimum, so qfrc_smooth + J^T efc (what mj_Euler integrates)
   * differs from H~ qacc by the residual; euler_damping takes it into account (H~ q = Ma,
   * kept up to date by the line searches every capped iteration ran) */
  e->res_valid = 0;
  if (capped || e->want_forces) {
    double jtf[NV];
    jt_force(e, e->efc_f, jtf);
    if (capped) {
      for (int i = 0; i < nv; i++) e->res[i] = Ma[i] - (e->frc[i] + jtf[i]);
      e->res_valid = 1;
    }
    if (e->want_forces)
      for (int i = 0; i < nv; i++) { e->last_smooth[i] = e->frc[i]; e->last_constraint[i] = jtf[i]; }
  }
}

/* ---- independent cross-check: the same soft-constraint problem in its dual form,
 * dense, solved by projected Gauss-Seidel (mj_solPGS: rows in order, ARinv, lock rows
 * unbounded, pyramid edges >= 0) for `sweeps` sweeps, warm-started from the forces at the
 * previous qacc (MuJoCo's warm start).  Test infrastructure only. ---- */
static void dense_H(const or_env* e, double H[NV][NV]) {
  const gm_model* m = &e->m;
  const otopo* T = &e->T;
  for (int i = 0; i < NV; i++) for (int j = 0; j < NV; j++) H[i][j] = 0;
  for (int d = 0; d < m->nv; d++) {
    double ev[NV], col[NV];
    for (int i = 0; i < NV; i++) ev[i] = (i == d) ? 1.0 : 0.0;
    smooth_matvec(e, ev, col);
    for (int i = 0; i < m->nv; i++) H[i][d] = col[i];
  }
  (void)T;
}
static void chol_solve(int n, double A[NV][NV], double* x) {   /* in-place Cholesky, then solve */
  for (int k = 0; k < n; k++) {
    double s = A[k][k];
    for (int j = 0; j < k; j++) s -= A[k][j] * A[k][j];
    A[k][k] = sqrt(s);
    for (int i = k + 1; i < n; i++) {
      double t = A[i][k];
      for (int j = 0; j < k; j++) t -= A[i][j] * A[k][j];
      A[i][k] = t / A[k][k];
    }
  }
  for (int i = 0; i < n; i++) { double s = x[i]; for (int j = 0; j < i; j++) s -= A[i][j] * x[j]; x[i] = s / A[i][i]; }
  for (int i = n - 1; i >= 0; i--) { double s = x[i]; for (int j = i + 1; j < n; j++) s -= A[j][i] * x[j]; x[i] = s / A[i][i]; }
}
static void ref_pgs_solve(or_env* e, int sweeps) {
  const gm_model* m = &e->m;
  const int nv = m->nv, n = e->nefc;
  static __thread double H[NV][NV], Lf[NV][NV], J[NE][NV], W[NE][NV], A[NE][NE];
  dense_H(e, H);
  double qs[NV];
  for (int i = 0; i < nv; i++) qs[i] = e->frc[i];
  memcpy(Lf, H, sizeof(Lf));
  chol_solve(nv, Lf, qs);
  /* dense Jacobian rows */
  for (int r = 0; r < n; r++) for (int i = 0; i < NV; i++) J[r][i] = 0;
  for (int r = 0; r < e->nl; r++) J[r][e->lock_row_dof[r]] = e->lock_row_a[r];
  for (int i = 0; i < nv; i++) {
    double ev[NV];
    for (int k = 0; k < NV; k++) ev[k] = (k == i) ? 1.0 : 0.0;
    double V[NB][6];
    body_vel(e, ev, V);
    for (int c = 0; c < e->ncon; c++) {
      double jv[4];
      contact_jv(e, c, V, jv);
      for (int ed = 0; ed < 4; ed++) J[e->nl + 4 * c + ed][i] = jv[ed];
    }
  }
  for (int r = 0; r < n; r++) {
    for (int i = 0; i < nv; i++) W[r][i] = J[r][i];
    memcpy(Lf, H, sizeof(Lf));
    chol_solve(nv, Lf, W[r]);
  }
  for (int r = 0; r < n; r++)
    for (int s = 0; s < n; s++) { double v = 0; for (int i = 0; i < nv; i++) v += J[r][i] * W[s][i]; A[r][s] = v; }
  double b[NE], f[NE], R[NE];
  for (int r = 0; r < n; r++) {
    double ja = 0;
    for (int i = 0; i < nv; i++) ja += J[r][i] * qs[i];
    b[r] = ja - e->efc_aref[r];
    R[r] = 1.0 / e->efc_D[r];
    /* warm start: the forces the previous qacc implies */
    double jw = 0;
    for (int i = 0; i < nv; i++) jw += J[r][i] * e->qacc_warm[i];
    const double jar = jw - e->efc_aref[r];
    f[r] = (e->efc_type[r] == 0 || jar < 0) ? -jar / R[r] : 0.0;
  }
  for (int it = 0; it < sweeps; it++)
    for (int r = 0; r < n; r++) {
      double g = b[r] + R[r] * f[r];
      for (int s = 0; s < n; s++) g += A[r][s] * f[s];
      double fn = f[r] - g / (A[r][r] + R[r]);
      if (e->efc_type[r] == 1 && fn < 0) fn = 0;
      f[r] = fn;
    }
  double jtf[NV];
  for (int i = 0; i < nv; i++) { jtf[i] = 0; for (int r = 0; r < n; r++) jtf[i] += J[r][i] * f[r]; }
  memcpy(Lf, H, sizeof(Lf));
  chol_solve(nv, Lf, jtf);
  for (int i = 0; i < nv; i++) e->qacc[i] = qs[i] + jtf[i];
  for (int r = 0; r < n; r++) e->efc_f[r] = f[r];
  for (int c = 0; c < e->ncon; c++) {
    const double* fe = &e->efc_f[e->nl + 4 * c];
    con_t* C = &e->con[c];
    C->force[0] = ((fe[0] + fe[1]) + fe[2]) + fe[3];
    C->force[1] = C->mu * (fe[0] - fe[1]);
    C->force[2] = C->mu * (fe[2] - fe[3]);
  }
  for (int i = 0; i < nv; i++) e->qacc_warm[i] = e->qacc[i];
  e->stat_it = sweeps;
}

/* =====================================================================
 * one physics substep: before_step + step + after_step (physics part),
 * myfunctions.cpp:1864-1908 -> mj_step1 / control / mj_step2 (the engine spec)
 * ===================================================================== */
/* A x = b for a symmetric positive definite 6 x 6 block, LDL^T with pivots 5 .. 0 (rows
 * eliminated last-first, as the device's serial version on lane 0), x overwrites b */
static void ldl6_solve(double A[6][6], double* b) {
  /* lower triangle only: A = U D U^T with U unit upper, U[i][k] kept at A[k][i] (i < k) */
  for (int k = 5; k >= 0; k--) {
    const double ik = 1.0 / A[k][k];
    double col[6];
    for (int i = 0; i < k; i++) col[i] = A[k][i];
    for (int i = 0; i < k; i++) {
      const double a = col[i] * ik;
      for (int j = 0; j <= i; j++) A[i][j] = A[i][j] - a * col[j];
      A[k][i] = a;
    }
  }
  for (int k = 5; k >= 0; k--)          /* U z = b */
    for (int i = 0; i < k; i++) b[i] = b[i] - A[k][i] * b[k];
  for (int k = 0; k < 6; k++) b[k] = b[k] / A[k][k];
  for (int k = 0; k < 6; k++)           /* U^T x = D^-1 z */
    for (int i = 0; i < k; i++) b[k] = b[k] - A[k][i] * b[i];
}
/* MuJoCo 2.1.5 mj_Euler's implicit joint damping (mujoco_actuators): qacc_e =
 * (M + h D)^-1 (qfrc_smooth + qfrc_constraint) = qacc - (M + h D)^-1 (h D qacc), qacc the
 * solve's (M qacc = qfrc_smooth + qfrc_constraint at its optimum).  The system on the
 * device's lanes (gm_newton.hip euler_damping): each finger chain block leaf-first LDL^T
 * on its DPP row with the base as the one border column, the palm one pivot, the base
 * pivot after the wave-summed Schur complement; the object (no damping, decoupled from the
 * gripper in M) takes no correction. */
static void euler_damping(const or_env* e, double* qe) {
  const gm_model* m = &e->m;
  const otopo* T = &e->T;
  const int CL = T->CL;
  const double h = m->timestep;
  double L[64][GM_CHAIN + 1], lb[64], ub[64], invd[64], y[64];
  for (int l = 0; l < 64; l++) {
    for (int j = 0; j <= CL; j++) L[l][j] = 0.0;
    lb[l] = 0.0; ub[l] = 0.0; invd[l] = 1.0; y[l] = 0.0;
  }
  for (int f = 0; f < 3; f++)
    for (int p = 1; p <= CL; p++) {
      const int l = 16 * f + p, d = T->dof_f0[f] + p - 1;
      const double hd = h * T->dof_damp[d];
      for (int j = 1; j <= CL; j++) L[l][j] = e->Hf[f][j <= p ? TRI(p, j) : TRI(j, p)];   /* full symmetric row */
      L[l][p] = L[l][p] + hd;
      lb[l] = e->Hf[f][TRI(p, 0)];
      y[l] = hd * e->qacc[d];
      if (e->res_valid) y[l] = y[l] + e->res[d];
    }
  const int lp = 56, lbase = 48;
  {
    const double hd = h * T->dof_damp[m->dof_palm];
    L[lp][1] = e->Hp[TRI(1, 1)] + hd;
    lb[lp] = e->Hp[TRI(1, 0)];
    y[lp] = hd * e->qacc[m->dof_palm];
    if (e->res_valid) y[lp] = y[lp] + e->res[m->dof_palm];
  }
  const double hdb = h * T->dof_damp[m->dof_base];
  const double bb = e->Hbb + hdb;
  y[lbase] = hdb * e->qacc[m->dof_base];
  if (e->res_valid) y[lbase] = y[lbase] + e->res[m->dof_base];
  /* chain factor, pivots CL .. 1, every lane of rows 0..2 in lock step */
  for (int k = CL; k >= 1; k--) {
    double hk[3][GM_CHAIN + 1], hkb[3], ihk[3];
    for (int f = 0; f < 3; f++) {
      const int lk = 16 * f + k;
      ihk[f] = 1.0 / L[lk][k];
      for (int j = 1; j < k; j++) hk[f][j] = L[lk][j];
      hkb[f] = lb[lk];
    }
    for (int l = 0; l < 48; l++) {
      const int f = l >> 4, p = l & 15;
      const int upd = p >= 1 && p < k, piv = p == k;
      const double a = L[l][k] * ihk[f];   /* the row's own pivot-column entry */
      const double aa = upd ? a : 0.0;
      const double sc = piv ? ihk[f] : 1.0;
      if (piv) ub[l] = lb[l];
      for (int j = 1; j < k; j++) L[l][j] = (L[l][j] - hk[f][j] * aa) * sc;
      lb[l] = (lb[l] - hkb[f] * aa) * sc;
      L[l][k] = upd ? a : L[l][k];
      if (piv) invd[l] = ihk[f];
    }
  }
  {
    const double ih = 1.0 / L[lp][1];
    ub[lp] = lb[lp];
    lb[lp] = lb[lp] * ih;
    invd[lp] = ih;
  }
  /* forward over the chains (leaf first) */
  for (int k = CL; k >= 1; k--)
    for (int f = 0; f < 3; f++) {
      const double yk = y[16 * f + k];
      for (int p = 1; p <= CL; p++) {
        const double Lc = (p < k) ? L[16 * f + p][k] : 0.0;
        y[16 * f + p] = y[16 * f + p] - Lc * yk;
      }
    }
  /* the base's two sums: per DPP row an inclusive Hillis-Steele scan of (lb ub, lb y) (the
   * row total lands on lane 15), then rows 0, 1, 2 and the palm in that order */
  double s1[64], s2[64];
  for (int l = 0; l < 64; l++) {
    const int f = l >> 4, p = l & 15;
    const int part = (f < 3 && p >= 1 && p <= CL) || l == lp;
    s1[l] = part ? lb[l] * ub[l] : 0.0;
    s2[l] = part ? lb[l] * y[l] : 0.0;
  }
  for (int off = 1; off < 16; off <<= 1) {
    double o1[64], o2[64];
    memcpy(o1, s1, sizeof(o1)); memcpy(o2, s2, sizeof(o2));
    for (int l = 0; l < 64; l++) {
      const int pos = l & 15, row = l & ~15;
      s1[l] = o1[l] + rshr(o1 + row, pos, off);
      s2[l] = o2[l] + rshr(o2 + row, pos, off);
    }
  }
  const double sch = ((s1[15] + s1[31]) + s1[47]) + s1[lp];
  const double fs = ((s2[15] + s2[31]) + s2[47]) + s2[lp];
  const double xb = (y[lbase] - fs) * (1.0 / (bb - sch));
  /* back substitution: D^-1, the border, then the chains root -> leaf */
  for (int f = 0; f < 3; f++) {
    for (int p = 1; p <= CL; p++) {
      const int l = 16 * f + p;
      y[l] = y[l] * invd[l];
      y[l] = y[l] - lb[l] * xb;
    }
    for (int j = 1; j < CL; j++) {
      const double xj = y[16 * f + j];
      for (int p = 1; p <= CL; p++) {
        const double Lr = (j < p) ? L[16 * f + p][j] : 0.0;
        y[16 * f + p] = y[16 * f + p] - Lr * xj;
      }
    }
  }
  y[lp] = y[lp] * invd[lp] - lb[lp] * xb;
  for (int d = 0; d < m->nv; d++) qe[d] = e->qacc[d];
  if (e->res_valid) {
    /* the object block of M (no damping, no coupling to the gripper): qacc_e = qacc - Moo^-1 r,
     * the 6 x 6 block (H~'s Ho, lower triangle) by LDL^T from the last row as the device's
     * lane 0 does it */
    double A[6][6], x[6];
    for (int k = 0; k < 6; k++)
      for (int l = 0; l <= k; l++) { A[k][l] = e->Ho[TRI(k, l)]; A[l][k] = A[k][l]; }
    for (int k = 0; k < 6; k++) x[k] = e->res[m->dof_obj + k];
    ldl6_solve(A, x);
    for (int k = 0; k < 6; k++) qe[m->dof_obj + k] = e->qacc[m->dof_obj + k] - x[k];
  }
  for (int f = 0; f < 3; f++)
    for (int p = 1; p <= CL; p++) qe[T->dof_f0[f] + p - 1] = e->qacc[T->dof_f0[f] + p - 1] - y[16 * f + p];
  qe[m->dof_palm] = e->qacc[m->dof_palm] - y[lp];
  qe[m->dof_base] = e->qacc[m->dof_base] - xb;
}

static void physics_substep(or_env* e) {
  const gm_model* m = &e->m;
  const double h = m->timestep;
  memcpy(e->qpos_pre, e->qpos, sizeof(e->qpos));
  fk(e);
  crb_rne(e);
  mass_and_forces(e);
  collision(e);
  constraint_setup(e);
  if (e->solver_pgs > 0) ref_pgs_solve(e, e->solver_pgs);
  else newton_solve(e);
  e->stat_solves++;
  e->stat_it_sum += e->stat_it;
  e->stat_ls_sum += e->stat_ls;
  if (e->stat_it > e->stat_it_max) e->stat_it_max = e->stat_it;
  if (e->ncon_total > e->stat_ncon_max) e->stat_ncon_max = e->ncon_total;
  e->stat_nefc_sum += e->nefc;
  /* mj_checkAcc -> mjWARN_BADQACC (is_sim_unstable, myfunctions.cpp:4233-4242) */
  for (int d = 0; d < m->nv; d++) if (!(fabs(e->qacc[d]) <= 1e10)) e->badqacc = 1;
  /* semi-implicit Euler (mj_Euler): with MuJoCo's actuator order the joint damping is
   * implicit here, qacc_e = (M + h D)^-1 (qfrc_smooth + qfrc_constraint) (euler_damping);
   * the folded scheme integrates the solve's qacc directly */
  double qe[NV];
  if (m->mujoco_actuators) euler_damping(e, qe);
  else for (int d = 0; d < m->nv; d++) qe[d] = e->qacc[d];
  for (int d = 0; d < m->nv; d++) e->qvel[d] += h * qe[d];
  for (int d = 0; d < m->dof_obj; d++) e->qpos[d] += h * e->qvel[d];
  {
    const int qa = m->dof_obj, da = m->dof_obj;
    for (int k = 0; k < 3; k++) e->qpos[qa + k] += h * e->qvel[da + k];
    double* q = &e->qpos[qa + 3];
    const double w[3] = {e->qvel[da + 3], e->qvel[da + 4], e->qvel[da + 5]};
    const double wn = sqrt(dot3(w, w));
    if (wn > 1e-15) {
      const double ang = wn * h;
      double sn, cs;
      gm_sincos(0.5 * ang, &sn, &cs);
      sn = sn / wn;
      const double dq[4] = {cs, w[0] * sn, w[1] * sn, w[2] * sn};
      quatmul(q, q, dq);
    }
    quatnorm_d(q);
    e->time += h;
  }
}
