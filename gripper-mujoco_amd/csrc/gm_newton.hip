// gm_newton.hip -- box-box collision and the constraint solve of the env-step kernel
// (included by gm_kernels.hip after the kinematics / dynamics stages).
//
// The constraint problem is MuJoCo's (mj_makeConstraint / mj_makeImpedance with the
// mj_diagApprox regulariser, pyramidal cones), solved to its unique optimum by MuJoCo's
// Newton method (mj_solNewton: primal, in qacc space, exact line search, warm start from
// the previous substep's qacc).  The Hessian H~ + J_a^T D_a J_a is assembled in spatial
// form -- per contact the 3x3 Q = sum_e D_e u_e u_e^T of its active pyramid edges, per
// body the 6x6 K = S Q S^T summed over the body's contacts, suffix-scanned along each
// finger chain like composite inertias -- so its cost follows the bodies, not the
// constraint rows, and no per-row Jacobian or Delassus matrix is ever formed.  It is
// factored on the DPP-row layout: each finger chain's block on its 16-lane row with the
// border [base, object 0..5] as extra columns (leaf-first LDL^T, row_newbcast pivots),
// Schur complements into the border, a 7x7 border LDL^T on row 3.
// oracle/physics.c restates every function here operation for operation (the oracle's
// lane emulation), so device and oracle agree bit for bit from the same state.

// ------------------------------------------------------------ box-box (mjc_BoxBox)
// Separating axes, then the face-clipped manifold (see oracle/physics.c bb_setup): the
// face case keeps up to 8 of 24 candidates (incident vertices inside the reference face,
// reference corners inside the incident face, edge crossings) below the reference face.
#define BB_NCAND 24
struct BBox {
  int kind;                     // 0 none, 1 face, 2 edge
  real n[3], pen, sgn;
  real crf[3], ru[3], rv[3], hu, hv;
  real V[4][3], cinc[3], ninc[3], pu[4], pv[4];
};

__device__ __forceinline__ void bb_setup(const GeomV& A, const GeomV& B, BBox& S, real* ea, real* eb, real* da,
                                         real* db) {
  S.kind = 0;
  const real d[3] = {B.c[0] - A.c[0], B.c[1] - A.c[1], B.c[2] - A.c[2]};
  real a[3][3], b[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int k = 0; k < 3; k++) { a[i][k] = A.R[3 * k + i]; b[i][k] = B.R[3 * k + i]; }
  real Ca[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) Ca[i][j] = fabs(dot3(a[i], b[j]));
  real best = 0;
  int code = -1;
#pragma unroll
  for (int i = 0; i < 3; i++) {
    const real rb = B.size[0] * Ca[i][0] + B.size[1] * Ca[i][1] + B.size[2] * Ca[i][2];
    const real pen = (A.size[i] + rb) - fabs(dot3(d, a[i]));
    if (pen < 0) return;
    if (code < 0 || pen < best) { best = pen; code = i; }
  }
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const real ra = A.size[0] * Ca[0][j] + A.size[1] * Ca[1][j] + A.size[2] * Ca[2][j];
    const real pen = (ra + B.size[j]) - fabs(dot3(d, b[j]));
    if (pen < 0) return;
    if (pen < best) { best = pen; code = 3 + j; }
  }
  real ebest = 0, eL[3] = {0, 0, 0};
  int ecode = -1;
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) {
      real L[3];
      cross3(L, a[i], b[j]);
      const real len2 = dot3(L, L);
      const real len = sqrt_n(len2);
      if (len < 1e-6) continue;
      const real il = rsq_n(len2);
      L[0] *= il; L[1] *= il; L[2] *= il;
      const real ra = A.size[0] * fabs(dot3(a[0], L)) + A.size[1] * fabs(dot3(a[1], L)) + A.size[2] * fabs(dot3(a[2], L));
      const real rb = B.size[0] * fabs(dot3(b[0], L)) + B.size[1] * fabs(dot3(b[1], L)) + B.size[2] * fabs(dot3(b[2], L));
      const real pen = (ra + rb) - fabs(dot3(d, L));
      if (pen < 0) return;
      if (ecode < 0 || pen < ebest) { ebest = pen; ecode = 3 * i + j; eL[0] = L[0]; eL[1] = L[1]; eL[2] = L[2]; }
    }
  if (ecode >= 0 && ebest < 0.95 * best) {
    const int i = ecode / 3, j = ecode % 3;
    real L[3] = {eL[0], eL[1], eL[2]};
    if (dot3(d, L) < 0) { L[0] = -L[0]; L[1] = -L[1]; L[2] = -L[2]; }
    S.kind = 2;
    S.pen = ebest;
    S.n[0] = L[0]; S.n[1] = L[1]; S.n[2] = L[2];
#pragma unroll
    for (int k = 0; k < 3; k++) { ea[k] = A.c[k]; eb[k] = B.c[k]; }
#pragma unroll
    for (int k = 0; k < 3; k++) {
      da[k] = (i == 0) ? a[0][k] : (i == 1) ? a[1][k] : a[2][k];
      db[k] = (j == 0) ? b[0][k] : (j == 1) ? b[1][k] : b[2][k];
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (k != i) {
        const real s = dot3(a[k], L) >= 0 ? A.size[k] : -A.size[k];
#pragma unroll
        for (int t = 0; t < 3; t++) ea[t] += s * a[k][t];
      }
      if (k != j) {
        const real s = dot3(b[k], L) >= 0 ? -B.size[k] : B.size[k];
#pragma unroll
        for (int t = 0; t < 3; t++) eb[t] += s * b[k][t];
      }
    }
    return;
  }
  const bool ref_is_a = code < 3;
  const int ri = ref_is_a ? code : code - 3;
  // reference / incident box data by selection (no pointer to a register array)
  real rc[3], ic[3], rs[3], is[3], ra[3][3], ia[3][3];
#pragma unroll
  for (int k = 0; k < 3; k++) {
    rc[k] = ref_is_a ? A.c[k] : B.c[k];
    ic[k] = ref_is_a ? B.c[k] : A.c[k];
    rs[k] = ref_is_a ? A.size[k] : B.size[k];
    is[k] = ref_is_a ? B.size[k] : A.size[k];
#pragma unroll
    for (int t = 0; t < 3; t++) { ra[k][t] = ref_is_a ? a[k][t] : b[k][t]; ia[k][t] = ref_is_a ? b[k][t] : a[k][t]; }
  }
  real rax[3], rau[3], rav[3];
  const int ui = (ri + 1) % 3, vi = (ri + 2) % 3;
#pragma unroll
  for (int t = 0; t < 3; t++) {
    rax[t] = ri == 0 ? ra[0][t] : ri == 1 ? ra[1][t] : ra[2][t];
    rau[t] = ui == 0 ? ra[0][t] : ui == 1 ? ra[1][t] : ra[2][t];
    rav[t] = vi == 0 ? ra[0][t] : vi == 1 ? ra[1][t] : ra[2][t];
  }
  const real rsi = ri == 0 ? rs[0] : ri == 1 ? rs[1] : rs[2];
  const real dd[3] = {ic[0] - rc[0], ic[1] - rc[1], ic[2] - rc[2]};
  const real s0 = dot3(dd, rax) >= 0 ? 1.0 : -1.0;
  S.kind = 1;
  S.pen = best;
  S.sgn = ref_is_a ? 1.0 : -1.0;
#pragma unroll
  for (int k = 0; k < 3; k++) S.n[k] = s0 * rax[k];
#pragma unroll
  for (int k = 0; k < 3; k++) { S.crf[k] = rc[k] + rsi * S.n[k]; S.ru[k] = rau[k]; S.rv[k] = rav[k]; }
  S.hu = ui == 0 ? rs[0] : ui == 1 ? rs[1] : rs[2];
  S.hv = vi == 0 ? rs[0] : vi == 1 ? rs[1] : rs[2];
  int jm = 0;
  real bm = fabs(dot3(S.n, ia[0]));
#pragma unroll
  for (int j = 1; j < 3; j++) { const real v = fabs(dot3(S.n, ia[j])); if (v > bm) { bm = v; jm = j; } }
  real iaj[3], ie1[3], ie2[3];
  const int e1 = (jm + 1) % 3, e2 = (jm + 2) % 3;
#pragma unroll
  for (int t = 0; t < 3; t++) {
    iaj[t] = jm == 0 ? ia[0][t] : jm == 1 ? ia[1][t] : ia[2][t];
    ie1[t] = e1 == 0 ? ia[0][t] : e1 == 1 ? ia[1][t] : ia[2][t];
    ie2[t] = e2 == 0 ? ia[0][t] : e2 == 1 ? ia[1][t] : ia[2][t];
  }
  const real isj = jm == 0 ? is[0] : jm == 1 ? is[1] : is[2];
  const real h1 = e1 == 0 ? is[0] : e1 == 1 ? is[1] : is[2];
  const real h2 = e2 == 0 ? is[0] : e2 == 1 ? is[1] : is[2];
  const real sj = dot3(S.n, iaj) >= 0 ? -1.0 : 1.0;
#pragma unroll
  for (int k = 0; k < 3; k++) { S.ninc[k] = sj * iaj[k]; S.cinc[k] = ic[k] + isj * S.ninc[k]; }
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const real su = (q == 1 || q == 2) ? 1.0 : -1.0, sv = (q >= 2) ? 1.0 : -1.0;
#pragma unroll
    for (int k = 0; k < 3; k++) S.V[q][k] = S.cinc[k] + (su * h1) * ie1[k] + (sv * h2) * ie2[k];
    const real r[3] = {S.V[q][0] - S.crf[0], S.V[q][1] - S.crf[1], S.V[q][2] - S.crf[2]};
    S.pu[q] = dot3(r, S.ru);
    S.pv[q] = dot3(r, S.rv);
  }
}
// face candidate i (see oracle/physics.c bb_face_cand); i compile-time after unrolling
__device__ __forceinline__ int bb_face_cand(const BBox& S, int i, real* P, real& depth) {
  if (i < 4) {
    if (!(fabs(S.pu[i]) <= S.hu && fabs(S.pv[i]) <= S.hv)) return 0;
    P[0] = S.V[i][0]; P[1] = S.V[i][1]; P[2] = S.V[i][2];
  } else if (i < 8) {
    const int m = i - 4;
    const real cu = (m == 1 || m == 2) ? S.hu : -S.hu, cv = (m >= 2) ? S.hv : -S.hv;
    real sgn_min = 0, sgn_max = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int q1 = (q + 1) & 3;
      const real ex = S.pu[q1] - S.pu[q], ey = S.pv[q1] - S.pv[q];
      const real cr = ex * (cv - S.pv[q]) - ey * (cu - S.pu[q]);
      if (q == 0) { sgn_min = cr; sgn_max = cr; }
      else { sgn_min = fmin(sgn_min, cr); sgn_max = fmax(sgn_max, cr); }
    }
    if (!(sgn_min >= 0 || sgn_max <= 0)) return 0;
    real Q[3];
#pragma unroll
    for (int k = 0; k < 3; k++) Q[k] = S.crf[k] + cu * S.ru[k] + cv * S.rv[k];
    const real den = dot3(S.ninc, S.n);
    if (fabs(den) < 1e-12) return 0;
    const real r[3] = {S.cinc[0] - Q[0], S.cinc[1] - Q[1], S.cinc[2] - Q[2]};
    const real t = div_n(dot3(S.ninc, r), den);
#pragma unroll
    for (int k = 0; k < 3; k++) P[k] = Q[k] + t * S.n[k];
  } else {
    const int q = (i - 8) >> 2, m = (i - 8) & 3;
    const int q1 = (q + 1) & 3;
    const real du = S.pu[q1] - S.pu[q], dv = S.pv[q1] - S.pv[q];
    real t;
    if (m < 2) {
      if (fabs(du) < 1e-15) return 0;
      const real bound = m == 0 ? -S.hu : S.hu;
      t = div_n(bound - S.pu[q], du);
      if (!(t > 0 && t < 1)) return 0;
      const real vt = S.pv[q] + t * dv;
      if (!(fabs(vt) < S.hv)) return 0;
    } else {
      if (fabs(dv) < 1e-15) return 0;
      const real bound = m == 2 ? -S.hv : S.hv;
      t = div_n(bound - S.pv[q], dv);
      if (!(t > 0 && t < 1)) return 0;
      const real ut = S.pu[q] + t * du;
      if (!(fabs(ut) < S.hu)) return 0;
    }
#pragma unroll
    for (int k = 0; k < 3; k++) P[k] = S.V[q][k] + t * (S.V[q1][k] - S.V[q][k]);
  }
  const real r[3] = {S.crf[0] - P[0], S.crf[1] - P[1], S.crf[2] - P[2]};
  depth = dot3(S.n, r);
  return depth > 0;
}
__device__ __forceinline__ void bb_face_hit(const BBox& S, const real* P, real depth, Hit& h) {
  h.dist = -depth;
#pragma unroll
  for (int k = 0; k < 3; k++) { h.pos[k] = P[k] + (0.5 * depth) * S.n[k]; h.n[k] = S.sgn * S.n[k]; }
}
__device__ __forceinline__ int bb_edge_hit(const BBox& S, const real* ea, const real* eb, const real* da,
                                           const real* db, Hit& h) {
  const real w[3] = {ea[0] - eb[0], ea[1] - eb[1], ea[2] - eb[2]};
  const real b = dot3(da, db), dd = dot3(da, w), e = dot3(db, w);
  const real den = 1.0 - b * b;
  if (!(den > 1e-12)) return 0;
  const real s = div_n(b * e - dd, den), t = div_n(e - b * dd, den);
  h.dist = -S.pen;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    const real pa = ea[k] + s * da[k], pb = eb[k] + t * db[k];
    h.pos[k] = 0.5 * (pa + pb);
    h.n[k] = S.n[k];
  }
  return 1;
}

// ------------------------------------------------------------ constraint rows
// the solimp sigmoid's general power (cold on the canonical model): one pow pair serves
// both halves; outlined so the inlined fast path stays small
__device__ __noinline__ real impedance_pow(real x, real mid, real pw) {
  const bool lo = x <= mid;
  const real t = pow(lo ? x : 1 - x, pw) / pow(lo ? mid : 1 - mid, pw - 1);
  return lo ? t : 1 - t;
}
// mj_makeImpedance's sigmoid, branch-free in the data (the branches left test model
// constants, wave-uniform): the same values as the early-return form, so several calls can
// interleave their dependency chains
__device__ __forceinline__ real impedance(const gm_model* __restrict__ m, real r) {
  const real dmin = m->solimp[0], dmax = m->solimp[1], width = m->solimp[2];
  const real mid = m->solimp[3], pw = m->solimp[4];
  if (dmin == dmax || width <= 1e-15) return dmin;
  const real x = div_n(fabs(r), width);
  real y;
  if (pw == 2) {   // MuJoCo's default power
    const bool lo = x <= mid;
    const real q = div_n(lo ? x * x : (1 - x) * (1 - x), lo ? mid : 1 - mid);
    y = lo ? q : 1 - q;
  } else if (pw == 1) {
    y = x;
  } else {
    y = impedance_pow(x, mid, pw);
  }
  real imp = dmin + y * (dmax - dmin);
  imp = (x >= 1) ? dmax : imp;
  imp = (x <= 0) ? dmin : imp;
  return imp;
}

// spatial velocity [angular; linear at the world origin] of every body for NVEC dof
// vectors v[0..NVEC) (LDS) into V[0..NVEC): chain prefix scans on the scan lanes plus the
// base, the object's free joint (two vectors scan interleaved: one pass of latency)
template <int CL, int NVEC>
__device__ void body_vel(SharedT<CL>& S, const real* const* v, real (*const* V)[6], const gm_model* __restrict__ m,
                         const GmTopo* __restrict__ T, int lane, bool obj_only = false) {
  // obj_only (wave-uniform): every contact is the object on the ground, so only the
  // object's velocity (and the world's zero) is read: the chain scans are skipped
  const int db = T->dof_base;
  const int grp = T->kl_grp[lane];
  const bool chain = grp >= 0 && grp <= 3;
  const int p = T->kl_cpos[lane];
  const int d = chain ? (grp < 3 ? T->dof_f0[grp] + p - 1 : T->dof_palm) : db;
  real cvb[NVEC][6], s[NVEC][6];
#pragma unroll
  for (int n = 0; n < NVEC; n++) {
    const real vb = v[n][db];
    const real vd = chain ? v[n][d] : 0.0;
#pragma unroll
    for (int k = 0; k < 6; k++) {
      cvb[n][k] = S.cdof[db][k] * vb;
      const real c = S.cdof[d][k];   // (d: the base dof off the chains; loaded, then selected)
      s[n][k] = (chain ? c : 0.0) * vd;
    }
  }
  if (!obj_only) {
#pragma unroll
    for (int off = 1; off < CL; off <<= 1)
#pragma unroll
      for (int n = 0; n < NVEC; n++)
#pragma unroll
        for (int k = 0; k < 6; k++) s[n][k] += row_shr(s[n][k], off);
  }
  const int b = T->lane_body[lane];
  if (chain && !obj_only) {
#pragma unroll
    for (int n = 0; n < NVEC; n++)
#pragma unroll
      for (int k = 0; k < 6; k++) V[n][b][k] = s[n][k] + cvb[n][k];
  } else if (lane == T->lane_base && !obj_only) {
#pragma unroll
    for (int n = 0; n < NVEC; n++)
#pragma unroll
      for (int k = 0; k < 6; k++) V[n][T->body_base][k] = cvb[n][k];
  } else if (b == T->body_obj) {
    const int d0 = T->dof_obj;
    real acc[NVEC][6];
#pragma unroll
    for (int n = 0; n < NVEC; n++)
#pragma unroll
      for (int t = 0; t < 6; t++) acc[n][t] = 0;
#pragma unroll
    for (int k0 = 0; k0 < 6; k0 += 3) {
      real co[18], vk[NVEC][3];   // three object dofs' subspaces and velocities, one batch
#pragma unroll
      for (int k = 0; k < 3; k++) {
#pragma unroll
        for (int t = 0; t < 6; t++) co[6 * k + t] = S.cdof[d0 + k0 + k][t];
#pragma unroll
        for (int n = 0; n < NVEC; n++) vk[n][k] = v[n][d0 + k0 + k];
      }
      keep_n<18>(co);
#pragma unroll
      for (int k = 0; k < 3; k++)
#pragma unroll
        for (int n = 0; n < NVEC; n++)
#pragma unroll
          for (int t = 0; t < 6; t++) acc[n][t] += co[6 * k + t] * vk[n][k];
    }
#pragma unroll
    for (int n = 0; n < NVEC; n++)
#pragma unroll
      for (int t = 0; t < 6; t++) V[n][b][t] = acc[n][t];
  } else if (lane == 0) {
#pragma unroll
    for (int n = 0; n < NVEC; n++)
#pragma unroll
      for (int k = 0; k < 6; k++) V[n][0][k] = 0.0;
  }
  GM_WAVE_SYNC();
}

// J v of contact c's 4 pyramid edges from the body velocities V (n + mu t1, n - mu t1,
// n + mu t2, n - mu t2)
template <int CL>
__device__ __forceinline__ void contact_jv(const SharedT<CL>& S, const real (*V)[6], const gm_model* __restrict__ m,
                                           int c, real* jv) {
  const real* C = S.con[c];
  const int b1 = S.cbody[c][0], b2 = S.cbody[c][1];
  const real pos[3] = {C[1], C[2], C[3]};
  real t1v[3], t2v[3];
  cross3(t1v, V[b1], pos);
  cross3(t2v, V[b2], pos);
  const real v1[3] = {V[b1][3] + t1v[0], V[b1][4] + t1v[1], V[b1][5] + t1v[2]};
  const real v2[3] = {V[b2][3] + t2v[0], V[b2][4] + t2v[1], V[b2][5] + t2v[2]};
  const real dv[3] = {v2[0] - v1[0], v2[1] - v1[1], v2[2] - v1[2]};
  const real n[3] = {C[4], C[5], C[6]}, t1[3] = {C[7], C[8], C[9]};
  real t2[3];
  cross3(t2, n, t1);
  const real mu = C[10];
  const real cn = dot3(n, dv), c1 = dot3(t1, dv), c2 = dot3(t2, dv);
  const real m1 = mu * c1, m2 = mu * c2;
  jv[0] = cn + m1; jv[1] = cn - m1; jv[2] = cn + m2; jv[3] = cn - m2;
}
// pyramid edge direction u_e of contact record C
__device__ __forceinline__ void edge_dir(const real* C, const real* t2, int ed, real* u) {
  const real* t = (ed >> 1) ? t2 : C + 7;
  const real mt[3] = {C[10] * t[0], C[10] * t[1], C[10] * t[2]};
  if (ed & 1) { u[0] = C[4] - mt[0]; u[1] = C[5] - mt[1]; u[2] = C[6] - mt[2]; }
  else { u[0] = C[4] + mt[0]; u[1] = C[5] + mt[1]; u[2] = C[6] + mt[2]; }
}
// K = S Q S^T, S = [skew(p); I]: [A xx yy zz xy xz yz | B row-major | Q xx yy zz xy xz yz]
__device__ __forceinline__ void spatial_K(const real* Q, const real* p, real* K) {
  const real Qm[3][3] = {{Q[0], Q[3], Q[4]}, {Q[3], Q[1], Q[5]}, {Q[4], Q[5], Q[2]}};
  real Bm[3][3];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    real c[3];
    cross3(c, p, Qm[j]);
    Bm[0][j] = c[0]; Bm[1][j] = c[1]; Bm[2][j] = c[2];
  }
  real Am[3][3];
#pragma unroll
  for (int i = 0; i < 3; i++) cross3(Am[i], p, Bm[i]);
  K[0] = Am[0][0]; K[1] = Am[1][1]; K[2] = Am[2][2]; K[3] = Am[0][1]; K[4] = Am[0][2]; K[5] = Am[1][2];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) K[6 + 3 * i + j] = Bm[i][j];
#pragma unroll
  for (int k = 0; k < 6; k++) K[15 + k] = Q[k];
}
__device__ __forceinline__ void symK_mul(const real* K, const real* v, real* y) {
  const real *A = K, *B = K + 6, *Q = K + 15;
  const real w0 = v[0], w1 = v[1], w2 = v[2], l0 = v[3], l1 = v[4], l2 = v[5];
  y[0] = A[0] * w0 + A[3] * w1 + A[4] * w2 + B[0] * l0 + B[1] * l1 + B[2] * l2;
  y[1] = A[3] * w0 + A[1] * w1 + A[5] * w2 + B[3] * l0 + B[4] * l1 + B[5] * l2;
  y[2] = A[4] * w0 + A[5] * w1 + A[2] * w2 + B[6] * l0 + B[7] * l1 + B[8] * l2;
  y[3] = B[0] * w0 + B[3] * w1 + B[6] * w2 + Q[0] * l0 + Q[3] * l1 + Q[4] * l2;
  y[4] = B[1] * w0 + B[4] * w1 + B[7] * w2 + Q[3] * l0 + Q[1] * l1 + Q[5] * l2;
  y[5] = B[2] * w0 + B[5] * w1 + B[8] * w2 + Q[4] * l0 + Q[5] * l1 + Q[2] * l2;
}

// xor butterfly over the wave: every lane ends with the same sum (oracle butterfly64)
__device__ __forceinline__ real wave_sum(real v) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) v = v + __shfl_xor(v, s);
  return v;
}

// H~ v on the tree blocks, lane = dof (oracle smooth_matvec); v, out in LDS
template <int CL>
__device__ void smooth_matvec(SharedT<CL>& S, const GmTopo* __restrict__ T, const real* v, real* out, int lane) {
  if (lane < T->nv) {
    const int d = lane, c = T->dof_grp[d], p = T->dof_p[d];
    real acc;
    if (c >= 0 && c < 3) {
      const real* H = S.Hf[c];
      const int f0 = T->dof_f0[c];
      acc = H[TRI(p, 0)] * v[T->dof_base];
#pragma unroll
      for (int j = 1; j <= CL; j++) {
        const real hv = H[(j <= p) ? TRI(p, j) : TRI(j, p)];
        acc = acc + hv * v[f0 + j - 1];
      }
    } else if (c == GM_GRP_BASE) {
      acc = S.Hbb * v[T->dof_base];
#pragma unroll
      for (int f = 0; f < 3; f++)
#pragma unroll
        for (int q = 1; q <= CL; q++) acc = acc + S.Hf[f][TRI(q, 0)] * v[T->dof_f0[f] + q - 1];
      acc = acc + S.Hp[TRI(1, 0)] * v[T->dof_palm];
    } else if (c == GM_GRP_PALM) {
      acc = S.Hp[TRI(1, 0)] * v[T->dof_base] + S.Hp[TRI(1, 1)] * v[T->dof_palm];
    } else {
      acc = 0;
#pragma unroll
      for (int l = 0; l < 6; l++) {
        const real hv = S.Ho[(l <= p) ? TRI(p, l) : TRI(l, p)];
        acc = acc + hv * v[T->dof_obj + l];
      }
    }
    out[d] = acc;
  }
  GM_WAVE_SYNC();
}

// ------------------------------------------------------------ Newton solve
// Row data lives with its lane: contact c's 4 edges on lane c (D, aref, jar at the
// iterate q, at the Newton point x), motor-lock row r on lane r (its own registers).
struct RowsT {
  real cD, caref[4], cjq[4], cjx[4];   // contact lane
  real lD, laref, ljq, ljx;            // lock lane
  int ldof;
};

// The motor-lock rows (1-dof joint equalities) of the constraint problem: impedance, the
// regulariser R = (1 - d) / d dof_invweight0 and the reference acceleration of each active
// lock, row r on lane r, into S.lrow_* and S.nl.  They need only qpos, qvel and the motion
// subspaces, so crb_rne issues them in its first basic block: their division chains fill
// the scans' latency instead of running as a phase of their own.
template <int CL, bool CAL>
__device__ __forceinline__ void lock_rows(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T, int lane) {
  const real h = CAL ? S.s.dt : m->timestep;
  real tc = m->solref[0];
  if (tc < 2 * h) tc = 2 * h;
  const real dr = m->solref[1], dmax = m->solimp[1];
  const real K = rcp_n(dmax * dmax * tc * tc * dr * dr);
  const real Bd = div_n(2.0, dmax * tc);
  // lock rows: row r (lane r) is the r-th active lock.  The lock behind each row is picked
  // branch-free from the (wave-uniform) active flags and its constants from uniform scalar
  // loads, and the weld's per-axis rows are evaluated side by side: no divergent search
  // loop, no per-lane global loads, three independent dependency chains instead of one.
  int nl = 0, k = 0, d = 0;
  real tran = 0.0;
#pragma unroll
  for (int kk = 0; kk < GM_MAX_LOCK; kk++) {
    const bool act = kk < T->nlock && S.s.lock_active[kk];
    const bool mine = act && nl == lane;
    k = mine ? kk : k;
    d = mine ? m->lock_dof[kk] : d;
    tran = mine ? T->lock_tran[kk] : tran;
    nl += act ? 1 : 0;
  }
  {
    const real pos = S.s.qpos[d] - S.s.lock_q[k];
    const real vel = S.s.qvel[d];
    // the reference's weld on a slide as one row on the dof (oracle constraint_setup):
    // per world axis r the weld row a_r qdot with its own impedance and the weld's
    // regulariser, summed in axis order: D = sum D_r a_r^2, D aref = sum D_r a_r aref_r
    real Da[3], ar[3], av[3];
    bool on[3];
#pragma unroll
    for (int r = 0; r < 3; r++) {
      const real a = S.cdof[d][3 + r];
      av[r] = a;
      on[r] = a != 0.0;
      const real pr = a * pos, vr = a * vel;
      const real imp = impedance(m, pr);
      real Rr = div_n(1 - imp, imp) * tran;
      if (Rr < 1e-15) Rr = 1e-15;
      Da[r] = rcp_n(Rr) * a;
      ar[r] = -Bd * vr - K * imp * pr;
    }
    real De = 0.0, Dar = 0.0;
#pragma unroll
    for (int r = 0; r < 3; r++) {
      De = on[r] ? De + Da[r] * av[r] : De;
      Dar = on[r] ? Dar + Da[r] * ar[r] : Dar;
    }
    // every lane stores (lanes past the active rows into the spare slot GM_MAX_LOCK): no
    // branch, so the whole computation stays in one basic block with the caller's
    const int slot = lane < nl ? lane : GM_MAX_LOCK;
    S.lrow_D[slot] = De;
    S.lrow_aref[slot] = div_n(Dar, De);
    S.lrow_dof[slot] = d;
  }
  S.nl = nl;   // (wave-uniform: every lane stores the same value)
}

// The contact rows of the constraint setup (mj_makeConstraint / mj_makeImpedance for the
// pyramid edges): body velocities at qvel (reference accelerations) and at the warm start
// (the first iterate's J q - aref) into V / V2, one fused pass; then per contact lane the
// edges' D = 1 / R (R = (1 - d) / d diagApprox, diagApprox = tran + mu^2 tran, tran = the two
// bodies' invweight0), their aref and the warm start's J q - aref.  The owner wave runs it
// inside constraint_setup; in a DUO workgroup the helper runs it right after its collider
// (duo_helper: it needs only the contacts, the motion subspaces and qvel / qacc_warm) and
// hands the rows over in LDS (duo_rows) -- the same code on the same operands.
template <int CL, bool CAL>
__device__ __forceinline__ void contact_rows(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T,
                                             int lane, real (*V)[6], real (*V2)[6], real& cD, real* caref, real* jq,
                                             bool& obj_only) {
  const real h = CAL ? S.s.dt : m->timestep;
  real tc = m->solref[0];
  if (tc < 2 * h) tc = 2 * h;
  const real dr = m->solref[1], dmax = m->solimp[1];
  const real K = rcp_n(dmax * dmax * tc * tc * dr * dr);
  const real Bd = div_n(2.0, dmax * tc);
  {
    const real* vv[2] = {S.s.qvel, S.s.qacc_warm};
    real (*VV[2])[6] = {V, V2};
    bool og = true;
    if (lane < S.ncon) {
      const int b1 = S.cbody[lane][0], b2 = S.cbody[lane][1];
      og = (b1 == 0 && b2 == T->body_obj) || (b2 == 0 && b1 == T->body_obj);
    }
    obj_only = __ballot(!og) == 0ull;
    body_vel<CL, 2>(S, vv, VV, m, T, lane, obj_only);
  }
#pragma unroll
  for (int e = 0; e < 4; e++) jq[e] = 0.0;
  cD = 0;
#pragma unroll
  for (int e = 0; e < 4; e++) caref[e] = 0;
  if (lane < S.ncon) {
    const real* C = S.con[lane];
    const int b1 = S.cbody[lane][0], b2 = S.cbody[lane][1];
    const real oiw = S.s.obj_invw[0], biw1 = m->body_invweight0[b1][0], biw2 = m->body_invweight0[b2][0];
    const real iw1 = (b1 == T->body_obj) ? oiw : biw1;
    const real iw2 = (b2 == T->body_obj) ? oiw : biw2;
    const real tran = iw1 + iw2;
    const real mu = C[10];
    const real diag = tran + (mu * mu) * tran;
    const real imp = impedance(m, C[0]);
    real Rr = div_n(1 - imp, imp) * diag;
    if (Rr < 1e-15) Rr = 1e-15;
    cD = rcp_n(Rr);
    real vel[4], jv[4];
    contact_jv<CL>(S, V, m, lane, vel);
    contact_jv<CL>(S, V2, m, lane, jv);
#pragma unroll
    for (int e = 0; e < 4; e++) {
      caref[e] = -Bd * vel[e] - K * imp * C[0];
      jq[e] = jv[e] - caref[e];
    }
  }
}

// DUO workgroups: the contact rows the helper formed (contact_rows), contact-lane-major
template <int CL>
struct DuoRows {
  real cD[GM_MAX_CON], caref[4][GM_MAX_CON], jq[4][GM_MAX_CON];
  int32_t obj_only;
};
template <int CL>
__device__ __forceinline__ DuoRows<CL>* duo_rows() {
  __shared__ DuoRows<CL> r;
  return &r;
}

// constraint setup (mj_makeConstraint / mj_makeImpedance): impedance, the regulariser
// R = (1 - d) / d diagApprox (lock rows: dof_invweight0; pyramid edges:
// tran + mu^2 tran, tran = the two bodies' invweight0), reference accelerations
template <int CL, bool CAL, bool DUO = false>
__device__ void constraint_setup(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T,
                                 int lane, RowsT& R, real* jq, real& jql, bool& obj_only, bool prof = false) {
  unsigned long long t0 = prof ? clock64() : 0;
  (void)t0;
  // lock rows: formed in crb_rne's first block (lock_rows below) and read back here
  const int nl = S.nl;
  R.lD = 0; R.laref = 0; R.ldof = 0;
  if (lane < GM_MAX_LOCK) { R.lD = S.lrow_D[lane]; R.laref = S.lrow_aref[lane]; R.ldof = S.lrow_dof[lane]; }
  if (lane >= nl) { R.lD = 0; R.laref = 0; R.ldof = 0; }
  if (lane == 0) S.nefc = nl + 4 * S.ncon;
#ifdef GM_PHASE_SPLIT_SETUP
  PH(15);   // developer split: lock rows
#endif
  if constexpr (DUO) {
    // formed by the helper wave after its collider (duo_helper), read after the barrier
    const DuoRows<CL>* dr = duo_rows<CL>();
    obj_only = dr->obj_only != 0;
    R.cD = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) { R.caref[e] = 0; jq[e] = 0.0; }
    if (lane < S.ncon) {
      R.cD = dr->cD[lane];
#pragma unroll
      for (int e = 0; e < 4; e++) { R.caref[e] = dr->caref[e][lane]; jq[e] = dr->jq[e][lane]; }
    }
  } else {
    contact_rows<CL, CAL>(S, m, T, lane, S.nw2.V, S.nw2.V2, R.cD, R.caref, jq, obj_only);
  }
  {
    const real qw = S.s.qacc_warm[R.ldof];   // (ldof = 0 off the lock lanes)
    jql = (lane < nl) ? qw - R.laref : 0.0;
  }
  GM_WAVE_SYNC();
#ifdef GM_PHASE_SPLIT_SETUP
  PH(11);   // developer split: the contact rows
#endif
}

// J v - aref for every row at the dof vector v (LDS); into jr (contact) / jl (lock)
template <int CL>
__device__ __forceinline__ void rows_jar(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T, bool obj_only,
                                         const real* v, int lane, const RowsT& R, real* jr, real& jl) {
  {
    const real* vv[1] = {v};
    real (*VV[1])[6] = {S.nw.V};
    body_vel<CL, 1>(S, vv, VV, m, T, lane, obj_only);
  }
  jl = (lane < S.nl) ? v[R.ldof] - R.laref : 0.0;
  if (lane < S.ncon) {
    real jv[4];
    contact_jv<CL>(S, S.nw.V, m, lane, jv);
#pragma unroll
    for (int e = 0; e < 4; e++) jr[e] = jv[e] - R.caref[e];
  } else {
#pragma unroll
    for (int e = 0; e < 4; e++) jr[e] = 0.0;
  }
}

// per-lane partial of a row sum (contact edges in order, then the lane's lock row) and the
// wave butterfly (oracle row_reduce)
__device__ __forceinline__ real row_sum(int lane, int ncon, int nl, const real* tc, real tl) {
  real a = 0.0;
  if (lane < ncon) a = ((tc[0] + tc[1]) + tc[2]) + tc[3];
  if (lane < nl) a = a + tl;
  return wave_sum(a);
}

// The Newton point x = H^-1 rhs for the active pattern (oracle newton_assemble +
// newton_factor_solve).  Lane roles: contact lanes build Q / F; scan lanes (GmTopo
// lane_body) sum their body's contacts and suffix-scan along the chains; factor lanes --
// finger chain rows on 16 f + p (p = 1..CL), border rows [base, obj0..5] on 48..54, the
// palm on 56 -- assemble H and rhs, factor, solve; x goes to S.xs.
#define GM_LANE_PALM_F 56
// RHS_ONLY: stop after the assembly and leave the right-hand side f + J_a^T (D aref)_a in S.xs
// (the capped-solve residual of newton_solve calls it with D aref replaced by the row forces,
// so S.xs = qfrc_smooth + J^T efc)
template <int CL, bool RHS_ONLY = false>
__device__ void newton_point(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T, int lane,
                             const RowsT& R, const bool* act, bool prof) {
  unsigned long long t0 = prof ? clock64() : 0;
  const int ncon = S.ncon, nl = S.nl;
  // ---- contact lanes: Q = sum_e D u u^T and F = sum_e D aref u over the active edges
  if (lane < ncon) {
    const real* C = S.con[lane];
    real t2[3];
    cross3(t2, C + 4, C + 7);
    real Q[6] = {0, 0, 0, 0, 0, 0}, F[3] = {0, 0, 0};
#pragma unroll
    for (int ed = 0; ed < 4; ed++) {
      real u[3];
      edge_dir(C, t2, ed, u);
      const real w = act[ed] ? R.cD : 0.0;
      const real du[3] = {w * u[0], w * u[1], w * u[2]};
      Q[0] += du[0] * u[0]; Q[1] += du[1] * u[1]; Q[2] += du[2] * u[2];
      Q[3] += du[0] * u[1]; Q[4] += du[0] * u[2]; Q[5] += du[1] * u[2];
      const real g = w * R.caref[ed];
      F[0] += g * u[0]; F[1] += g * u[1]; F[2] += g * u[2];
    }
    real* qf = S.nw.QF[lane];
#pragma unroll
    for (int k = 0; k < 6; k++) qf[k] = Q[k];
    qf[6] = F[0]; qf[7] = F[1]; qf[8] = F[2];
  }
  GM_WAVE_SYNC();
  // ---- scan lanes: the body's contacts with the object.  Contacts of gripper bodies with
  // the ground (rare) are added in a second pass below, so the common path keeps one
  // 27-value composite per lane in registers instead of two.
  const int b = T->lane_body[lane];
  real Ko[21], Fo[6];
#pragma unroll
  for (int k = 0; k < 21; k++) Ko[k] = 0;
#pragma unroll
  for (int k = 0; k < 6; k++) Fo[k] = 0;
  bool have_g = false;
  // the lane's (up to two) object pairs' contacts, in pair order, as one loop (one set of
  // accumulator phis instead of one per pair)
  int cs[2] = {0, 0}, ns[2] = {0, 0};
#pragma unroll
  for (int s = 0; s < 2; s++) {
    const int pr = T->lane_opair[lane][s];
    const int pg = T->lane_gpair[lane][s];
    if (pg >= 0 && S.pair_cnt[pg] > 0 && S.pair_off[pg] < ncon) have_g = true;
    if (pr >= 0) {
      const int c0 = S.pair_off[pr];
      int c1 = c0 + S.pair_cnt[pr];
      if (c1 > ncon) c1 = ncon;
      cs[s] = c0;
      ns[s] = c1 > c0 ? c1 - c0 : 0;
    }
  }
  const bool have_o = ns[0] + ns[1] > 0;
  {
    for (int t = 0; t < ns[0] + ns[1]; t++) {
      const int c = t < ns[0] ? cs[0] + t : cs[1] + (t - ns[0]);
      const real* qf = S.nw.QF[c];
      const real pos[3] = {S.con[c][1], S.con[c][2], S.con[c][3]};
      const real sg = (S.cbody[c][1] == b) ? 1.0 : -1.0;
      real Kc[21], Fs[6];
      spatial_K(qf, pos, Kc);
      cross3(Fs, pos, qf + 6);
      Fs[3] = qf[6]; Fs[4] = qf[7]; Fs[5] = qf[8];
#pragma unroll
      for (int k = 0; k < 21; k++) Ko[k] += Kc[k];
#pragma unroll
      for (int k = 0; k < 6; k++) Fo[k] += sg * Fs[k];
    }
  }
  const bool any_g = __ballot(have_g) != 0ull;
  // no gripper body touches the object (wave-uniform): the gripper rows' composites are
  // zero and their Hessian entries are H~'s own
  const bool any_o = __ballot(have_o) != 0ull;
  PH(3);
  // the object's ground contacts (its other contacts reach it through the base composite)
  if (lane == T->lane_obj) {
    real Kgo[21], Fgo[6];
#pragma unroll
    for (int k = 0; k < 21; k++) Kgo[k] = 0;
#pragma unroll
    for (int k = 0; k < 6; k++) Fgo[k] = 0;
    const int pr = T->pair_gobj;
    if (pr >= 0) {
      const int c0 = S.pair_off[pr];
      int c1 = c0 + S.pair_cnt[pr];
      if (c1 > ncon) c1 = ncon;
      for (int c = c0; c < c1; c++) {
        const real* qf = S.nw.QF[c];
        const real pos[3] = {S.con[c][1], S.con[c][2], S.con[c][3]};
        const real sg = (S.cbody[c][1] == T->body_obj) ? 1.0 : -1.0;
        real Kc[21], Fs[6];
        spatial_K(qf, pos, Kc);
        cross3(Fs, pos, qf + 6);
        Fs[3] = qf[6]; Fs[4] = qf[7]; Fs[5] = qf[8];
#pragma unroll
        for (int k = 0; k < 21; k++) Kgo[k] += Kc[k];
#pragma unroll
        for (int k = 0; k < 6; k++) Fgo[k] += sg * Fs[k];
      }
    }
#pragma unroll
    for (int k = 0; k < 21; k++) S.go[k] = Kgo[k];
#pragma unroll
    for (int k = 0; k < 6; k++) S.go[21 + k] = Fgo[k];
  }
  // ---- suffix sums along the chains (composite, like Ic)
  if (any_o) {
#pragma unroll
    for (int off = 1; off < CL; off <<= 1) {
#pragma unroll
      for (int k = 0; k < 21; k++) Ko[k] += row_shl(Ko[k], off);
#pragma unroll
      for (int k = 0; k < 6; k++) Fo[k] += row_shl(Fo[k], off);
    }
  }
  // ---- chain roots (fingers at position 1, the palm) to the stage (which sits after the
  // per-contact Q / F in the union: the ground pass below still reads them)
  {
    const int root = (lane == 1) ? 0 : (lane == 17) ? 1 : (lane == 33) ? 2 : (lane == 49) ? 3 : -1;
    if (root >= 0) {
      real* st = S.st.root[root];
#pragma unroll
      for (int k = 0; k < 21; k++) st[k] = Ko[k];
#pragma unroll
      for (int k = 0; k < 6; k++) st[42 + k] = Fo[k];
    }
  }
  GM_WAVE_SYNC();
  // ---- base composites (the four roots in order) and the object's totals
  if (lane < 27) {
    const int k = lane < 21 ? lane : 42 + lane - 21;
    real acc = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) acc += S.st.root[c][k];
    S.st.comp[k] = acc;
  }
  GM_WAVE_SYNC();
  if (lane < 27) {
    // Koo = KBo + Kgo (21), Fobj = Fgo - FBo (6)
    S.st.oo[lane] = (lane < 21) ? S.st.comp[lane] + S.go[lane] : S.go[lane] - S.st.comp[42 + lane - 21];
  }
  GM_WAVE_SYNC();
  PH(4);
  // ---- H and rhs on the factor lanes
  real h[CL + 1], hb[7], rhs = 0;
#pragma unroll
  for (int j = 0; j <= CL; j++) h[j] = 0;
#pragma unroll
  for (int k = 0; k < 7; k++) hb[k] = 0;
  const int rowf = lane >> 4, p = lane & 15;
  const real* cdb = S.cdof[T->dof_base];
  if (rowf < 3 && p >= 1 && p <= CL) {
    const int d = T->dof_f0[rowf] + p - 1;
    const real* H = S.Hf[rowf];
    if (any_o) {
      real cd[6], y[6], Hr[CL + 1];
#pragma unroll
      for (int k = 0; k < 6; k++) cd[k] = S.cdof[d][k];
#pragma unroll
      for (int j = 0; j <= CL; j++) Hr[j] = H[TRI(p, j)];   // (the row, in range for every p)
      keep_n<CL + 1>(Hr);
      symK_mul(Ko, cd, y);
      // (all CL entries computed and kept for j <= p; the motion subspace of chain position
      // j is lane j's cd, taken by row_newbcast instead of an LDS round trip per entry)
#pragma unroll
      for (int j = 1; j <= CL; j++) {
        real cj[6];
#pragma unroll
        for (int k = 0; k < 6; k++) cj[k] = row_bcast(cd[k], j);
        const real v = Hr[j] + dot6(cj, y);
        keep(v);
        h[j] = (j <= p) ? v : h[j];
      }
      hb[0] = Hr[0] + dot6(cdb, y);
      // the object's six motion subspaces (wave-uniform reads), in two batches of three
#pragma unroll
      for (int k0 = 0; k0 < 6; k0 += 3) {
        real co[18];
#pragma unroll
        for (int k = 0; k < 3; k++)
#pragma unroll
          for (int t = 0; t < 6; t++) co[6 * k + t] = S.cdof[T->dof_obj + k0 + k][t];
        keep_n<18>(co);
#pragma unroll
        for (int k = 0; k < 3; k++) hb[1 + k0 + k] = -dot6(co + 6 * k, y);
      }
      rhs = S.frc[d] + dot6(cd, Fo);
    } else {
      real Hr[CL + 1];
#pragma unroll
      for (int j = 0; j <= CL; j++) Hr[j] = H[TRI(p, j)];
      keep_n<CL + 1>(Hr);
#pragma unroll
      for (int j = 1; j <= CL; j++) h[j] = (j <= p) ? Hr[j] : h[j];
      hb[0] = Hr[0];
      rhs = S.frc[d];
    }
  } else if (lane == GM_LANE_PALM_F && !any_o) {
    h[1] = S.Hp[TRI(1, 1)];
    hb[0] = S.Hp[TRI(1, 0)];
    rhs = S.frc[T->dof_palm];
  } else if (lane == GM_LANE_PALM_F) {
    const int d = T->dof_palm;
    const real* st = S.st.root[3];
    real K0[27], y[6];   // the palm root's composite (21) then its cdof (6), one batch
#pragma unroll
    for (int k = 0; k < 21; k++) K0[k] = st[k];
#pragma unroll
    for (int k = 0; k < 6; k++) K0[21 + k] = S.cdof[d][k];
    keep_n<27>(K0);
    const real* cd = K0 + 21;
    symK_mul(K0, cd, y);
    h[1] = S.Hp[TRI(1, 1)] + dot6(cd, y);
    hb[0] = S.Hp[TRI(1, 0)] + dot6(cdb, y);
#pragma unroll
    for (int k0 = 0; k0 < 6; k0 += 3) {
      real co[18];   // (the object's subspaces, wave-uniform, in two batches)
#pragma unroll
      for (int k = 0; k < 3; k++)
#pragma unroll
        for (int t = 0; t < 6; t++) co[6 * k + t] = S.cdof[T->dof_obj + k0 + k][t];
      keep_n<18>(co);
#pragma unroll
      for (int k = 0; k < 3; k++) hb[1 + k0 + k] = -dot6(co + 6 * k, y);
    }
    rhs = S.frc[d] + dot6(cd, st + 42);
  } else if (lane >= 48 && lane < 55) {
    const int i = lane - 48;
    const real* cp = S.st.comp;
    real yob[6] = {0, 0, 0, 0, 0, 0};
    if (any_o) {
      real KBo[21];
#pragma unroll
      for (int k = 0; k < 21; k++) KBo[k] = cp[k];
      keep_n<21>(KBo);
      symK_mul(KBo, cdb, yob);
    }
    if (i == 0) {
      hb[0] = any_o ? S.Hbb + dot6(cdb, yob) : S.Hbb;
      rhs = any_o ? S.frc[T->dof_base] + dot6(cdb, cp + 42) : S.frc[T->dof_base];
    } else {
      const int k = i - 1;
      real KC[27], yk[6];   // Koo (21) then the row's cdof (6), loaded in one batch
#pragma unroll
      for (int t = 0; t < 21; t++) KC[t] = S.st.oo[t];
#pragma unroll
      for (int t = 0; t < 6; t++) KC[21 + t] = S.cdof[T->dof_obj + k][t];
      keep_n<27>(KC);
      const real* cok = KC + 21;
      symK_mul(KC, cok, yk);
      hb[0] = -dot6(cok, yob);
#pragma unroll
      for (int l0 = 0; l0 < 6; l0 += 3) {
        real co[18];   // three of the object's motion subspaces (wave-uniform), one batch
#pragma unroll
        for (int l = 0; l < 3; l++)
#pragma unroll
          for (int t = 0; t < 6; t++) co[6 * l + t] = S.cdof[T->dof_obj + l0 + l][t];
        keep_n<18>(co);
#pragma unroll
        for (int l = 0; l < 3; l++) {
          const int l2 = l0 + l;
          const real v = S.Ho[TRI(k, l2)] + dot6(co + 6 * l, yk);
          keep(v);
          hb[1 + l2] = (l2 <= k) ? v : hb[1 + l2];
        }
      }
      rhs = S.frc[T->dof_obj + k] + dot6(cok, S.st.oo + 21);
    }
  }
  // ---- contacts of gripper bodies with the ground (wave-uniform, rare): their composite
  // Kg is added to the chain rows' and the base's entries (the object rows do not see it)
  if (__builtin_expect(any_g, 0)) {   // cold: keep it out of the hot code's cache lines
    real Kg[21], Fg[6];
#pragma unroll
    for (int k = 0; k < 21; k++) Kg[k] = 0;
#pragma unroll
    for (int k = 0; k < 6; k++) Fg[k] = 0;
#pragma unroll
    for (int s = 0; s < 2; s++) {
      const int pr = T->lane_gpair[lane][s];
      if (pr < 0) continue;
      const int c0 = S.pair_off[pr];
      int c1 = c0 + S.pair_cnt[pr];
      if (c1 > ncon) c1 = ncon;
      for (int c = c0; c < c1; c++) {
        const real* qf = S.nw.QF[c];
        const real pos[3] = {S.con[c][1], S.con[c][2], S.con[c][3]};
        const real sg = (S.cbody[c][1] == b) ? 1.0 : -1.0;
        real Kc[21], Fs[6];
        spatial_K(qf, pos, Kc);
        cross3(Fs, pos, qf + 6);
        Fs[3] = qf[6]; Fs[4] = qf[7]; Fs[5] = qf[8];
#pragma unroll
        for (int k = 0; k < 21; k++) Kg[k] += Kc[k];
#pragma unroll
        for (int k = 0; k < 6; k++) Fg[k] += sg * Fs[k];
      }
    }
#pragma unroll
    for (int off = 1; off < CL; off <<= 1) {
#pragma unroll
      for (int k = 0; k < 21; k++) Kg[k] += row_shl(Kg[k], off);
#pragma unroll
      for (int k = 0; k < 6; k++) Fg[k] += row_shl(Fg[k], off);
    }
    const int root = (lane == 1) ? 0 : (lane == 17) ? 1 : (lane == 33) ? 2 : (lane == 49) ? 3 : -1;
    if (root >= 0) {
      real* st = S.st.root[root];
#pragma unroll
      for (int k = 0; k < 21; k++) st[21 + k] = Kg[k];
#pragma unroll
      for (int k = 0; k < 6; k++) st[48 + k] = Fg[k];
    }
    GM_WAVE_SYNC();
    const bool chainrow = rowf < 3 && p >= 1 && p <= CL;
    if (lane == GM_LANE_PALM_F) {
#pragma unroll
      for (int k = 0; k < 21; k++) Kg[k] = S.st.root[3][21 + k];
#pragma unroll
      for (int k = 0; k < 6; k++) Fg[k] = S.st.root[3][48 + k];
    } else if (lane == 48) {
#pragma unroll
      for (int k = 0; k < 21; k++) Kg[k] = ((S.st.root[0][21 + k] + S.st.root[1][21 + k]) + S.st.root[2][21 + k]) + S.st.root[3][21 + k];
#pragma unroll
      for (int k = 0; k < 6; k++) Fg[k] = ((S.st.root[0][48 + k] + S.st.root[1][48 + k]) + S.st.root[2][48 + k]) + S.st.root[3][48 + k];
    }
    if (chainrow || lane == GM_LANE_PALM_F || lane == 48) {
      const int d = chainrow ? T->dof_f0[rowf] + p - 1 : lane == 48 ? T->dof_base : T->dof_palm;
      real cd[6], yg[6];
#pragma unroll
      for (int k = 0; k < 6; k++) cd[k] = S.cdof[d][k];
      symK_mul(Kg, cd, yg);
      if (chainrow) {
#pragma unroll
        for (int j = 1; j <= CL; j++)
          if (j <= p) h[j] += dot6(S.cdof[T->dof_f0[rowf] + j - 1], yg);
      } else if (lane == GM_LANE_PALM_F) {
        h[1] += dot6(cd, yg);
      }
      hb[0] += dot6(cdb, yg);
      rhs += dot6(cd, Fg);
    }
  }
  // motor-lock rows (1-dof joint equalities): D on the diagonal, D aref on the rhs
  for (int r = 0; r < nl; r++) {
    const int d = __builtin_amdgcn_readlane(R.ldof, r);
    const real lD = readlane_real(R.lD, r), lR = readlane_real(R.lD * R.laref, r);
    if (T->dof_grp[d] < 3) {
      const int f = T->dof_grp[d], pd = T->dof_p[d];
      if (rowf == f && p == pd) {
#pragma unroll
        for (int j = 1; j <= CL; j++) if (j == pd) h[j] += lD;
        rhs += lR;
      }
    } else if (lane == GM_LANE_PALM_F) {
      h[1] += lD;
      rhs += lR;
    }
  }
  if constexpr (RHS_ONLY) {
    if (rowf < 3 && p >= 1 && p <= CL) S.xs[T->dof_f0[rowf] + p - 1] = rhs;
    else if (lane == GM_LANE_PALM_F) S.xs[T->dof_palm] = rhs;
    else if (lane >= 48 && lane < 55) S.xs[lane == 48 ? T->dof_base : T->dof_obj + lane - 49] = rhs;
    GM_WAVE_SYNC();
    return;
  }
  GM_WAVE_SYNC();   // the stage is read; the factor's transfers reuse the union
  PH(7);
  // ---- factor: finger chains (rows 0..2), pivots CL .. 1
  real invd = 1.0;
  if (lane < 48) {
#pragma unroll
    for (int k = CL; k >= 1; k--) {
      const real hkk = row_bcast(h[k], k);
      const real ihk = rcp_piv(hkk);
      real hk[CL + 1], hkb[7];
#pragma unroll
      for (int j = 1; j < k; j++) hk[j] = row_bcast(h[j], k);
#pragma unroll
      for (int t = 0; t < 7; t++) hkb[t] = row_bcast(hb[t], k);
      const bool upd = p >= 1 && p < k, piv = p == k;
      real Hpk = 0.0;
#pragma unroll
      for (int j = 1; j < k; j++) Hpk = (p == j) ? hk[j] : Hpk;
      const real a = Hpk * ihk;
      const real aa = upd ? a : 0.0;
      if (piv && rowf < 3) {
        real* ub = S.fs.lbub[rowf][k - 1] + 7;
#pragma unroll
        for (int t = 0; t < 7; t++) ub[t] = hb[t];
      }
      // (the pivot row's scaling by 1 / d_k is applied once after the loop: no later step
      // changes the row, whose updates from here on subtract exact zeros)
#pragma unroll
      for (int j = 1; j < k; j++) h[j] = h[j] - hk[j] * aa;
#pragma unroll
      for (int t = 0; t < 7; t++) hb[t] = hb[t] - hkb[t] * aa;
      h[k] = upd ? a : h[k];
      invd = piv ? ihk : invd;
    }
#pragma unroll
    for (int j = 1; j < CL; j++) h[j] = (j < p) ? h[j] * invd : h[j];
#pragma unroll
    for (int t = 0; t < 7; t++) hb[t] = hb[t] * invd;
    if (rowf < 3 && p >= 1 && p <= CL) {
      real* lb = S.fs.lbub[rowf][p - 1];
#pragma unroll
      for (int t = 0; t < 7; t++) lb[t] = hb[t];
    }
  } else if (lane == GM_LANE_PALM_F) {
    const real ih = rcp_piv(h[1]);
    real* pl = S.fs.plb;
#pragma unroll
    for (int t = 0; t < 7; t++) { pl[7 + t] = hb[t]; hb[t] = hb[t] * ih; pl[t] = hb[t]; }
    invd = ih;
  } else if (lane >= 48 && lane < 55) {
    // border rows to the entry transfer: lower triangle, row-major
    const int i = lane - 48;
#pragma unroll
    for (int j = 0; j < 7; j++)
      if (j <= i) S.fs.bbx[i * (i + 1) / 2 + j] = hb[j];
  }
  GM_WAVE_SYNC();
  // Schur complements: one lane per border entry (i, j), elimination order
  if (lane < 28) {
    int i = 0;
#pragma unroll
    for (int t = 1; t < 7; t++) i += (lane >= t * (t + 1) / 2) ? 1 : 0;
    const int j = lane - i * (i + 1) / 2;
    // one partial sum per finger chain: three independent dependent-chains of CL terms
    real acc[3] = {0.0, 0.0, 0.0};
    // (the transfers read four pivots at a time, one batch of loads per group)
#pragma unroll
    for (int k0 = CL; k0 >= 1; k0 -= 4) {
      real lv[24];
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int f = 0; f < 3; f++) {
          const int k = (k0 - q >= 1) ? k0 - q : 1;
          lv[6 * q + 2 * f] = S.fs.lbub[f][k - 1][i];
          lv[6 * q + 2 * f + 1] = S.fs.lbub[f][k - 1][7 + j];
        }
      keep_n<24>(lv);
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int f = 0; f < 3; f++)
          if (k0 - q >= 1) acc[f] = acc[f] + lv[6 * q + 2 * f] * lv[6 * q + 2 * f + 1];
    }
    real v = S.fs.bbx[lane];
    v = (((v - acc[0]) - acc[1]) - acc[2]) - S.fs.plb[i] * S.fs.plb[7 + j];
    S.fs.bbx[lane] = v;
  }
  GM_WAVE_SYNC();
  const int bi = lane - 48;
  const bool border = lane >= 48 && lane < 55;
  if (border) {
#pragma unroll
    for (int j = 0; j < 7; j++)
      if (j <= bi) hb[j] = S.fs.bbx[bi * (bi + 1) / 2 + j];
    // border LDL^T: pivots 6 .. 0 (row 3 lanes 48 + k)
#pragma unroll
    for (int k = 6; k >= 0; k--) {
      const real ihk = rcp_piv(row_bcast(hb[k], k));
      real bk[7];
#pragma unroll
      for (int j = 0; j < k; j++) bk[j] = row_bcast(hb[j], k);
      const bool upd = bi < k, piv = bi == k;
      real Bik = 0.0;
#pragma unroll
      for (int j = 0; j < k; j++) Bik = (bi == j) ? bk[j] : Bik;
      const real a = Bik * ihk;
      const real aa = upd ? a : 0.0;
#pragma unroll
      for (int j = 0; j < k; j++) hb[j] = hb[j] - bk[j] * aa;   // (pivot row scaled after the loop)
      hb[k] = upd ? a : hb[k];
      invd = piv ? ihk : invd;
    }
#pragma unroll
    for (int j = 0; j < 6; j++) hb[j] = (j < bi) ? hb[j] * invd : hb[j];
  }
  PH(14);
  // ---- solve: forward (chains leaf first, border sums, border), D, backward
  real y = rhs;
  if (lane < 48) {
#pragma unroll
    for (int k = CL; k >= 1; k--) {
      const real yk = row_bcast(y, k);
      const real Lc = (p >= 1 && p < k) ? h[k] : 0.0;
      y = y - Lc * yk;
    }
    if (rowf < 3 && p >= 1 && p <= CL) S.fs.ych[rowf][p - 1] = y;
  } else if (lane == GM_LANE_PALM_F) {
    S.fs.ypalm = y;
  }
  GM_WAVE_SYNC();
  if (border) {
    real acc[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int k0 = CL; k0 >= 1; k0 -= 4) {   // (four pivots' transfers per batch of loads)
      real lv[24];
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int f = 0; f < 3; f++) {
          const int k = (k0 - q >= 1) ? k0 - q : 1;
          lv[6 * q + 2 * f] = S.fs.lbub[f][k - 1][bi];
          lv[6 * q + 2 * f + 1] = S.fs.ych[f][k - 1];
        }
      keep_n<24>(lv);
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int f = 0; f < 3; f++)
          if (k0 - q >= 1) acc[f] = acc[f] + lv[6 * q + 2 * f] * lv[6 * q + 2 * f + 1];
    }
    y = (((y - acc[0]) - acc[1]) - acc[2]) - S.fs.plb[bi] * S.fs.ypalm;
#pragma unroll
    for (int k = 6; k >= 0; k--) {
      const real yk = row_bcast(y, k);
      const real Lc = (bi < k) ? hb[k] : 0.0;
      y = y - Lc * yk;
    }
  }
  y = y * invd;
  if (border) {
#pragma unroll
    for (int j = 0; j < 6; j++) {
      const real xj = row_bcast(y, j);
      const real Lr = (j < bi) ? hb[j] : 0.0;
      y = y - Lr * xj;
    }
  }
  // the border solution to every lane (row 3 lanes 48..54)
  real xb[7];
#pragma unroll
  for (int t = 0; t < 7; t++) xb[t] = readlane_real(y, 48 + t);
  if (lane < 48) {
#pragma unroll
    for (int t = 0; t < 7; t++) y = y - hb[t] * xb[t];
#pragma unroll
    for (int j = 1; j < CL; j++) {
      const real xj = row_bcast(y, j);
      const real Lr = (j < p) ? h[j] : 0.0;
      y = y - Lr * xj;
    }
    if (rowf < 3 && p >= 1 && p <= CL) S.xs[T->dof_f0[rowf] + p - 1] = y;
  } else if (lane == GM_LANE_PALM_F) {
#pragma unroll
    for (int t = 0; t < 7; t++) y = y - hb[t] * xb[t];
    S.xs[T->dof_palm] = y;
  } else if (border) {
    S.xs[bi == 0 ? T->dof_base : T->dof_obj + bi - 1] = y;
  }
  GM_WAVE_SYNC();
#ifdef GM_PHASE_SPLIT_NARROW
  PH(14);
#else
  PH(24);
#endif
}

// mj_solNewton restated (oracle newton_solve): warm start, Newton point on the active
// pattern, accept when the pattern at x is unchanged (x is then the exact optimum), else
// an exact line search along x - q; contact forces and the warm start at the end.
template <int CL, bool CAL, bool DUO = false>
__device__ __forceinline__ void newton_solve(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T, int lane,
                             bool prof) {
  unsigned long long t0 = prof ? clock64() : 0;
  RowsT R;
  real jq[4], jql;
  bool obj_only;
  constraint_setup<CL, CAL, DUO>(S, m, T, lane, R, jq, jql, obj_only, prof);
#ifdef GM_PHASE_SPLIT_SETUP
  if (prof) t0 = clock64();   // the split phases above were charged inside; the rest: contact rows
#endif
  PH(11);
  const int ncon = S.ncon, nl = S.nl, nv = T->nv;
  const bool clane = lane < ncon;
  if (lane < nv) S.qacc[lane] = S.s.qacc_warm[lane];
  GM_WAVE_SYNC();
#ifdef GM_PHASE_SPLIT_NARROW
  PH(11);
#else
  PH(12);
#endif
  int it = 0, nls = 0;
  bool capped = true;   // no Newton point accepted within GM_NEWTON_MAXIT iterations
  bool ls_cap = false;  // a line search ran GM_NEWTON_MAXLS evaluations without settling
  const int maxit = (m->newton_maxit > 0 && m->newton_maxit < GM_NEWTON_MAXIT) ? m->newton_maxit : GM_NEWTON_MAXIT;
  for (it = 0; it < maxit; it++) {
    bool act[4];
#pragma unroll
    for (int e = 0; e < 4; e++) act[e] = clane && jq[e] < 0;
    PH(13);
    newton_point<CL>(S, m, T, fresh_lane(), R, act, prof);
    if (prof) t0 = clock64();
    real jx[4], jxl;
    rows_jar<CL>(S, m, T, obj_only, S.xs, lane, R, jx, jxl);
    bool differ = false;
#pragma unroll
    for (int e = 0; e < 4; e++) differ = differ || (clane && ((jx[e] < 0) != act[e]));
    if (__builtin_expect(__ballot(differ) == 0ull, 1)) {
      if (lane < nv) S.qacc[lane] = S.xs[lane];
#pragma unroll
      for (int e = 0; e < 4; e++) jq[e] = jx[e];
      jql = jxl;
      it++;
      capped = false;
      break;
    }
    // exact line search along d = x - q (d overwrites x); H~ q formed when first needed
    // (only iteration 0 reaches here with q unchanged: the oracle does the same)
    if (it == 0) smooth_matvec<CL>(S, T, S.qacc, S.Ma, lane);
    if (lane < nv) S.xs[lane] = S.xs[lane] - S.qacc[lane];
    GM_WAVE_SYNC();
    smooth_matvec<CL>(S, T, S.xs, S.Mv, lane);
    const real xl = S.xs[lane];   // (lanes past nv read the next LDS vector; selected away)
    const real dd = lane < nv ? xl : 0.0;
    const real g0 = wave_sum(lane < nv ? dd * (S.Ma[lane] - S.frc[lane]) : 0.0);
    const real h0 = wave_sum(lane < nv ? dd * S.Mv[lane] : 0.0);
    real dj[4];
#pragma unroll
    for (int e = 0; e < 4; e++) dj[e] = jx[e] - jq[e];
    const real djl = jxl - jql;
    real alpha = 1.0, lo = 0.0, hi = 0.0;
    bool hi_set = false, newton = false, have_prev = false;
    unsigned prev = 0;
    int ls = 0;
    for (; ls < GM_NEWTON_MAXLS; ls++) {
      nls++;
      unsigned pat = 0;
      real tg[4], th[4];
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const real j = jq[e] + alpha * dj[e];
        const bool a = clane && j < 0;
        pat |= (unsigned)a << e;
        tg[e] = a ? (R.cD * j) * dj[e] : 0.0;
        th[e] = a ? (R.cD * dj[e]) * dj[e] : 0.0;
      }
      const real jl = jql + alpha * djl;
      const real tgl = (R.lD * jl) * djl, thl = (R.lD * djl) * djl;   // lock rows: always active
      const bool same_piece = have_prev && __ballot(pat != prev) == 0ull;
      if (newton && same_piece) break;
      const real g = (g0 + alpha * h0) + row_sum(lane, ncon, nl, tg, tgl);
      const real hh = h0 + row_sum(lane, ncon, nl, th, thl);
      if (g == 0.0) break;
      if (g < 0) lo = alpha; else { hi = alpha; hi_set = true; }
      if (!(hh > 0)) break;
      real an = alpha - div_n(g, hh);
      newton = true;
      if (!(an > lo) || (hi_set && !(an < hi))) { an = hi_set ? 0.5 * (lo + hi) : 2.0 * alpha; newton = false; }
      prev = pat;
      have_prev = true;
      alpha = an;
    }
    ls_cap = ls_cap || ls == GM_NEWTON_MAXLS;   // wave-uniform: every exit test above is
    if (lane < nv) {
      S.qacc[lane] = S.qacc[lane] + alpha * S.xs[lane];
      S.Ma[lane] = S.Ma[lane] + alpha * S.Mv[lane];
    }
#pragma unroll
    for (int e = 0; e < 4; e++) jq[e] = jq[e] + alpha * dj[e];
    jql = jql + alpha * djl;
    GM_WAVE_SYNC();
  }
  PH(13);
  // A capped solve (wave-uniform, rare: none in the benchmarks): qacc is no optimum, so what
  // mj_Euler integrates, qfrc_smooth + J^T efc, differs from H~ qacc by the residual
  // r = H~ qacc - qfrc_smooth - J^T efc.  J^T efc is the Newton right-hand side with the row
  // forces in place of D aref (efc = -D jar on the active rows: caref := -jq); H~ qacc is Ma,
  // which the line search of every capped iteration kept up to date.  r goes to S.Mv for
  // euler_damping; the object rows (decoupled from the gripper in M, undamped) take their
  // correction Moo^-1 r right here on lane 0 (oracle/physics.c ldl6_solve, same order).
  if (lane == 0) S.res_valid = capped ? 1 : 0;
  if (capped) {
    RowsT Rc = R;
    bool ac[4];
#pragma unroll
    for (int e = 0; e < 4; e++) { Rc.caref[e] = -jq[e]; ac[e] = clane && jq[e] < 0; }
    Rc.laref = -jql;
    newton_point<CL, true>(S, m, T, fresh_lane(), Rc, ac, false);
    if (lane < nv) S.Mv[lane] = S.Ma[lane] - S.xs[lane];
    GM_WAVE_SYNC();
    if (lane == 0) {
      real A[6][6], x[6];
      for (int k = 0; k < 6; k++)
        for (int l = 0; l <= k; l++) A[k][l] = S.Ho[TRI(k, l)];
      for (int k = 0; k < 6; k++) x[k] = S.Mv[T->dof_obj + k];
      for (int k = 5; k >= 0; k--) {
        const real ik = 1.0 / A[k][k];
        real col[6];
        for (int i = 0; i < k; i++) col[i] = A[k][i];
        for (int i = 0; i < k; i++) {
          const real a = col[i] * ik;
          for (int j = 0; j <= i; j++) A[i][j] = A[i][j] - a * col[j];
          A[k][i] = a;
        }
      }
      for (int k = 5; k >= 0; k--)
        for (int i = 0; i < k; i++) x[i] = x[i] - A[k][i] * x[k];
      for (int k = 0; k < 6; k++) x[k] = x[k] / A[k][k];
      for (int k = 0; k < 6; k++)
        for (int i = 0; i < k; i++) x[k] = x[k] - A[k][i] * x[i];
      for (int k = 0; k < 6; k++) S.Mv[T->dof_obj + k] = x[k];
    }
    GM_WAVE_SYNC();
  }
  // constraint forces at the solution and the contact-frame forces (mj_contactForce)
  real fe[4];
#pragma unroll
  for (int e = 0; e < 4; e++) fe[e] = (clane && jq[e] < 0) ? -(R.cD * jq[e]) : 0.0;
  if (clane) {
    real* C = S.con[lane];
    const real mu = C[10];
    C[11] = ((fe[0] + fe[1]) + fe[2]) + fe[3];
    C[12] = mu * (fe[0] - fe[1]);
    C[13] = mu * (fe[2] - fe[3]);
#pragma unroll
    for (int e = 0; e < 4; e++) S.dbg.efc[nl + 4 * lane + e] = fe[e];
  }
  if (lane < nl) S.dbg.efc[lane] = -(R.lD * jql);
  if (lane < nv) S.s.qacc_warm[lane] = S.qacc[lane];
  if (lane == 0) {
    S.work_nefc += nl + 4 * ncon;
    S.work_newton += it;
    if (capped || ls_cap) S.s.newton_caps += 1;   // (the oracle counts the same, physics.c newton_solve)
    if (prof) { S.tph[28] += nl + 4 * ncon; S.tph[30] += it; S.tph[31] += nls; }
  }
  GM_WAVE_SYNC();
}

// ------------------------------------------------------------ mj_Euler's implicit damping
// MuJoCo 2.1.5's actuator order (gm_model::mujoco_actuators): the PD forces are explicit
// (mass_and_forces), the constraint solve runs on M + armature, and mj_Euler integrates
// qacc_e = (M + h D)^-1 (qfrc_smooth + qfrc_constraint) = qacc - (M + h D)^-1 (h D qacc)
// (M qacc = qfrc_smooth + qfrc_constraint at the solve's optimum).  The gripper's M + h D on
// the factor lanes: each finger chain block leaf-first on its DPP row with the base as the
// single border column (row_newbcast pivots, as newton_point with a one-wide border), the
// palm one pivot; the base pivot's two sums (Schur complement sum lb ub, forward sum lb y)
// are one two-value segmented scan per DPP row plus the three row totals and the palm read
// back as scalars, so the base solve is computed wave-uniformly.  The object has no damping
// and no coupling to the gripper in M: its rows take no correction.  qacc_e goes to S.xs
// (free after the solve); oracle/physics.c euler_damping restates it lane for lane.
// The factor half: L (chain rows, scaled), lb (the base column, scaled), 1 / d on the pivot
// lanes, and the base pivot's Schur sum (returned, wave-uniform).  It reads only M's blocks
// (mass_and_forces) and the damping, so a DUO workgroup's helper wave runs it during the
// constraint solve (duo_helper) and hands it over in LDS; the one-wave kernel keeps it in
// registers.  The same operations either way.
template <int CL>
__device__ __forceinline__ real euler_factor(const SharedT<CL>& S, const GmTopo* __restrict__ T, real h, int lane,
                                             real (&L)[CL + 1], real& lb, real& invd) {
  const int rowf = lane >> 4, p = lane & 15;
  const bool chainrow = rowf < 3 && p >= 1 && p <= CL;
  const bool palm = lane == GM_LANE_PALM_F;
  lb = 0.0;
#pragma unroll
  for (int j = 0; j <= CL; j++) L[j] = 0.0;
  if (chainrow) {
    const real* H = S.Hf[rowf];
    const int d = T->dof_f0[rowf] + p - 1;
    const real hd = h * T->dof_damp[d];
    {
      // the full symmetric row (M's upper part read from its lower triangle): the factor
      // then takes each pivot's column entry from the lane's own row
      real Hr[CL + 1];
#pragma unroll
      for (int j = 1; j <= CL; j++) Hr[j] = H[j <= p ? TRI(p, j) : TRI(j, p)];
      Hr[0] = Hr[1];
      keep_n<CL + 1>(Hr);
#pragma unroll
      for (int j = 1; j <= CL; j++) L[j] = Hr[j];
    }
#pragma unroll
    for (int j = 1; j <= CL; j++) L[j] = (j == p) ? L[j] + hd : L[j];
    lb = H[TRI(p, 0)];
  } else if (palm) {
    const int d = T->dof_palm;
    const real hd = h * T->dof_damp[d];
    L[1] = S.Hp[TRI(1, 1)] + hd;
    lb = S.Hp[TRI(1, 0)];
  }
  invd = 1.0;
  real ub = 0.0;
  if (lane < 48) {
#pragma unroll
    for (int k = CL; k >= 1; k--) {
      const real ihk = rcp_piv(row_bcast(L[k], k));
      real hk[CL + 1];
#pragma unroll
      for (int j = 1; j < k; j++) hk[j] = row_bcast(L[j], k);
      const real hkb = row_bcast(lb, k);
      const bool upd = p >= 1 && p < k, piv = p == k;
      const real a = L[k] * ihk;   // (the lane's own row holds the pivot column: full symmetric rows)
      const real aa = upd ? a : 0.0;
      ub = piv ? lb : ub;
#pragma unroll
      for (int j = 1; j < k; j++) L[j] = L[j] - hk[j] * aa;   // (pivot row scaled after the loop)
      lb = lb - hkb * aa;
      L[k] = upd ? a : L[k];
      invd = piv ? ihk : invd;
    }
#pragma unroll
    for (int j = 1; j < CL; j++) L[j] = (j < p) ? L[j] * invd : L[j];
    lb = lb * invd;
  } else if (palm) {
    const real ih = rcp_piv(L[1]);
    ub = lb;
    lb = lb * ih;
    invd = ih;
  }
  // the base pivot's Schur sum: per DPP row an inclusive scan of lb ub (lane 15 of the row
  // holds the row total; lanes outside the chain hold zeros), then rows 0, 1, 2 and the palm
  const bool part = chainrow || palm;
  real s1 = part ? lb * ub : 0.0;
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) {
    const real t1 = row_shr(s1, off);
    s1 += t1;
  }
  return ((readlane_real(s1, 15) + readlane_real(s1, 31)) + readlane_real(s1, 47)) + readlane_real(s1, 56);
}

// The solve half: qacc_e = qacc - (M + h D)^-1 (h D qacc [- r on a capped solve]) into S.xs.
template <int CL>
__device__ __forceinline__ void euler_solve(SharedT<CL>& S, const GmTopo* __restrict__ T, real h, int lane,
                                            const real (&L)[CL + 1], real lb, real invd, real sch) {
  const int rowf = lane >> 4, p = lane & 15;
  const bool chainrow = rowf < 3 && p >= 1 && p <= CL;
  const bool palm = lane == GM_LANE_PALM_F;
  const bool res = S.res_valid != 0;   // a capped solve's residual in S.Mv (newton_solve)
  real y = 0.0;
  if (chainrow) {
    const int d = T->dof_f0[rowf] + p - 1;
    const real hd = h * T->dof_damp[d];
    y = hd * S.qacc[d];
    if (res) y = y + S.Mv[d];
  } else if (palm) {
    const int d = T->dof_palm;
    const real hd = h * T->dof_damp[d];
    y = hd * S.qacc[d];
    if (res) y = y + S.Mv[d];
  }
  // the base row (wave-uniform: one scalar dof)
  const int db = T->dof_base;
  const real hdb = h * T->dof_damp[db];
  const real bb = S.Hbb + hdb;
  const real yb0 = res ? hdb * S.qacc[db] + S.Mv[db] : hdb * S.qacc[db];
  if (lane < 48) {
    // forward over the chains, leaf first
#pragma unroll
    for (int k = CL; k >= 1; k--) {
      const real yk = row_bcast(y, k);
      const real Lc = (p >= 1 && p < k) ? L[k] : 0.0;
      y = y - Lc * yk;
    }
  }
  // the base pivot's forward sum, as the Schur sum (euler_factor)
  const bool part = chainrow || palm;
  real s2 = part ? lb * y : 0.0;
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) {
    const real t2 = row_shr(s2, off);
    s2 += t2;
  }
  const real fs = ((readlane_real(s2, 15) + readlane_real(s2, 31)) + readlane_real(s2, 47)) + readlane_real(s2, 56);
  const real xb = (yb0 - fs) * rcp_piv(bb - sch);
  // back substitution: D^-1, the border column, then the chains root -> leaf
  y = y * invd;
  y = y - lb * xb;
  if (lane < 48) {
#pragma unroll
    for (int j = 1; j < CL; j++) {
      const real xj = row_bcast(y, j);
      const real Lr = (j < p) ? L[j] : 0.0;
      y = y - Lr * xj;
    }
  }
  if (chainrow) {
    const int d = T->dof_f0[rowf] + p - 1;
    S.xs[d] = S.qacc[d] - y;
  } else if (palm) {
    S.xs[T->dof_palm] = S.qacc[T->dof_palm] - y;
  } else if (lane == 48) {
    S.xs[db] = S.qacc[db] - xb;
  } else if (lane >= 57 && lane < 63) {
    const int d = T->dof_obj + lane - 57;
    S.xs[d] = res ? S.qacc[d] - S.Mv[d] : S.qacc[d];
  }
  GM_WAVE_SYNC();
}

template <int CL>
__device__ __forceinline__ void euler_damping(SharedT<CL>& S, const GmTopo* __restrict__ T, real h, int lane) {
  real L[CL + 1], lb, invd;
  const real sch = euler_factor<CL>(S, T, h, lane, L, lb, invd);
  euler_solve<CL>(S, T, h, lane, L, lb, invd, sch);
}
