// gm_kernels.hip -- the MI355X (gfx950) batched env-step hot path.
//
// One 64-lane workgroup (one wavefront) per env.  A launch runs a whole
// MjClass::action_step() (mjclass.cpp:1483-1508): S = sim_steps_per_action
// physics substeps, each = MuJoCo-style mj_step1 / control / mj_step2
// (myfunctions.cpp:1873-1898) + after_step/update_all (1900-1908, 2110-2284)
// + monitor_sensors (mjclass.cpp:741-898), then sense_gripper_state,
// update_env, get_observation, is_done and reward -- without leaving the chip.
// Per-env state is moved HBM -> LDS once at entry and back once at exit; all
// per-substep working data (kinematics, mass matrix, contacts, constraint
// rows) stays in LDS / VGPRs.  Lane mapping per stage:
//   - kinematic chains (3 fingers, palm, object): one lane per chain
//   - mass-matrix rows, bias/passive/actuator forces: one lane per dof
//   - collision: one lane per candidate geom pair (63 pairs <= 64 lanes)
//   - constraint rows (pyramid edges + motor locks): one lane per row; the
//     row's Delassus column A[:, j] lives in that lane's VGPRs and projected
//     Gauss-Seidel broadcasts each row's update with v_readlane (no LDS, no
//     reductions in the inner loop)
//   - reference scalar logic (stepper in fp64, events, RNG): lane 0
// The algorithm is the engine spec restated in oracle/oracle.c (fp64); this
// file is the fp64 device implementation of the same spec (MuJoCo's mjtNum is double),
// with fp32 only where the reference itself uses float (sensor windows, observations).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "gm_state.h"
#include "gm_math.h"
#include "gm_policy_net.h"

#define NT 64
// Phase boundary inside one env's physics.  Every kernel that runs the substep is launched
// with one 64-lane wavefront per workgroup (NT), and a wave's LDS operations complete in
// issue order, so a lane's read issued after another lane's write sees it: the boundary
// only has to stop the compiler moving LDS accesses across it.  __syncthreads' workgroup
// fence is lowered to an s_waitcnt lgkmcnt(0) drain at every boundary, stalling the wave
// on loads whose results it does not yet need.
#define GM_WAVE_SYNC() do { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); \
                            __builtin_amdgcn_wave_barrier(); } while (0)
// Synchronisation of the env's own work, which one wave does: __syncthreads' fences around
// a wave barrier instead of s_barrier.  For the 64-thread workgroups this is what
// __syncthreads lowers to anyway; in a DUO workgroup (gm_step_kernel<.., true>: a second,
// helper wave runs the collider concurrently, duo_helper) the helper is parked at its own
// s_barrier handshake and must not be counted by the owner wave's bookkeeping syncs.
#define GM_ENV_SYNC() do { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); \
                           __builtin_amdgcn_wave_barrier(); \
                           __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup"); } while (0)
// The lane id, opaque to the compiler: each phase derives its lane predicates (chain row,
// border, contact lane, ...) from its own copy, so they are recomputed per phase instead of
// being computed once per substep and held live (in spilled SGPR pairs) across all of them.
__device__ __forceinline__ int fresh_lane() {
  int lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  return lane;
}
// Pins a value's computation to the current block: the optimizer otherwise sinks the
// operands of a select or a conditional store (LDS loads, dot products) into a divergent
// branch per entry, each with its own load -> wait -> use chain.
__device__ __forceinline__ void keep(double x) { asm volatile("" ::"v"(x)); }
// ... and a batch of up to 13 values at once: their loads are all issued before the one
// wait (the scheduler otherwise issues each just before its use, one latency per entry)
template <int N>
__device__ __forceinline__ void keep_n(const double* a) {
  static_assert(N >= 1 && N <= 28, "keep_n: 1..28 values");
#define GM_K(i) "v"(a[(i) < N ? (i) : 0])
  if constexpr (N <= 13) {
    asm volatile("" ::GM_K(0), GM_K(1), GM_K(2), GM_K(3), GM_K(4), GM_K(5), GM_K(6), GM_K(7), GM_K(8), GM_K(9),
                 GM_K(10), GM_K(11), GM_K(12));
  } else {
    asm volatile("" ::GM_K(0), GM_K(1), GM_K(2), GM_K(3), GM_K(4), GM_K(5), GM_K(6), GM_K(7), GM_K(8), GM_K(9),
                 GM_K(10), GM_K(11), GM_K(12), GM_K(13), GM_K(14), GM_K(15), GM_K(16), GM_K(17), GM_K(18),
                 GM_K(19), GM_K(20), GM_K(21), GM_K(22), GM_K(23), GM_K(24), GM_K(25), GM_K(26), GM_K(27));
  }
#undef GM_K
}
#define GM_CQ_NB 16      // priority buckets per XCD of the chunked env-step (gm_step_kernel)
#define GM_BB_SLOTS 18   // box-box hit slots in the LDS union (18 x 256 B; SharedT asserts it fits
                         // inside the union's CL-independent chain-root stage, so it never grows LDS)
// gm_step_kernel is instantiated per finger chain length (CL = n_seg + 2) so every chain
// recursion is unrolled into registers; GM_NSEG_LIST is the set compiled in.
#ifndef GM_NSEG_LIST
#define GM_NSEG_LIST X(5) X(6) X(7) X(8) X(9) X(10)
#endif
#define CLMAX (GM_MAX_SEG + 2)
#define TRI(p, q) ((p) * ((p) + 1) / 2 + (q))
#define TRIF ((CLMAX + 1) * (CLMAX + 2) / 2)
#define CW (CL + 8)   // compact row: obj[6], base, chain[CL] (+1 scratch slot); needs CL in scope
#define PI_F 3.14159265358979f

// `real` is the dynamics type: fp64, MuJoCo's mjtNum.  Kinematics, dynamics, collision
// geometry and the PGS solve all run in it (see DESIGN.md "Precision").
typedef double real;
// Env-step bookkeeping (sense / events / obs / done / reward) is inlined into the kernel;
// the substep loop is one outlined call per env-step (substep_loop).
#define GM_EPI_ATTR __device__

struct DebugOut {
  int32_t* ncon;      // [n_envs]
  double* contact;    // [n_envs][GM_MAX_CON][16]
  double* efc_force;  // [n_envs][GM_MAX_EFC]
  double* qacc;       // [n_envs][GM_MAX_DOF]
  unsigned long long* phase;   // [n_envs][GM_NPHASE] shader-clock cycles per phase (profiling)
  int32_t* nefc;      // [n_envs]
  double* wrench;     // [n_envs][6] the live object's cfrc_ext, [force; torque]
};
#define GM_NPHASE 32   // 0-27 shader clocks (see gmx.env PHASES), 28: sum of nefc, 29: substeps running MPR,
                       // 30: Newton iterations, 31: line-search evaluations

// Per-env LDS image, sized for the compile-time finger chain length CL = n_seg + 2:
// NB = 3 CL + 4 bodies (world, base, 3 x CL finger links, palm, object),
// NV = 3 CL + 8 dofs (base, 3 x CL, palm, free object).  gm_create checks the model.
template <int CL>
struct __align__(16) SharedT {
  static constexpr int NB = 3 * CL + 4;
  static constexpr int NV = 3 * CL + 8;
  static constexpr int TRIC = (CL + 1) * (CL + 2) / 2;
  GmEnvHot s;                     // the env's state minus its sensor windows
  real lock_pre[GM_MAX_LOCK];     // pre-integration qpos of the lock dofs (weld re-anchoring)
  real lrow_D[GM_MAX_LOCK + 1], lrow_aref[GM_MAX_LOCK + 1];   // lock rows (lock_rows; + a spare slot)
  int32_t lrow_dof[GM_MAX_LOCK + 2];
  real qacc[NV];                  // the Newton iterate; the substep's qacc at the end
  real xs[NV];                    // the Newton point x (line search: the step d = x - q)
  real Ma[NV], Mv[NV];            // H~ q and H~ d
  real xpos[NB][3];
  real xquat[NB][4];   // normalised body orientations; xmat = quat2mat(xquat)
  real Hf[3][TRIC], Hp[3], Ho[21], Hbb;   // H~ tree blocks (finger rows p = 0 base .. CL)
  real cdof[NV][6];
  real frc[NV];                   // smooth force: passive + PD actuation - bias
  real go[27];                    // the object's ground-contact K (21) and force (6)
  // contact record: dist, pos[3], normal[3], t1[3] (t2 = normal x t1), mu, force[3]
  // (contact frame, after the solve)
  real con[GM_MAX_CON][14];
  int16_t cgeom[GM_MAX_CON][2];   // canonical (geom1, geom2)
  int16_t cbody[GM_MAX_CON][2];   // their bodies
  int16_t pair_off[GM_MAX_PAIR], pair_cnt[GM_MAX_PAIR];   // contact slots of each candidate pair
  // LDS shared in time: the dynamics scratch is dead once H~ and the forces are formed; the
  // Newton stages then reuse it (body velocities + per-contact Q / F; the chain-root stage;
  // the factor's transfers; the debug copy of the row forces)
  union {
    struct {                  // kinematics .. mass matrix
      union {                 // composite inertia accumulates in place over cinert
        real cinert[NB][10];
        real Ic[NB][10];
      };
      real cfrc[NB][6];
      real chain_f[5][6], chain_I[5][10];   // chain-root sums for the base body
    };
    struct { real QF[GM_MAX_CON][9]; real V[NB][6]; } nw;
    struct { real V[NB][6]; real V2[NB][6]; } nw2;   // setup: qvel and warm-start velocities
    // the chain-root stage sits after the per-contact Q / F (the ground pass re-reads them)
    struct { real qf_[GM_MAX_CON][9]; real root[4][54]; real comp[54]; real oo[27]; } st;
    struct { real lbub[3][CL][14]; real plb[14]; real bbx[28]; real ych[3][CL]; real ypalm; } fs;
    struct { real efc[GM_MAX_EFC]; } dbg;
    // collision: the face-clipped box-box hits of pass 1 (point, depth), one slot of 8 per
    // face-case lane in lane order, for pass 2 to write without re-deriving the manifold
    struct { real hit[GM_BB_SLOTS][8][4]; } cl;
  };
  static_assert(sizeof(real[GM_BB_SLOTS][8][4]) <= sizeof(real) * (GM_MAX_CON * 9 + 4 * 54 + 54 + 27),
                "box-box hit slots must fit inside the chain-root stage (st): they may not grow the union");
  int32_t ncon, nefc, nl, overflow;
  int32_t res_valid;              // newton_solve: a capped solve's residual sits in Mv (euler_damping)
  int32_t duo_cmd;                // DUO workgroups: 1 = the helper wave runs this substep's collider, 0 = exit
  int32_t work_nefc, work_mpr, work_newton;   // this env-step's rows / MPR substeps / Newton iterations
  int32_t stp_fixed;              // update_all: `next` is a fixed point of the stepper this env-step (see there)
  float forces[32];            // extract_forces_faster results (see extract_forces)
  int32_t have_forces;
  float gauge_tmp[3];
  int32_t bend_ready;             // monitor_sensors: the bending gauges read this substep
  double next_read;               // substep_loop: sim time after which a sensor becomes ready
  unsigned long long tph[GM_NPHASE];
  GmEnvState* gs;                 // the env's record in HBM (sensor windows read / written there)
};

// per-phase shader-clock accounting (gm_step_profiled); needs `prof`, `lane`, `t0` in scope
#define PH(k) do { MARK(k); if (__builtin_expect(prof, 0)) { unsigned long long t_ = clock64(); if (lane == 0) S.tph[k] += t_ - t0; t0 = t_; } } while (0)
// developer marker for static per-phase instruction counts (GM_ISA_MARKERS builds: an
// s_nop 15 / s_nop k pair at every PH(k) in the disassembly)
#ifdef GM_ISA_MARKERS
#define MARK(k) asm volatile("s_nop 15\n\ts_nop " #k)
#else
#define MARK(k) do { } while (0)
#endif
// developer split of the narrowphase (GM_PHASE_SPLIT_NARROW builds): each collider branch
// charges its own clocks to slot k from its first active lane (the branches are divergent)
#ifdef GM_PHASE_SPLIT_NARROW
#define NB_BEGIN() const unsigned long long tb_ = prof ? clock64() : 0
#define NB_END(k) do { if (prof) { const unsigned long long te_ = clock64(); \
    if (lane == (int)__builtin_ctzll(__ballot(1))) S.tph[k] += te_ - tb_; } } while (0)
#else
#define NB_BEGIN() do { } while (0)
#define NB_END(k) do { } while (0)
#endif

// ------------------------------------------------------------ small math
// Correctly rounded fp64 sqrt, reciprocal and quotient on the compiler's own expansions
// (v_rsq_f64 / v_rcp_f64 and the same FMA refinement steps, operation for operation) minus
// their range pre-/post-scaling and special-value fix-ups, which cost a third of the
// instructions and sit on the dependent chain.  Bit-identical to sqrt(x), 1.0 / b and a / b
// wherever the scaling is inactive: x >= 2^-767 or x == +-0; |a|, |b|, |a / b| roughly
// inside [2^-900, 2^900] -- every call site's operands are lengths in metres, masses,
// pivots and contact quantities.  (b == 0 gives NaN where the library gives inf; every
// caller guards its zero case or is in a blown-up state already.)  -DGM_LIBM_DIVSQRT
// selects the library operations.
#ifndef GM_LIBM_DIVSQRT
__device__ __forceinline__ double sqrt_n(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = y * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  double d = fma(-g, g, x);
  h = fma(h, r, h);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  g = fma(d, h, g);
  return x == 0.0 ? x : g;
}
// 1 / sqrt(x) for normal x > 0: v_rsq_f64 and two Newton steps (normalising directions in
// the physics substep); rcp_piv: a factor pivot's reciprocal, two Newton steps without the
// final correction.  The calibration build (GM_CAL_TU: stability verdicts compared with the
// oracle candidate for candidate) takes the correctly rounded forms instead.
#ifndef GM_CAL_TU
__device__ __forceinline__ double rsq_n(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  double e = fma(-hx * y, y, 0.5);
  y = fma(y, e, y);
  e = fma(-hx * y, y, 0.5);
  return fma(y, e, y);
}
#endif
__device__ __forceinline__ double rcp_refined(double b) {
  double r = __builtin_amdgcn_rcp(b);
  double e = fma(-b, r, 1.0);
  r = fma(r, e, r);
  e = fma(-b, r, 1.0);
  return fma(r, e, r);
}
__device__ __forceinline__ double rcp_n(double b) {
  const double r = rcp_refined(b);
  return fma(fma(-b, r, 1.0), r, r);
}
__device__ __forceinline__ double div_n(double a, double b) {
  const double r = rcp_refined(b);
  const double q = a * r;
  return fma(fma(-b, q, a), r, q);
}
#ifdef GM_CAL_TU
__device__ __forceinline__ double rsq_n(double x) { return rcp_n(sqrt_n(x)); }
__device__ __forceinline__ double rcp_piv(double b) { return rcp_n(b); }
#else
__device__ __forceinline__ double rcp_piv(double b) { return rcp_refined(b); }
#endif
#else
__device__ __forceinline__ double sqrt_n(double x) { return sqrt(x); }
__device__ __forceinline__ double rsq_n(double x) { return 1.0 / sqrt(x); }
__device__ __forceinline__ double rcp_piv(double b) { return 1.0 / b; }
__device__ __forceinline__ double rcp_n(double b) { return 1.0 / b; }
__device__ __forceinline__ double div_n(double a, double b) { return a / b; }
#endif

__device__ __forceinline__ void ld3(float* r, const double* a) { r[0] = (float)a[0]; r[1] = (float)a[1]; r[2] = (float)a[2]; }
__device__ __forceinline__ void ld3(double* r, const double* a) { r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; }
__device__ __forceinline__ void ld4(double* r, const double* a) { r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3]; }
__device__ __forceinline__ void ld4(float* r, const double* a) { r[0] = (float)a[0]; r[1] = (float)a[1]; r[2] = (float)a[2]; r[3] = (float)a[3]; }

#include "gm_fphelpers.inc"
template <int CL>
__device__ __forceinline__ void body_R(const SharedT<CL>& S, int b, real* R) {
  const real q[4] = {S.xquat[b][0], S.xquat[b][1], S.xquat[b][2], S.xquat[b][3]};
  quat2mat(R, q);
}   // (one definition: ADL on SharedT would make a second one ambiguous)

// ------------------------------------------------------------ topology helpers
// chain c: 0..2 finger, 3 palm, 4 object.  Chain lengths (positions >= 1).
__device__ __forceinline__ int chain_len(const GmTopo* T, int c) { return c < 3 ? T->CL : (c == 3 ? 1 : 6); }
__device__ __forceinline__ int chain_body(const GmTopo* T, int c, int p) {
  if (c < 3) return T->body_f0[c] + p - 1;
  if (c == 3) return T->body_palm;
  return T->body_obj;
}
__device__ __forceinline__ int chain_dof(const GmTopo* T, int c, int p) {
  if (c < 3) return T->dof_f0[c] + p - 1;
  if (c == 3) return T->dof_palm;
  return T->dof_obj + p;   // object uses positions 0..5
}
// H/L storage accessor: chain c, positions p >= q (object: 0..5, others: 0 = base)

// ============================================================ kinematics
// mj_kinematics restated (oracle.c fk): phase A, one lane per body, the hinge joint
// rotations (the only transcendental work) ; phase B, one lane per chain, the pose
// recursion root -> leaf entirely in registers (chain length compile-time, unrolled,
// every model constant load independent of the recursion) ; phase C, one lane per
// body / dof / geom: rotation matrices, world-origin spatial inertias, motion
// subspaces, geom poses.
struct Pose { real p[3], q[4], R[9]; };


// Segmented-scan shuffles inside a 16-lane DPP row (chains live on the scan lanes of
// GmTopo::lane_body): row_shr / row_shl by a compile-time distance, 0 shifted in at the
// row edge.  A VALU op with a DPP modifier, no LDS round trip (ds_bpermute).
template <int CTRL>
__device__ __forceinline__ real dpp_move(real x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// value from the lane `off` positions lower in the row (off in 1, 2, 4, 8)
__device__ __forceinline__ real row_shr(real x, int off) {
  switch (off) {
    case 1: return dpp_move<0x111>(x);
    case 2: return dpp_move<0x112>(x);
    case 4: return dpp_move<0x114>(x);
    default: return dpp_move<0x118>(x);
  }
}
// value from the lane `off` positions higher in the row
__device__ __forceinline__ real row_shl(real x, int off) {
  switch (off) {
    case 1: return dpp_move<0x101>(x);
    case 2: return dpp_move<0x102>(x);
    case 4: return dpp_move<0x104>(x);
    default: return dpp_move<0x108>(x);
  }
}
// row_newbcast is the one DPP control the 64-bit data path takes (gfx90a+ DP-ALU DPP):
// one v_mov_b64_dpp instead of two 32-bit halves
template <int CTRL>
__device__ __forceinline__ real dpp_bcast64(real x) {
  return __builtin_amdgcn_update_dpp(0.0, x, CTRL, 0xF, 0xF, true);
}
// value of position k of this lane's 16-lane DPP row (row_newbcast:k), k compile-time
// after unrolling
__device__ __forceinline__ real row_bcast(real x, int k) {
  switch (k) {
    case 0: return dpp_bcast64<0x150>(x);
    case 1: return dpp_bcast64<0x151>(x);
    case 2: return dpp_bcast64<0x152>(x);
    case 3: return dpp_bcast64<0x153>(x);
    case 4: return dpp_bcast64<0x154>(x);
    case 5: return dpp_bcast64<0x155>(x);
    case 6: return dpp_bcast64<0x156>(x);
    case 7: return dpp_bcast64<0x157>(x);
    case 8: return dpp_bcast64<0x158>(x);
    case 9: return dpp_bcast64<0x159>(x);
    case 10: return dpp_bcast64<0x15A>(x);
    case 11: return dpp_bcast64<0x15B>(x);
    case 12: return dpp_bcast64<0x15C>(x);
    case 13: return dpp_bcast64<0x15D>(x);
    case 14: return dpp_bcast64<0x15E>(x);
    default: return dpp_bcast64<0x15F>(x);
  }
}
__device__ __forceinline__ real readlane_real(real x, int l) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane((int)b, l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__host__ __device__ constexpr int gm_pair_batches(int CL) { return CL <= 10 ? 1 : 2; }

// The physics substep (kinematics .. integrate, the collider and the constraint solver)
// is compiled with FMA contraction: its dot products and small matrix products issue as
// fused multiply-adds (fewer fp64 instructions and shorter dependent chains, -11 % kernel
// time).  The oracle evaluates the same expressions unfused, so device and oracle physics
// agree to ~1e-12 per substep instead of bit for bit (tests/test_grasp_parity.py bounds);
// everything after the namespace -- stepper, sensors, events, observations, resets and
// spawns -- keeps contraction off and stays bit-exact.  The calibration build (gm_calib.hip)
// keeps it off too: its timestep search compares stability verdicts at the edge of
// stability, candidate for candidate with the oracle.
#ifdef GM_CAL_TU
#pragma clang fp contract(off)
#else
#pragma clang fp contract(fast)
#endif
namespace gmf {
#define GM_FP_PHYSICS
#include "gm_fphelpers.inc"
#undef GM_FP_PHYSICS

template <int CL>
__device__ __forceinline__ void kinematics(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T, int lane,
                           bool prof = false) {
  unsigned long long t0 = prof ? clock64() : 0;
  // A: local transform of every body (model constants + its joint), lane = body:
  //    slide  p = bpos + R(bquat) axis q,  quat = bquat
  //    hinge  p = bpos,                    quat = bquat (x) (cos q/2, axis sin q/2)
  // every constant below is one load from the lane's flattened GmTopo entry (identity
  // transform and no joint on lanes without a body)
  real lp[3], lq[4], ax[3] = {0, 0, 0};
  const int b = T->lane_body[lane];   // scan-lane layout (GmTopo::lane_body)
  const int type = T->kl_type[lane];
  ld3(lp, T->kl_pos[lane]);
  ld4(lq, T->kl_quat[lane]);
  if (type >= 0) {
    const real qv = S.s.qpos[T->kl_qadr[lane]];
    ld3(ax, T->kl_axis[lane]);
    if (type == GM_JNT_SLIDE) {
      real R[9], wa[3];
      quat2mat(R, lq);
      mulmv3(wa, R, ax);
      lp[0] += wa[0] * qv; lp[1] += wa[1] * qv; lp[2] += wa[2] * qv;
    } else if (type == GM_JNT_HINGE) {
      real sn, cs;
      gm_sincos(0.5 * qv, &sn, &cs);   // shared with the oracle (gm_math.h)
      const real ql[4] = {cs, ax[0] * sn, ax[1] * sn, ax[2] * sn};
      quatmul(lq, lq, ql);
    }
  }
#if defined(GM_PHASE_SPLIT_PGS) || defined(GM_PHASE_SPLIT_COLL) || defined(GM_PHASE_SPLIT_SETUP) || defined(GM_PHASE_SPLIT_NARROW)
  PH(0);
#else
  PH(15);
#endif
  // B: poses.  The base is the world's child; along each finger / palm chain the
  // local transforms are composed by a segmented inclusive scan (root-side operand on
  // the left: (p_a, q_a) o (p_b, q_b) = (p_a + R(q_a) p_b, q_a (x) q_b)), then the base
  // pose is applied and the orientation renormalised.  Every body other than the world has
  // a scan lane (chain links, palm, base, object), which keeps its pose in registers for C.
  const int bb = T->body_base;
  const int grp = T->kl_grp[lane];
  const bool chain = grp >= 0 && grp <= 3;
  const bool is_obj = b == T->body_obj;
  real xp[3], xq[4];
  {
    const int lb = T->lane_base;
    real bpos[3], bq[4];
#pragma unroll
    for (int k = 0; k < 3; k++) bpos[k] = readlane_real(lp[k], lb);
#pragma unroll
    for (int k = 0; k < 4; k++) bq[k] = readlane_real(lq[k], lb);
    quatnorm(bq);
    real bR[9];
    quat2mat(bR, bq);
    const int p = T->kl_cpos[lane];
#pragma unroll
    for (int off = 1; off < CL; off <<= 1) {
      real np[3], nq[4];
#pragma unroll
      for (int k = 0; k < 3; k++) np[k] = row_shr(lp[k], off);
#pragma unroll
      for (int k = 0; k < 4; k++) nq[k] = row_shr(lq[k], off);
      if (p > off) {
        real R[9], t[3], q[4];
        quat2mat(R, nq);
        mulmv3(t, R, lp);
        quatmul(q, nq, lq);
        lp[0] = np[0] + t[0]; lp[1] = np[1] + t[1]; lp[2] = np[2] + t[2];
        lq[0] = q[0]; lq[1] = q[1]; lq[2] = q[2]; lq[3] = q[3];
      }
    }
    if (chain) {
      real t[3];
      mulmv3(t, bR, lp);
      quatmul(xq, bq, lq);
      quatnorm(xq);
      xp[0] = bpos[0] + t[0]; xp[1] = bpos[1] + t[1]; xp[2] = bpos[2] + t[2];
    } else if (is_obj) {
      // object: free joint, pose straight from qpos
      const int qa = T->qadr_obj;
      xq[0] = S.s.qpos[qa + 3]; xq[1] = S.s.qpos[qa + 4]; xq[2] = S.s.qpos[qa + 5]; xq[3] = S.s.qpos[qa + 6];
      quatnorm(xq);
      xp[0] = S.s.qpos[qa]; xp[1] = S.s.qpos[qa + 1]; xp[2] = S.s.qpos[qa + 2];
    } else {   // the base lane (the rest hold no body and store nothing)
      xp[0] = bpos[0]; xp[1] = bpos[1]; xp[2] = bpos[2];
      xq[0] = bq[0]; xq[1] = bq[1]; xq[2] = bq[2]; xq[3] = bq[3];
    }
  }
#if defined(GM_PHASE_SPLIT_PGS) || defined(GM_PHASE_SPLIT_COLL) || defined(GM_PHASE_SPLIT_SETUP) || defined(GM_PHASE_SPLIT_NARROW)
  PH(0);
#else
  PH(16);
#endif
  // C, on the body's scan lane from the pose in registers: the pose itself, the
  // world-origin spatial inertia and the motion subspace of the body's dof(s) (the
  // object's six)
  if (b > 0) {
    real R[9];
    quat2mat(R, xq);
    S.xpos[b][0] = xp[0]; S.xpos[b][1] = xp[1]; S.xpos[b][2] = xp[2];
#pragma unroll
    for (int k = 0; k < 4; k++) S.xquat[b][k] = xq[k];
    real ip[3], c[3];
    ld3(ip, m->body_ipos[b]);
    mulmv3(c, R, ip);
    c[0] += xp[0]; c[1] += xp[1]; c[2] += xp[2];
    real I[3] = {(real)m->body_inertia[b][0], (real)m->body_inertia[b][1], (real)m->body_inertia[b][2]};
    real mass = (real)m->body_mass[b];
    if (is_obj) {
      mass = S.s.obj_mass;
      I[0] = S.s.obj_inertia[0]; I[1] = S.s.obj_inertia[1]; I[2] = S.s.obj_inertia[2];
    }
    real Iw[9];
#pragma unroll
    for (int i = 0; i < 3; i++)
#pragma unroll
      for (int k = 0; k < 3; k++)
        Iw[3 * i + k] = R[3 * i] * I[0] * R[3 * k] + R[3 * i + 1] * I[1] * R[3 * k + 1] + R[3 * i + 2] * I[2] * R[3 * k + 2];
    const real cc = dot3(c, c);
    real* ci = S.cinert[b];
    ci[0] = Iw[0] + mass * (cc - c[0] * c[0]);
    ci[1] = Iw[4] + mass * (cc - c[1] * c[1]);
    ci[2] = Iw[8] + mass * (cc - c[2] * c[2]);
    ci[3] = Iw[1] - mass * c[0] * c[1];
    ci[4] = Iw[2] - mass * c[0] * c[2];
    ci[5] = Iw[5] - mass * c[1] * c[2];
    ci[6] = mass * c[0]; ci[7] = mass * c[1]; ci[8] = mass * c[2];
    ci[9] = mass;
    if (is_obj) {
      // free joint: translations along the world axes, rotations about the body axes
      // through the body origin
      const int d0 = T->dof_obj;
#pragma unroll
      for (int k = 0; k < 3; k++) {
        real* cd = S.cdof[d0 + k];
        cd[0] = cd[1] = cd[2] = 0; cd[3] = cd[4] = cd[5] = 0; cd[3 + k] = 1;
      }
#pragma unroll
      for (int k = 0; k < 3; k++) {
        real* cd = S.cdof[d0 + 3 + k];
        const real w[3] = {R[k], R[3 + k], R[6 + k]};
        cd[0] = w[0]; cd[1] = w[1]; cd[2] = w[2];
        cross3(cd + 3, xp, w);
      }
    } else {
      // the body's one joint (slide / hinge; kl_axis = the joint's dof axis)
      const int d = chain ? (grp < 3 ? T->dof_f0[grp] + T->kl_cpos[lane] - 1 : T->dof_palm) : T->dof_base;
      real* cd = S.cdof[d];
      real wa[3];
      mulmv3(wa, R, ax);
      if (type == GM_JNT_SLIDE) {
        cd[0] = cd[1] = cd[2] = 0; cd[3] = wa[0]; cd[4] = wa[1]; cd[5] = wa[2];
      } else {
        cd[0] = wa[0]; cd[1] = wa[1]; cd[2] = wa[2];
        cross3(cd + 3, xp, wa);   // anchor at the body origin in this model
      }
    }
  }
  GM_WAVE_SYNC();
}

// ============================================================ CRB + RNE
// mj_rne (bias forces, world-origin spatial algebra) and mj_crb (composite inertias):
// forward velocity / bias-acceleration recursion and body forces per chain, then
// leaf -> root running sums in registers; chain-root totals meet at the base body.
template <int CL>
__device__ __forceinline__ void body_force(SharedT<CL>& S, int b, const real* cvel, const real* cacc) {
  real ci[10], t1[6], t2[6], f[6];
#pragma unroll
  for (int k = 0; k < 10; k++) ci[k] = S.cinert[b][k];
  inert_mul(f, ci, cacc);
  inert_mul(t1, ci, cvel);
  cross_force(t2, cvel, t1);
#pragma unroll
  for (int k = 0; k < 6; k++) S.cfrc[b][k] = f[k] + t2[k];
}
template <int CL>
__device__ __forceinline__ void rne_fwd(SharedT<CL>& S, int b, int d, real* cvel, real* cacc) {
  real cd[6], cdd[6];
#pragma unroll
  for (int k = 0; k < 6; k++) cd[k] = S.cdof[d][k];
  cross_motion(cdd, cvel, cd);
  const real qv = S.s.qvel[d];
#pragma unroll
  for (int k = 0; k < 6; k++) { cvel[k] += cd[k] * qv; cacc[k] += cdd[k] * qv; }
  body_force(S, b, cvel, cacc);
}
// backward running sums over bodies b0 .. b0+L-1 (leaf = last); writes cfrc / Ic
template <int L, int CL>
__device__ __forceinline__ void chain_sums(SharedT<CL>& S, int b0, real* fs, real* Is) {
#pragma unroll
  for (int k = 0; k < 6; k++) fs[k] = 0;
#pragma unroll
  for (int k = 0; k < 10; k++) Is[k] = 0;
#pragma unroll
  for (int p = L; p >= 1; p--) {
    const int b = b0 + p - 1;
#pragma unroll
    for (int k = 0; k < 6; k++) { fs[k] += S.cfrc[b][k]; S.cfrc[b][k] = fs[k]; }
#pragma unroll
    for (int k = 0; k < 10; k++) { Is[k] = S.cinert[b][k] + (p < L ? Is[k] : 0.0); S.Ic[b][k] = Is[k]; }
  }
}

template <int CL, bool CAL>
__device__ __forceinline__ void lock_rows(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T, int lane);
template <int CL, bool CAL>
__device__ __forceinline__ void crb_rne(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T, int lane,
                        bool prof = false) {
  unsigned long long t0 = prof ? clock64() : 0;
  // the constraint problem's lock rows ride in this phase's first block (see lock_rows)
  lock_rows<CL, CAL>(S, m, T, lane);
  // Lanes = bodies.  Along each finger / palm chain the velocities and bias accelerations
  // are segmented prefix sums and the composite forces / inertias segmented suffix sums
  // (Hillis-Steele over the chain position, shuffles within the wave); the base body is
  // the common root and the free object is handled by its own lane.
  const int db = T->dof_base;
  const real qdb = S.s.qvel[db];
  real cvb[6], cab[6];
#pragma unroll
  for (int k = 0; k < 6; k++) { cvb[k] = S.cdof[db][k] * qdb; cab[k] = 0; }
  cab[3] = -(real)m->gravity[0]; cab[4] = -(real)m->gravity[1]; cab[5] = -(real)m->gravity[2];

  const int b = T->lane_body[lane];   // scan-lane layout (GmTopo::lane_body)
  const int grp = T->kl_grp[lane];
  const bool chain = grp >= 0 && grp <= 3;
  const int p = T->kl_cpos[lane];
  const int d = chain ? (grp < 3 ? T->dof_f0[grp] + p - 1 : T->dof_palm) : db;
  real cd[6], v[6];
  // (operands loaded on every lane -- d is the base dof off the chains -- and selected: a
  // select instead of a divergent branch around each load)
  const real qvd = S.s.qvel[d];
  const real qd = chain ? qvd : 0.0;
#pragma unroll
  for (int k = 0; k < 6; k++) { const real c = S.cdof[d][k]; cd[k] = chain ? c : 0.0; v[k] = cd[k] * qd; }
  // The scans add their shifted operand unconditionally: every source outside a lane's
  // chain segment holds an exact zero (the empty position 0 of each finger row, the base
  // lane before the palm, the no-body lanes past the chain end, the zero-inertia object
  // lane, and DPP's bound_ctrl zero past the row edge), so the old p > off / p + off <= Lc
  // selects only cost two v_cndmask per double per step.  The sums of nonzero terms keep
  // the scan's association; only the sign of an exactly-zero entry can differ.
  // velocities: inclusive prefix along the chain, then the base contribution
  real cv[6];
#pragma unroll
  for (int k = 0; k < 6; k++) cv[k] = v[k];
#pragma unroll
  for (int off = 1; off < CL; off <<= 1) {
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const real nb = row_shr(cv[k], off);
      cv[k] += nb;
    }
  }
  real cvp[6];
#pragma unroll
  for (int k = 0; k < 6; k++) {
    const real nb = row_shr(cv[k], 1);
    cvp[k] = cvb[k] + (p > 1 ? nb : 0.0);
    cv[k] += cvb[k];
  }
  // bias accelerations: prefix of (cvel_parent x cdof) qd
  real ca[6];
  cross_motion(ca, cvp, cd);
#pragma unroll
  for (int k = 0; k < 6; k++) ca[k] *= qd;
#pragma unroll
  for (int off = 1; off < CL; off <<= 1) {
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const real nb = row_shr(ca[k], off);
      ca[k] += nb;
    }
  }
#pragma unroll
  for (int k = 0; k < 6; k++) ca[k] += cab[k];
  // body forces I a + v x* (I v), then suffix sums of forces and inertias
  real ci[10], f[6];
#pragma unroll
  for (int k = 0; k < 10; k++) { const real c = S.cinert[b < 0 ? 0 : b][k]; ci[k] = chain ? c : 0.0; }
  {
    real t1[6], t2[6];
    inert_mul(f, ci, ca);
    inert_mul(t1, ci, cv);
    cross_force(t2, cv, t1);
#pragma unroll
    for (int k = 0; k < 6; k++) f[k] += t2[k];
  }
#pragma unroll
  for (int off = 1; off < CL; off <<= 1) {
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const real nb = row_shl(f[k], off);
      f[k] += nb;
    }
#pragma unroll
    for (int k = 0; k < 10; k++) {
      const real nb = row_shl(ci[k], off);
      ci[k] += nb;
    }
  }
  if (chain) {
#pragma unroll
    for (int k = 0; k < 6; k++) S.cfrc[b][k] = f[k];
#pragma unroll
    for (int k = 0; k < 10; k++) S.Ic[b][k] = ci[k];
    if (p == 1) {
#pragma unroll
      for (int k = 0; k < 6; k++) S.chain_f[grp][k] = f[k];
#pragma unroll
      for (int k = 0; k < 10; k++) S.chain_I[grp][k] = ci[k];
    }
  }
  if (b == T->body_obj) {
    // object: free joint on one body
    const int d0 = T->dof_obj;
    real cvel[6], cacc[6];
#pragma unroll
    for (int k = 0; k < 6; k++) { cvel[k] = 0; cacc[k] = 0; }
    cacc[3] = -(real)m->gravity[0]; cacc[4] = -(real)m->gravity[1]; cacc[5] = -(real)m->gravity[2];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const real qv = S.s.qvel[d0 + k];
#pragma unroll
      for (int t = 0; t < 6; t++) cvel[t] += S.cdof[d0 + k][t] * qv;
    }
    real cdd[3][6];
#pragma unroll
    for (int k = 0; k < 3; k++) cross_motion(cdd[k], cvel, S.cdof[d0 + 3 + k]);
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const real qv = S.s.qvel[d0 + 3 + k];
#pragma unroll
      for (int t = 0; t < 6; t++) cvel[t] += S.cdof[d0 + 3 + k][t] * qv;
    }
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const real qv = S.s.qvel[d0 + 3 + k];
#pragma unroll
      for (int t = 0; t < 6; t++) cacc[t] += cdd[k][t] * qv;
    }
    body_force(S, b, cvel, cacc);
  }
  GM_WAVE_SYNC();
#ifdef GM_PHASE_SPLIT_NARROW
  PH(1);
#else
  PH(17);
#endif
  // base body: its own inertia / force plus the four chain roots, one lane per value
  // (lanes 0..9 the composite inertia, 10..15 the force; the base's own body force is
  // formed on every lane from its uniform operands, the same operations as body_force)
  {
    const int bb = T->body_base;
    real ci[10], t1[6], t2[6], fo[6];
#pragma unroll
    for (int k = 0; k < 10; k++) ci[k] = S.cinert[bb][k];
    inert_mul(fo, ci, cab);
    inert_mul(t1, ci, cvb);
    cross_force(t2, cvb, t1);
#pragma unroll
    for (int k = 0; k < 6; k++) fo[k] = fo[k] + t2[k];
    const bool isI = lane < 10;
    const int k = isI ? lane : (lane < 16 ? lane - 10 : 0);
    real own = ci[0];
#pragma unroll
    for (int t = 1; t < 10; t++) own = (lane == t) ? ci[t] : own;
#pragma unroll
    for (int t = 0; t < 6; t++) own = (lane == 10 + t) ? fo[t] : own;
    real acc = own;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const real vI = S.chain_I[c][k], vf = S.chain_f[c][k];
      acc += isI ? vI : vf;
    }
    if (lane < 16) {
      real* dst = isI ? &S.Ic[bb][k] : &S.cfrc[bb][k];
      *dst = acc;
    }
  }
  GM_WAVE_SYNC();
}

// ============================================================ mass matrix rows + forces
__device__ __forceinline__ void ctrl_gains(const gm_model* __restrict__ m, const GmTopo* __restrict__ T, int d,
                                           real* kp, real* kd) {
  *kp = 0; *kd = 0;
  for (int f = 0; f < 3; f++) {
    if (d == m->dof_pris[f]) { *kp = (real)m->kp_gripper[0]; *kd = (real)m->kd_gripper[0]; }
    if (d == m->dof_rev[f]) { *kp = (real)m->kp_gripper[1]; *kd = (real)m->kd_gripper[1]; }
  }
  if (d == m->dof_palm) { *kp = (real)m->kp_gripper[2]; *kd = (real)m->kd_gripper[2]; }
  if (d == m->dof_base) { *kp = (real)m->kp_base[2]; *kd = (real)m->kd_base[2]; }
}

// lane per dof: H row entries (compact), bias/passive/actuator force
// CAL: the calibration variant (per-env timestep, tip load); the env-step kernel is CAL = false
template <int CL, bool CAL>
__device__ __forceinline__ void mass_and_forces(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T, int lane) {
  if (lane < T->nv) {
    const int d = lane;
    const int b = T->dof_body[d];
    const int c = T->dof_grp[d];
    const int p = T->dof_p[d];
    real add;
    if constexpr (CAL) {   // H~ diagonal for this env's timestep (same operations as the host fold)
      const real h = S.s.dt;
      add = T->dof_arm[d] + h * T->dof_dsum[d];
      add += h * h * T->dof_ksum[d];
    } else {
      add = T->dof_add[d];
    }
    real cd[6], F[6];
#pragma unroll
    for (int k = 0; k < 6; k++) cd[k] = S.cdof[d][k];
    inert_mul(F, S.Ic[b], cd);
    if (c == GM_GRP_BASE) {
      S.Hbb = dot6(cd, F) + add;
    } else {
      // object and chain rows share one loop (one pass of the wave instead of two
      // divergent ones): row p of the object block or of the chain's block
      const bool objd = c == GM_GRP_OBJECT;
      const int d0 = objd ? T->dof_obj : (c < 3) ? T->dof_f0[c] : T->dof_palm;
      real* Hrow = objd ? &S.Ho[TRI(p, 0)] : (c < 3) ? &S.Hf[c][TRI(p, 0)] : &S.Hp[TRI(p, 0)];
#pragma unroll
      for (int q = 0; q <= CL; q++) {
        int dq = objd ? d0 + q : (q == 0) ? T->dof_base : d0 + q - 1;
        dq = dq < SharedT<CL>::NV ? dq : SharedT<CL>::NV - 1;
        real v = dot6(S.cdof[dq], F);
        if (q == p) v += add;
        keep(v);
        if (q <= p) Hrow[q] = v;
      }
    }
    // forces: passive springs/damping, PD control (target_.next, base target), RNE bias
    const real bias = dot6(cd, S.cfrc[b]);
    const real qp = S.s.qpos[d], qv = S.s.qvel[d];
    real pas = 0;
    pas -= T->dof_stiff[d] * qp;
    pas -= T->dof_damp[d] * qv;
    const int tgt = T->dof_target[d];
    real act = 0;
    if (tgt != 0) {
      const real target = tgt == 1 ? S.s.next.x : tgt == 2 ? S.s.next.th : tgt == 3 ? S.s.next.z : S.s.base[2];
      act = -((qp - target) * T->dof_kp[d] + qv * T->dof_kd[d]);
    }
    real frc = pas + act - bias;
    if (CAL && S.s.tip_force != 0.0 && (c < 3 || c == GM_GRP_BASE)) {
      // calibration tip load: resolve_segment_forces -> apply_segment_force
      // (myfunctions.cpp:1642-1727) pulls each finger's tip link at its centre of mass
      // along the finger's rest bending direction; J^T F for the dofs above that link
#pragma unroll
      for (int f = 0; f < 3; f++) {
        if (c < 3 && f != c) continue;
        const int bt = m->body_tip[f];
        real R[9], ip[3], pc[3], wxp[3];
        body_R(S, bt, R);
        ld3(ip, m->body_ipos[bt]);
        mulmv3(pc, R, ip);
        pc[0] += S.xpos[bt][0]; pc[1] += S.xpos[bt][1]; pc[2] += S.xpos[bt][2];
        const real F[3] = {S.s.tip_force * m->tip_dir[f][0], S.s.tip_force * m->tip_dir[f][1],
                           S.s.tip_force * m->tip_dir[f][2]};
        cross3(wxp, cd, pc);
        const real col[3] = {cd[3] + wxp[0], cd[4] + wxp[1], cd[5] + wxp[2]};
        frc += dot3(col, F);
      }
    }
    S.frc[d] = frc;
  }
  GM_WAVE_SYNC();
}

// ============================================================ collision
struct Hit { real dist, pos[3], n[3]; };

__device__ void make_frame(real* F, const real* n) {
  real a[3] = {0, 0, 0};
  if (fabs(n[0]) < 0.5) a[0] = 1; else a[1] = 1;
  real d = dot3(a, n);
  real t1[3] = {a[0] - d * n[0], a[1] - d * n[1], a[2] - d * n[2]};
  const real il = rsq_n(dot3(t1, t1));
  t1[0] *= il; t1[1] *= il; t1[2] *= il;
  real t2[3];
  cross3(t2, n, t1);
  F[0] = n[0]; F[1] = n[1]; F[2] = n[2];
  F[3] = t1[0]; F[4] = t1[1]; F[5] = t1[2];
  F[6] = t2[0]; F[7] = t2[1]; F[8] = t2[2];
}

struct GeomV { int type; real size[3]; real c[3]; real R[9]; real rbound; real friction; };

// world pose of a geom on body b with local pose (gp, gq) (oracle.c fk, geom part),
// computed where a pair lane needs it
template <int CL>
__device__ __forceinline__ void geom_pose(SharedT<CL>& S, int b, const double* gpos, const double* gquat, real* c,
                                          real* Rw) {
  real R[9];
  if (b == 0) {
    R[0] = 1; R[1] = 0; R[2] = 0; R[3] = 0; R[4] = 1; R[5] = 0; R[6] = 0; R[7] = 0; R[8] = 1;
  } else {
    body_R(S, b, R);
  }
  real gp[3], t[3], gq[4], Rg[9];
  ld3(gp, gpos);
  mulmv3(t, R, gp);
  const real bp0 = b == 0 ? 0.0 : S.xpos[b][0], bp1 = b == 0 ? 0.0 : S.xpos[b][1], bp2 = b == 0 ? 0.0 : S.xpos[b][2];
  c[0] = bp0 + t[0]; c[1] = bp1 + t[1]; c[2] = bp2 + t[2];
  ld4(gq, gquat);
  quat2mat(Rg, gq);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int k = 0; k < 3; k++)
      Rw[3 * i + k] = R[3 * i] * Rg[k] + R[3 * i + 1] * Rg[3 + k] + R[3 * i + 2] * Rg[6 + k];
}

// geom slot sl (0: pair_a, 1: pair_b) of candidate pair pr from the pair's flattened
// constants (GmTopo pr_*); the live object's geom reads its type and size from the env
template <int CL>
__device__ __forceinline__ void load_pair_geom(SharedT<CL>& S, const GmTopo* __restrict__ T, int pr, int sl, GeomV& G) {
  const int t = T->pr_type[pr][sl];
  if (t < 0) {
    G.type = S.s.obj_type;
    G.size[0] = S.s.obj_size[0]; G.size[1] = S.s.obj_size[1]; G.size[2] = S.s.obj_size[2];
    G.rbound = S.s.obj_rbound; G.friction = S.s.obj_friction;
  } else {
    G.type = t;
    ld3(G.size, T->pr_size[pr][sl]);
    G.rbound = (real)T->pr_rbound[pr][sl];
    G.friction = (real)T->pr_fric[pr][sl];
  }
  geom_pose(S, T->pr_body[pr][sl], T->pr_pos[pr][sl], T->pr_quat[pr][sl], G.c, G.R);
}

// plane-X multi-contact generators: k-th candidate point (returns 0 if none)
__device__ __forceinline__ int plane_box_point(const GeomV& P, const GeomV& B, int i, Hit& h) {
  real nz[3] = {P.R[2], P.R[5], P.R[8]};
  real s[3] = {(i & 1) ? B.size[0] : -B.size[0], (i & 2) ? B.size[1] : -B.size[1], (i & 4) ? B.size[2] : -B.size[2]};
  real v[3];
  mulmv3(v, B.R, s);
  v[0] += B.c[0]; v[1] += B.c[1]; v[2] += B.c[2];
  real dv[3] = {v[0] - P.c[0], v[1] - P.c[1], v[2] - P.c[2]};
  real d = dot3(dv, nz);
  if (!(d < 0)) return 0;
  h.dist = d;
  for (int k = 0; k < 3; k++) { h.pos[k] = v[k] - 0.5 * d * nz[k]; h.n[k] = nz[k]; }
  return 1;
}
// per-pair part of the plane-cylinder rim test (the rim frame: axis a, w = the in-plane
// direction towards the plane, a x w), computed once per pair instead of once per rim
// point -- the same operations, so the same values
struct CylFrame { real nz[3], a[3], w[3], axw[3]; };
__device__ __forceinline__ void cyl_frame(const GeomV& P, const GeomV& Cy, CylFrame& F) {
  F.nz[0] = P.R[2]; F.nz[1] = P.R[5]; F.nz[2] = P.R[8];
  F.a[0] = Cy.R[2]; F.a[1] = Cy.R[5]; F.a[2] = Cy.R[8];
  real na = dot3(F.nz, F.a);
  real w[3] = {-F.nz[0] + na * F.a[0], -F.nz[1] + na * F.a[1], -F.nz[2] + na * F.a[2]};
  const real lw2 = dot3(w, w);
  const real lw = sqrt_n(lw2), ilw = rsq_n(lw2);   // (independent: the test and the scale)
  if (lw < 1e-6) { w[0] = Cy.R[0]; w[1] = Cy.R[3]; w[2] = Cy.R[6]; }
  else { w[0] = w[0] * ilw; w[1] = w[1] * ilw; w[2] = w[2] * ilw; }
  F.w[0] = w[0]; F.w[1] = w[1]; F.w[2] = w[2];
  cross3(F.axw, F.a, F.w);
}
__device__ __forceinline__ int plane_cyl_point(const GeomV& P, const GeomV& Cy, const CylFrame& F, int i, Hit& h) {
  const real* nz = F.nz;
  const real* a = F.a;
  real r = Cy.size[0], hh = Cy.size[1];
  int s = i >> 2, k = i & 3;
  real sg = s == 0 ? 1.0 : -1.0;
  real dir[3];
  if (k == 0) { dir[0] = F.w[0]; dir[1] = F.w[1]; dir[2] = F.w[2]; }
  else if (k == 1) { dir[0] = F.axw[0]; dir[1] = F.axw[1]; dir[2] = F.axw[2]; }
  else if (k == 2) { dir[0] = -F.w[0]; dir[1] = -F.w[1]; dir[2] = -F.w[2]; }
  else { dir[0] = -F.axw[0]; dir[1] = -F.axw[1]; dir[2] = -F.axw[2]; }
  real v[3];
  for (int t = 0; t < 3; t++) v[t] = Cy.c[t] + sg * hh * a[t] + r * dir[t];
  real dv[3] = {v[0] - P.c[0], v[1] - P.c[1], v[2] - P.c[2]};
  real d = dot3(dv, nz);
  if (!(d < 0)) return 0;
  h.dist = d;
  for (int t = 0; t < 3; t++) { h.pos[t] = v[t] - 0.5 * d * nz[t]; h.n[t] = nz[t]; }
  return 1;
}
__device__ __forceinline__ int plane_sphere(const GeomV& P, const GeomV& Sp, Hit& h) {
  real nz[3] = {P.R[2], P.R[5], P.R[8]};
  real r = Sp.size[0];
  real dv[3] = {Sp.c[0] - P.c[0], Sp.c[1] - P.c[1], Sp.c[2] - P.c[2]};
  real dist = dot3(dv, nz) - r;
  if (!(dist < 0)) return 0;
  h.dist = dist;
  for (int k = 0; k < 3; k++) { h.pos[k] = Sp.c[k] - nz[k] * (r + 0.5 * dist); h.n[k] = nz[k]; }
  return 1;
}
__device__ __forceinline__ int sphere_box(const GeomV& Sp, const GeomV& B, Hit& h) {
  const real* R = B.R;
  const real* hs = B.size;
  real r = Sp.size[0];
  real dv[3] = {Sp.c[0] - B.c[0], Sp.c[1] - B.c[1], Sp.c[2] - B.c[2]};
  real cl[3];
  mulmtv3(cl, R, dv);
  real q[3];
  int inside = 1;
  for (int k = 0; k < 3; k++) {
    q[k] = cl[k];
    if (q[k] > hs[k]) { q[k] = hs[k]; inside = 0; }
    if (q[k] < -hs[k]) { q[k] = -hs[k]; inside = 0; }
  }
  real nl[3], dist, ql[3];
  if (!inside) {
    real df[3] = {cl[0] - q[0], cl[1] - q[1], cl[2] - q[2]};
    const real l2 = dot3(df, df);
    real l = sqrt_n(l2);
    if (l < 1e-12) return 0;
    dist = l - r;
    if (!(dist < 0)) return 0;
    const real il = rsq_n(l2);
    nl[0] = -df[0] * il; nl[1] = -df[1] * il; nl[2] = -df[2] * il;
    ql[0] = q[0]; ql[1] = q[1]; ql[2] = q[2];
  } else {
    int kmin = 0;
    real best = hs[0] - fabs(cl[0]);
    for (int k = 1; k < 3; k++) { real v = hs[k] - fabs(cl[k]); if (v < best) { best = v; kmin = k; } }
    const real clk = kmin == 0 ? cl[0] : (kmin == 1 ? cl[1] : cl[2]);
    const real hsk = kmin == 0 ? hs[0] : (kmin == 1 ? hs[1] : hs[2]);
    real sg = clk >= 0 ? 1.0 : -1.0;
    dist = -(best + r);
#pragma unroll
    for (int k = 0; k < 3; k++) {
      nl[k] = (k == kmin) ? -sg : 0.0;
      ql[k] = (k == kmin) ? sg * hsk : cl[k];
    }
  }
  real n[3], qw[3];
  mulmv3(n, R, nl);
  mulmv3(qw, R, ql);
  h.dist = dist;
  for (int k = 0; k < 3; k++) {
    qw[k] += B.c[k];
    real sp = Sp.c[k] + n[k] * r;
    h.pos[k] = 0.5 * (qw[k] + sp);
    h.n[k] = n[k];
  }
  return 1;
}

// ---- MPR ----
struct SV { real v[3], p1[3], p2[3]; };
// TYPE: the geom type when known at compile time (mpr's cylinder-box instance), -1 = read it
template <int TYPE = -1>
__device__ __forceinline__ void support_geom(const GeomV& G, const real* d, real* out) {
  real dl[3];
  mulmtv3(dl, G.R, d);
  real pl[3] = {0, 0, 0};
  const int type = TYPE >= 0 ? TYPE : G.type;
  // face / rim-line ties take the centre (oracle.c support_geom, GM_SUPPORT_TIE)
  if (type == GM_GEOM_BOX) {
    for (int k = 0; k < 3; k++) pl[k] = fabs(dl[k]) < GM_SUPPORT_TIE ? 0.0 : (dl[k] >= 0 ? G.size[k] : -G.size[k]);
  } else if (type == GM_GEOM_CYLINDER) {
    const real rr2 = dl[0] * dl[0] + dl[1] * dl[1];
    if (rr2 > 1e-24) { const real irr = rsq_n(rr2); pl[0] = (G.size[0] * dl[0]) * irr; pl[1] = (G.size[0] * dl[1]) * irr; }
    pl[2] = fabs(dl[2]) < GM_SUPPORT_TIE ? 0.0 : (dl[2] >= 0 ? G.size[1] : -G.size[1]);
  } else if (type == GM_GEOM_SPHERE) {
    const real l2 = dot3(dl, dl);
    real l = sqrt_n(l2);
    if (l > 1e-12) { const real il = rsq_n(l2); pl[0] = (dl[0] * G.size[0]) * il; pl[1] = (dl[1] * G.size[0]) * il; pl[2] = (dl[2] * G.size[0]) * il; }
  }
  mulmv3(out, G.R, pl);
  out[0] += G.c[0]; out[1] += G.c[1]; out[2] += G.c[2];
}
template <int TA, int TB>
__device__ __forceinline__ void mpr_support(const GeomV& A, const GeomV& B, const real* d, SV& sv) {
  real nd[3] = {-d[0], -d[1], -d[2]};
  support_geom<TA>(A, d, sv.p1);
  support_geom<TB>(B, nd, sv.p2);
  sv.v[0] = sv.p1[0] - sv.p2[0]; sv.v[1] = sv.p1[1] - sv.p2[1]; sv.v[2] = sv.p1[2] - sv.p2[2];
}
__device__ __forceinline__ int fzero(real x) { return fabs(x) < 1e-12; }
// (1 / |d| as one refined reciprocal square root: half the dependent chain of sqrt then
// reciprocal; the oracle's 1 / sqrt(x) rounds twice, this once -- the MPR iterates agree to
// the last bits, the collider's contacts to ~1e-15 relative)
__device__ __forceinline__ void normalize3(real* d) {
  const real l2 = dot3(d, d);
  if (l2 > 0) { const real il = rsq_n(l2); d[0] *= il; d[1] *= il; d[2] *= il; }
}
// The simplex vertices are four named values (not an array), conditional vertex copies
// are per-component selects and every helper is inlined, so the whole MPR state stays in
// VGPRs (an indexable array, or a branch between whole-struct copies, goes to scratch).
__device__ __forceinline__ void sv_take(SV& dst, const SV& src, bool c) {
#pragma unroll
  for (int k = 0; k < 3; k++) {
    dst.v[k] = c ? src.v[k] : dst.v[k];
    dst.p1[k] = c ? src.p1[k] : dst.p1[k];
    dst.p2[k] = c ? src.p2[k] : dst.p2[k];
  }
}
__device__ __forceinline__ void portal_dir(const SV& P1, const SV& P2, const SV& P3, real* dir) {
  real a[3] = {P2.v[0] - P1.v[0], P2.v[1] - P1.v[1], P2.v[2] - P1.v[2]};
  real b[3] = {P3.v[0] - P1.v[0], P3.v[1] - P1.v[1], P3.v[2] - P1.v[2]};
  cross3(dir, a, b);
  normalize3(dir);
}
__device__ __forceinline__ void expand_portal(const SV& P0, SV& P1, SV& P2, SV& P3, const SV& v4) {
  real v4v0[3];
  cross3(v4v0, v4.v, P0.v);
  const bool s1 = dot3(P1.v, v4v0) > 0;
  const bool s2 = dot3(P2.v, v4v0) > 0;
  const bool s3 = dot3(P3.v, v4v0) > 0;
  // d1 > 0: (d2 > 0 ? P1 : P3) = v4;  else: (d3 > 0 ? P2 : P1) = v4
  sv_take(P1, v4, s1 ? s2 : !s3);
  sv_take(P2, v4, !s1 && s3);
  sv_take(P3, v4, s1 && !s2);
}
__device__ __forceinline__ int reach_tol(const SV& P1, const SV& P2, const SV& P3, const SV& v4, const real* dir, real tol) {
  real dv1 = dot3(P1.v, dir), dv2 = dot3(P2.v, dir), dv3 = dot3(P3.v, dir), dv4 = dot3(v4.v, dir);
  real d1 = dv4 - dv1, d2 = dv4 - dv2, d3 = dv4 - dv3;
  real dd = fmin(fmin(d1, d2), d3);
  return dd < tol || fabs(dd - tol) < 1e-12;
}
__device__ __forceinline__ void tri_closest_origin(const real* a, const real* b, const real* c, real* out) {
  real ab[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]};
  real ac[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
  real ap[3] = {-a[0], -a[1], -a[2]};
  real d1 = dot3(ab, ap), d2 = dot3(ac, ap);
  if (d1 <= 0 && d2 <= 0) { out[0] = a[0]; out[1] = a[1]; out[2] = a[2]; return; }
  real bp[3] = {-b[0], -b[1], -b[2]};
  real d3 = dot3(ab, bp), d4 = dot3(ac, bp);
  if (d3 >= 0 && d4 <= d3) { out[0] = b[0]; out[1] = b[1]; out[2] = b[2]; return; }
  real vc = d1 * d4 - d3 * d2;
  if (vc <= 0 && d1 >= 0 && d3 <= 0) { real v = div_n(d1, d1 - d3); for (int k = 0; k < 3; k++) out[k] = a[k] + v * ab[k]; return; }
  real cp[3] = {-c[0], -c[1], -c[2]};
  real d5 = dot3(ab, cp), d6 = dot3(ac, cp);
  if (d6 >= 0 && d5 <= d6) { out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; return; }
  real vb = d5 * d2 - d1 * d6;
  if (vb <= 0 && d2 >= 0 && d6 <= 0) { real w = div_n(d2, d2 - d6); for (int k = 0; k < 3; k++) out[k] = a[k] + w * ac[k]; return; }
  real va = d3 * d6 - d5 * d4;
  if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
    real w = div_n(d4 - d3, (d4 - d3) + (d5 - d6));
    for (int k = 0; k < 3; k++) out[k] = b[k] + w * (c[k] - b[k]);
    return;
  }
  real den = rcp_n(va + vb + vc);
  real v = vb * den, w = vc * den;
  for (int k = 0; k < 3; k++) out[k] = a[k] + ab[k] * v + ac[k] * w;
}
__device__ __forceinline__ void mpr_pos(const SV& P0, const SV& P1, const SV& P2, const SV& P3, real* pos) {
  real dir[3];
  portal_dir(P1, P2, P3, dir);
  real t[3];
  cross3(t, P1.v, P2.v); real b0 = dot3(t, P3.v);
  cross3(t, P3.v, P2.v); real b1 = dot3(t, P0.v);
  cross3(t, P0.v, P1.v); real b2 = dot3(t, P3.v);
  cross3(t, P2.v, P1.v); real b3 = dot3(t, P0.v);
  real sum = b0 + b1 + b2 + b3;
  if (sum <= 0) {
    b0 = 0;
    cross3(t, P2.v, P3.v); b1 = dot3(t, dir);
    cross3(t, P3.v, P1.v); b2 = dot3(t, dir);
    cross3(t, P1.v, P2.v); b3 = dot3(t, dir);
    sum = b1 + b2 + b3;
  }
  real inv = rcp_n(sum);
  real p1[3] = {0, 0, 0}, p2[3] = {0, 0, 0};
#pragma unroll
  for (int k = 0; k < 3; k++) {
    p1[k] += b0 * P0.p1[k]; p2[k] += b0 * P0.p2[k];
    p1[k] += b1 * P1.p1[k]; p2[k] += b1 * P1.p2[k];
    p1[k] += b2 * P2.p1[k]; p2[k] += b2 * P2.p2[k];
    p1[k] += b3 * P3.p1[k]; p2[k] += b3 * P3.p2[k];
  }
  for (int k = 0; k < 3; k++) pos[k] = 0.5 * (p1[k] + p2[k]) * inv;
}
// TA, TB: the two geoms' types when known at compile time (-1: read per lane)
template <int TA = -1, int TB = -1>
__device__ __forceinline__ int mpr(const GeomV& A, const GeomV& B, real tol, int maxit, Hit& h) {
  SV P0, P1, P2, P3;
  for (int k = 0; k < 3; k++) { P0.v[k] = A.c[k] - B.c[k]; P0.p1[k] = A.c[k]; P0.p2[k] = B.c[k]; }
  if (fzero(P0.v[0]) && fzero(P0.v[1]) && fzero(P0.v[2])) P0.v[0] += 1e-5;
  real d[3] = {-P0.v[0], -P0.v[1], -P0.v[2]};
  normalize3(d);
  mpr_support<TA, TB>(A, B, d, P1);
  if (dot3(P1.v, d) <= 0) return 0;
  cross3(d, P0.v, P1.v);
  if (fzero(sqrt_n(dot3(d, d)))) {
    real l1 = sqrt_n(dot3(P1.v, P1.v));
    if (fzero(l1)) return 0;
    h.dist = -l1;
    real il = rcp_n(l1);
    for (int k = 0; k < 3; k++) { h.n[k] = P1.v[k] * il; h.pos[k] = 0.5 * (P1.p1[k] + P1.p2[k]); }
    return 1;
  }
  normalize3(d);
  mpr_support<TA, TB>(A, B, d, P2);
  if (dot3(P2.v, d) <= 0) return 0;
  real va[3], vb[3];
  for (int k = 0; k < 3; k++) { va[k] = P1.v[k] - P0.v[k]; vb[k] = P2.v[k] - P0.v[k]; }
  cross3(d, va, vb);
  normalize3(d);
  if (dot3(d, P0.v) > 0) {
    const SV t = P1;
    sv_take(P1, P2, true); sv_take(P2, t, true);
    d[0] = -d[0]; d[1] = -d[1]; d[2] = -d[2];
  }
  int it = 0;
  for (;;) {
    mpr_support<TA, TB>(A, B, d, P3);
    if (dot3(P3.v, d) <= 0) return 0;
    cross3(va, P1.v, P3.v);
    const bool c2 = dot3(va, P0.v) < -1e-12;
    cross3(va, P3.v, P2.v);
    const bool c1 = !c2 && dot3(va, P0.v) < -1e-12;
    sv_take(P2, P3, c2);
    sv_take(P1, P3, c1);
    if (!(c1 || c2)) break;
    for (int k = 0; k < 3; k++) { va[k] = P1.v[k] - P0.v[k]; vb[k] = P2.v[k] - P0.v[k]; }
    cross3(d, va, vb);
    normalize3(d);
    if (++it > maxit) return 0;
  }
  it = 0;
  for (;;) {
    portal_dir(P1, P2, P3, d);
    if (dot3(d, P1.v) >= -1e-12) break;
    SV v4;
    mpr_support<TA, TB>(A, B, d, v4);
    real dv4 = dot3(v4.v, d);
    if (!(fzero(dv4) || dv4 > 0)) return 0;
    if (reach_tol(P1, P2, P3, v4, d, tol)) return 0;
    expand_portal(P0, P1, P2, P3, v4);
    if (++it > maxit) return 0;
  }
  it = 0;
  for (;;) {
    portal_dir(P1, P2, P3, d);
    SV v4;
    mpr_support<TA, TB>(A, B, d, v4);
    if (reach_tol(P1, P2, P3, v4, d, tol) || it > maxit) {
      real cp[3];
      tri_closest_origin(P1.v, P2.v, P3.v, cp);
      const real dp2 = dot3(cp, cp);
      real depth = sqrt_n(dp2);
      if (fzero(depth)) return 0;
      h.dist = -depth;
      real id = rsq_n(dp2);
      h.n[0] = cp[0] * id; h.n[1] = cp[1] * id; h.n[2] = cp[2] * id;
      mpr_pos(P0, P1, P2, P3, h.pos);
      return depth > 0;
    }
    expand_portal(P0, P1, P2, P3, v4);
    it++;
  }
}

// canonical (geom1, geom2): lower type first, then lower id
__device__ __forceinline__ void canon_pair(int a, int b, int ta, int tb, int& g1, int& g2) {
  if (ta > tb || (ta == tb && a > b)) { g1 = b; g2 = a; } else { g1 = a; g2 = b; }
}

// pass 2 stores the hit (depth, point, normal), friction and the geom/body ids; the contact
// frame's tangent and the zeroed tail are filled by collision()'s lane-per-contact epilogue
template <int CL>
__device__ __forceinline__ void write_contact(SharedT<CL>& S, int slot, int g1, int g2, int b1, int b2, const Hit& h,
                                              real mu) {
  real* C = S.con[slot];
  C[0] = h.dist;
  C[1] = h.pos[0]; C[2] = h.pos[1]; C[3] = h.pos[2];
  C[4] = h.n[0]; C[5] = h.n[1]; C[6] = h.n[2];
  C[10] = mu;
  S.cgeom[slot][0] = (int16_t)g1; S.cgeom[slot][1] = (int16_t)g2;
  S.cbody[slot][0] = (int16_t)b1; S.cbody[slot][1] = (int16_t)b2;
}


#include "gm_newton.hip"

// hit: the box-box hit slots (S.cl.hit, in the union; a DUO workgroup's helper wave passes
// its own array, the union being live with crb_rne's composites while it runs)
template <int CL>
__device__ __forceinline__ bool collision(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T, int lane,
                          bool prof, real (*hit)[8][4]) {
  unsigned long long t0 = prof ? clock64() : 0;
  (void)t0;
  // one lane per candidate pair, in batches of 64 pairs: the 6 N + 15 pairs fit one batch
  // for N <= 8 (CL <= 10), N = 9, 10 take two (gm_create checks npair against this);
  // contacts keep the pair order across batches
  constexpr int NBATCH = gm_pair_batches(CL);
  int written = 0;
  bool ran_mpr = false;   // profiling: a lane of this env ran the convex (MPR) collider
  // (not unrolled: with two batches (N = 9, 10) the unrolled copies held each other's
  // collider state live and the pair loop spilled ~1 K scratch operations per substep)
#pragma nounroll
  for (int bi = 0; bi < NBATCH; bi++) {
    const int pr = bi * NT + lane;
    int cnt = 0, kind = 0, g1 = 0, g2 = 0, b1 = 0, b2 = 0;
    unsigned hm = 0;   // multi-point colliders: the counted candidates (pass 2 revisits only these)
    Hit single;
    GeomV A, B;
    CylFrame cf;
    BBox bbs;
    int bslot = -1;          // box-box face case: this lane's hit slot (S.cl), -1 = none
    real bn[3] = {0, 0, 0}, bsg = 0;   // and its manifold normal / sign
    real ea[3], eb[3], da[3], db[3];
    if (pr < T->npair) {
      const int a = T->pr_g[pr][0], b = T->pr_g[pr][1];
      const int ta0 = T->pr_type[pr][0], tb0 = T->pr_type[pr][1];
      const int ta = ta0 < 0 ? S.s.obj_type : ta0, tb = tb0 < 0 ? S.s.obj_type : tb0;
      canon_pair(a, b, ta, tb, g1, g2);
      const int s1 = (g1 == a) ? 0 : 1;
      b1 = T->pr_body[pr][s1]; b2 = T->pr_body[pr][1 - s1];   // kept with the contact (LDS)
      load_pair_geom(S, T, pr, s1, A);
      load_pair_geom(S, T, pr, 1 - s1, B);
#ifdef GM_PHASE_SPLIT_COLL
      PH(15);   // developer split: pair setup + geom poses
#endif
      bool pass;
      if (A.type == GM_GEOM_PLANE) {
        real nz[3] = {A.R[2], A.R[5], A.R[8]};
        real dv[3] = {B.c[0] - A.c[0], B.c[1] - A.c[1], B.c[2] - A.c[2]};
        pass = !(dot3(dv, nz) > B.rbound);
      } else {
        real dv[3] = {B.c[0] - A.c[0], B.c[1] - A.c[1], B.c[2] - A.c[2]};
        real rr = A.rbound + B.rbound;
        pass = !(dot3(dv, dv) > rr * rr);
      }
      if (pass) {
        if (A.type == GM_GEOM_PLANE) {
          NB_BEGIN();
          if (B.type == GM_GEOM_SPHERE) { kind = 1; cnt = plane_sphere(A, B, single); }
          else if (B.type == GM_GEOM_BOX) {
            kind = 2;
            Hit t;
            for (int i = 0; i < 8 && cnt < 4; i++) {
              const int ok = plane_box_point(A, B, i, t);
              hm |= (unsigned)ok << i;
              cnt += ok;
            }
          } else if (B.type == GM_GEOM_CYLINDER) {
            kind = 3;
            Hit t;
            cyl_frame(A, B, cf);
            for (int i = 0; i < 8 && cnt < 4; i++) {
              const int ok = plane_cyl_point(A, B, cf, i, t);
              hm |= (unsigned)ok << i;
              cnt += ok;
            }
          }
          NB_END(15);
        } else if (A.type == GM_GEOM_SPHERE && B.type == GM_GEOM_BOX) {
          NB_BEGIN();
          kind = 1; cnt = sphere_box(A, B, single);
          NB_END(16);
        } else if (A.type == GM_GEOM_BOX && B.type == GM_GEOM_BOX) {
          NB_BEGIN();
          // mjc_BoxBox: separating axes, then the face-clipped manifold or one edge contact
          bb_setup(A, B, bbs, ea, eb, da, db);
          if (bbs.kind == 1) {
            kind = 4;
            // this lane's hit slot: its rank among the face-case lanes (the active lanes here)
            const unsigned long long fb = __ballot(1);
            const int rank = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(fb >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)fb, 0u));
            bslot = rank < GM_BB_SLOTS ? rank : -1;
#pragma unroll
            for (int i = 0; i < BB_NCAND; i++) {
              if (cnt < 8) {
                real P[3], dep;
                const int ok = bb_face_cand(bbs, i, P, dep);
                if (ok && bslot >= 0) {
                  real* hs = hit[bslot][cnt];
                  hs[0] = P[0]; hs[1] = P[1]; hs[2] = P[2]; hs[3] = dep;
                }
                hm |= (unsigned)ok << i;
                cnt += ok;
              }
            }
            bn[0] = bbs.n[0]; bn[1] = bbs.n[1]; bn[2] = bbs.n[2]; bsg = bbs.sgn;
          } else if (bbs.kind == 2) {
            kind = 1; cnt = bb_edge_hit(bbs, ea, eb, da, db, single);
          }
          NB_END(17);
        } else {
          NB_BEGIN();
          ran_mpr = true;
          // a cylinder against a box (the gripper's links against a cylinder object) on every
          // MPR lane: the instance with the support types fixed, no type test per support call
          const bool cb = A.type == GM_GEOM_CYLINDER && B.type == GM_GEOM_BOX;
          if (__ballot(!cb) == 0ull)
            cnt = mpr<GM_GEOM_CYLINDER, GM_GEOM_BOX>(A, B, (real)m->mpr_tolerance, m->mpr_iterations, single);
          else
            cnt = mpr(A, B, (real)m->mpr_tolerance, m->mpr_iterations, single);
          kind = 1;
          if (cnt && !(single.dist < 0)) cnt = 0;
          NB_END(12);
        }
      }
    }
#ifdef GM_PHASE_SPLIT_COLL
    PH(16);   // developer split: broadphase + narrowphase
#endif
    // contact slots: exclusive prefix sum of the per-lane counts (0..8, four bits) from
    // four ballots -- no LDS round trip
    int off = written, total = 0;
#pragma unroll
    for (int bit = 0; bit < 4; bit++) {
      const unsigned long long bal = __ballot((cnt >> bit) & 1);
      off += (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u)) << bit;
      total += __popcll(bal) << bit;
    }
    if (pr < T->npair) { S.pair_off[pr] = (int16_t)off; S.pair_cnt[pr] = (int16_t)cnt; }
    if (cnt > 0) {
      NB_BEGIN();
      real mu = fmax(A.friction, B.friction);
      if (kind == 1) {
        if (off < GM_MAX_CON) write_contact(S, off, g1, g2, b1, b2, single, mu);
      } else if (kind == 4 && bslot >= 0) {
        // the stored hits, in candidate order as pass 1 found them (bb_face_hit's operations)
        for (int w = 0; w < cnt; w++) {
          const real* hs = hit[bslot][w];
          const real dep = hs[3];
          Hit t;
          t.dist = -dep;
#pragma unroll
          for (int k = 0; k < 3; k++) { t.pos[k] = hs[k] + (0.5 * dep) * bn[k]; t.n[k] = bsg * bn[k]; }
          if (off + w < GM_MAX_CON) write_contact(S, off + w, g1, g2, b1, b2, t, mu);
        }
      } else if (kind == 4) {
        // (more face-case lanes than slots: the counted candidates again)
        int w = 0;
#pragma unroll
        for (int i = 0; i < BB_NCAND; i++) {
          if ((hm >> i) & 1u) {
            real P[3], dep;
            Hit t;
            bb_face_cand(bbs, i, P, dep);
            bb_face_hit(bbs, P, dep, t);
            if (off + w < GM_MAX_CON) write_contact(S, off + w, g1, g2, b1, b2, t, mu);
            w++;
          }
        }
      } else {
        Hit t;
        int w = 0;
        while (hm) {   // the counted corners in index order, as pass 1 found them
          const int i = __builtin_ctz(hm);
          hm &= hm - 1;
          if (kind == 2) plane_box_point(A, B, i, t);
          else plane_cyl_point(A, B, cf, i, t);
          if (off + w < GM_MAX_CON) write_contact(S, off + w, g1, g2, b1, b2, t, mu);
          w++;
        }
      }
      NB_END(24);
    }
    written += total;
  }
  const bool any_mpr = __ballot(ran_mpr) != 0;
  if (lane == 0 && any_mpr) {
    S.work_mpr += 1;
    if (prof) S.tph[29] += 1;
  }
  // contact frames, one contact per lane (GM_MAX_CON <= 64): the normal and a tangent, as
  // make_frame builds them; the rest of the frame is implied by the two
  static_assert(GM_MAX_CON <= NT, "contact frames: one lane per contact");
  const int ncon = written < GM_MAX_CON ? written : GM_MAX_CON;
  GM_WAVE_SYNC();
  if (lane < ncon) {
    real* C = S.con[lane];
    const real n[3] = {C[4], C[5], C[6]};
    real F[9];
    make_frame(F, n);
    C[7] = F[3]; C[8] = F[4]; C[9] = F[5];
    C[11] = 0; C[12] = 0; C[13] = 0;
  }
  if (lane == 0) {
    S.ncon = ncon;
    S.overflow = written > GM_MAX_CON;
  }
  GM_WAVE_SYNC();
  return any_mpr;
}

// DUO workgroups: the helper wave's euler_factor results, lane-major ([j][64]: L[1..CL], lb,
// 1 / d), then the base pivot's Schur sum
template <int CL>
__device__ __forceinline__ real* duo_ef() {
  __shared__ real ef[64 * (CL + 2) + 1];
  return ef;
}

// ============================================================ integrate
template <int CL, bool CAL, bool DUO = false>
__device__ __forceinline__ void integrate(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T, int lane) {
  const real h = CAL ? S.s.dt : m->timestep;
  if constexpr (CAL) {
    // mj_checkAcc's mjWARN_BADQACC (is_sim_unstable, myfunctions.cpp:4233-4242): a
    // non-finite or |qacc| > mjMAXVAL acceleration; sticky until the next reset
    const bool bad = lane < T->nv && !(fabs(S.qacc[lane]) <= 1e10);
    if (__ballot(bad) != 0ull && lane == 0) S.s.badqacc = 1;
  }
  // mj_Euler: under MuJoCo's actuator order the joint damping is implicit here
  // (euler_damping: qacc_e = (M + h D)^-1 (qfrc_smooth + qfrc_constraint) into S.xs)
  const bool mj = m->mujoco_actuators != 0;
  if constexpr (DUO) {
    // the helper factored M + h D during the constraint solve (duo_helper); third barrier
    __syncthreads();
    if (mj) {
      const int ln = fresh_lane();
      const real* ef = duo_ef<CL>();
      real L[CL + 1];
      L[0] = 0.0;
#pragma unroll
      for (int j = 1; j <= CL; j++) L[j] = ef[(j - 1) * 64 + ln];
      euler_solve<CL>(S, T, h, ln, L, ef[CL * 64 + ln], ef[(CL + 1) * 64 + ln], ef[64 * (CL + 2)]);
    }
  } else {
    if (mj) euler_damping<CL>(S, T, h, fresh_lane());
  }
  if (lane < T->nv) S.s.qvel[lane] += h * (mj ? S.xs[lane] : S.qacc[lane]);
  GM_WAVE_SYNC();
  if (lane < T->nv && lane < T->dof_obj) {
    S.s.qpos[lane] += h * S.s.qvel[lane];   // slides/hinges: qposadr == dofadr before the object
  }
  if (lane == 0) {
    int qa = T->qadr_obj, da = T->dof_obj;
    for (int k = 0; k < 3; k++) S.s.qpos[qa + k] += h * S.s.qvel[da + k];
    real* q = &S.s.qpos[qa + 3];
    real w[3] = {S.s.qvel[da + 3], S.s.qvel[da + 4], S.s.qvel[da + 5]};
    // (sqrt_n / div_n: the library operations' results wherever their range scaling is
    // inactive -- a |w| below 2^-383 takes the branch either way)
    real wn = sqrt_n(dot3(w, w));
    if (wn > 1e-15) {
      real ang = wn * h;
      real sn, cs;
      gm_sincos(0.5 * ang, &sn, &cs);
      sn = div_n(sn, wn);
      real dq[4] = {cs, w[0] * sn, w[1] * sn, w[2] * sn};
      quatmul(q, q, dq);
    }
    quatnorm(q);
    S.s.time += h;
  }
  GM_WAVE_SYNC();
}

}  // namespace gmf
#pragma clang fp contract(off)
using gmf::kinematics;
using gmf::crb_rne;
using gmf::mass_and_forces;
using gmf::collision;
using gmf::newton_solve;
using gmf::integrate;
using gmf::euler_factor;
using gmf::duo_ef;
using gmf::contact_rows;
using gmf::duo_rows;
using gmf::DuoRows;

// ============================================================ reference scalar logic (lane 0)
// luke::Gripper in fp64 (gripper.cpp), bit-for-bit the same operations as the reference
#define G_XY_MIN 49e-3
#define G_XY_MAX 134e-3
#define G_Z_MIN 0e-3
#define G_Z_MAX 165e-3
#define G_TOL 1e-4
#define G_LEAD 35e-3
__device__ __forceinline__ double g_xy_step_m() { return 4.0 / (1.0 * 400 * 1e3); }
__device__ __forceinline__ double g_z_step_m() { return 4.8768 / (1 * 400 * 1e3); }
__device__ __forceinline__ double g_calc_th(double x, double y) { return asin((y - x) / G_LEAD) * 1; }
__device__ __forceinline__ double g_calc_y(const GmGrip& g, double th) { return g.x + 1 * G_LEAD * sin(th); }
__device__ __forceinline__ int g_xs(const GmGrip& g) { return (int)round((G_XY_MAX - g.x) / g_xy_step_m()); }
__device__ __forceinline__ int g_ys(const GmGrip& g) { return (int)round((G_XY_MAX - g.y) / g_xy_step_m()); }
__device__ __forceinline__ int g_zs(const GmGrip& g) { return (int)round(g.z / g_z_step_m()); }
__device__ __forceinline__ double g_th_deg(const GmGrip& g) { return (180.0 / 3.14159265358979323846) * g_calc_th(g.x, g.y); }
__device__ int g_update_xy(GmGrip& g) {
  const double to_rad = 3.14159265358979323846 / 180.0;
  const double th_min = -40 * to_rad, th_max = 40 * to_rad;
  const double hyp = sqrt(pow(235e-3, 2) + pow(35.0e-3, 2));
  const double rest = atan(35.0e-3 / 235e-3);
  int wl = 1;
  if (g.x > G_XY_MAX + G_TOL) { g.x = G_XY_MAX; wl = 0; }
  if (g.x < G_XY_MIN - G_TOL) { g.x = G_XY_MIN; wl = 0; }
  if (g.y > G_XY_MAX + G_TOL) { g.y = G_XY_MAX; wl = 0; }
  if (g.y < G_XY_MIN - G_TOL) { g.y = G_XY_MIN; wl = 0; }
  double nth = g_calc_th(g.x, g.y);
  if (nth > th_max) { nth = th_max; g.y = g_calc_y(g, th_max); wl = 0; }
  if (nth < th_min) { nth = th_min; g.y = g_calc_y(g, th_min); wl = 0; }
  g.th = nth;
  double th_lim = (asin((-1.0 - g.x) / hyp) + rest) * 1;
  if (g.th < th_lim) { g.y = g_calc_y(g, th_lim); g.th = th_lim; wl = 0; }
  g.sx = g_xs(g);
  g.sy = g_ys(g);
  return wl;
}
__device__ int g_update_z(GmGrip& g) {
  int wl = 1;
  if (g.z > G_Z_MAX + G_TOL) { g.z = G_Z_MAX; wl = 0; }
  if (g.z < G_Z_MIN - G_TOL) { g.z = G_Z_MIN; wl = 0; }
  g.sz = g_zs(g);
  return wl;
}
__device__ void g_reset(GmGrip& g) {
  g.x = G_XY_MAX - 1.0 * (4 * 1e-3 / 1.0);
  g.y = g.x;
  g.z = G_Z_MIN + 1.0 * (4.8768 * 1e-3 / 1);
  int a = g_update_xy(g); int b = g_update_z(g); (void)a; (void)b;
}
__device__ int g_set_xyz_m_rad(GmGrip& g, double x, double th, double z) {
  g.x = x; g.y = g_calc_y(g, th);
  int in_lim = g_update_xy(g);
  g.z = z;
  return g_update_z(g) ? in_lim : 0;
}
__device__ int g_set_xyz_m(GmGrip& g, double x, double y, double z) {
  g.x = x; g.y = y; g.z = z;
  int a = g_update_xy(g); int b = g_update_z(g);
  return a * b;
}
__device__ int g_set_xyz_step(GmGrip& g, int xs, int ys, int zs) {
  g.x = G_XY_MAX - g_xy_step_m() * xs; g.y = G_XY_MAX - g_xy_step_m() * ys;
  int in_lim = g_update_xy(g);
  g.z = g_z_step_m() * zs;
  return g_update_z(g) ? in_lim : 0;
}
__device__ int g_step_to(GmGrip& g, const GmGrip& t, int num) {
  int fin = 1;
  int xg = t.sx - g.sx, yg = t.sy - g.sy, zg = t.sz - g.sz;
  if (xg < 0) { if (-xg > num) { xg = -num; fin = 0; } } else if (xg > num) { xg = num; fin = 0; }
  if (yg < 0) { if (-yg > num) { yg = -num; fin = 0; } } else if (yg > num) { yg = num; fin = 0; }
  if (zg < 0) { if (-zg > num) { zg = -num; fin = 0; } } else if (zg > num) { zg = num; fin = 0; }
  g_set_xyz_step(g, g.sx + xg, g.sy + yg, g.sz + zg);
  return fin;
}

// update_all: update_stepper / update_constraints (myfunctions.cpp:2129-2284), antiroll
template <int CL>
GM_EPI_ATTR void update_all(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T, int lane) {
  GmEnvHot& s = S.s;
  const bool stepping = s.time > s.last_step_time + m->time_per_step;   // uniform (LDS broadcast)
  // Once a stepper update left `next` bit for bit unchanged, every later one in this
  // env-step does too (`end` only changes between env-steps, and g_step_to is a pure
  // function of the two grippers), and the lock-toggle tests see the same (end, next) as
  // that update did, so their flags already match: only the step time moves.
  const bool fixed = stepping && S.stp_fixed;
  int nx = 0, ny = 0, nz = 0;
  if (stepping && !fixed) {
    // the end (lane 0) and next (lane 1) grippers' step counts and angle in one pass of
    // the wave instead of two serial evaluations on lane 0 (an asin and two divisions each)
    const GmGrip& g = (lane & 1) ? s.next : s.end;
    const int xs = g_xs(g), zs = g_zs(g);
    const double th = g_th_deg(g);
    nx = __builtin_amdgcn_readlane(xs, 0) != __builtin_amdgcn_readlane(xs, 1);
    ny = !(fabs(readlane_real(th, 0) - readlane_real(th, 1)) < 5e-1);
    nz = __builtin_amdgcn_readlane(zs, 0) != __builtin_amdgcn_readlane(zs, 1);
  }
  if (lane == 0) {
    if (fixed) {
      s.last_step_time = s.time;
    } else if (stepping) {
      if (nx != s.old_x) {
        for (int k = 0; k < T->nlock; k++)
          if (m->lock_kind[k] == 0) { s.lock_active[k] = !nx; if (!nx) s.lock_q[k] = S.lock_pre[k]; }
        s.old_x = nx;
      }
      if (ny != s.old_y) s.old_y = ny;   // revolute locks disabled (myfunctions.cpp:479)
      if (nz != s.old_z) {
        for (int k = 0; k < T->nlock; k++)
          if (m->lock_kind[k] == 2) { s.lock_active[k] = !nz; if (!nz) s.lock_q[k] = S.lock_pre[k]; }
        s.old_z = nz;
      }
      s.last_step_time = s.time;
      const GmGrip before = s.next;
      g_step_to(s.next, s.end, m->stepper_num_steps);
      const GmGrip& a = s.next;
      S.stp_fixed = __double_as_longlong(a.x) == __double_as_longlong(before.x) &&
                    __double_as_longlong(a.y) == __double_as_longlong(before.y) &&
                    __double_as_longlong(a.z) == __double_as_longlong(before.z) &&
                    __double_as_longlong(a.th) == __double_as_longlong(before.th) && a.sx == before.sx &&
                    a.sy == before.sy && a.sz == before.sz;
    }
    const real* v = &s.qvel[T->dof_obj];
    real mag = sqrt_n(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);   // (= sqrt wherever it decides anything)
    if (mag < 1e-6) for (int k = 0; k < 6; k++) s.qvel[T->dof_obj + k] = 0;
  }
  GM_WAVE_SYNC();
}

// ---- RNG: minstd_rand0 + generate_canonical (libstdc++), per-env stream ----
__device__ __forceinline__ uint32_t lcg_next(uint32_t& s) {
  s = (uint32_t)(((uint64_t)s * 16807ull) % 2147483647ull);
  return s;
}
__device__ float unif01(uint32_t& s) {
  const float r = 2147483646.0f;
  float sum = (float)(lcg_next(s) - 1u) * 1.0f;
  float ret = sum / r;
  if (ret >= 1.0f) ret = __int_as_float(0x3F7FFFFF);  // nextafterf(1, 0)
  return ret * (1.0f - 0.0f) + 0.0f;
}
__device__ double canon_d(uint32_t& s) {
  const double r = 2147483646.0;
  double sum = 0.0, tmp = 1.0;
  for (int k = 0; k < 2; k++) { sum += (double)(lcg_next(s) - 1u) * tmp; tmp *= r; }
  double ret = sum / tmp;
  if (ret >= 1.0) ret = __longlong_as_double(0x3FEFFFFFFFFFFFFFLL);  // nextafter(1, 0)
  return ret;
}

// ---- sensors (mjclass.h:155-241) ----
// SlidingWindow::add / read_element on a ring of GM_RING readings (the window itself
// lives in the env's HBM record, GmEnvState::ring; its write index in the hot state)
typedef float (*RingRef)[GM_RING];
__device__ __forceinline__ void ring_add(GmEnvHot& s, RingRef R, int st, float x) {
  int i = s.ring_i[st] + 1;
  if (i > GM_RING - 1) i = 0;
  s.ring_i[st] = i;
  R[st][i] = x;
}
__device__ __forceinline__ float ring_read(const GmEnvHot& s, RingRef R, int st, int n) {
  int idx = s.ring_i[st] - n;
  while (idx < 0) idx += GM_RING;
  return R[st][idx];
}
__device__ __forceinline__ float ring_latest(const GmEnvHot& s, RingRef R, int st) {
  return s.ring_i[st] == -1 ? R[st][0] : R[st][s.ring_i[st]];
}
__device__ float s_normalise(const gm_sensor& ss, float v) {
  if (!ss.use_normalisation) return v;
  if (ss.normalise <= 0) return v < 0 ? -1.0f : 1.0f;
  else if (v > ss.normalise) return 1.0f;
  if (v < -ss.normalise) return -1.0f;
  return v / ss.normalise;
}
__device__ float s_noise(GmEnvHot& s, const gm_sensor& ss, int slot, float value, int i) {
  if (!ss.use_noise) return value;
  const float two_pi = (float)(2.0 * 3.14159265358979323846);
  const float eps = 1.1920928955078125e-07f;
  float mu = s.rand_mu[slot][i - 1];
  if (ss.noise_std < eps) {
    float noise = mu + ss.noise_mag * (2 * unif01(s.rng) - 1);
    value += noise;
  } else {
    float u1, u2;
    do { u1 = unif01(s.rng); } while (u1 <= eps);
    u2 = unif01(s.rng);
    float mag = (float)(ss.noise_std * sqrt(-2.0 * (double)logf(u1)));
    float z0 = mag * cosf(two_pi * u2) + mu;
    value += z0;
  }
  if (value > 1) value = 1;
  else if (value < -1) value = -1;
  return value;
}
__device__ int s_ready(GmEnvHot& s, const gm_sensor& ss, int slot) {
  double tbr = (double)(1 / ss.read_rate);
  if (s.time > s.last_read[slot] + tbr) { s.last_read[slot] = s.time; return 1; }
  return 0;
}

// The earliest sim time at which one of monitor_sensors' four sensors becomes ready:
// s_ready's test is time > last_read + tbr, so time <= min over the sensors of
// (last_read + tbr) means none is, with the same operands and the same rounding.
__device__ __forceinline__ double next_sensor_read(const GmEnvHot& s, const gm_settings& st) {
  const gm_sensor* ss[4] = {&st.bending_gauge, &st.axial_gauge, &st.palm_sensor, &st.wrist_sensor_Z};
  const int slot[4] = {SL_BEND, SL_AXIAL, SL_PALM, SL_WRISTZ};
  double t = __builtin_inf();
  for (int k = 0; k < 4; k++) {
    const double tk = s.last_read[slot[k]] + (double)(1 / ss[k]->read_rate);
    t = tk < t ? tk : t;
  }
  return t;
}

// bending gauge: cubic least squares through the N+1 joint points, evaluated at
// gauge.xpos (read_armadillo_gauge, myfunctions.cpp:2699-2795).  Evaluated in fp64
// (two reads per env-step at 10 Hz: negligible cost): the fitted value at 50 mm is
// ~16x smaller than the tip deflection, so an fp32 fit would cost ~3e-5 relative.
// Householder QR on a centred/scaled abscissa -- the same least-squares solution as
// the reference's arma::polyfit on the raw Vandermonde.
template <int NS>
__device__ float gauge_reading(const gm_model* __restrict__ m, const real* q) {
  constexpr int P = NS + 1;
  const double Ls = m->segment_length;
  double X[P], Yv[P];
  X[0] = m->fixed_first_segment ? Ls : 0.0;
  Yv[0] = 0;
  double cum = 0;
#pragma unroll
  for (int i = 0; i < NS; i++) {
    cum = (i == 0) ? (double)q[0] : cum + (double)q[i];
    double sn, cs;
    gm_sincos(cum, &sn, &cs);
    X[i + 1] = X[i] + Ls * cs;
    Yv[i + 1] = Yv[i] + Ls * sn;
  }
  const double half = 0.5 * m->finger_length;
  const double ihalf = 1.0 / half;
  double A[P][4], b[P];
#pragma unroll
  for (int i = 0; i < P; i++) {
    const double t = (X[i] - half) * ihalf;
    A[i][0] = t * t * t; A[i][1] = t * t; A[i][2] = t; A[i][3] = 1.0;
    b[i] = Yv[i];
  }
  // Householder QR of the (centred) Vandermonde system, as LAPACK's dgels under arma::polyfit
#pragma unroll
  for (int k = 0; k < 4; k++) {
    double nrm = 0;
#pragma unroll
    for (int i = k; i < P; i++) nrm += A[i][k] * A[i][k];
    nrm = sqrt(nrm);
    const double alpha = A[k][k] > 0 ? -nrm : nrm;
    double v[P];
#pragma unroll
    for (int i = 0; i < P; i++) v[i] = (i >= k) ? A[i][k] : 0.0;
    v[k] -= alpha;
    double vv = 0;
#pragma unroll
    for (int i = k; i < P; i++) vv += v[i] * v[i];
    if (vv < 1e-300) continue;
    const double ivv = 2.0 / vv;
#pragma unroll
    for (int j = k; j < 4; j++) {
      double sacc = 0;
#pragma unroll
      for (int i = k; i < P; i++) sacc += v[i] * A[i][j];
      sacc *= ivv;
#pragma unroll
      for (int i = k; i < P; i++) A[i][j] -= sacc * v[i];
    }
    double sacc = 0;
#pragma unroll
    for (int i = k; i < P; i++) sacc += v[i] * b[i];
    sacc *= ivv;
#pragma unroll
    for (int i = k; i < P; i++) b[i] -= sacc * v[i];
  }
  double coeff[4];
#pragma unroll
  for (int k = 3; k >= 0; k--) {
    double sacc = b[k];
#pragma unroll
    for (int j = k + 1; j < 4; j++) sacc -= A[k][j] * coeff[j];
    coeff[k] = sacc / A[k][k];
  }
  const double tg = (m->gauge_xpos - half) * ihalf;
  const double y = ((coeff[0] * tg + coeff[1]) * tg + coeff[2]) * tg + coeff[3];
  return (float)y * 1000;
}

// extract_forces_faster (objecthandler.cpp:737-992) over the last substep's contacts.
// forces[]: obj_loc f1,f2,f3,palm (12) | obj ground global (3) | all_loc f1,f2,f3 x (3),
//           all_loc palm x (1) | gnd_loc f1,f2,f3 x (3)
template <int CL>
__device__ void extract_forces(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T) {
  real og[5][3], ag[4][3], gg[3][3];
  for (int a = 0; a < 5; a++) for (int k = 0; k < 3; k++) og[a][k] = 0;
  for (int a = 0; a < 4; a++) for (int k = 0; k < 3; k++) ag[a][k] = 0;
  for (int a = 0; a < 3; a++) for (int k = 0; k < 3; k++) gg[a][k] = 0;
  for (int i = 0; i < S.ncon; i++) {
    const real* C = S.con[i];
    int c1 = m->geom_class[S.cgeom[i][0]], c2 = m->geom_class[S.cgeom[i][1]];
    int w_obj = (c1 == GM_CLS_OBJECT || c2 == GM_CLS_OBJECT);
    int w_f0 = (c1 == GM_CLS_FINGER1 || c2 == GM_CLS_FINGER1);
    int w_f1 = (c1 == GM_CLS_FINGER2 || c2 == GM_CLS_FINGER2);
    int w_f2 = (c1 == GM_CLS_FINGER3 || c2 == GM_CLS_FINGER3);
    int w_palm = (c1 == GM_CLS_PALM || c2 == GM_CLS_PALM);
    int w_gnd = (c1 == GM_CLS_GROUND || c2 == GM_CLS_GROUND);
    real g[3];
    real Fr[9];
    Fr[0] = C[4]; Fr[1] = C[5]; Fr[2] = C[6]; Fr[3] = C[7]; Fr[4] = C[8]; Fr[5] = C[9];
    cross3(Fr + 6, Fr, Fr + 3);
    for (int k = 0; k < 3; k++) g[k] = Fr[k] * C[11] + Fr[3 + k] * C[12] + Fr[6 + k] * C[13];
    int wf[3] = {w_f0, w_f1, w_f2};
    if (w_obj) {
      for (int f = 0; f < 3; f++) if (wf[f]) for (int k = 0; k < 3; k++) og[f][k] += g[k];
      if (w_palm) for (int k = 0; k < 3; k++) og[3][k] += g[k];
      if (w_gnd) for (int k = 0; k < 3; k++) og[4][k] += g[k];
    }
    for (int f = 0; f < 3; f++)
      if (wf[f]) {
        for (int k = 0; k < 3; k++) ag[f][k] += g[k];
        if (w_gnd) for (int k = 0; k < 3; k++) gg[f][k] += g[k];
      }
    if (w_palm) for (int k = 0; k < 3; k++) ag[3][k] += g[k];
  }
  float* F = S.forces;
  for (int f = 0; f < 4; f++) {
    int b = f < 3 ? T->body_finger[f] : T->body_palm;
    real Rb[9];
    body_R(S, b, Rb);
    real loc[3];
    mulmtv3(loc, Rb, og[f]);
    F[3 * f] = (float)loc[0]; F[3 * f + 1] = (float)loc[1]; F[3 * f + 2] = (float)loc[2];
    real al[3];
    mulmtv3(al, Rb, ag[f]);
    if (f < 3) F[15 + f] = (float)al[0]; else F[18] = (float)al[0];
    if (f < 3) { real gl[3]; mulmtv3(gl, Rb, gg[f]); F[19 + f] = (float)gl[0]; }
  }
  F[12] = (float)og[4][0]; F[13] = (float)og[4][1]; F[14] = (float)og[4][2];
}

// mj_rnePostConstraint's cfrc_ext for the live object (myfunctions.cpp:1905), as
// ObjectHandler::get_object_net_force_faster reads it (objecthandler.cpp:543-565): each
// contact's world force (frame^T * contact-frame force) acts on geom2, its reaction on
// geom1; torques about the object's centre of mass.  out = [force; torque] (the
// reference's swapped order).  Lane-parallel over contacts, wave-reduced.
template <int CL>
__device__ void object_net_wrench(SharedT<CL>& S, const GmTopo* __restrict__ T, int lane, real* out) {
  real w[6] = {0, 0, 0, 0, 0, 0};
  if (lane < S.ncon) {
    const real* C = S.con[lane];
    const int g1 = S.cgeom[lane][0], g2 = S.cgeom[lane][1];
    const real sgn = (g2 == T->geom_obj) ? 1.0 : (g1 == T->geom_obj) ? -1.0 : 0.0;
    real Fr[9], g[3], r[3], t[3];
    Fr[0] = C[4]; Fr[1] = C[5]; Fr[2] = C[6]; Fr[3] = C[7]; Fr[4] = C[8]; Fr[5] = C[9];
    cross3(Fr + 6, Fr, Fr + 3);
    for (int k = 0; k < 3; k++) g[k] = Fr[k] * C[11] + Fr[3 + k] * C[12] + Fr[6 + k] * C[13];
    const int bo = T->body_obj;
    for (int k = 0; k < 3; k++) r[k] = C[1 + k] - S.xpos[bo][k];
    cross3(t, r, g);
    for (int k = 0; k < 3; k++) { w[k] = sgn * g[k]; w[3 + k] = sgn * t[k]; }
  }
  // contact order sum (lane 0 accumulates in index order, as the oracle does)
  for (int k = 0; k < 6; k++) {
    real acc = 0;
    for (int i = 0; i < GM_MAX_CON; i++) acc += readlane_real(w[k], i);
    out[k] = acc;
  }
}

// MjClass::monitor_sensors (mjclass.cpp:741-898)
template <int CL>
GM_EPI_ATTR void monitor_sensors(SharedT<CL>& S, const gm_model* __restrict__ m, const gm_config* __restrict__ C,
                                const GmTopo* __restrict__ T, int lane) {
  // (per-env LDS fields, no function-scope __shared__: substep_loop and monitor_sensors are
  // reached from two kernels, and such variables would cost a per-kernel offset lookup)
  if (lane == 0) S.bend_ready = s_ready(S.s, C->s.bending_gauge, SL_BEND);
  GM_WAVE_SYNC();
  const int bend_ready = S.bend_ready;
  if (bend_ready && lane < 3) S.gauge_tmp[lane] = gauge_reading<CL - 2>(m, &S.s.qpos[T->dof_f0[lane] + 2]);
  GM_WAVE_SYNC();
  if (lane == 0) {
    GmEnvHot& s = S.s;
  RingRef R = S.gs->ring;
    const gm_settings& st = C->s;
    int have = 0;
    if (bend_ready) {
      float g[3] = {S.gauge_tmp[0], S.gauge_tmp[1], S.gauge_tmp[2]};
      for (int f = 0; f < 3; f++) ring_add(s, R, ST_SI_GAUGE + f, (float)(g[f] * C->sim_gauge_raw_to_N_factor));
      for (int f = 0; f < 3; f++) g[f] = s_normalise(st.bending_gauge, g[f]);
      for (int f = 0; f < 3; f++) g[f] = s_noise(s, st.bending_gauge, SL_BEND, g[f], f + 1);
      for (int f = 0; f < 3; f++) ring_add(s, R, ST_GAUGE + f, g[f]);
    }
    if (s_ready(s, st.axial_gauge, SL_AXIAL)) {
      if (!have) { extract_forces(S, m, T); have = 1; }
      float a[3] = {S.forces[15], S.forces[16], S.forces[17]};
      for (int f = 0; f < 3; f++) ring_add(s, R, ST_SI_AXIAL + f, a[f]);
      for (int f = 0; f < 3; f++) a[f] = s_normalise(st.axial_gauge, a[f]);
      for (int f = 0; f < 3; f++) a[f] = s_noise(s, st.axial_gauge, SL_AXIAL, a[f], f + 1);
      for (int f = 0; f < 3; f++) ring_add(s, R, ST_AXIAL + f, a[f]);
    }
    if (s_ready(s, st.palm_sensor, SL_PALM)) {
      if (!have) { extract_forces(S, m, T); have = 1; }
      float p = S.forces[18];
      p *= st.palm_scale_factor;
      ring_add(s, R, ST_SI_PALM, p);
      p = s_normalise(st.palm_sensor, p);
      p = s_noise(s, st.palm_sensor, SL_PALM, p, 1);
      ring_add(s, R, ST_PALM, p);
    }
    if (s_ready(s, st.wrist_sensor_Z, SL_WRISTZ)) {
      float z = 0.0f;
      z -= st.wrist_sensor_Z.raw_value_offset;
      ring_add(s, R, ST_SI_WZ, z);
      z = s_normalise(st.wrist_sensor_Z, z);
      z = s_noise(s, st.wrist_sensor_Z, SL_WRISTZ, z, 1);
      ring_add(s, R, ST_WZ, z);
    }
  }
  GM_WAVE_SYNC();
}

// ============================================================ one full substep
template <int CL, bool CAL, bool DUO>
__device__ __forceinline__ void physics_substep_body(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T,
                                                     int lane, bool prof) {
  unsigned long long t0 = prof ? clock64() : 0;
  if (lane < T->nlock) S.lock_pre[lane] = S.s.qpos[m->lock_dof[lane]];
  kinematics<CL>(S, m, T, fresh_lane(), prof);
  PH(0);
  if constexpr (DUO) {
    // the collider needs only the poses: the helper wave runs it (duo_helper) while this
    // wave forms the inertia and forces; the two barriers are the handshake
    if (lane == 0) S.duo_cmd = 1;
    __syncthreads();
    crb_rne<CL, CAL>(S, m, T, fresh_lane(), prof);
    PH(1);
    mass_and_forces<CL, CAL>(S, m, T, fresh_lane());
    PH(2);
    __syncthreads();
  } else {
    crb_rne<CL, CAL>(S, m, T, fresh_lane(), prof);
    PH(1);
    mass_and_forces<CL, CAL>(S, m, T, fresh_lane());
    PH(2);
    collision(S, m, T, fresh_lane(), prof, S.cl.hit);
  }
  PH(5);
  newton_solve<CL, CAL, DUO>(S, m, T, fresh_lane(), prof);
  PH(6);
  integrate<CL, CAL, DUO>(S, m, T, fresh_lane());
  PH(8);
}

#define GM_AS_LDS __attribute__((address_space(3)))
#define GM_AS_GLOBAL __attribute__((address_space(1)))
// One substep, outlined: its own register allocation (the fused kernel around it keeps
// the env-step epilogue's state), parameters typed with their address spaces so the body
// issues global loads for the model and LDS instructions for the per-env image rather
// than generic (flat) accesses that would serialise the two.
#define GM_AS_CONST __attribute__((address_space(4)))
// The model and topology pointers arrive in VGPRs (callee ABI); read back as wave-uniform
// constant-address-space pointers, every access with a uniform index is a scalar load
// through the scalar cache instead of a vector memory round trip.
template <typename P>
__device__ __forceinline__ const GM_AS_CONST P* uniform_const_ptr(const GM_AS_GLOBAL P* p) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return (const GM_AS_CONST P*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
// The substep loop: one outlined call per env-step.  Its own register allocation (the
// kernel around it keeps the env-step epilogue's state), parameters typed with their
// address spaces so the body issues scalar / global loads for the model and LDS
// instructions for the per-env image rather than generic (flat) accesses.  The
// callee-saved registers it uses are saved and restored once per env-step (an outlined
// call per substep paid that, ~92 VGPRs x 64 lanes x 2, every substep: 12 GB of scratch
// traffic per 4096-env launch).  update_all and monitor_sensors are small calls of
// their own inside the loop, so the loop body keeps the physics' register allocation.
// Built with MachineLICM off (gmx/build.py): hoisting the sincos / polynomial constant
// materialisations out of the loop would hold them live across the whole body and spill.
template <int CL>
__device__ __noinline__ void update_all_call(GM_AS_LDS SharedT<CL>* S_, const GM_AS_GLOBAL gm_model* m_,
                                             const GM_AS_GLOBAL GmTopo* T_, int lane) {
  update_all<CL>(*(SharedT<CL>*)S_, (const gm_model*)uniform_const_ptr(m_), (const GmTopo*)uniform_const_ptr(T_), lane);
}
template <int CL>
__device__ __noinline__ void monitor_call(GM_AS_LDS SharedT<CL>* S_, const GM_AS_GLOBAL gm_model* m_,
                                          const GM_AS_GLOBAL gm_config* C_, const GM_AS_GLOBAL GmTopo* T_, int lane) {
  monitor_sensors<CL>(*(SharedT<CL>*)S_, (const gm_model*)uniform_const_ptr(m_), (const gm_config*)uniform_const_ptr(C_),
                      (const GmTopo*)uniform_const_ptr(T_), lane);
}
// Preemption test of the chunked env-step (chunked_env_steps): every `every` substeps the
// loop yields when the predicted work left in this env, own * left / total (the env's last
// dispatch cost, shader clocks / 64, spread evenly over its substeps), has dropped below the
// next unstarted env's cost -- longest-remaining-work-first at substep granularity.
struct GmPreempt {
  const uint32_t* fresh_head;   // the queue's next-unstarted index (agent-scope loads)
  const int32_t* order;
  const uint32_t* cost;
  uint32_t n, own;
  int left, total, every;       // every = 0: never yield
  int margin;                   // percent
  // the XCD's yielded envs: a running env also yields to the best bucket when that bucket's
  // lower edge (cmax * b / GM_CQ_NB) exceeds its own work left by cmargin percent (< 0: off)
  const uint32_t* bq;
  uint32_t cmax;
  int cmargin;
  int prio;                     // > 0: the wave's issue priority follows the work left (job_prio)
  int steps;                    // env-steps per job: the cost array holds per-env-step costs
};
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// The wave's VALU issue priority from its job's predicted work left (rem, in the cost array's
// units) against the launch's heaviest job (cmax): 0..3 in quarters.  Two waves share a SIMD's
// issue and it goes by priority, then age (MI355X_MICROARCH.md, two waves per SIMD) -- the
// persistent grid's waves never change age, so without this the job with the most work left
// runs at the younger wave's pace on half the SIMDs.  Longest-remaining-work-first, at issue.
__device__ __forceinline__ void job_prio(uint64_t rem, uint32_t cmax, int mode) {
  if (mode <= 0) return;
  const uint32_t p = __builtin_amdgcn_readfirstlane((uint32_t)(rem * 4u / (uint64_t)(cmax ? cmax : 1u)));
  if (p >= 3) __builtin_amdgcn_s_setprio(3);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else if (p == 1) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}
// Claim the next entry of a yielded-env bucket (head at b[0], tail at b[1]; lane 0): the head
// advances only while it is below the tail, so every claimed slot was reserved by a producer
// that is about to store it -- two waves that saw the same last entry cannot both claim, and
// the loser parks on no slot that a future yield would have to fill.  Returns the slot or -1.
__device__ __forceinline__ int64_t claim_bucket(uint32_t* b) {
  uint32_t h = ld_agent(b);
  for (;;) {
    if (h >= ld_agent(b + 1)) return -1;
    if (__hip_atomic_compare_exchange_strong(b, &h, h + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      return (int64_t)h;
  }
}
// returns the substeps run (nsub unless the preemption test yielded).  PROF = false
// compiles the per-phase clock reads (PH) out: no uniform branch at every phase boundary,
// so the scheduler's regions span them (the env-step kernel's chunked path runs this one)
template <int CL, bool CAL, bool PROF, bool DUO = false>
__device__ __noinline__ int substep_loop(GM_AS_LDS SharedT<CL>* S_, const GM_AS_GLOBAL gm_model* m_,
                                         const GM_AS_GLOBAL GmTopo* T_, const GM_AS_GLOBAL gm_config* C_, int lane_in,
                                         bool prof_in, int nsub_in, bool settle_in, GmPreempt pre) {
  // nothing but scalars is carried across the loop body: the loop bounds and flags are
  // wave-uniform (SGPRs), the lane id is recomputed, the next sensor-read time lives in LDS
  SharedT<CL>& S = *(SharedT<CL>*)S_;
  const GM_AS_CONST gm_model* m_s = uniform_const_ptr(m_);
  const GM_AS_CONST GmTopo* T_s = uniform_const_ptr(T_);
  const gm_config* C = (const gm_config*)uniform_const_ptr(C_);
  const int nsub = __builtin_amdgcn_readfirstlane(nsub_in);
  const bool prof = PROF && __builtin_amdgcn_readfirstlane((int)prof_in) != 0;
  const bool settle = __builtin_amdgcn_readfirstlane((int)settle_in) != 0;
  (void)lane_in;
  const int every = CAL ? 0 : __builtin_amdgcn_readfirstlane(pre.every);
  if (__lane_id() == 0) S.next_read = (settle || CAL) ? 0.0 : next_sensor_read(S.s, C->s);
  GM_WAVE_SYNC();
  int i = 0;
#pragma nounroll
  for (; i < nsub; i++) {
    if (every > 0 && i > 0 && i % every == 0) {
      // work left in the units of the cost array, times pre.total
      const uint64_t left = (uint64_t)__builtin_amdgcn_readfirstlane(pre.own) *
                            (uint64_t)(__builtin_amdgcn_readfirstlane(pre.left) - i);
      const uint64_t total = (uint64_t)__builtin_amdgcn_readfirstlane(pre.total);
      const int pm = __builtin_amdgcn_readfirstlane(pre.prio);
      if (pm > 0) job_prio(left / (total ? total : 1u), __builtin_amdgcn_readfirstlane(pre.cmax), pm);
      const uint32_t fh = __builtin_amdgcn_readfirstlane(ld_agent(pre.fresh_head));
      const uint32_t n = __builtin_amdgcn_readfirstlane(pre.n);
      if (fh < n) {
        const uint64_t next = (uint64_t)__builtin_amdgcn_readfirstlane(pre.cost[pre.order[fh]]) *
                              (uint64_t)__builtin_amdgcn_readfirstlane(pre.steps);
        // (with a margin: a yield costs a state hand-off)
        if (left * (uint64_t)(100 + __builtin_amdgcn_readfirstlane(pre.margin)) < next * total * 100u) break;
      }
      const int cm = __builtin_amdgcn_readfirstlane(pre.cmargin);
      if (cm >= 0) {
        const int ln = __lane_id();
        uint32_t hb = 0, tb = 0;
        if (ln < GM_CQ_NB) { hb = ld_agent(pre.bq + ln * 32); tb = ld_agent(pre.bq + ln * 32 + 1); }
        const unsigned long long ne = __ballot(ln < GM_CQ_NB && hb < tb);
        if (ne) {
          const uint64_t b = 63 - __builtin_clzll(ne);
          const uint64_t lower = b * (uint64_t)__builtin_amdgcn_readfirstlane(pre.cmax) / GM_CQ_NB;
          if (left * (uint64_t)(100 + cm) < lower * total * 100u) break;
        }
      }
    }
    // opaque per iteration: nothing derived from the lane id or the model / topology
    // pointers is hoisted out of the loop and held live across the whole body
    int lane;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
    // (the opaque copy keeps the constant address space: every model / topology access
    // stays a scalar load when its index is uniform, a global load otherwise -- a generic
    // pointer would make them flat loads that wait on LDS traffic too)
    const GM_AS_CONST gm_model* mc = m_s;
    const GM_AS_CONST GmTopo* Tc = T_s;
    asm volatile("" : "+s"(mc), "+s"(Tc));
    const gm_model* m = (const gm_model*)mc;
    const GmTopo* T = (const GmTopo*)Tc;
    if (CAL && S.s.tip_force != 0.0 && lane < T->nlock && m->lock_kind[lane] == 0) {
      S.s.lock_active[lane] = 1;
      S.s.lock_q[lane] = S.lock_pre[lane];
    }
    const unsigned long long tc = prof ? clock64() : 0;
    physics_substep_body<CL, CAL, DUO>(S, m, T, lane, prof);
    unsigned long long t0 = prof ? clock64() : 0;
    if (prof && lane == 0) S.tph[22] += t0 - tc;
    update_all<CL>(S, m, T, fresh_lane());
    PH(9);
    if (!settle && !CAL && S.s.time > S.next_read) {
      monitor_call<CL>((GM_AS_LDS SharedT<CL>*)&S, (const GM_AS_GLOBAL gm_model*)(uintptr_t)m,
                       (const GM_AS_GLOBAL gm_config*)(uintptr_t)C, (const GM_AS_GLOBAL GmTopo*)(uintptr_t)T, __lane_id());
      if (__lane_id() == 0) S.next_read = next_sensor_read(S.s, C->s);
      GM_WAVE_SYNC();
    }
    PH(10);
    if (CAL && S.s.badqacc) break;
  }
  return i;
}

// ============================================================ env-step epilogue (lane 0)
__device__ __forceinline__ float normalise_between(float val, float mn, float mx) {
  if (val > mx) return 1.0f;
  else if (val < mn) return -1.0f;
  return 2 * (val - mn) / (mx - mn) - 1;
}

template <int CL>
GM_EPI_ATTR void sense_gripper_state(SharedT<CL>& S, const gm_model* __restrict__ m, const gm_config* __restrict__ C) {
  GmEnvHot& s = S.s;
  RingRef R = S.gs->ring;
  const gm_settings& st = C->s;
  const double* bmn = C->base_min;
  const double* bmx = C->base_max;
  double gx = normalise_between((float)s.end.x, (float)G_XY_MIN, (float)G_XY_MAX);
  double gy = normalise_between((float)s.end.y, (float)G_XY_MIN, (float)G_XY_MAX);
  double gz = normalise_between((float)s.end.z, (float)G_Z_MIN, (float)G_Z_MAX);
  double bx = normalise_between((float)s.base[0], (float)bmn[0], (float)bmx[0]);
  double by = normalise_between((float)s.base[1], (float)bmn[1], (float)bmx[1]);
  double bz = normalise_between((float)s.base[2], (float)bmn[2], (float)bmx[2]);
  double byaw = normalise_between((float)s.base[5], (float)bmn[5], (float)bmx[5]);
  gx = s_noise(s, st.motor_state_sensor, SL_MOTOR, (float)gx, 1);
  gy = s_noise(s, st.motor_state_sensor, SL_MOTOR, (float)gy, 2);
  gz = s_noise(s, st.motor_state_sensor, SL_MOTOR, (float)gz, 3);
  bx = s_noise(s, st.base_state_sensor_XY, SL_BASEXY, (float)bx, 1);
  by = s_noise(s, st.base_state_sensor_XY, SL_BASEXY, (float)by, 2);
  bz = s_noise(s, st.base_state_sensor_Z, SL_BASEZ, (float)bz, 1);
  byaw = s_noise(s, st.base_state_sensor_yaw, SL_YAW, (float)byaw, 1);
  ring_add(s, R, ST_MOTOR + 0, (float)gx);
  ring_add(s, R, ST_MOTOR + 1, (float)gy);
  ring_add(s, R, ST_MOTOR + 2, (float)gz);
  ring_add(s, R, ST_BASE + 0, (float)bx);
  ring_add(s, R, ST_BASE + 1, (float)by);
  ring_add(s, R, ST_BASE + 2, (float)bz);
  ring_add(s, R, ST_YAW, (float)byaw);
  // MAT cartesian contact points (get_fingerend_and_palm_xyz, myfunctions.cpp:3622-3688)
  double fsi[3] = {ring_latest(s, R, ST_SI_GAUGE), ring_latest(s, R, ST_SI_GAUGE + 1), ring_latest(s, R, ST_SI_GAUGE + 2)};
  double psi = ring_latest(s, R, ST_SI_PALM);
  double fx = s.end.x, fth = g_calc_th(s.end.x, s.end.y), pz = s.end.z;
  const double PI23 = 3.14159265358979323846 * (2.0 / 3.0);
  double ang[3] = {0.0, PI23, 2 * PI23};
  double unt = m->fingertip_clearance - s.base[2];
  double lift = m->finger_length * (1 - cos(fth));
  double tilted = unt + lift;
  const double ft = 0.2;
  for (int i = 0; i < 3; i++) {
    double tilt_x = fx - m->finger_length * sin(fth);
    double defl = fsi[i] * pow(m->finger_length, 3) / (3 * m->finger_EI);
    double fin_x = tilt_x + defl * cos(fth);
    double px = -fin_x * sin(ang[i] + s.base[5]) + s.base[0];
    double py = -fin_x * cos(ang[i] + s.base[5]) + s.base[1];
    double pzz = tilted - defl * sin(fth);
    bool on = fabs(fsi[i]) > ft;
    ring_add(s, R, ST_CART + 3 * i + 0, (float)(on ? px : 0.0));
    ring_add(s, R, ST_CART + 3 * i + 1, (float)(on ? py : 0.0));
    ring_add(s, R, ST_CART + 3 * i + 2, (float)(on ? pzz : 0.0));
  }
  bool pon = psi > ft;
  ring_add(s, R, ST_CART + 9, (float)(pon ? s.base[0] : 0.0));
  ring_add(s, R, ST_CART + 10, (float)(pon ? s.base[1] : 0.0));
  ring_add(s, R, ST_CART + 11, (float)(pon ? unt + 165e-3 - pz : 0.0));
}

__device__ float mag3f(const float* v) { return (float)sqrt((double)v[0] * v[0] + (double)v[1] * v[1] + (double)v[2] * v[2]); }

// MjClass::update_env (mjclass.cpp:966-1346) + update_events (5437-5469)
template <int CL>
GM_EPI_ATTR void update_env(SharedT<CL>& S, const gm_model* __restrict__ m, const gm_config* __restrict__ C,
                           const GmTopo* __restrict__ T) {
  GmEnvHot& s = S.s;
  RingRef R = S.gs->ring;
  const gm_settings& st = C->s;
  const double ftol = 1e-5;
  extract_forces(S, m, T);
  const float* F = S.forces;
  int qa = T->qadr_obj;
  double ox = s.qpos[qa], oy = s.qpos[qa + 1], oz = s.qpos[qa + 2];
  double relx = s.base[0] - ox, rely = s.base[1] - oy;
  float dist_from_gripper = (float)sqrt(pow(relx, 2) + pow(rely, 2));
  float f1m = mag3f(F + 0), f2m = mag3f(F + 3), f3m = mag3f(F + 6), pm = mag3f(F + 9), gm = mag3f(F + 12);
  float palm_axial = F[9];
  float lift_height = (float)(oz - (double)s.start_qpos[2]);
  float avg_finger = (float)(0.33333 * (f1m + f2m + f3m));
  float mn = F[1];
  if (F[4] < mn) mn = F[4];
  if (F[7] < mn) mn = F[7];
  float peak_lat = -1 * mn;
  float ov_avg = 0, ov_palm = 0, ov_lift = 0;
  if (avg_finger > ov_avg) ov_avg = avg_finger;
  if (palm_axial > ov_palm) ov_palm = palm_axial;
  if (peak_lat > s.grp_peak_lateral) s.grp_peak_lateral = peak_lat;
  if (lift_height > ov_lift) ov_lift = lift_height;
  float gripper_z_height = (float)(-1 * s.base[2]);
  float ga = F[19];
  if (F[20] < ga) ga = F[20];
  if (F[21] < ga) ga = F[21];
  float grp_peak_axial = -1 * ga;
  float g1 = ring_latest(s, R, ST_SI_GAUGE), g2 = ring_latest(s, R, ST_SI_GAUGE + 1), g3 = ring_latest(s, R, ST_SI_GAUGE + 2);
  float last_palm = ring_latest(s, R, ST_SI_PALM), last_wrist = ring_latest(s, R, ST_SI_WZ);
  float max_gauge = g1 > g2 ? g1 : g2;
  max_gauge = max_gauge > g3 ? max_gauge : g3;
  float avg_gauge = (float)((1.0 / 3.0) * (g1 + g2 + g3));
  int* B = s.bev_value;
  B[GM_EV_step_num] = 1;
  double closest = dist_from_gripper;
  int o_lifted = 0, o_oob = 0, o_l2h = 0, o_th = 0, o_stable = 0;
  if (gm < ftol && 0.0f < ftol) { B[GM_EV_lifted] = 1; o_lifted = 1; }
  if (ox > st.oob_distance || ox < -st.oob_distance || oy > st.oob_distance || oy < -st.oob_distance) { B[GM_EV_oob] = 1; o_oob = 1; }
  if (ov_lift > st.lift_height - ftol && o_lifted && !o_oob) { B[GM_EV_lifted_to_height] = 1; o_l2h = 1; }
  if (o_l2h && gripper_z_height > st.gripper_target_height - ftol) { B[GM_EV_target_height] = 1; o_th = 1; }
  if (f1m > ftol || f2m > ftol || f3m > ftol || pm > ftol) B[GM_EV_object_contact] = 1;
  if (f1m > st.stable_finger_force && f2m > st.stable_finger_force && f3m > st.stable_finger_force &&
      f1m < st.stable_finger_force_lim && f2m < st.stable_finger_force_lim && f3m < st.stable_finger_force_lim &&
      pm > st.stable_palm_force && pm < st.stable_palm_force_lim && B[GM_EV_lifted]) {
    B[GM_EV_object_stable] = 1; o_stable = 1;
  }
  if (o_stable && o_th) B[GM_EV_stable_height] = 1;
  if (s.termination_signal_sent) {
    if (st.lifted_termination.done) {
      if (o_l2h) B[GM_EV_lifted_termination] = 1; else B[GM_EV_failed_termination] = 1;
    } else {
      if (B[GM_EV_stable_height]) B[GM_EV_stable_termination] = 1; else B[GM_EV_failed_termination] = 1;
    }
  }
  if (dist_from_gripper < st.XY_distance_threshold) B[GM_EV_within_XY_distance] = 1;
  if (dist_from_gripper < closest) closest = dist_from_gripper;
  {
    int* R = s.bev_row;
    int v = (!R[GM_EV_dropped] * !B[GM_EV_lifted] * R[GM_EV_lifted]) ? 1
            : (B[GM_EV_lifted] ? 0 : (R[GM_EV_dropped] ? R[GM_EV_dropped] + 1 : 0));
    B[GM_EV_dropped] = v != 0;
  }
  float* Lv = s.lev_value;
  Lv[GM_LEV_exceed_axial] = grp_peak_axial;
  Lv[GM_LEV_exceed_lateral] = s.grp_peak_lateral;
  Lv[GM_LEV_palm_force] = ov_palm * B[GM_EV_lifted];
  Lv[GM_LEV_exceed_palm] = ov_palm;
  Lv[GM_LEV_finger_force] = ov_avg;
  Lv[GM_LEV_finger1_force] = f1m;
  Lv[GM_LEV_finger2_force] = f2m;
  Lv[GM_LEV_finger3_force] = f3m;
  Lv[GM_LEV_ground_force] = gm;
  Lv[GM_LEV_good_bend_sensor] = avg_gauge;
  Lv[GM_LEV_exceed_bend_sensor] = max_gauge;
  Lv[GM_LEV_dangerous_bend_sensor] = max_gauge;
  Lv[GM_LEV_good_palm_sensor] = last_palm;
  Lv[GM_LEV_exceed_palm_sensor] = last_palm;
  Lv[GM_LEV_dangerous_palm_sensor] = last_palm;
  Lv[GM_LEV_exceed_wrist_sensor] = last_wrist;
  Lv[GM_LEV_dangerous_wrist_sensor] = last_wrist;
  Lv[GM_LEV_action_penalty_lin] /= (float)(C->n_actions - st.use_termination_action);
  Lv[GM_LEV_action_penalty_sq] /= (float)(C->n_actions - st.use_termination_action);
  Lv[GM_LEV_object_XY_distance] = (float)(-closest);
  {
    int k = 0;
#define GM_BR(n, r, d, t)                                                                         \
    if (B[k] && st.n.reward >= (1.0 - 1e-5) && st.n.done && s.bev_row[k] + 1 >= st.n.trigger)    \
      B[GM_EV_successful_grasp] = 1;                                                              \
    k++;
#include "gm_settings.def"
  }
  // update_events
  for (int k = 0; k < GM_N_BINARY; k++) {
    s.bev_row[k] = s.bev_row[k] * s.bev_value[k] + s.bev_value[k];
    s.bev_abs[k] += s.bev_value[k];
    s.bev_last[k] = s.bev_value[k];
    s.bev_value[k] = 0;
  }
  {
    int k = 0;
#define GM_LR(n, r, d, t, a, b, o)                                                         \
    {                                                                                      \
      int active = (Lv[k] > st.n.min && (Lv[k] < st.n.overshoot || st.n.overshoot < 0));   \
      s.lev_row[k] = s.lev_row[k] * active + active;                                       \
      s.lev_abs[k] += active;                                                              \
      s.lev_last[k] = Lv[k];                                                               \
      Lv[k] = 0.0f;                                                                        \
    }                                                                                      \
    k++;
#include "gm_settings.def"
  }
}

__device__ int sample_stream(const GmEnvHot& s, RingRef R, int mode, int st, const gm_sensor& ss, float* out) {
  int prev = ss.prev_steps, rps = ss.readings_per_step, total = ss.total_readings;
  if (mode == GM_SAMPLE_RAW) {
    int n = total - 1;
    for (int j = n - 1, k = 0; j >= 0; j--, k++) out[k] = ring_read(s, R, st, j);
    return n;
  }
  out[0] = ring_read(s, R, st, total - 1);
  for (int i = 0; i < prev; i++) {
    int first = total - 1 - i * rps;
    out[2 * i + 2] = ring_read(s, R, st, first - rps);
    float a = out[2 * i], b = out[2 * i + 2];
    float r;
    if (mode == GM_SAMPLE_CHANGE) r = b - a;
    else if (mode == GM_SAMPLE_AVERAGE) {
      float acc = 0;
      for (int j = 0; j < rps + 1; j++) acc += ring_read(s, R, st, first - j);
      r = acc / (rps + 1);
    } else if (mode == GM_SAMPLE_MEDIAN) {
      float v[GM_RING + 1];
      int nv = rps + 1;
      for (int j = 0; j < nv; j++) v[j] = ring_read(s, R, st, first - j);
      for (int x = 1; x < nv; x++) { float t = v[x]; int y = x - 1; while (y >= 0 && v[y] > t) { v[y + 1] = v[y]; y--; } v[y + 1] = t; }
      int hn = nv / 2;
      float med = v[hn];
      if (!(nv & 1)) med = (v[hn - 1] + med) / 2.0f;
      r = med;
    } else if (mode == GM_SAMPLE_SIGN) {
      float ch = b - a;
      r = ch > 1e-6f ? 1.0f : (ch < -1e-6f ? -1.0f : 0.0f);
    } else if (mode == GM_SAMPLE_SCALED_CHANGE) {
      float sc = (b - a) / 0.07f;
      r = sc > 1.0f ? 1.0f : (sc < -1.0f ? -1.0f : sc);
    } else {
      float ch = fabsf(b - a);
      float sc = (b - a) * ch * (1.0f / (0.10f * 0.10f));
      r = sc > 1.0f ? 1.0f : (sc < -1.0f ? -1.0f : sc);
    }
    out[2 * i + 1] = r;
  }
  return 2 * prev + 1;
}

// MjClass::get_observation (mjclass.cpp:1707-1959)
__device__ int get_obs(const GmEnvHot& s, RingRef R, const gm_config* __restrict__ C, float* out) {
  const gm_settings& st = C->s;
  int sf = C->sensor_fcn, tf = C->state_fcn, n = 0;
  if (st.bending_gauge.in_use) for (int f = 0; f < 3; f++) n += sample_stream(s, R, sf, ST_GAUGE + f, st.bending_gauge, out + n);
  if (st.axial_gauge.in_use) for (int f = 0; f < 3; f++) n += sample_stream(s, R, sf, ST_AXIAL + f, st.axial_gauge, out + n);
  if (st.palm_sensor.in_use) n += sample_stream(s, R, sf, ST_PALM, st.palm_sensor, out + n);
  if (st.wrist_sensor_XY.in_use) {
    n += sample_stream(s, R, sf, ST_WX, st.wrist_sensor_XY, out + n);
    n += sample_stream(s, R, sf, ST_WY, st.wrist_sensor_XY, out + n);
  }
  if (st.wrist_sensor_Z.in_use) n += sample_stream(s, R, sf, ST_WZ, st.wrist_sensor_XY, out + n);
  if (st.motor_state_sensor.in_use) for (int k = 0; k < 3; k++) n += sample_stream(s, R, tf, ST_MOTOR + k, st.motor_state_sensor, out + n);
  if (st.base_state_sensor_XY.in_use) for (int k = 0; k < 2; k++) n += sample_stream(s, R, tf, ST_BASE + k, st.base_state_sensor_XY, out + n);
  if (st.base_state_sensor_Z.in_use) n += sample_stream(s, R, tf, ST_BASE + 2, st.base_state_sensor_Z, out + n);
  if (st.base_state_sensor_yaw.in_use) n += sample_stream(s, R, tf, ST_YAW, st.base_state_sensor_yaw, out + n);
  if (st.cartesian_contacts_XYZ.in_use)
    for (int k = 0; k < 12; k++) n += sample_stream(s, R, GM_SAMPLE_CHANGE, ST_CART + k, st.cartesian_contacts_XYZ, out + n);
  return n;
}

// get_obs with one stream per lane (the env-step epilogue): every lane walks the same
// in-use stream list, in get_obs's order, to find its stream's sampler, settings and
// output offset, then all streams are sampled at once -- the serial version's arithmetic
// per stream, without its chain of dependent window reads on one lane.
__device__ void get_obs_lanes(const GmEnvHot& s, RingRef R, const gm_config* __restrict__ C, float* out, int lane) {
  const gm_settings& st = C->s;
  const int sf = C->sensor_fcn, tf = C->state_fcn;
  int k = 0, n = 0, my_mode = 0, my_st = -1, my_n = 0;
  const gm_sensor* my_ss = nullptr;
  auto visit = [&](bool in_use, int count, int mode, int st0, const gm_sensor& ss) {
    if (!in_use) return;
    const int size = (mode == GM_SAMPLE_RAW) ? ss.total_readings - 1 : 2 * ss.prev_steps + 1;
    for (int c = 0; c < count; c++) {
      if (k == lane) { my_mode = mode; my_st = st0 + c; my_ss = &ss; my_n = n; }
      n += size;
      k++;
    }
  };
  visit(st.bending_gauge.in_use, 3, sf, ST_GAUGE, st.bending_gauge);
  visit(st.axial_gauge.in_use, 3, sf, ST_AXIAL, st.axial_gauge);
  visit(st.palm_sensor.in_use, 1, sf, ST_PALM, st.palm_sensor);
  visit(st.wrist_sensor_XY.in_use, 1, sf, ST_WX, st.wrist_sensor_XY);
  visit(st.wrist_sensor_XY.in_use, 1, sf, ST_WY, st.wrist_sensor_XY);
  visit(st.wrist_sensor_Z.in_use, 1, sf, ST_WZ, st.wrist_sensor_XY);   // XY's counts (quirk, as get_obs)
  visit(st.motor_state_sensor.in_use, 3, tf, ST_MOTOR, st.motor_state_sensor);
  visit(st.base_state_sensor_XY.in_use, 2, tf, ST_BASE, st.base_state_sensor_XY);
  visit(st.base_state_sensor_Z.in_use, 1, tf, ST_BASE + 2, st.base_state_sensor_Z);
  visit(st.base_state_sensor_yaw.in_use, 1, tf, ST_YAW, st.base_state_sensor_yaw);
  visit(st.cartesian_contacts_XYZ.in_use, 12, GM_SAMPLE_CHANGE, ST_CART, st.cartesian_contacts_XYZ);
  if (my_st >= 0) sample_stream(s, R, my_mode, my_st, *my_ss, out + my_n);
}

GM_EPI_ATTR int is_done(const GmEnvHot& s, const gm_config* __restrict__ C) {
  const gm_settings& st = C->s;
  int k = 0;
  int done = 0;
#define GM_BR(n, r, d, t) if (st.n.done && s.bev_row[k] >= st.n.done) done = 1; k++;
#include "gm_settings.def"
  k = 0;
#define GM_LR(n, r, d, t, a, b, o) if (st.n.done && s.lev_row[k] >= st.n.done) done = 1; k++;
#include "gm_settings.def"
  if (st.cap_reward && st.quit_if_cap_exceeded) {
    if (s.cumulative_reward - 1e-5 < st.reward_cap_lower_bound) done = 1;
    if (s.cumulative_reward + 1e-5 > st.reward_cap_upper_bound) done = 1;
  }
  return done;
}

__device__ float linear_reward(float val, float mn, float mx, float overshoot) {
  if (val < mn) return 0.0f;
  if (val > mx) {
    if (overshoot < mx) return 1.0f;
    if (val > overshoot) return 0.0f;
    mn = 0; mx = overshoot - mx; val = overshoot - val;
  }
  return (val - mn) / (mx - mn);
}
__device__ float reward(GmEnvHot& s, const gm_config* __restrict__ C) {
  const gm_settings& st = C->s;
  float r = 0;
  int k = 0;
#define GM_BR(n, rr, d, t) if (s.bev_row[k] >= st.n.trigger) r += st.n.reward; k++;
#include "gm_settings.def"
  k = 0;
#define GM_LR(n, rr, d, t, a, b, o)                                                        \
  if (s.lev_row[k] >= st.n.trigger) {                                                      \
    float fr = linear_reward(s.lev_last[k], st.n.min, st.n.max, st.n.overshoot);           \
    r += st.n.reward * fr;                                                                 \
  }                                                                                        \
  k++;
#include "gm_settings.def"
  s.cumulative_reward += r;
  if (s.cumulative_reward < st.reward_cap_lower_bound && st.cap_reward) {
    r += st.reward_cap_lower_bound - s.cumulative_reward;
    s.cumulative_reward = st.reward_cap_lower_bound;
  }
  if (s.cumulative_reward > st.reward_cap_upper_bound && st.cap_reward) {
    r += st.reward_cap_upper_bound - s.cumulative_reward;
    s.cumulative_reward = st.reward_cap_upper_bound;
  }
  return r;
}

// ============================================================ kernels
// action_step's tail after the substeps: sense_gripper_state, update_env, the observation,
// is_done and reward (mjclass.cpp:1483-1508, MjEnv.py:2170-2220)
template <int CL>
__device__ __forceinline__ void env_step_epilogue(SharedT<CL>& S, const gm_model* __restrict__ m,
                                                  const gm_config* __restrict__ C, const GmTopo* __restrict__ T,
                                                  float* __restrict__ obs, float* __restrict__ rew,
                                                  uint8_t* __restrict__ done, int env, int lane, bool prof,
                                                  unsigned long long& t0) {
  if (lane == 0) {
    S.s.extra_substeps = 0;
    S.s.overflow = S.overflow;
    sense_gripper_state(S, m, C);
    PH(18);
    update_env(S, m, C, T);
    PH(19);
    S.s.num_action_steps += 1;
  }
  GM_WAVE_SYNC();   // lane 0's window appends (HBM) and indices (LDS) before the samplers
  get_obs_lanes(S.s, S.gs->ring, C, obs + (size_t)env * C->n_obs, lane);
  PH(20);
  if (lane == 0) {
    int d = is_done(S.s, C);
    float r = reward(S.s, C);
    S.s.done = d;
    S.s.reward = r;
    rew[env] = r;
    done[env] = (uint8_t)d;
    PH(21);
  }
}

template <int CL>
__device__ __forceinline__ void load_state(SharedT<CL>& S, GmEnvState* __restrict__ g, int lane) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(g);
  uint32_t* dst = reinterpret_cast<uint32_t*>(&S.s);
  for (int i = lane; i < GM_HOT_WORDS; i += NT) dst[i] = src[i];
  S.gs = g;
  GM_ENV_SYNC();
}
template <int CL>
__device__ __forceinline__ void store_state(const SharedT<CL>& S, GmEnvState* __restrict__ g, int lane) {
  GM_ENV_SYNC();
  const uint32_t* src = reinterpret_cast<const uint32_t*>(&S.s);
  uint32_t* dst = reinterpret_cast<uint32_t*>(g);
  for (int i = lane; i < GM_HOT_WORDS; i += NT) dst[i] = src[i];
}

// ---------------------------------------------------------------- chunked env-step
// gm_step as a persistent work queue over env CHUNKS of a few substeps (DESIGN.md §5,
// "Chunked dispatch").  One env-step is ~2.9 ms on a wave; with 4096 envs on 2048 resident
// waves, whole env-steps leave the chip partly idle for the last third of the launch (the
// last env starts ~5 ms in).  Here a wave runs one chunk of an env, stores the env's hot
// state and hands the env on; any wave of the same XCD continues it.  Results are
// bit-identical to the one-shot kernel: the substeps, their order and the epilogue are the
// same code on the same state.
//
// Scheduling: envs start in descending predicted cost (the previous env-step's); a running
// env yields (at most max_yields times per env-step) when an unstarted env has clearly more
// work than it has left, and yielded envs wait in priority buckets by predicted work left;
// a free wave takes the larger of the best bucket's head and the next unstarted env --
// longest-remaining-work-first at substep granularity (tools/sim_dispatch.py).
//
// Hand-off (MI355X_MICROARCH.md, inter-workgroup visibility): an env's chunks all run on
// the XCD that started it (each XCD has its own continuation buckets, a wave serves those
// of the XCD it runs on, read from HW_REG_XCC_ID), so the L2 is shared between producer and
// consumer.  Producer: plain stores of the state and carry, s_waitcnt vmcnt(0), then the
// ring entry by an agent-scope (sc1) store.  Consumer: sc1 poll of the entry, agent-scope
// acquire (invalidates its CU's L1) and its wait, then plain loads.
struct GmChunkCarry {        // what a chunk hands the next besides the hot state
  int32_t sub_done, nsub;
  int32_t work_nefc, work_mpr, work_newton, stp_fixed;
  uint32_t clk;              // s_memtime / 64 summed over this env-step's chunks
  int32_t yielded;           // yields so far this env-step (at most GmChunkQ::max_yields)
  int32_t steps_left;        // env-steps of this launch's job still to run, the current one included
  int32_t step_idx;          // index of the current env-step in the launch (rollout records)
  int32_t job_yields;        // yields over the whole job (gm_chunk_job_stats)
};
// counters (zeroed by gm_dispatch_order_kernel before every launch), one 128-B line each:
// ring r = x * GM_CQ_NB + bucket: [r * 32] its head, [r * 32 + 1] its tail; GM_CQ_FRESH the
// next unstarted env, GM_CQ_DONE envs finished, + 1 yields, + 2 resumes, + 4 resumes on another
// XCD, + 5 claims whose ring slot was still empty (the producer between its tail increment and
// its entry store), + 6 polls those claims made; GM_CQ_LAST the previous launch's
// [GM_CQ_FRESH ..] (39 words, diagnostics)
#define GM_CQ_FRESH (8 * GM_CQ_NB * 32)
#define GM_CQ_DONE (GM_CQ_FRESH + 32)
#define GM_CQ_CMAX (GM_CQ_DONE + 3)   // this launch's bucket scale (written by the order kernel)
#define GM_CQ_WORDS (GM_CQ_FRESH + 64)
#define GM_CQ_LAST GM_CQ_WORDS
#define GM_CQ_ALLOC (GM_CQ_WORDS + 64)
struct GmChunkQ {
  uint32_t* ctr;             // GM_CQ_ALLOC words
  uint64_t* ring;            // [8 * GM_CQ_NB][cap] (predicted work left << 32) | (env + 1), 0 = empty
  GmChunkCarry* carry;       // [n_envs]
  int cap;                   // ring slots per XCD: n_envs + launched waves
  int chunk;                 // substeps between preemption tests
  int margin;                // yield when work left * (100 + margin) < next unstarted env's * 100
  int max_yields;            // per env per env-step
  int cmargin;               // yield to a yielded env with cmargin percent more work left (< 0: off)
  unsigned long long* st;    // [0] first pick, [1] first pick that found no unstarted env,
                             // [2] last env finished (100 MHz clock), [3] wave-busy, [4] wave
                             // polling (sums, 100 MHz ticks); [8 ..] the previous launch's;
                             // [16 + w] when workgroup w finished its last piece of work
  // rollout (gm_rollout; act_mode < 0: one plain env-step per env, gm_step): each env runs
  // `steps` env-steps in a row, every one of them the per-step API's sequence -- driver actions
  // (gm_scripted_actions / gm_random_actions) -> set_continous_action -> action_step + obs /
  // done / reward -> gm_autoreset_episodes' episode-end record and reset
  int steps;
  int act_mode;              // 0 scripted grasp mix, 1 uniform random, -1 none
  uint64_t act_seed;
  float jitter;
  int max_ep;                // truncation (num_action_steps >= max_ep), <= 0 off
  gm_episode_end* rec;       // [steps][n_envs] episode-end records (may be NULL)
  const double* eq;          // the settled equilibrium (calibrate_reset) for the resets
  const gm_object* objs;
  int n_objects;
  int scene_tries;
  const gm_spawn_params* scene;
  GmSpawnRand sr;
  int steal;                 // an idle wave may resume a yielded env of another XCD
  int prio;                  // > 0: issue priority by predicted work left (job_prio)
  // act_mode 2: the DQN policy picks each env-step's discrete action on the env's own wave
  // (gm_policy_rollout; gp_select_one = gm_policy_kernel's select_action for one env)
  const float* pparams;      // packed network (gm_policy_pack layout)
  GpNet pnet;
  const float* peps;         // [steps] exploration threshold per env-step of the launch
  uint64_t pseed, pdecision; // the policy's seed and the first env-step's decision index
};
__device__ __forceinline__ void st_agent(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t add_agent(uint32_t* p, uint32_t v) {
  return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// what survives a reset (see reset_env)
struct GmResetKeep {
  uint32_t rng;
  int32_t ox, oy, oz, episode, newton_caps;
};
__device__ __noinline__ void reset_env(GmEnvHot& s, GmEnvState& rec, GmResetKeep keep, const gm_model* __restrict__ m,
                                       const gm_config* __restrict__ C, const GmTopo* __restrict__ T,
                                       const double* __restrict__ eq_qpos, const gm_spawn* __restrict__ spawn,
                                       const gm_object* __restrict__ objs, int n_objects, int env,
                                       const gm_spawn_params* __restrict__ scene, int scene_tries, GmSpawnRand sr,
                                       uint16_t* sh_pxy, uint16_t* sh_prot, int lane);
__device__ void set_action_one(GmEnvHot& s, const gm_model* __restrict__ m, const gm_config* __restrict__ C,
                               int action, float frac);
// the grasp program's inputs (gm_state.h gm_program_fraction) from an env's state and its
// SI sensor windows
__device__ __forceinline__ gm_program_in program_input(const GmEnvHot& s, RingRef R, const gm_model* __restrict__ m) {
  gm_program_in in;
  in.x = s.end.x; in.y = s.end.y; in.z = s.end.z;
  in.base_z = s.base[2];
  in.q_base = s.qpos[m->jnt_qposadr[m->body_jnt[m->body_base]]];
  in.q_palm = s.qpos[m->jnt_qposadr[m->body_jnt[m->body_palm]]];
  in.obj_z = s.qpos[m->jnt_qposadr[m->body_jnt[m->body_obj]] + 2];
  in.obj_top = gm_program_obj_top(s.obj_type, s.obj_size);
  in.z_root = m->body_pos[m->body_base][2];
  in.palm_drop = (m->finger_length - 165e-3) + 0.004;
  const float g0 = ring_latest(s, R, ST_SI_GAUGE), g1 = ring_latest(s, R, ST_SI_GAUGE + 1),
              g2 = ring_latest(s, R, ST_SI_GAUGE + 2);
  in.g_max = fmaxf(g0, fmaxf(g1, g2));
  in.palm = ring_latest(s, R, ST_SI_PALM);
  return in;
}
// the driver's fraction for action i of kind `kind` (modes: 0 scripted grasp mix, 1 uniform
// random, 3 grasp program, 4 the program in 1 episode of 4 and the scripted mix otherwise)
__device__ __forceinline__ float driver_fraction(const GmEnvHot& s, RingRef R, const gm_model* __restrict__ m,
                                                 const gm_config* __restrict__ C, int mode, uint64_t seed, float jitter,
                                                 int64_t gid, int i, int kind) {
  if (mode == 3 || (mode == 4 && gm_program_episode(seed, gid, s.episode))) {
    if (kind < 0) return 0.0f;
    const gm_action* acts[GM_N_ACTION_KINDS] = {
#define GM_AA(n, u, vv, sg) &C->s.n,
#include "gm_settings.def"
    };
    const gm_program_in in = program_input(s, R, m);
    return gm_program_fraction(&in, kind, acts[kind]->value, acts[kind]->sign);
  }
  if (mode == 0 || mode == 4) return gm_script_fraction(seed, gid, s.episode, s.num_action_steps, i, kind, jitter);
  return gm_random_fraction(seed, gid, s.episode, s.num_action_steps, i);
}
// the rollout driver's actions for the env's next env-step (lane 0): the same fractions
// gm_scripted_actions / gm_random_actions / gm_program_actions produce, applied as
// gm_set_action applies them
__device__ __noinline__ void driver_actions(GmEnvHot& s, RingRef R, const gm_model* __restrict__ m,
                                            const gm_config* __restrict__ C, int mode, uint64_t seed, float jitter,
                                            int64_t gid) {
  const int na = C->n_actions;
  float f[GM_ACTION_CODE_COUNT];
  // every fraction from the state before any action moves a target (the program reads them)
  for (int i = 0; i < na; i++) {
    const int code = C->action_options[i];
    const int kind = (code >= 0 && code < GM_ACTION_TERMINATION) ? code / 3 : -1;
    float v = driver_fraction(s, R, m, C, mode, seed, jitter, gid, i, kind);
    f[i] = v < -1.0f ? -1.0f : (v > 1.0f ? 1.0f : v);
  }
  for (int i = 0; i < na; i++) set_action_one(s, m, C, i, f[i]);
}

// the persistent loop of gm_step_kernel's chunked mode (a mode of the one kernel, not a
// kernel of its own: substep_loop keeps its single caller and so its constant LDS base)
template <int CL, bool DUO>
__device__ __forceinline__ void chunked_env_steps(SharedT<CL>& S, GmEnvState* __restrict__ states,
                                                  const gm_model* __restrict__ m, const gm_config* __restrict__ C,
                                                  const GmTopo* __restrict__ T, float* __restrict__ obs,
                                                  float* __restrict__ rew, uint8_t* __restrict__ done, int n_envs,
                                                  const int32_t* __restrict__ order, uint32_t* __restrict__ cost,
                                                  const GmChunkQ& q, int lane) {
  int xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 7;
  uint32_t* bq = q.ctr + xcc * GM_CQ_NB * 32;                    // this XCD's bucket counters
  uint64_t* ring = q.ring + (size_t)xcc * GM_CQ_NB * q.cap;      // and rings
  uint32_t* fresh_head = q.ctr + GM_CQ_FRESH;
  uint32_t* n_done = q.ctr + GM_CQ_DONE;
  const uint32_t n = (uint32_t)n_envs;
  // bucket scale: the heaviest env's last cost + 1, snapshot by gm_dispatch_order_kernel, so
  // every wave of the launch buckets alike (costs of this launch go to the second half)
  // (costs are per env-step: a job of q.steps env-steps is predicted at q.steps times its env's)
  const uint32_t cmax = q.ctr[GM_CQ_CMAX] * (uint32_t)(q.steps > 1 ? q.steps : 1);
  unsigned long long busy = 0, poll = 0, last_end = 0;
  bool first = true, saw_empty = false;
  for (;;) {
    if (q.prio > 0) __builtin_amdgcn_s_setprio(0);   // looking for work: the partner wave first
    const unsigned long long tw = __builtin_amdgcn_s_memrealtime();
    // take work (lane 0): a continuation queued on this XCD first, else a fresh env in
    // cost order; -1 once every env has finished its env-step
    int pick = -1, fresh = 0;
    for (;;) {
      // bucket occupancy, one lane per bucket; the highest non-empty bucket is the best
      // yielded env (its exact work left rides in the entry; an entry still in flight
      // reads 0 and counts as large)
      uint32_t hb = 0, tb = 0;
      if (lane < GM_CQ_NB) { hb = ld_agent(bq + lane * 32); tb = ld_agent(bq + lane * 32 + 1); }
      const unsigned long long ne = __ballot(lane < GM_CQ_NB && hb < tb);
      const uint32_t fh = __builtin_amdgcn_readfirstlane(ld_agent(fresh_head));
      const bool have_f = fh < n;
      if (!have_f && !saw_empty) {
        saw_empty = true;
        if (lane == 0)
          __hip_atomic_fetch_min(q.st + 1, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const int bsel = ne ? 63 - __builtin_clzll(ne) : -1;
      bool take_c = bsel >= 0;
      if (take_c && have_f) {
        const uint32_t h = __builtin_amdgcn_readlane(hb, bsel);
        const uint64_t e = ld_agent64(ring + (size_t)bsel * q.cap + h % (uint32_t)q.cap);
        take_c = e == 0ull || (uint64_t)(uint32_t)(e >> 32) >= (uint64_t)cost[order[fh]] * (uint64_t)(q.steps > 1 ? q.steps : 1);
      }
      if (take_c) {
        int got = 0;
        if (lane == 0) {
          uint64_t* rb = ring + (size_t)bsel * q.cap;
          const int64_t c = claim_bucket(bq + bsel * 32);
          if (c >= 0) {
            got = 1;
            const uint32_t i = (uint32_t)c % (uint32_t)q.cap;
            uint64_t v;
            uint32_t polls = 0;
            // acquire: pairs with the producer's release store of this entry
            while ((v = __hip_atomic_load(rb + i, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) == 0ull &&
                   ld_agent(n_done) < n) {
              __builtin_amdgcn_s_sleep(2);
              polls++;
            }
            if (polls) { add_agent(q.ctr + GM_CQ_DONE + 5, 1u); add_agent(q.ctr + GM_CQ_DONE + 6, polls); }
            if (v != 0ull) {
              st_agent(rb + i, 0ull);
              add_agent(q.ctr + GM_CQ_DONE + 2, 1u);
              pick = (int)(uint32_t)v - 1;
            }
          }
        }
        if (__builtin_amdgcn_readfirstlane(got)) break;   // pick < 0: everything finished while waiting
        continue;                                          // the entry went to another wave: poll again
      }
      if (have_f) {
        if (lane == 0) {
          const uint32_t i = add_agent(fresh_head, 1u);
          if (i < n) { pick = order[i]; fresh = 1; }
        }
        if (__builtin_amdgcn_readfirstlane(pick) >= 0) break;
      } else if (q.steal) {
        // nothing unstarted and nothing yielded on this XCD: the best yielded env of another
        // XCD (its hot state was published with an agent-scope release, the acquire below
        // makes it visible here; same-XCD resumption is only the faster case).  Lane l looks
        // at XCD l / 8, buckets 15 - l % 8 and 7 - l % 8.
        const int x2 = lane >> 3;
        const uint32_t* bq2 = q.ctr + x2 * GM_CQ_NB * 32;
        const int bh = 15 - (lane & 7), bl = 7 - (lane & 7);
        const bool other = x2 != xcc;
        const bool nh = other && ld_agent(bq2 + bh * 32) < ld_agent(bq2 + bh * 32 + 1);
        const bool nl = other && ld_agent(bq2 + bl * 32) < ld_agent(bq2 + bl * 32 + 1);
        const unsigned long long mh = __ballot(nh), ml = __ballot(nl);
        if (mh | ml) {
          // the highest non-empty bucket over the other XCDs (lowest lane among equals)
          int src = -1, sb = -1;
          for (int r = 0; r < 8 && src < 0; r++) {   // bucket 15 - r in the high half, lanes with lane % 8 == r
            const unsigned long long m8 = mh & (0x0101010101010101ull << r);
            if (m8) { src = (int)__builtin_ctzll(m8) >> 3; sb = 15 - r; }
          }
          for (int r = 0; r < 8 && src < 0; r++) {
            const unsigned long long m8 = ml & (0x0101010101010101ull << r);
            if (m8) { src = (int)__builtin_ctzll(m8) >> 3; sb = 7 - r; }
          }
          int got = 0;
          if (lane == 0) {
            uint32_t* sbq = q.ctr + src * GM_CQ_NB * 32;
            uint64_t* rb = q.ring + (size_t)src * GM_CQ_NB * q.cap + (size_t)sb * q.cap;
            const int64_t c = claim_bucket(sbq + sb * 32);
            if (c >= 0) {
              got = 1;
              const uint32_t i = (uint32_t)c % (uint32_t)q.cap;
              uint64_t v;
              uint32_t polls = 0;
              while ((v = __hip_atomic_load(rb + i, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) == 0ull &&
                     ld_agent(n_done) < n) {
                __builtin_amdgcn_s_sleep(2);
                polls++;
              }
              if (polls) { add_agent(q.ctr + GM_CQ_DONE + 5, 1u); add_agent(q.ctr + GM_CQ_DONE + 6, polls); }
              if (v != 0ull) {
                st_agent(rb + i, 0ull);
                add_agent(q.ctr + GM_CQ_DONE + 2, 1u);
                add_agent(q.ctr + GM_CQ_DONE + 4, 1u);   // steals
                pick = (int)(uint32_t)v - 1;
              }
            }
          }
          if (__builtin_amdgcn_readfirstlane(got)) break;   // pick < 0: everything finished while waiting
        }
      }
      if (__builtin_amdgcn_readfirstlane(ld_agent(n_done)) >= n) break;
      __builtin_amdgcn_s_sleep(2);
    }
    pick = __builtin_amdgcn_readfirstlane(pick);
    fresh = __builtin_amdgcn_readfirstlane(fresh);
    const unsigned long long tp = __builtin_amdgcn_s_memrealtime();
    poll += tp - tw;
    if (pick < 0) break;
    if (first && lane == 0)
      __hip_atomic_fetch_min(q.st, tp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    first = false;
    const int env = pick;
    uint64_t* env_t = reinterpret_cast<uint64_t*>(q.st) + 16 + gridDim.x + 2 * (size_t)env;   // gm_chunk_timeline
    if (fresh && lane == 0) st_agent(env_t, tp);
    const unsigned long long t_start = __builtin_amdgcn_s_memtime();
    if (!fresh) {
      // lane 0's acquire load saw the entry; the fence extends that acquire to the whole
      // wave's loads of the env's state (another CU of this XCD stored it) below
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    GmEnvState* g = states + env;
    load_state(S, g, lane);
    GmChunkCarry cr;
    if (fresh) {
      cr.sub_done = 0;
      cr.nsub = C->sim_steps_per_action + S.s.extra_substeps;
      cr.work_nefc = 0; cr.work_mpr = 0; cr.work_newton = 0; cr.stp_fixed = 0;
      cr.clk = 0;
      cr.yielded = 0;
      cr.steps_left = q.steps;
      cr.step_idx = 0;
      cr.job_yields = 0;
    } else {
      // agent-scope loads: never served by a scalar cache that the acquire does not reach
      const uint32_t* src = reinterpret_cast<const uint32_t*>(q.carry + env);
      uint32_t* dst = reinterpret_cast<uint32_t*>(&cr);
#pragma unroll
      for (int w = 0; w < (int)(sizeof(GmChunkCarry) / 4); w++) dst[w] = ld_agent(src + w);
    }
    if (lane == 0) {
      S.work_nefc = cr.work_nefc; S.work_mpr = cr.work_mpr; S.work_newton = cr.work_newton;
      S.stp_fixed = cr.stp_fixed;
    }
    GM_ENV_SYNC();
    const uint64_t own = (uint64_t)cost[env] * (uint64_t)(q.steps > 1 ? q.steps : 1);   // the job's predicted cost
    const int s_nom = C->sim_steps_per_action;
    bool finished = false;
    for (;;) {   // the env-steps of this pick
      if (cr.sub_done == 0 && q.act_mode >= 0) {
        // a new env-step of a rollout: the driver's actions first (they may add the
        // termination lift's substeps), as gm_set_action before gm_step
        if (q.act_mode == 2) {
          // gm_policy_act on this env alone: select_action from its current observation,
          // then set_discrete_action (the LDS scratch: the dynamics union, dead between
          // env-steps)
          static_assert(sizeof(S.st) >= sizeof(float) * 2 * (GP_MAX_WIDTH + 4), "policy activations fit the union");
          const int a = gp_select_one(obs + (size_t)env * C->n_obs, q.pparams, q.pnet, q.peps[cr.step_idx], q.pseed,
                                      q.pdecision + (uint64_t)cr.step_idx, (uint64_t)(q.sr.env_offset + env),
                                      reinterpret_cast<float*>(&S.st), lane);
          if (lane == 0) {
            set_action_one(S.s, m, C, a, 0.0f);
            S.stp_fixed = 0;
          }
        } else if (lane == 0) {
          driver_actions(S.s, g->ring, m, C, q.act_mode, q.act_seed, q.jitter, q.sr.env_offset + env);
          S.stp_fixed = 0;
        }
        GM_ENV_SYNC();
        cr.nsub = C->sim_steps_per_action + S.s.extra_substeps;
      }
      // run to the end of the env-step unless an unstarted env has become the longer job
      // (work left counted over the launch's whole job of env-steps)
      const int left = cr.nsub - cr.sub_done;
      const int job_left = (cr.steps_left - 1) * s_nom + left;
      const int job_total = q.steps > 1 ? q.steps * s_nom : cr.nsub;
      const uint32_t est = (uint32_t)(own > 0xFFFFFFFFull ? 0xFFFFFFFFull : own);
      const GmPreempt pre{fresh_head, order, cost, n, est, job_left, job_total,
                          cr.yielded < q.max_yields ? q.chunk : 0, q.margin, bq, cmax, q.cmargin, q.prio,
                          q.steps > 1 ? q.steps : 1};
      job_prio((uint64_t)est * (uint64_t)job_left / (uint64_t)(job_total > 0 ? job_total : 1), cmax, q.prio);
      const int k = substep_loop<CL, false, false, DUO>((GM_AS_LDS SharedT<CL>*)&S, (const GM_AS_GLOBAL gm_model*)m,
                                            (const GM_AS_GLOBAL GmTopo*)T, (const GM_AS_GLOBAL gm_config*)C, lane,
                                            false, left, false, pre);
      cr.sub_done += k;
      if (cr.sub_done < cr.nsub) break;   // yielded
      unsigned long long t0 = 0;
      env_step_epilogue(S, m, C, T, obs, rew, done, env, lane, false, t0);
      if (q.act_mode >= 0) {
        // gm_autoreset_episodes on this env: the episode-end record, then MjEnv.reset
        const int r = __builtin_amdgcn_readfirstlane(
            (S.s.done || (q.max_ep > 0 && S.s.num_action_steps >= q.max_ep)) ? 1 : 0);
        if (lane == 0 && q.rec) {
          gm_episode_end e;
          e.ret = r ? S.s.cumulative_reward : __builtin_nanf("");
          e.length = r ? S.s.num_action_steps : 0;
          e.success = (r && S.s.bev_last[GM_EV_successful_grasp]) ? 1 : 0;
          e.pad[0] = e.pad[1] = e.pad[2] = 0;
          q.rec[(size_t)cr.step_idx * n + env] = e;
        }
        if (r) {
          GM_ENV_SYNC();   // lane 0's epilogue writes (RNG, counters) before every lane reads them
          const GmResetKeep keep{S.s.rng, S.s.old_x, S.s.old_y, S.s.old_z, S.s.episode + 1, S.s.newton_caps};
          GM_ENV_SYNC();   // every lane has read what survives before the image is cleared
          static_assert(sizeof(S.st) >= sizeof(uint16_t) * (GM_SPAWN_MAX_XY + GM_SPAWN_MAX_ROT),
                        "spawn search buffers alias the (dead between env-steps) dynamics union");
          uint16_t* sh_pxy = reinterpret_cast<uint16_t*>(&S.st);
          reset_env(S.s, *g, keep, m, C, T, q.eq, nullptr, q.objs, q.n_objects, env, q.scene, q.scene_tries, q.sr,
                    sh_pxy, sh_pxy + GM_SPAWN_MAX_XY, lane);
          get_obs_lanes(S.s, g->ring, C, obs + (size_t)env * C->n_obs, lane);
        }
      }
      cr.steps_left -= 1;
      cr.step_idx += 1;
      if (cr.steps_left <= 0) { finished = true; break; }
      cr.sub_done = 0;
      cr.yielded = 0;
      GM_ENV_SYNC();
    }
    if (finished) {
      if (cost && lane == 0) {
        // the dispatch cost (see gm_step_kernel): clocks of this job's chunks, blended with
        // the work model
        const uint32_t now = cr.clk + (uint32_t)((__builtin_amdgcn_s_memtime() - t_start) >> 6);
        const uint32_t model = 14000u * (uint32_t)q.steps + 19u * (uint32_t)S.work_nefc + 188u * (uint32_t)S.work_mpr +
                               940u * (uint32_t)S.work_newton;
        // recorded for the next launch's order, per env-step (whatever the next launch's job length)
        cost[n + env] = ((now >> 1) + (model >> 1)) / (uint32_t)(q.steps > 1 ? q.steps : 1);
        // diagnostics (gm_chunk_job_stats): the job's busy clocks / 64 and its yields
        __hip_atomic_store(&q.carry[env].clk, now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&q.carry[env].job_yields, cr.job_yields, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      store_state(S, g, lane);
      if (lane == 0) {
        add_agent(n_done, 1u);
        st_agent(env_t + 1, __builtin_amdgcn_s_memrealtime());
        __hip_atomic_fetch_max(q.st + 2, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      store_state(S, g, lane);
      if (lane == 0) {
        cr.work_nefc = S.work_nefc; cr.work_mpr = S.work_mpr; cr.work_newton = S.work_newton;
        cr.stp_fixed = S.stp_fixed;
        cr.yielded += 1;
        cr.job_yields += 1;
        cr.clk += (uint32_t)((__builtin_amdgcn_s_memtime() - t_start) >> 6);
        q.carry[env] = cr;
      }
      // publish (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms): the wave's
      // state / carry stores drained, then lane 0's agent-scope release (the XCD L2 written
      // back, so a consumer on ANY XCD sees the bytes after its acquire), drained again
      // before the ring entry's relaxed agent store
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      GM_ENV_SYNC();
      if (lane == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int job_total = q.steps > 1 ? q.steps * s_nom : cr.nsub;
        const int job_left = (cr.steps_left - 1) * s_nom + (cr.nsub - cr.sub_done);
        const uint64_t rem = own * (uint64_t)job_left / (uint64_t)job_total;
        add_agent(q.ctr + GM_CQ_DONE + 1, 1u);
        const uint32_t b = rem * GM_CQ_NB / cmax < GM_CQ_NB - 1 ? (uint32_t)(rem * GM_CQ_NB / cmax) : GM_CQ_NB - 1;
        const uint32_t t = add_agent(bq + b * 32 + 1, 1u) % (uint32_t)q.cap;
        __hip_atomic_store(ring + (size_t)b * q.cap + t,
                           ((rem > 0xFFFFFFFFull ? 0xFFFFFFFFull : rem) << 32) | ((uint64_t)env + 1u), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    GM_ENV_SYNC();   // LDS image reused by the next pick
    last_end = __builtin_amdgcn_s_memrealtime();
    busy += last_end - tp;
  }
  if (lane == 0) {
    __hip_atomic_fetch_add(q.st + 3, busy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(q.st + 4, poll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // this workgroup's last work (gm_chunk_timeline), its XCD in the top four bits
    st_agent(reinterpret_cast<uint64_t*>(q.st) + 16 + blockIdx.x, last_end | ((uint64_t)xcc << 60));
  }
}
// mode 0: action_step + obs/done/reward; mode 1: calibrate_reset settle (400 substeps,
// no sensors); mode 2: one full substep with diagnostics
#ifndef GM_WPS
#define GM_WPS 2   // waves per SIMD the register allocation is held to
#endif
// DUO workgroups (small batches, gm_capi.hip launch_step): the second wave of the
// workgroup runs each substep's collider for the env the first wave owns, between the
// first two barriers of physics_substep_body, with its own box-box hit slots, then the
// factor of integrate's Euler damping solve while the owner runs the constraint solve
// (third barrier, in integrate); duo_cmd = 0 releases it.
template <int CL>
__device__ __forceinline__ void duo_helper(SharedT<CL>& S, const gm_model* __restrict__ m, const GmTopo* __restrict__ T) {
  __shared__ real hit[GM_BB_SLOTS][8][4];
  for (;;) {
    __syncthreads();
    if (S.duo_cmd == 0) return;
    collision<CL>(S, m, T, fresh_lane(), false, hit);
    {
      // the constraint setup's contact rows for the owner (contact_rows), the body
      // velocities in the hit slots (dead once the contacts are written).  (Measured: only
      // on the substeps whose collider ran no MPR, the owner forming them on the rest, was
      // no better: tools/duo_rows_ab.sh, profiles/r06_ab_duo_rows.txt)
      static_assert(sizeof(hit) >= sizeof(real) * 12 * SharedT<CL>::NB, "two velocity sets fit the hit slots");
      const int ln = fresh_lane();
      real (*V)[6] = reinterpret_cast<real (*)[6]>(&hit[0][0][0]);
      real cD, caref[4], jq[4];
      bool oo;
      contact_rows<CL, false>(S, m, T, ln, V, V + SharedT<CL>::NB, cD, caref, jq, oo);
      DuoRows<CL>* dr = duo_rows<CL>();
      if (ln < GM_MAX_CON) {
        dr->cD[ln] = cD;
#pragma unroll
        for (int e = 0; e < 4; e++) { dr->caref[e][ln] = caref[e]; dr->jq[e][ln] = jq[e]; }
      }
      if (ln == 0) dr->obj_only = oo ? 1 : 0;
    }
    __syncthreads();
    // M is formed (the owner wave's mass_and_forces ran before the barrier): the Euler
    // damping factor for integrate, while the owner runs the constraint solve
    if (m->mujoco_actuators != 0) {
      const int ln = fresh_lane();
      real L[CL + 1], lb, invd;
      const real sch = euler_factor<CL>(S, T, m->timestep, ln, L, lb, invd);
      real* ef = duo_ef<CL>();
#pragma unroll
      for (int j = 1; j <= CL; j++) ef[(j - 1) * 64 + ln] = L[j];
      ef[CL * 64 + ln] = lb;
      ef[(CL + 1) * 64 + ln] = invd;
      if (ln == 0) ef[64 * (CL + 2)] = sch;
    }
    __syncthreads();
  }
}
template <int CL, bool CAL, bool DUO>
__device__ __forceinline__ void step_kernel_body(SharedT<CL>& S,
    GmEnvState* __restrict__ states, const gm_model* __restrict__ m, const gm_config* __restrict__ C,
    const GmTopo* __restrict__ T, float* __restrict__ obs, float* __restrict__ rew,
    uint8_t* __restrict__ done, int n_envs, int mode, DebugOut dbg, const int32_t* __restrict__ order,
    uint32_t* __restrict__ cost, const GmChunkQ& q, int lane) {
  if constexpr (!CAL) {
    if (q.chunk > 0) {   // chunked work queue (gm_step): the grid is the resident wave slots
      chunked_env_steps<CL, DUO>(S, states, m, C, T, obs, rew, done, n_envs, order, cost, q, lane);
      return;
    }
  }
  if ((int)blockIdx.x >= n_envs) return;
  // cost-sorted dispatch: workgroups start in blockIdx order, so the envs that were the
  // most expensive last env-step are started first (longest-processing-time list
  // scheduling over the resident slots; see gm_dispatch_order_kernel)
  const int env = order ? order[blockIdx.x] : (int)blockIdx.x;
  const unsigned long long t_start = cost ? __builtin_amdgcn_s_memtime() : 0;
  load_state(S, states + env, lane);
  const bool settle = (mode == 1);          // calibrate_reset settle: 400 substeps, no sensors
  const bool calib = CAL;                   // calibration run (mode 3): S.s.cal_steps substeps, no sensors
  const bool prof = !settle && dbg.phase != nullptr;
  if (prof && lane < GM_NPHASE) S.tph[lane] = 0;
  // profiling timeline: start / end on the 100 MHz constant clock and the wave's CU, for
  // the dispatch-occupancy analysis (tools/tail_bench.py)
  if (prof && lane == 0) { S.tph[25] = __builtin_amdgcn_s_memrealtime(); S.tph[27] = __smid(); }
  if (lane == 0) { S.work_nefc = 0; S.work_mpr = 0; S.work_newton = 0; S.stp_fixed = 0; }
  const unsigned long long t_kernel = prof ? clock64() : 0;
  GM_ENV_SYNC();
  const int nsub = settle ? 400 : calib ? S.s.cal_steps : (mode == 2) ? 1 : C->sim_steps_per_action + S.s.extra_substeps;
  // a calibration run starts from a reset's mj_forward pose
  if (calib && lane < T->nlock) S.lock_pre[lane] = S.s.qpos[m->lock_dof[lane]];
  int ran;
  if constexpr (DUO) {   // (profiled: the owner wave's clocks; its "collision" is the wait for the helper)
    ran = prof ? substep_loop<CL, CAL, true, true>((GM_AS_LDS SharedT<CL>*)&S, (const GM_AS_GLOBAL gm_model*)m,
                                                   (const GM_AS_GLOBAL GmTopo*)T, (const GM_AS_GLOBAL gm_config*)C, lane,
                                                   prof, nsub, settle, GmPreempt{})
               : substep_loop<CL, CAL, false, true>((GM_AS_LDS SharedT<CL>*)&S, (const GM_AS_GLOBAL gm_model*)m,
                                                    (const GM_AS_GLOBAL GmTopo*)T, (const GM_AS_GLOBAL gm_config*)C, lane,
                                                    false, nsub, settle, GmPreempt{});
  } else {
    ran = prof ? substep_loop<CL, CAL, true>((GM_AS_LDS SharedT<CL>*)&S, (const GM_AS_GLOBAL gm_model*)m,
                                             (const GM_AS_GLOBAL GmTopo*)T, (const GM_AS_GLOBAL gm_config*)C, lane,
                                             prof, nsub, settle, GmPreempt{})
               : substep_loop<CL, CAL, false>((GM_AS_LDS SharedT<CL>*)&S, (const GM_AS_GLOBAL gm_model*)m,
                                              (const GM_AS_GLOBAL GmTopo*)T, (const GM_AS_GLOBAL gm_config*)C, lane,
                                              false, nsub, settle, GmPreempt{});
  }
  // a calibration run reports the substeps it made (the unstable one included: the loop
  // stops right after it, as the reference's retry resumes after it)
  if (calib && lane == 0) S.s.cal_steps = S.s.badqacc ? ran + 1 : ran;
  if (settle || calib) {
    store_state(S, states + env, lane);
    return;
  }
  if (mode == 2) {
    if (lane == 0) { dbg.ncon[env] = S.ncon; dbg.nefc[env] = S.nefc; }
    if (lane < GM_MAX_CON) {
      double* o = dbg.contact + ((size_t)env * GM_MAX_CON + lane) * 16;
      for (int k = 0; k < 16; k++) o[k] = 0;
      if (lane < S.ncon) {
        const real* Cc = S.con[lane];
        o[0] = Cc[0];
        for (int k = 0; k < 3; k++) o[1 + k] = Cc[1 + k];
        for (int k = 0; k < 6; k++) o[4 + k] = Cc[4 + k];
        cross3(o + 10, Cc + 4, Cc + 7);
        o[13] = S.cgeom[lane][0]; o[14] = S.cgeom[lane][1]; o[15] = Cc[10];
      }
    }
    for (int r = lane; r < GM_MAX_EFC; r += NT)
      dbg.efc_force[(size_t)env * GM_MAX_EFC + r] = r < S.nefc ? S.dbg.efc[r] : 0.0;
    if (lane < GM_MAX_DOF) dbg.qacc[(size_t)env * GM_MAX_DOF + lane] = lane < T->nv ? S.qacc[lane] : 0.0;
    {
      real w[6];
      object_net_wrench(S, T, lane, w);
      if (lane == 0) for (int k = 0; k < 6; k++) dbg.wrench[(size_t)env * 6 + k] = w[k];
    }
    store_state(S, states + env, lane);
    return;
  }
  unsigned long long t0 = prof ? clock64() : 0;
  env_step_epilogue(S, m, C, T, obs, rew, done, env, lane, prof, t0);
  if (prof) {
    if (lane == 0) {
      S.tph[23] = clock64() - t_kernel;   // whole env-step on this wave
      S.tph[26] = __builtin_amdgcn_s_memrealtime();
    }
    GM_ENV_SYNC();
    if (lane < GM_NPHASE) dbg.phase[(size_t)env * GM_NPHASE + lane] = S.tph[lane];
  }
  if (cost && lane == 0) {
    // next env-step's dispatch cost: the measured one (shader clocks / 64; it carries
    // co-residency noise) averaged with a work model of this env-step (a fixed part, the
    // Hessian work per constraint row, each Newton iteration, the convex collider's
    // latency per substep that ran it; fitted on the C3 workload, tools/tail_bench.py): the blend orders the
    // next launch closer to its true costs than either alone (LPT makespan 1.17 vs 1.21
    // of the ideal on recorded costs)
    const uint32_t now = (uint32_t)((__builtin_amdgcn_s_memtime() - t_start) >> 6);
    const uint32_t model = 14000u + 19u * (uint32_t)S.work_nefc + 188u * (uint32_t)S.work_mpr +
                           940u * (uint32_t)S.work_newton;
    cost[n_envs + env] = (now >> 1) + (model >> 1);   // recorded for the next launch's order
  }
  store_state(S, states + env, lane);
}
template <int CL, bool CAL, bool DUO = false>
__global__ __launch_bounds__(DUO ? 2 * NT : NT, GM_WPS) void gm_step_kernel(
    GmEnvState* __restrict__ states, const gm_model* __restrict__ m, const gm_config* __restrict__ C,
    const GmTopo* __restrict__ T, float* __restrict__ obs, float* __restrict__ rew,
    uint8_t* __restrict__ done, int n_envs, int mode, DebugOut dbg, const int32_t* __restrict__ order,
    uint32_t* __restrict__ cost, GmChunkQ q) {
  __shared__ SharedT<CL> S;
  if constexpr (DUO) {
    static_assert(!CAL, "DUO workgroups run the env-step only");
    if (threadIdx.x >= NT) {
      duo_helper<CL>(S, m, T);
      return;
    }
  }
  step_kernel_body<CL, CAL, DUO>(S, states, m, C, T, obs, rew, done, n_envs, mode, dbg, order, cost, q, (int)threadIdx.x);
  if constexpr (DUO) {
    // every path of the owner wave ends here: release the helper
    if (threadIdx.x == 0) S.duo_cmd = 0;
    __syncthreads();
  }
}


// Dispatch order for the next env-step: envs by descending cost of their last env-step
// (shader clocks / 64, written by gm_step_kernel), bucketed into 256 cost classes.
// One 1024-thread workgroup; the order only changes which env a workgroup slot runs
// first, never any result.
#ifndef GM_CAL_TU   // env-step translation unit only
extern "C" __global__ __launch_bounds__(1024) void gm_dispatch_order_kernel(uint32_t* __restrict__ cost,
                                                                            int32_t* __restrict__ order, int n,
                                                                            uint32_t* __restrict__ chunk_ctr,
                                                                            unsigned long long* __restrict__ chunk_st) {
  __shared__ uint32_t cnt[256];
  __shared__ uint32_t cmax;
  const int t = threadIdx.x;
  if (chunk_ctr && t < 39) chunk_ctr[GM_CQ_LAST + t] = chunk_ctr[GM_CQ_FRESH + t];   // last launch's, for diagnostics
  __syncthreads();
  if (chunk_ctr)
    for (int w = t; w < GM_CQ_WORDS; w += 1024) chunk_ctr[w] = 0;   // the chunked launch's queue counters
  if (chunk_st && t < 8) {
    chunk_st[8 + t] = chunk_st[t];
    chunk_st[t] = (t < 2) ? ~0ull : 0ull;
  }
  if (t < 256) cnt[t] = 0;
  if (t == 0) cmax = 1;
  __syncthreads();
  uint32_t m = 1;
  for (int i = t; i < n; i += 1024) {
    const uint32_t c = cost[n + i];   // the costs the last launch recorded become current
    cost[i] = c;
    m = max(m, c);
  }
  atomicMax(&cmax, m);
  __syncthreads();
  const uint64_t cm = (uint64_t)cmax + 1;
  if (chunk_ctr && t == 0) chunk_ctr[GM_CQ_CMAX] = (uint32_t)cm;
  for (int i = t; i < n; i += 1024) {
    const int b = 255 - (int)(((uint64_t)cost[i] * 256) / cm);
    atomicAdd(&cnt[b], 1u);
  }
  __syncthreads();
  {
    // exclusive prefix over the 256 buckets: shuffle scans in the first four waves, then
    // each wave's offset from the wave totals (a serial loop on one thread took ~10 us)
    __shared__ uint32_t wsum[4];
    const uint32_t v = (t < 256) ? cnt[t] : 0u;
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(inc, o);
      if ((t & 63) >= o) inc += u;
    }
    if (t < 256 && (t & 63) == 63) wsum[t >> 6] = inc;
    __syncthreads();
    if (t < 256) {
      uint32_t base = 0;
      for (int w = 0; w < (t >> 6); w++) base += wsum[w];
      cnt[t] = base + inc - v;
    }
  }
  __syncthreads();
  for (int i = t; i < n; i += 1024) {
    const int b = 255 - (int)(((uint64_t)cost[i] * 256) / cm);
    order[atomicAdd(&cnt[b], 1u)] = i;
  }
}
#endif

// ---------------------------------------------------------------- actions
// MjClass::set_action for every action index (mjclass.cpp:1528-1630); one thread per env.
__device__ int move_base_target_m(GmEnvHot& s, const gm_config* __restrict__ C, double x, double y, double z) {
  double* b = s.base;
  b[0] += x; b[1] += y; b[2] += z;
  int wl = 1;
  for (int k = 0; k < 3; k++) {
    if (b[k] > C->base_max[k]) { b[k] = C->base_max[k]; wl = 0; }
    if (b[k] < C->base_min[k]) { b[k] = C->base_min[k]; wl = 0; }
  }
  return wl;
}
__device__ int call_action(GmEnvHot& s, const gm_config* __restrict__ C, int kind, double v) {
  const gm_action* acts[GM_N_ACTION_KINDS] = {
#define GM_AA(n, u, vv, sg) &C->s.n,
#include "gm_settings.def"
  };
  v *= acts[kind]->sign;
  switch (kind) {
    case GM_ACT_gripper_X: return g_set_xyz_m(s.end, s.end.x + v, s.end.y, s.end.z);
    case GM_ACT_gripper_Y: return g_set_xyz_m(s.end, s.end.x, s.end.y + v, s.end.z);
    case GM_ACT_gripper_prismatic_X: return g_set_xyz_m_rad(s.end, s.end.x + v, s.end.th, s.end.z);
    case GM_ACT_gripper_revolute_Y: return g_set_xyz_m_rad(s.end, s.end.x, s.end.th + v, s.end.z);
    case GM_ACT_gripper_Z: return g_set_xyz_m(s.end, s.end.x, s.end.y, s.end.z + v);
    case GM_ACT_base_X: return move_base_target_m(s, C, v, 0, 0);
    case GM_ACT_base_Y: return move_base_target_m(s, C, 0, v, 0);
    case GM_ACT_base_Z: return move_base_target_m(s, C, 0, 0, v);
    case GM_ACT_base_roll:
    case GM_ACT_base_pitch: return 1;
    default: {
      s.base[5] += v;
      int wl = 1;
      if (s.base[5] > C->base_max[5]) { s.base[5] = C->base_max[5]; wl = 0; }
      if (s.base[5] < C->base_min[5]) { s.base[5] = C->base_min[5]; wl = 0; }
      return wl;
    }
  }
}
__device__ void set_action_one(GmEnvHot& s, const gm_model* __restrict__ m, const gm_config* __restrict__ C,
                               int action, float frac) {
  const gm_settings& st = C->s;
  int wl = 1;
  s.termination_signal_sent = 0;
  if (action < 0 || action >= C->n_actions) return;
  int code = C->action_options[action];
  if (code == GM_ACTION_TERMINATION) {
    float value = st.continous_actions ? frac : 1.0f;
    if (value > st.termination_threshold) {
      s.termination_signal_sent = 1;
      if (st.lift_on_termination) {
        s.base[2] = -C->base_max[2];
        if (s.base[2] > C->base_max[2]) s.base[2] = C->base_max[2];
        if (s.base[2] < C->base_min[2]) s.base[2] = C->base_min[2];
        s.extra_substeps += C->sim_steps_per_action * 2;
      }
    }
    wl = 1;
  } else {
    const gm_action* acts[GM_N_ACTION_KINDS] = {
#define GM_AA(n, u, vv, sg) &st.n,
#include "gm_settings.def"
    };
    int kind = code / 3, sub = code % 3;
    if (sub == 0) wl = call_action(s, C, kind, acts[kind]->value);
    else if (sub == 1) wl = call_action(s, C, kind, -1 * acts[kind]->value);
    else {
      wl = call_action(s, C, kind, acts[kind]->value * frac);
      s.lev_value[GM_LEV_action_penalty_lin] += fabsf(frac);
      s.lev_value[GM_LEV_action_penalty_sq] += (frac * frac);
    }
  }
  // get_fingertip_z_height (myfunctions.cpp:3608-3620)
  float straight = (float)(-C->base_min[2] - s.base[2]);
  float tip_lift = (float)(m->finger_length * (1 - cos(g_calc_th(s.end.x, s.end.y))));
  float hgt = straight + tip_lift;
  float fz = (float)(hgt + C->base_min[2]);
  if (fz < st.fingertip_min_mm * 1e-3) wl = 0;
  s.bev_value[GM_EV_exceed_limits] = s.bev_value[GM_EV_exceed_limits] || !wl;
}

#ifndef GM_CAL_TU   // env-step translation unit only
extern "C" __global__ void gm_action_kernel(GmEnvState* __restrict__ states, const gm_model* __restrict__ m,
                                            const gm_config* __restrict__ C, const float* __restrict__ cont,
                                            const int32_t* __restrict__ disc, int n_envs) {
  int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  GmEnvState& s = states[env];
  if (cont) {
    for (int i = 0; i < C->n_actions; i++) {
      float f = cont[(size_t)env * C->n_actions + i];
      if (f < -1.0f) f = -1.0f; else if (f > 1.0f) f = 1.0f;
      set_action_one(s, m, C, i, f);
    }
  } else {
    set_action_one(s, m, C, disc[env], 0.0f);
  }
}
#endif

// ---------------------------------------------------------------- scripted grasp mix
// The benchmark's / parity tests' synthetic driver (gmx.GraspScript mirrors it on the
// host bit for bit): per env and episode, phase lengths drawn from the counter-based
// hash (seed, global env id, episode) -- close the fingers, squeeze (tilt the tips), press
// the palm, lift the base -- indexed by the env's own episode step (num_action_steps),
// plus uniform jitter per (step, action).  Continuous action fractions in [-1, 1] for
// the in-use actions (MjClass::set_continous_action order).
#ifndef GM_CAL_TU   // env-step translation unit only
extern "C" __global__ void gm_scripted_action_kernel(const GmEnvState* __restrict__ states, const gm_config* __restrict__ C,
                                                     float* __restrict__ out, int n_envs, uint64_t seed,
                                                     long long env_offset, float jitter) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  const GmEnvState& s = states[env];
  const int na = C->n_actions;
  for (int i = 0; i < na; i++) {
    const int code = C->action_options[i];
    const int kind = (code >= 0 && code < GM_ACTION_TERMINATION) ? code / 3 : -1;
    out[(size_t)env * na + i] = gm_script_fraction(seed, env_offset + env, s.episode, s.num_action_steps, i, kind, jitter);
  }
}
#endif

// the driver's actions for the current state of every env (gm_program_actions): modes 3
// (grasp program) and 4 (program / scripted mix), thread per env
#ifndef GM_CAL_TU   // env-step translation unit only
extern "C" __global__ void gm_program_action_kernel(const GmEnvState* __restrict__ states, const gm_model* __restrict__ m,
                                                    const gm_config* __restrict__ C, float* __restrict__ out, int n_envs,
                                                    uint64_t seed, long long env_offset, float jitter, int mode) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  const GmEnvState& s = states[env];
  const int na = C->n_actions;
  for (int i = 0; i < na; i++) {
    const int code = C->action_options[i];
    const int kind = (code >= 0 && code < GM_ACTION_TERMINATION) ? code / 3 : -1;
    const float v = driver_fraction(s, const_cast<RingRef>(s.ring), m, C, mode, seed, jitter, env_offset + env, i, kind);
    out[(size_t)env * na + i] = v < -1.0f ? -1.0f : (v > 1.0f ? 1.0f : v);
  }
}
#endif

// uniform random action fractions (gm_random_actions; the rollout's random mode): U[-1, 1)
// per (env, episode, episode step, action) from the counter-based hash (gm_state.h)
#ifndef GM_CAL_TU   // env-step translation unit only
extern "C" __global__ void gm_random_action_kernel(const GmEnvState* __restrict__ states, const gm_config* __restrict__ C,
                                                   float* __restrict__ out, int n_envs, uint64_t seed,
                                                   long long env_offset) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  const GmEnvState& s = states[env];
  const int na = C->n_actions;
  for (int i = 0; i < na; i++)
    out[(size_t)env * na + i] = gm_random_fraction(seed, env_offset + env, s.episode, s.num_action_steps, i);
}
#endif

// ---------------------------------------------------------------- reset + spawn
// MjClass::spawn_object -> ObjectHandler::spawn_object (mjclass.cpp:2352-2420,
// objecthandler.cpp:403-428): live object, pose on the ground at (x, y), z-rotation
__device__ void spawn_object(GmEnvHot& s, const GmTopo* __restrict__ T, const gm_object* __restrict__ objs,
                             int n_objects, gm_spawn sp) {
  int oi = sp.object_index;
  if (oi < 0 || oi >= n_objects) oi = 0;
  const gm_object& o = objs[oi];
  s.obj_index = oi;
  s.obj_type = o.type;
  s.obj_size[0] = o.size[0]; s.obj_size[1] = o.size[1]; s.obj_size[2] = o.size[2];
  s.obj_mass = o.mass;
  s.obj_friction = o.friction;
  double I0, I1, I2, rb, restz;
  if (o.type == GM_GEOM_BOX) {
    double a = 2 * o.size[0], bb = 2 * o.size[1], c = 2 * o.size[2];
    I0 = o.mass * (bb * bb + c * c) / 12; I1 = o.mass * (a * a + c * c) / 12; I2 = o.mass * (a * a + bb * bb) / 12;
    rb = sqrt(o.size[0] * o.size[0] + o.size[1] * o.size[1] + o.size[2] * o.size[2]);
    restz = o.size[2];
  } else if (o.type == GM_GEOM_CYLINDER) {
    double r = o.size[0], hh = 2 * o.size[1];
    I0 = I1 = o.mass * (3 * r * r + hh * hh) / 12; I2 = o.mass * r * r / 2;
    rb = sqrt(o.size[0] * o.size[0] + o.size[1] * o.size[1]);
    restz = o.size[1];
  } else {
    double r = o.size[0];
    I0 = I1 = I2 = 2 * o.mass * r * r / 5;
    rb = r;
    restz = r;
  }
  s.obj_inertia[0] = I0; s.obj_inertia[1] = I1; s.obj_inertia[2] = I2;
  s.obj_rbound = rb;
  s.obj_rest_z = restz;
  // body_invweight0 of the live object (mj_setConst at qpos0; oracle object_invweight)
  s.obj_invw[0] = 1.0 / o.mass;
  s.obj_invw[1] = ((1.0 / I0 + 1.0 / I1) + 1.0 / I2) / 3.0;
  int qa = T->qadr_obj;
  double x2, w2;
  gm_sincos(-sp.zrot / 2.0, &x2, &w2);   // shared with the oracle (gm_math.h)
  double q4[4] = {x2, 0, 0, w2};   // reference QPos quirk: qx lands in MuJoCo's w slot
  double nq = sqrt(q4[0] * q4[0] + q4[1] * q4[1] + q4[2] * q4[2] + q4[3] * q4[3]);
  s.qpos[qa + 0] = sp.x;
  s.qpos[qa + 1] = sp.y;
  s.qpos[qa + 2] = restz + 1e-6;
  for (int k = 0; k < 4; k++) s.qpos[qa + 3 + k] = q4[k] / nq;
  for (int k = 0; k < 7; k++) s.start_qpos[k] = s.qpos[qa + k];
  for (int k = 0; k < 6; k++) s.qvel[T->dof_obj + k] = 0;
}

// MjEnv auto-reset bookkeeping (MjEnv.py:616-637, 2170-2263): an env whose episode
// terminated (is_done) or truncated (num_action_steps >= max_episode_steps) hands its
// episode return to `returns` and is flagged for gm_reset_kernel.
// ---------------------------------------------------------------- spawn_into_scene
// MjClass::spawn_into_scene(SpawnParams) (mjclass.cpp:2475-2654), one thread per env.
//
// std::uniform_int_distribution<unsigned long>{a, b} driven by minstd_rand0, as libstdc++
// implements it (bits/uniform_int_dist.h): the engine's range 2^31 - 3 is neither 2^32 - 1
// nor 2^64 - 1, so the downscaling branch takes the two-division rejection path.
__device__ uint64_t uid_minstd(uint32_t& st, uint64_t a, uint64_t b) {
  const uint64_t urngrange = 2147483646ull - 1ull;   // max() - min()
  const uint64_t urange = b - a;
  uint64_t ret;
  if (urngrange > urange) {
    // every operand is below 2^31 here: 32-bit division, the same quotients as the
    // 64-bit ones libstdc++ computes (a 64-bit divide is a long software sequence)
    const uint32_t uerange = (uint32_t)urange + 1u;
    const uint32_t scaling = (uint32_t)urngrange / uerange;
    const uint32_t past = uerange * scaling;
    uint32_t r32;
    do r32 = lcg_next(st) - 1u; while (r32 >= past);
    ret = r32 / scaling;
  } else {
    ret = (uint64_t)lcg_next(st) - 1ull;   // urange == urngrange (grids are far smaller)
  }
  return ret + a;
}
// std::shuffle(first, first + n, minstd_rand0) as libstdc++ implements it
// (bits/stl_algo.h): when the engine range allows, positions are drawn two at a time
// from one uniform_int over [0, (k + 1)(k + 2) - 1] (__gen_two_uniform_ints), with a
// single leading {0, 1} draw for even n.  Shuffling indices permutes exactly like
// shuffling the elements.  (n <= GM_SPAWN_MAX_XY: the pair range and its quotients fit
// 32 bits.)
__device__ __forceinline__ void shuffle_minstd(uint16_t* v, int n, uint32_t& st) {
  if (n <= 0) return;
  const uint64_t urngrange = 2147483645ull, urange = (uint64_t)n;
  if (urngrange / urange >= urange) {
    int i = 1;
    if ((urange % 2) == 0) {
      const int j = (int)uid_minstd(st, 0, 1);
      const uint16_t t = v[i]; v[i] = v[j]; v[j] = t;
      i++;
    }
    while (i != n) {
      const uint32_t r = (uint32_t)i + 1u;
      const uint32_t x = (uint32_t)uid_minstd(st, 0, (uint64_t)r * (r + 1) - 1);
      const int p1 = (int)(x / (r + 1u)), p2 = (int)(x % (r + 1u));
      uint16_t t = v[i]; v[i] = v[p1]; v[p1] = t;
      i++;
      t = v[i]; v[i] = v[p2]; v[p2] = t;
      i++;
    }
  } else {
    for (int i = 1; i < n; i++) {
      const int j = (int)uid_minstd(st, 0, (uint64_t)i);
      const uint16_t t = v[i]; v[i] = v[j]; v[j] = t;
    }
  }
}
// luke::Box2d (customtypes.h:35-172): corners counter-clockwise from bottom-left
struct Box2 { double x[4], y[4]; };
__device__ void box_init_centre(Box2& b, double cx, double cy, double width, double height) {
  const double hw = width / 2.0, hh = height / 2.0;
  b.x[0] = cx - hw; b.y[0] = cy - hh;
  b.x[1] = cx + hw; b.y[1] = cy - hh;
  b.x[2] = cx + hw; b.y[2] = cy + hh;
  b.x[3] = cx - hw; b.y[3] = cy + hh;
}
__device__ void box_rotate(Box2& b, double theta) {
  const double cx = (b.x[0] + b.x[1] + b.x[2] + b.x[3]) / 4.0;
  const double cy = (b.y[0] + b.y[1] + b.y[2] + b.y[3]) / 4.0;
  const double c = cos(theta), s = sin(theta);
  for (int i = 0; i < 4; i++) {
    const double nx = cx + (b.x[i] - cx) * c - (b.y[i] - cy) * s;
    const double ny = cy + (b.x[i] - cx) * s + (b.y[i] - cy) * c;
    b.x[i] = nx; b.y[i] = ny;
  }
}
__device__ bool box_inbounds(const Box2& b, double xmin, double ymin, double xmax, double ymax) {
  for (int i = 0; i < 4; i++)
    if (b.x[i] < xmin || b.x[i] > xmax || b.y[i] < ymin || b.y[i] > ymax) return false;
  return true;
}
// Box2d::overlapsWith: SAT over this box's four edge normals only, with the reference's
// "containsOther" bookkeeping (true only if no axis separates by more than zero)
__device__ bool box_overlaps(const Box2& a, const Box2& o, double gap) {
  bool contains = true;
  for (int i = 0; i < 4; i++) {
    const int j = (i + 1) % 4;
    double px = -(a.y[j] - a.y[i]), py = a.x[j] - a.x[i];
    const double len = sqrt(px * px + py * py);
    px /= len; py /= len;
    double min1 = a.x[0] * px + a.y[0] * py, max1 = min1;
    double min2 = o.x[0] * px + o.y[0] * py, max2 = min2;
    for (int k = 1; k < 4; k++) {
      const double p1 = a.x[k] * px + a.y[k] * py;
      const double p2 = o.x[k] * px + o.y[k] * py;
      if (p1 < min1) min1 = p1;
      if (p1 > max1) max1 = p1;
      if (p2 < min2) min2 = p2;
      if (p2 > max2) max2 = p2;
    }
    if (max1 + gap < min2 || max2 + gap < min1) return false;
    if (max1 < min2 || max2 < min1) contains = false;
  }
  return contains;
}
// "Task object i" xyz bounding box (objecthandler.cpp:91-110): full extents of the
// synthetic object's geom (the MJCF numerics are unavailable)
__device__ __host__ inline void object_bbox(const gm_object& o, double* xyz) {
  if (o.type == GM_GEOM_BOX) { xyz[0] = 2 * o.size[0]; xyz[1] = 2 * o.size[1]; xyz[2] = 2 * o.size[2]; }
  else if (o.type == GM_GEOM_CYLINDER) { xyz[0] = xyz[1] = 2 * o.size[0]; xyz[2] = 2 * o.size[1]; }
  else { xyz[0] = xyz[1] = xyz[2] = 2 * o.size[0]; }
}
// returns 1 and spawns on success; 0 when no candidate pose is free
// pxy / prot: the shuffled grids' work buffers (GM_SPAWN_MAX_XY / GM_SPAWN_MAX_ROT entries):
// LDS in the reset kernel (its one working lane would otherwise wait on a scratch round
// trip per swap), private arrays in the thread-per-env kernel
__device__ __forceinline__ int spawn_into_scene_dev(GmEnvHot& s, const gm_model* __restrict__ m,
                                                    const GmTopo* __restrict__ T, const gm_object* __restrict__ objs,
                                                    int n_objects, const gm_spawn_params& p, int index,
                                                    uint16_t* pxy, uint16_t* prot) {
  const int num_x = (int)(((2 * p.xrange) / p.xy_increment) + 1);
  const int num_y = (int)(((2 * p.yrange) / p.xy_increment) + 1);
  const int num_r = (int)(((2 * p.rotrange) / p.rot_increment) + 1);
  const int nxy = num_x * num_y;
  if (num_x < 1 || num_y < 1 || num_r < 1 || nxy > GM_SPAWN_MAX_XY || num_r > GM_SPAWN_MAX_ROT) return 0;
  for (int i = 0; i < nxy; i++) pxy[i] = (uint16_t)i;
  for (int i = 0; i < num_r; i++) prot[i] = (uint16_t)i;
  {
    uint32_t rng = s.rng;   // in a register through both shuffles, not the env's HBM record
    if (nxy > 1) shuffle_minstd(pxy, nxy, rng);
    if (num_r > 1) shuffle_minstd(prot, num_r, rng);
    s.rng = rng;
  }
  // object footprint
  int oi = index;
  if (oi < 0 || oi >= n_objects) oi = 0;
  double bb[3];
  object_bbox(objs[oi], bb);
  // initial fingertip boxes: Env::reset (mjclass.h:895-904) from
  // get_finger_hook_locations (myfunctions.cpp:3717-3761), straight fingers at the target
  Box2 tips[3];
  {
    const double PI_23 = M_PI * (2.0 / 3.0);
    const double angles[3] = {0.0, PI_23, 2 * PI_23};
    const double fing_x = s.end.x;
    const double hook_th = m->hook_angle_degrees * (M_PI / 180.000);
    for (int i = 0; i < 3; i++) {
      const double hook_x = 0.5 * m->hook_length * sin(hook_th);
      const double x = -(fing_x - hook_x) * sin(angles[i]) + s.base[0];
      const double y = -(fing_x - hook_x) * cos(angles[i]) + s.base[1];
      box_init_centre(tips[i], x, y, m->finger_width, m->hook_length);
      box_rotate(tips[i], -angles[i]);
    }
  }
  const int total = nxy > num_r ? nxy : num_r;
  int ixy = -1, ir = -1;
  for (int i = 0; i < total; i++) {
    ixy += 1; ir += 1;
    if (ixy >= nxy) ixy = 0;
    if (ir >= num_r) ir = 0;
    const int kx = pxy[ixy] / num_y, ky = pxy[ixy] % num_y;
    const double px = num_x > 1 ? -p.xrange + kx * p.xy_increment + p.x : p.x;
    const double py = num_y > 1 ? -p.yrange + ky * p.xy_increment + p.y : p.y;
    const double pr = num_r > 1 ? -p.rotrange + prot[ir] * p.rot_increment + p.zrot : p.zrot;
    Box2 ob;
    box_init_centre(ob, px, py, bb[0], bb[1]);
    box_rotate(ob, pr);
    if (!box_inbounds(ob, p.xmin, p.ymin, p.xmax, p.ymax)) continue;
    bool good = true;
    for (int f = 0; f < 3 && good; f++)
      if (box_overlaps(ob, tips[f], p.smallest_gap)) good = false;
    if (!good) continue;
    spawn_object(s, T, objs, n_objects, gm_spawn{index, px, py, pr});
    return 1;
  }
  return 0;
}

#ifndef GM_CAL_TU   // env-step translation unit only
extern "C" __global__ void gm_spawn_into_scene_kernel(GmEnvState* __restrict__ states, const gm_model* __restrict__ m,
                                                      const GmTopo* __restrict__ T, const gm_object* __restrict__ objs,
                                                      int n_objects, const uint8_t* __restrict__ mask,
                                                      const gm_spawn_params* __restrict__ params, int n_params,
                                                      uint8_t* __restrict__ ok, int n_envs) {
  const int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  if (mask && !mask[env]) { if (ok) ok[env] = 0; return; }
  const gm_spawn_params p = params[n_params == 1 ? 0 : env];
  uint16_t pxy[GM_SPAWN_MAX_XY], prot[GM_SPAWN_MAX_ROT];
  const int r = spawn_into_scene_dev(states[env], m, T, objs, n_objects, p, p.index, pxy, prot);
  if (ok) ok[env] = (uint8_t)r;
}
#endif

#ifndef GM_CAL_TU   // env-step translation unit only
extern "C" __global__ void gm_autoreset_mask_kernel(const GmEnvState* __restrict__ states,
                                                    const uint8_t* __restrict__ done, int max_steps,
                                                    uint8_t* __restrict__ mask, float* __restrict__ returns,
                                                    gm_episode_end* __restrict__ episodes, int n_envs) {
  int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  const GmEnvState& s = states[env];
  uint8_t r = (done[env] || (max_steps > 0 && s.num_action_steps >= max_steps)) ? 1 : 0;
  mask[env] = r;
  const float ret = r ? s.cumulative_reward : __builtin_nanf("");
  if (returns) returns[env] = ret;
  if (episodes) {
    // successful_grasp (mjclass.cpp:1295-1322): this env-step's event value, which
    // update_events leaves in bev_last
    gm_episode_end e;
    e.ret = ret;
    e.length = r ? s.num_action_steps : 0;
    e.success = (r && s.bev_last[GM_EV_successful_grasp]) ? 1 : 0;
    e.pad[0] = e.pad[1] = e.pad[2] = 0;
    episodes[env] = e;
  }
}
#endif

// MjClass::reset (mjclass.cpp:434-486) -> luke::reset / calibrate_reset (non-first call),
// configure_settings RNG draws, random_base_Z_movement, then spawn_object.
#ifndef GM_CAL_TU   // env-step translation unit only
// The whole reset of one env by one wave on an LDS image `s` of its hot state (rec: its HBM
// record, whose sensor windows are cleared in place): the image is cleared with coalesced
// 16-byte stores, then lane 0 runs the reference's serial reset (RNG draws, spawn search --
// pxy / prot: LDS work buffers of GM_SPAWN_MAX_XY / GM_SPAWN_MAX_ROT entries).  What survives
// a reset (the per-env RNG stream, the function-static stepper flags -- a reference quirk --,
// the episode counter, the solver diagnostics) comes in as arguments, read by the caller
// before the clear.  Used by gm_reset_kernel and by the rollout's in-kernel auto-reset.
__device__ __noinline__ void reset_env(GmEnvHot& s, GmEnvState& rec, GmResetKeep keep, const gm_model* __restrict__ m,
                                       const gm_config* __restrict__ C, const GmTopo* __restrict__ T,
                                       const double* __restrict__ eq_qpos, const gm_spawn* __restrict__ spawn,
                                       const gm_object* __restrict__ objs, int n_objects, int env,
                                       const gm_spawn_params* __restrict__ scene, int scene_tries, GmSpawnRand sr,
                                       uint16_t* sh_pxy, uint16_t* sh_prot, int lane) {
  {
    static_assert(sizeof(GmEnvState) % 16 == 0 && sizeof(GmEnvHot) % 16 == 0, "records move in 16-byte words");
    uint4* hw = reinterpret_cast<uint4*>(&s);
    for (int i = lane; i < GM_HOT_WORDS / 4; i += 64) hw[i] = make_uint4(0u, 0u, 0u, 0u);
    uint4* w = reinterpret_cast<uint4*>(&rec);
    for (int i = GM_HOT_WORDS / 4 + lane; i < GM_STATE_WORDS / 4; i += 64) w[i] = make_uint4(0u, 0u, 0u, 0u);
  }
  GM_ENV_SYNC();
  if (lane == 0) {   // the reference's serial reset on lane 0
    const int32_t episode = keep.episode;
    s.rng = keep.rng; s.old_x = keep.ox; s.old_y = keep.oy; s.old_z = keep.oz;
    s.episode = episode;
    s.newton_caps = keep.newton_caps;
    g_reset(s.end); g_reset(s.next);
    for (int k = 0; k < GM_MAX_QPOS; k++) s.qpos[k] = m->qpos0[k];
    s.time = 0; s.last_step_time = 0;
    s.dt = m->timestep;
    for (int d = 0; d < T->nv; d++) {
      bool motor = (d == m->dof_base || d == m->dof_palm);
      for (int f = 0; f < 3; f++) motor = motor || d == m->dof_pris[f] || d == m->dof_rev[f];
      if (motor) s.qpos[d] = eq_qpos[d];
    }
    for (int k = 0; k < T->nlock; k++) { s.lock_active[k] = 1; s.lock_q[k] = m->qpos0[m->lock_dof[k]]; }
    for (int st = 0; st < GM_NSTREAM; st++) s.ring_i[st] = -1;
    // apply_noise_params: mean draws, SS order then the state sensors again
    {
      const gm_settings& st = C->s;
      const gm_sensor* ss[SL_N] = {&st.motor_state_sensor, &st.base_state_sensor_Z, &st.base_state_sensor_XY,
                                   &st.base_state_sensor_yaw, &st.bending_gauge, &st.axial_gauge, &st.palm_sensor,
                                   &st.wrist_sensor_XY, &st.wrist_sensor_Z, &st.cartesian_contacts_XYZ};
      uint32_t g = s.rng;   // the draws below run on a register copy of the stream
      for (int k = 0; k < SL_N; k++)
        for (int i = 0; i < 3; i++) {
          s.rand_mu[k][i] = ss[k]->noise_mu * (2 * unif01(g) - 1);
        }
      int order[5] = {SL_MOTOR, SL_BASEXY, SL_BASEZ, SL_YAW, SL_CART};
      for (int k = 0; k < 5; k++)
        for (int i = 0; i < 3; i++) {
          s.rand_mu[order[k]][i] = ss[order[k]]->noise_mu * (2 * unif01(g) - 1);
        }
      s.rng = g;
    }
    {
      double size = C->s.base_position_noise;
      uint32_t g = s.rng;
      double u = canon_d(g);
      s.rng = g;
      double z = u * (size - (-size)) + (-size);
      s.base[2] = z;
      if (s.base[2] > C->base_max[2]) s.base[2] = C->base_max[2];
      if (s.base[2] < C->base_min[2]) s.base[2] = C->base_min[2];
      s.qpos[m->dof_base] = s.base[2] + eq_qpos[m->dof_base];
    }
    gm_spawn sp = spawn ? spawn[env] : gm_spawn{0, 0.0, 0.0, 0.0};
    if (sr.enable && !spawn) {
      // MjEnv._spawn_object's generator draws: object index, then the "old method" pose
      // (integer mm offsets, one of {0, 60, 120} deg plus integer-degree noise)
      const int64_t gid = sr.env_offset + env;
      const int nm = sr.position_noise_mm, nd = sr.rotation_noise_deg;
      sp.object_index = gm_spawn_int(sr.seed, gid, episode, 0, 0, n_objects - 1);
      sp.x = gm_spawn_int(sr.seed, gid, episode, 1, -nm, nm) * 1e-3;
      sp.y = gm_spawn_int(sr.seed, gid, episode, 2, -nm, nm) * 1e-3;
      const int noise_deg = gm_spawn_int(sr.seed, gid, episode, 3, -nd, nd);
      const int opt = gm_spawn_int(sr.seed, gid, episode, 4, 0, 2);
      sp.zrot = (60 * opt + noise_deg) * (M_PI / 180.0);
    }
    bool placed = false;
    if (scene) {
      // MjEnv._spawn_object (MjEnv.py:1177-1267): spawn_into_scene up to scene_tries times,
      // then the "old method" pose from the spawn table
      for (int t = 0; t < scene_tries && !placed; t++)
        placed = spawn_into_scene_dev(s, m, T, objs, n_objects, *scene, sp.object_index, sh_pxy, sh_prot);
    }
    if (!placed) spawn_object(s, T, objs, n_objects, sp);
    s.done = 0;
    s.reward = 0;
  }
  GM_ENV_SYNC();
}

// One wave per env (grid = n_envs workgroups of 64; unmasked envs exit at once): the new
// record's hot part is built in LDS (lane 0's serial reset reads back what it wrote many
// times over) and stored to HBM in one coalesced sweep; the sensor windows are cleared in
// place.
extern "C" __global__ __launch_bounds__(64) void gm_reset_kernel(
    GmEnvState* __restrict__ states, const gm_model* __restrict__ m, const gm_config* __restrict__ C,
    const GmTopo* __restrict__ T, const double* __restrict__ eq_qpos, const uint8_t* __restrict__ mask,
    const gm_spawn* __restrict__ spawn, const gm_object* __restrict__ objs, int n_objects, int n_envs,
    const gm_spawn_params* __restrict__ scene, int scene_tries, float* __restrict__ obs, GmSpawnRand sr) {
  __shared__ uint16_t sh_pxy[GM_SPAWN_MAX_XY], sh_prot[GM_SPAWN_MAX_ROT];   // spawn grid shuffles
  const int env = blockIdx.x;
  if (env >= n_envs) return;
  if (mask && !mask[env]) return;
  __shared__ uint4 hot_words[GM_HOT_WORDS / 4];
  GmEnvHot& s = *reinterpret_cast<GmEnvHot*>(hot_words);
  GmEnvState& rec = states[env];
  // keep the per-env RNG stream and the function-static stepper flags (quirk)
  const GmResetKeep keep{rec.rng, rec.old_x, rec.old_y, rec.old_z, rec.episode + 1, rec.newton_caps};
  reset_env(s, rec, keep, m, C, T, eq_qpos, spawn, objs, n_objects, env, scene, scene_tries, sr, sh_pxy, sh_prot,
            (int)threadIdx.x);
  // MjEnv.reset returns _next_observation() of the fresh episode (MjEnv.py:2222-2263):
  // the observation buffer holds the reset env's sensor windows, not the last episode's;
  // sampled one stream per lane as in the env-step epilogue
  {
    uint4* w = reinterpret_cast<uint4*>(&rec);
    for (int i = threadIdx.x; i < GM_HOT_WORDS / 4; i += 64) w[i] = hot_words[i];
  }
  if (obs) get_obs_lanes(s, rec.ring, C, obs + (size_t)env * C->n_obs, threadIdx.x);
}
#endif

// settle initialisation (keyframe, targets home, locks off, flags true) for env 0
#ifndef GM_CAL_TU   // env-step translation unit only
extern "C" __global__ void gm_settle_init_kernel(GmEnvState* __restrict__ states, const gm_model* __restrict__ m,
                                                 const GmTopo* __restrict__ T, const gm_object* __restrict__ objs) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  GmEnvState& s = states[0];
  uint32_t* w = reinterpret_cast<uint32_t*>(&s);
  for (int i = 0; i < GM_STATE_WORDS; i++) w[i] = 0;
  g_reset(s.end); g_reset(s.next);
  for (int k = 0; k < GM_MAX_QPOS; k++) s.qpos[k] = m->qpos0[k];
  s.dt = m->timestep;
  s.old_x = s.old_y = s.old_z = 1;
  for (int st = 0; st < GM_NSTREAM; st++) s.ring_i[st] = -1;
  const gm_object& o = objs[0];
  s.obj_type = o.type;
  s.obj_size[0] = o.size[0]; s.obj_size[1] = o.size[1]; s.obj_size[2] = o.size[2];
  s.obj_mass = o.mass;
  s.obj_friction = o.friction;
  if (o.type == GM_GEOM_BOX) {
    double a = 2 * o.size[0], bb = 2 * o.size[1], c = 2 * o.size[2];
    s.obj_inertia[0] = (o.mass * (bb * bb + c * c) / 12); s.obj_inertia[1] = (o.mass * (a * a + c * c) / 12);
    s.obj_inertia[2] = (o.mass * (a * a + bb * bb) / 12);
    s.obj_rbound = sqrt(o.size[0] * o.size[0] + o.size[1] * o.size[1] + o.size[2] * o.size[2]);
  } else if (o.type == GM_GEOM_CYLINDER) {
    double r = o.size[0], hh = 2 * o.size[1];
    s.obj_inertia[0] = s.obj_inertia[1] = (o.mass * (3 * r * r + hh * hh) / 12);
    s.obj_inertia[2] = (o.mass * r * r / 2);
    s.obj_rbound = sqrt(o.size[0] * o.size[0] + o.size[1] * o.size[1]);
  } else {
    double r = o.size[0];
    s.obj_inertia[0] = s.obj_inertia[1] = s.obj_inertia[2] = (2 * o.mass * r * r / 5);
    s.obj_rbound = r;
  }
  s.obj_invw[0] = 1.0 / o.mass;
  s.obj_invw[1] = ((1.0 / s.obj_inertia[0] + 1.0 / s.obj_inertia[1]) + 1.0 / s.obj_inertia[2]) / 3.0;
}
#endif

// per-env initialisation after the settle: RNG seeds and settled stepper flags
#ifndef GM_CAL_TU   // env-step translation unit only
extern "C" __global__ void gm_init_envs_kernel(GmEnvState* __restrict__ states, uint32_t base_seed, long long env_offset,
                                               int n_envs, double dt) {
  int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  GmEnvState& s = states[env];
  s.dt = dt;
  uint64_t seed = ((uint64_t)base_seed + (uint64_t)(env_offset + env) * 1000003ull) % 2147483647ull;
  s.rng = seed == 0 ? 1u : (uint32_t)seed;
  s.old_x = s.old_y = s.old_z = 0;
}
#endif

// spawn only (MjClass::spawn_object after MjClass::reset, MjEnv.py:1212-1267)
#ifndef GM_CAL_TU   // env-step translation unit only
// MjClass::set_motor_target -> Gripper::set_xyz_m on the env's target (thread per env)
extern "C" __global__ void gm_motor_target_kernel(GmEnvState* __restrict__ states, const uint8_t* __restrict__ mask,
                                                  const double* __restrict__ xyz, int per_env,
                                                  uint8_t* __restrict__ in_limits, int n_envs) {
  int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  if (mask && !mask[env]) return;
  const double* t = xyz + (per_env ? 3 * env : 0);
  in_limits[env] = (uint8_t)g_set_xyz_m(states[env].end, t[0], t[1], t[2]);
}
// the latest sim_sensors_SI_ readings (finger 1..3 gauges, palm, wrist Z), thread per env
extern "C" __global__ void gm_sensor_si_kernel(const GmEnvState* __restrict__ states, float* __restrict__ out, int n_envs) {
  int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  const GmEnvState& s = states[env];
  RingRef R = const_cast<RingRef>(s.ring);
  const int st[5] = {ST_SI_GAUGE, ST_SI_GAUGE + 1, ST_SI_GAUGE + 2, ST_SI_PALM, ST_SI_WZ};
  for (int k = 0; k < 5; k++) out[5 * env + k] = ring_latest(s, R, st[k]);
}
extern "C" __global__ void gm_spawn_kernel(GmEnvState* __restrict__ states, const GmTopo* __restrict__ T,
                                           const uint8_t* __restrict__ mask, const gm_spawn* __restrict__ spawn,
                                           const gm_object* __restrict__ objs, int n_objects, int n_envs) {
  int env = blockIdx.x * blockDim.x + threadIdx.x;
  if (env >= n_envs) return;
  if (mask && !mask[env]) return;
  spawn_object(states[env], T, objs, n_objects, spawn[env]);
}
#endif
