// gm_state.h -- per-env persistent state in HBM and the device model view.
//
// One EnvState per env, array-of-structs: the fused step kernel runs one
// 64-lane workgroup per env and moves the whole struct HBM<->LDS with fully
// coalesced 4-byte-per-lane sweeps at launch entry/exit.  Plain C as well as C++: the
// CPU oracle (oracle/oracle.c, test infrastructure) imports / exports this struct so
// parity tests can hand the device's fp64 state to it verbatim.  Everything an
// MjClass instance carries between action_step() calls (mjclass.h:1554-1833,
// myfunctions.cpp:464-473 globals, the function-static flags the reference
// keeps across resets) lives here.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include "gripper_mi355x.h"

#define GM_NSTREAM 37          // sensor ring streams, see stream ids below
// stream ids (observation windows, then SI windows)
enum {
  ST_GAUGE = 0,      // 3
  ST_AXIAL = 3,      // 3
  ST_PALM = 6,
  ST_WX = 7,
  ST_WY = 8,
  ST_WZ = 9,
  ST_MOTOR = 10,     // 3
  ST_BASE = 13,      // 3 (x, y, z)
  ST_YAW = 16,
  ST_CART = 17,      // 12
  ST_SI_GAUGE = 29,  // 3
  ST_SI_AXIAL = 32,  // 3
  ST_SI_PALM = 35,
  ST_SI_WZ = 36
};
// sensor slots in settings (SS) order, used for last_read_time / rand_mu
enum { SL_MOTOR = 0, SL_BASEZ, SL_BASEXY, SL_YAW, SL_BEND, SL_AXIAL, SL_PALM, SL_WRISTXY, SL_WRISTZ, SL_CART, SL_N };

typedef struct GmGrip GmGrip;
typedef struct GmEnvHot GmEnvHot;
typedef struct GmEnvState GmEnvState;
typedef struct GmTopo GmTopo;

struct GmGrip {            // luke::Gripper (gripper.h:11-198)
  double x, y, z, th;
  int32_t sx, sy, sz, pad;
};

// Everything but the sensor windows: the part of the state the step kernel stages into
// LDS (GmEnvHot is the leading part of GmEnvState, field for field).
#define GM_ENV_HOT_FIELDS                                                              \
  /* ---- doubles first (8-byte aligned) ---- */                                       \
  double time;                                                                         \
  double last_step_time;                                                               \
  GmGrip end, next;                                                                    \
  double base[6];                                                                      \
  double last_read[SL_N];                                                              \
  double qpos[GM_MAX_QPOS];      /* fp64 like MuJoCo's mjtNum (reference physics type) */ \
  double qvel[GM_MAX_DOF];                                                             \
  double qacc_warm[GM_MAX_DOF];  /* mjData qacc_warmstart: the last substep's qacc */   \
  double lock_q[GM_MAX_LOCK];                                                          \
  double start_qpos[7];                                                                \
  double obj_size[3];                                                                  \
  double obj_mass, obj_inertia[3], obj_friction, obj_rbound, obj_rest_z;               \
  double obj_invw[2];            /* the live object's body_invweight0 (trans, rot) */   \
  double dt;                     /* this env's timestep (per env for calibration) */   \
  double tip_force;              /* calibration tip load, N; 0 = off */                \
  /* ---- floats ---- */                                                               \
  float rand_mu[SL_N][3];                                                              \
  float lev_value[GM_N_LINEAR];                                                        \
  float lev_last[GM_N_LINEAR];                                                         \
  float cumulative_reward;                                                             \
  float grp_peak_lateral;                                                              \
  float reward;                                                                        \
  /* ---- ints ---- */                                                                 \
  int32_t ring_i[GM_NSTREAM];                                                          \
  int32_t bev_value[GM_N_BINARY];                                                      \
  int32_t bev_last[GM_N_BINARY];                                                       \
  int32_t bev_row[GM_N_BINARY];                                                        \
  int32_t bev_abs[GM_N_BINARY];                                                        \
  int32_t lev_row[GM_N_LINEAR];                                                        \
  int32_t lev_abs[GM_N_LINEAR];                                                        \
  int32_t lock_active[GM_MAX_LOCK];                                                    \
  int32_t old_x, old_y, old_z;                                                         \
  int32_t num_action_steps;                                                            \
  int32_t termination_signal_sent;                                                     \
  int32_t extra_substeps;        /* termination lift substeps pending (2 * S) */       \
  int32_t obj_type;                                                                    \
  int32_t obj_index;                                                                   \
  int32_t done;                                                                        \
  int32_t overflow;                                                                    \
  uint32_t rng;                                                                        \
  int32_t cal_steps;             /* calibration launch: substeps to run */             \
  int32_t badqacc;               /* mjWARN_BADQACC: non-finite or |qacc| > 1e10 seen */ \
  int32_t episode;               /* resets since gm_create (keys the spawn draws) */   \
  int32_t newton_caps;           /* constraint solves that hit GM_NEWTON_MAXIT / _MAXLS */ \
  int32_t pad_end[GM_HOT_PAD];

// pad words so the hot part is a multiple of 16 B (see GM_STATE_WORDS below)
#define GM_HOT_PAD 1
struct GmEnvHot { GM_ENV_HOT_FIELDS };

// The sensor windows (SlidingWindow, mjclass.h:155-241) are the state's tail: GM_RING
// readings per stream, read and written in place in HBM by the kernel's lane-0 sensor
// code (once per sensor reading / observation), never staged into LDS.
#ifdef __cplusplus
struct GmEnvState : GmEnvHot {
  float ring[GM_NSTREAM][GM_RING];
};
#else
struct GmEnvState {
  GM_ENV_HOT_FIELDS
  float ring[GM_NSTREAM][GM_RING];
};
#endif

// word counts for HBM<->LDS sweeps (the hot part) and whole-state clears
#define GM_HOT_WORDS ((int)(sizeof(GmEnvHot) / 4))
#define GM_STATE_WORDS ((int)(sizeof(GmEnvState) / 4))
// multiples of 16 B: the LDS image (SharedT) places its double arrays right after the
// hot state, and 16-byte alignment keeps their paired accesses as single ds_*_b128 ops
// (an 8-byte shift measured 5-15% slower across every phase)
#ifdef __cplusplus
static_assert(sizeof(GmEnvHot) % 16 == 0, "GmEnvHot must be 16-byte padded");
static_assert(sizeof(GmEnvState) % 16 == 0, "GmEnvState must be 16-byte padded");
static_assert(sizeof(GmEnvState) == sizeof(GmEnvHot) + sizeof(float) * GM_NSTREAM * GM_RING, "rings follow the hot part");
#else
_Static_assert(sizeof(GmEnvHot) % 16 == 0, "GmEnvHot must be 16-byte padded");
_Static_assert(sizeof(GmEnvState) % 16 == 0, "GmEnvState must be 16-byte padded");
_Static_assert(offsetof(GmEnvState, ring) == sizeof(GmEnvHot), "rings follow the hot part");
#endif

// MjEnv._spawn_object's Python-side draws (MjEnv.py:1177-1267: object index, and the
// "old method" pose when spawn_into_scene fails) made on the device from a counter-based
// hash of (seed, global env id, episode, draw) -- splitmix64, identical on the host
// (gmx.spawn_draws) -- so they do not depend on sharding and leave the reference's C++
// RNG stream (GmEnvState::rng) untouched.
typedef struct GmSpawnRand {
  uint64_t seed;
  int32_t enable;
  int32_t position_noise_mm;     // object_position_noise_mm (MjEnv default 10)
  int32_t rotation_noise_deg;    // object_rotation_noise_deg (MjEnv default 5)
  int32_t pad;
  int64_t env_offset;            // global id of env 0 of this context
} GmSpawnRand;

static inline
#ifdef __HIPCC__
__host__ __device__
#endif
uint64_t gm_splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
// uniform integer in [lo, hi] from draw k of (seed, gid, episode)
static inline
#ifdef __HIPCC__
__host__ __device__
#endif
int32_t gm_spawn_int(uint64_t seed, int64_t gid, int32_t episode, int k, int32_t lo, int32_t hi) {
  const uint64_t h = gm_splitmix64(seed + (uint64_t)gid * 0xD1B54A32D192ED03ull +
                                   (uint64_t)(uint32_t)episode * 0x8CB92BA72F3D8DD7ull +
                                   (uint64_t)k * 0x9E3779B97F4A7C15ull);
  const uint64_t span = (uint64_t)(hi - lo + 1);
  return lo + (int32_t)(((h >> 32) * span) >> 32);
}

// scripted grasp mix (gm_scripted_actions; host mirror gmx.GraspScript; the CPU oracle's
// bench sample uses it too): action fraction for action index i of kind `kind` at episode
// step k
static inline
#ifdef __HIPCC__
__host__ __device__
#endif
float gm_script_fraction(uint64_t seed, int64_t gid, int32_t ep, int32_t k, int i, int kind,
                                                    float jitter) {
  const int close_n = gm_spawn_int(seed, gid, ep, 16, 34, 45);
  const int tilt_n = gm_spawn_int(seed, gid, ep, 17, 0, 25);
  const float tilt_dir = gm_spawn_int(seed, gid, ep, 18, 0, 4) < 4 ? -1.0f : 1.0f;
  const int palm_n = gm_spawn_int(seed, gid, ep, 19, 0, 15);
  const int t1 = close_n, t2 = t1 + tilt_n, t3 = t2 + palm_n;
  float a = 0.0f;
  if (kind == GM_ACT_gripper_prismatic_X && k < t1) a = 1.0f;
  if (kind == GM_ACT_gripper_revolute_Y && k >= t1 && k < t2) a = tilt_dir;
  if (kind == GM_ACT_gripper_Z && k >= t2 && k < t3) a = 1.0f;
  if (kind == GM_ACT_base_Z && k >= t3) a = -1.0f;
  if (jitter > 0.0f) {
    const int u = gm_spawn_int(seed, gid, ep, 32 + 8 * k + i, 0, 1 << 20);
    a += jitter * ((float)u * (2.0f / (float)(1 << 20)) - 1.0f);
  }
  return a > 1.0f ? 1.0f : (a < -1.0f ? -1.0f : a);
}

// uniform random action fraction in [-1, 1) for action index i of env-step k (the rollout
// driver's random mode, gm_random_actions; host mirror gmx.random_fractions): 24 bits of a
// counter-based hash of (seed, global env id, episode, k, i), so draws do not depend on
// sharding or launch boundaries
static inline
#ifdef __HIPCC__
__host__ __device__
#endif
float gm_random_fraction(uint64_t seed, int64_t gid, int32_t ep, int32_t k, int i) {
  const uint64_t h = gm_splitmix64(seed * 0xA24BAED4963EE407ull + (uint64_t)gid * 0xD1B54A32D192ED03ull +
                                   (uint64_t)(uint32_t)ep * 0x8CB92BA72F3D8DD7ull +
                                   (uint64_t)(uint32_t)k * 0x9E3779B97F4A7C15ull + (uint64_t)i * 0xF1357AEA2E62A9C5ull);
  return (float)(h >> 40) * (2.0f / 16777216.0f) - 1.0f;
}

// Grasp-lift-hold program (rollout action modes 3 / 4, gm_program_actions; the CPU oracle's
// or_program_actions; tests/grasp_program.py drives the oracle with it): a closed-loop
// driver that takes an episode through the reference's whole success chain
// (mjclass.cpp:1148-1210, 1295-1322: lifted -> lifted_to_height -> target_height ->
// object_stable -> stable_height -> successful_grasp).  Stateless: the phase is read off
// the env's targets and its latest SI readings each env-step, so it resumes anywhere:
//   close   prismatic X until a gauge reads GM_PROG_G_TOUCH or x reaches GM_PROG_X_CLOSE;
//   squeeze tilt the tips inward (y below x) until a gauge reads GM_PROG_G_SQUEEZE or y hits
//           its limit -- the fixed hooks meet the object under its widest section;
//   lift    the base up to GM_PROG_BASE_LIFT (gripper_z_height > gripper_target_height);
//   palm    lower the palm onto the object (full speed until 1 mm from its top, then in
//           proportion to the gap), then hold the palm reading near GM_PROG_PALM_HOLD
//           (stable_palm_force band [1, 4] N) -- object_stable and stable_height fire.
// The palm's approach uses the object's pose and size (a scripted test driver may, a
// policy could not).  Fractions are for the canonical action signs (close = -x, inward =
// -th, palm down = +z, lift = -base z), mapped through each action's sign; arithmetic is
// adds, subtracts and divides only (no contractible multiply-add), so the device and the
// oracle decide on the same bits.
#define GM_PROG_X_CLOSE 58.5e-3
#define GM_PROG_Y_MIN 49.5e-3
#define GM_PROG_Z_HOME 4.8768e-3        /* luke::Gripper::z_home (gripper.h:50) */
#define GM_PROG_BASE_LIFT (-24e-3)
#define GM_PROG_G_TOUCH 0.2f
#define GM_PROG_G_SQUEEZE 1.5f
#define GM_PROG_PALM_ON 1.0f
#define GM_PROG_PALM_HOLD 2.5f
typedef struct gm_program_in {
  double x, y, z;              // gripper target (luke::Gripper end: x, y, palm z)
  double base_z;               // base target z (+ve down)
  double q_base, q_palm;       // base and palm joint positions
  double obj_z, obj_top;       // object centre height and its centre-to-top extent
  double z_root, palm_drop;    // base origin height at q = 0; palm face below it at q = 0
  float g_max, palm;           // largest finger gauge and palm sensor: latest SI readings, N
} gm_program_in;
static inline
#ifdef __HIPCC__
__host__ __device__
#endif
float gm_program_fraction(const gm_program_in* in, int kind, double value, int sign) {
  const float p = in->palm < 0.0f ? -in->palm : in->palm;
  const int inward = (in->y - in->x) < -1e-9;
  int want;
  float c;
  if (in->z > GM_PROG_Z_HOME + 0.5e-3 || in->base_z <= GM_PROG_BASE_LIFT + 1e-6) {
    want = GM_ACT_gripper_Z;
    if (p >= GM_PROG_PALM_ON) {
      c = (GM_PROG_PALM_HOLD - p) / 5.0f;
      c = c > 0.25f ? 0.25f : (c < -0.25f ? -0.25f : c);
    } else {
      const double face = ((in->z_root - in->q_base) - in->palm_drop) - in->q_palm;
      const double gap = face - (in->obj_z + in->obj_top);
      double f = (gap + 1e-3) / value;
      f = f > 1.0 ? 1.0 : (f < 0.05 ? 0.05 : f);
      c = (float)f;
    }
  } else if (in->base_z < -1e-6 || (inward && (in->g_max >= GM_PROG_G_SQUEEZE || in->y <= GM_PROG_Y_MIN))) {
    want = GM_ACT_base_Z;
    c = 1.0f;
  } else if (inward || in->g_max >= GM_PROG_G_TOUCH || in->x <= GM_PROG_X_CLOSE) {
    want = GM_ACT_gripper_revolute_Y;
    c = 1.0f;
  } else {
    want = GM_ACT_gripper_prismatic_X;
    c = 1.0f;
  }
  if (kind != want) return 0.0f;
  // canonical direction -> fraction: an action moves its target by sign * value * fraction
  const float s = sign < 0 ? -1.0f : 1.0f;
  return kind == GM_ACT_gripper_Z ? c * s : -c * s;
}
// the live object's centre-to-top extent (MuJoCo sizes: sphere r; cylinder r, half height;
// box half sizes)
static inline
#ifdef __HIPCC__
__host__ __device__
#endif
double gm_program_obj_top(int type, const double* size) {
  return type == GM_GEOM_SPHERE ? size[0] : (type == GM_GEOM_CYLINDER ? size[1] : size[2]);
}
// rollout action mode 4 (the benchmark mix): the program drives 1 episode in 4 of each env
// (draw 21 of the episode's counter-based hash), the scripted grasp mix the rest
static inline
#ifdef __HIPCC__
__host__ __device__
#endif
int gm_program_episode(uint64_t seed, int64_t gid, int32_t ep) {
  return gm_spawn_int(seed, gid, ep, 21, 0, 3) == 0;
}

// Topology derived from gm_model on the host (the canonical gripper tree):
// dof/body of chain position p in finger chain f is first + p - 1 (p >= 1),
// position 0 of every finger / palm chain is the base dof.
struct GmTopo {
  int32_t N, CL, nbody, nv, nq, ngeom, npair, nlock;
  int32_t body_base, dof_base;
  int32_t body_f0[3], dof_f0[3];       // first chain body / dof (intermediate / prismatic)
  int32_t body_palm, dof_palm, body_obj, dof_obj, qadr_obj, geom_obj;
  int32_t body_finger[3];              // "finger_f" bodies (local force frames)
  int32_t geom_group[GM_MAX_GEOM];     // 0..2 finger, 3 palm, 5 object, -1 world
  int32_t geom_cpos[GM_MAX_GEOM];      // chain position of the geom's body (fingers / palm)
  int32_t body_group[GM_MAX_BODY];
  int32_t body_cpos[GM_MAX_BODY];
  // scan lanes: finger f's chain position p (1..CL) sits on lane 16 f + p, so a chain
  // lies inside one 16-lane DPP row; row 3 holds the base (48), palm (49, position 1)
  // and object (50).  -1: no body on that lane.
  int32_t lane_body[64];
  int32_t lane_base;
  // per-dof constants folded on the host (one load level in the substep)
  int32_t dof_body[GM_MAX_DOF];
  int32_t dof_grp[GM_MAX_DOF];         // 0..2 finger, 3 palm, 4 base, 5 object
  int32_t dof_p[GM_MAX_DOF];           // chain position (object: 0..5)
  int32_t dof_target[GM_MAX_DOF];      // PD target: 0 none, 1 next.x, 2 next.th, 3 next.z, 4 base z
  double dof_add[GM_MAX_DOF];          // armature + h (damping + kd) [+ h^2 kp]; springs are explicit
  // the same addition's parts, formed per env from its own timestep h (calibration)
  double dof_arm[GM_MAX_DOF], dof_dsum[GM_MAX_DOF], dof_ksum[GM_MAX_DOF];
  double dof_stiff[GM_MAX_DOF];        // 0 for the free joint
  double dof_damp[GM_MAX_DOF];
  double dof_kp[GM_MAX_DOF], dof_kd[GM_MAX_DOF];
  // Model constants flattened per lane on the host, so a phase issues all of a lane's
  // loads at one level instead of body -> joint -> qpos chains of dependent loads.
  // per scan lane (lane_body): the body's joint and local transform
  int32_t kl_type[64];                 // joint type, -1: no body / welded
  int32_t kl_qadr[64];                 // the joint's qpos address
  int32_t kl_grp[64];                  // body group, -1: no body
  int32_t kl_cpos[64];                 // chain position (fingers / palm), else 0
  double kl_pos[64][3], kl_quat[64][4], kl_axis[64][3];   // body_pos / body_quat / jnt_axis
  // per dof: its joint's type, index inside the joint, axis
  int32_t dof_jtype[GM_MAX_DOF], dof_k[GM_MAX_DOF];
  double dof_axis[GM_MAX_DOF][3];
  // per candidate pair, both geoms (slot 0 = pair_a, 1 = pair_b); the live object's
  // geom has type -1 (its type, size, rbound and friction come from the env state)
  int32_t pr_g[GM_MAX_PAIR][2], pr_type[GM_MAX_PAIR][2], pr_body[GM_MAX_PAIR][2];
  double pr_pos[GM_MAX_PAIR][2][3], pr_quat[GM_MAX_PAIR][2][4], pr_size[GM_MAX_PAIR][2][3];
  double pr_rbound[GM_MAX_PAIR][2], pr_fric[GM_MAX_PAIR][2];
  // per motor lock: the locked dof's group and chain position
  int32_t lock_grp[GM_MAX_LOCK], lock_cpos[GM_MAX_LOCK];
  // Newton Hessian assembly: per scan lane, the pairs of the lane body's geoms with the
  // object / the ground (-1: none; the object lane holds none, its ground contacts come
  // from pair_gobj); lane_obj is the object's scan lane
  int32_t lane_opair[64][2], lane_gpair[64][2];
  int32_t pair_gobj, lane_obj;
  // per motor lock: its weld's regulariser sum, body_invweight0 of the slide's two bodies
  double lock_tran[GM_MAX_LOCK];
};
