/* gripper_mi355x.h -- C ABI of the MI355X-native batched gripper env-step path.
 *
 * This is the drop-in boundary that replaces the per-env MjClass hot path which
 * the reference exposes through pybind11 (src/bind.cpp:32-205, compiled to
 * rl/env/mjpy/bind.so by Makefile:22,31,155-156).  Every entry point below names
 * the reference interface it replaces.  Conventions:
 *   - plain C types and pointers only; no C++ exceptions cross the ABI;
 *   - every call returns GM_OK (0) or a negative GM_E* code, and the per-context
 *     message is available from gm_last_error(ctx) (the Python facade raises
 *     RuntimeError with it, as pybind11's default translator does for
 *     std::runtime_error in the reference);
 *   - host buffers are owned by the caller; `on_device != 0` means the pointer is
 *     a HIP device pointer on the context's device (zero-copy torch tensors);
 *   - one context per HIP stream; calls on one context are not reentrant.
 *
 * The interface data types (settings, model, object descriptors) are plain POD
 * structs; tests/ hand the same structs to the CPU oracle in oracle/.
 */
#ifndef GRIPPER_MI355X_H_
#define GRIPPER_MI355X_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ limits */
#define GM_MAX_SEG    10      /* finger segment joints N (reference: 5..10)   */
#define GM_MAX_BODY   40
#define GM_MAX_DOF    44      /* 3 (N + 2) + 8 for N = 10                    */
#define GM_MAX_QPOS   48
#define GM_MAX_GEOM   40
#define GM_MAX_PAIR   80      /* 6 N + 15 candidate pairs; a lane per pair per 64-pair batch */
#define GM_MAX_CON    32      /* contacts kept per env per substep (box-box: up to 8 per pair) */
#define GM_MAX_EFC    (4 * GM_MAX_CON + GM_MAX_LOCK)   /* rows: motor locks + 4 pyramid edges per contact */
#define GM_NEWTON_MAXIT 16    /* Newton iterations per substep (cap; converged runs stop earlier) */
#define GM_NEWTON_MAXLS 16    /* exact line-search evaluations per Newton iteration (cap)          */
#define GM_MAX_LOCK   4       /* prismatic x3 + palm (revolute locks disabled) */
#define GM_MAX_OBJSET 64      /* objects in one synthetic object set          */
#define GM_RING       64      /* sensor window: last 64 readings per stream (1 + rps * prev_steps <= 64) */
#define GM_CHAIN      (GM_MAX_SEG + 2)  /* dofs per finger chain below base   */
/* MPR support-point tie band: a unit direction whose body-frame component along a box
 * face normal / cylinder axis is below this picks the face centre (see support_geom) */
#define GM_SUPPORT_TIE 1e-9

/* ------------------------------------------------------------------ errors */
#define GM_OK            0
#define GM_E_ARG        -1
#define GM_E_HIP        -2
#define GM_E_STATE      -3
#define GM_E_NOEXT      -4
#define GM_E_RANGE      -5

/* ------------------------------------------------------------- geom types */
/* numbering follows MuJoCo's mjtGeom so the (geom1, geom2) canonical order
 * "lower type first, then lower id" is the one the reference's contact signs
 * depend on (hard part 3). */
#define GM_GEOM_PLANE    0
#define GM_GEOM_SPHERE   2
#define GM_GEOM_CAPSULE  3
#define GM_GEOM_CYLINDER 5
#define GM_GEOM_BOX      6

/* contact classes: Contact::check_involves() prefixes (objecthandler.h:117-129) */
#define GM_CLS_NONE    0
#define GM_CLS_FINGER1 1
#define GM_CLS_FINGER2 2
#define GM_CLS_FINGER3 3
#define GM_CLS_PALM    4
#define GM_CLS_GROUND  5
#define GM_CLS_OBJECT  6

/* joint types (MuJoCo mjtJoint numbering) */
#define GM_JNT_FREE   0
#define GM_JNT_SLIDE  2
#define GM_JNT_HINGE  3

/* body chain groups: which compact Jacobian block a body's dofs live in */
#define GM_GRP_WORLD  -1
#define GM_GRP_FINGER0 0
#define GM_GRP_PALM    3
#define GM_GRP_BASE    4
#define GM_GRP_OBJECT  5

/* ------------------------------------------------------------ settings */
typedef struct gm_sensor {            /* MjType::Sensor, mjclass.h:79-241 */
  int32_t in_use;
  float   normalise;
  float   read_rate;
  int32_t use_normalisation;
  int32_t use_noise;
  float   raw_value_offset;
  float   noise_mag;
  float   noise_mu;
  float   noise_std;
  int32_t noise_overriden;
  int32_t prev_steps;
  int32_t readings_per_step;
  int32_t total_readings;
} gm_sensor;

typedef struct gm_action {            /* MjType::ActionSetting, mjclass.h:458-572 */
  int32_t in_use;
  int32_t continous;
  double  value;
  int32_t sign;
} gm_action;

typedef struct gm_binary_reward {     /* MjType::BinaryReward, mjclass.h:649-663 */
  float   reward;
  int32_t done;
  int32_t trigger;
} gm_binary_reward;

typedef struct gm_linear_reward {     /* MjType::LinearReward, mjclass.h:665-684 */
  float   reward;
  int32_t done;
  int32_t trigger;
  float   min;
  float   max;
  float   overshoot;
} gm_linear_reward;

typedef struct gm_settings {          /* MjType::Settings, mjclass.h:736-779 */
#define GM_XX(n, t, v) t n;
#define GM_SS(n, u, nm, r) gm_sensor n;
#define GM_AA(n, u, v, s) gm_action n;
#define GM_BR(n, r, d, t) gm_binary_reward n;
#define GM_LR(n, r, d, t, a, b, o) gm_linear_reward n;
#include "gm_settings.def"
} gm_settings;

/* event indices, in settings order (binary first, then linear) */
enum {
#define GM_BR(n, r, d, t) GM_EV_##n,
#include "gm_settings.def"
  GM_N_BINARY
};
enum {
#define GM_LR(n, r, d, t, a, b, o) GM_LEV_##n,
#include "gm_settings.def"
  GM_N_LINEAR
};
enum {
#define GM_AA(n, u, v, s) GM_ACT_##n,
#include "gm_settings.def"
  GM_N_ACTION_KINDS
};
/* action codes, MjType::Action (mjclass.h:40-63): 3 per action kind + termination */
#define GM_ACTION_CODE_COUNT (3 * GM_N_ACTION_KINDS + 1)
#define GM_ACTION_TERMINATION (3 * GM_N_ACTION_KINDS)

/* sample modes, MjType::Sample (mjclass.h:66-76) */
#define GM_SAMPLE_RAW 0
#define GM_SAMPLE_CHANGE 1
#define GM_SAMPLE_AVERAGE 2
#define GM_SAMPLE_MEDIAN 3
#define GM_SAMPLE_SIGN 4
#define GM_SAMPLE_SCALED_CHANGE 5
#define GM_SAMPLE_SCALED_CHANGE_SQ 6

/* Derived configuration: what MjClass::configure_settings() (mjclass.cpp:97-314)
 * and Settings::update_sensor_settings() (mjclass.cpp:5236-5265) compute from
 * gm_settings.  Built on the host by gm_configure(); shared by all envs. */
typedef struct gm_config {
  gm_settings s;
  int32_t n_actions;
  int32_t action_options[GM_ACTION_CODE_COUNT];
  int32_t sensor_fcn;                 /* sample mode for sensors            */
  int32_t state_fcn;                  /* sample mode for state sensors      */
  int32_t sensor_fcn_state_override;  /* reference quirk mjclass.cpp:204-206 */
  int32_t sim_steps_per_action;
  int32_t n_obs;
  double  timestep;
  double  sim_gauge_raw_to_N_factor;  /* mjclass.cpp:281                    */
  double  base_min[6];                /* x,y,z,roll,pitch,yaw (myfunctions.cpp:245-261) */
  double  base_max[6];
} gm_config;

/* ------------------------------------------------------------ model */
typedef struct gm_model_params {      /* numerics the MJCF would carry (myfunctions.cpp:836-953) */
  int32_t n_seg;                      /* N finger segment joints              */
  double  finger_length;              /* 235e-3                               */
  double  finger_width;               /* 28e-3                                */
  double  finger_thickness;           /* 0.86e-3 (baseline yaml)              */
  double  finger_E;                   /* 193e9                                */
  double  hook_length;                /* 35e-3                                */
  double  hook_angle_degrees;         /* 75                                   */
  double  fingertip_clearance;        /* 10e-3                                */
  double  segment_inertia_scaling;    /* 50                                   */
  double  timestep;                   /* 3.187e-3 (test.cpp:207)              */
  int32_t pgs_iterations;             /* sweeps of the oracle's PGS cross-check */
  double  collision_half_thickness;   /* finger plate collision half-thickness */
  /* segment hinge damping d = segment_damping * N^-segment_damping_power and armature
   * a = segment_armature * N^-segment_armature_power (absent from the reference sources:
   * fitted to its measured stable timesteps, tests/test_calibration.py) */
  double  segment_damping;
  double  segment_damping_power;
  double  segment_armature;
  double  segment_armature_power;
  /* actuators (the reference writes ctrl to MJCF motors, luke::control myfunctions.cpp:1912-2057):
   * 1 = MuJoCo 2.1.5's order -- the PD forces explicit between mj_step1 and mj_step2, the
   * constraint solve on M + armature, joint damping implicit in mj_Euler; 0 = the PD gains
   * and joint damping folded implicitly into the solve's matrix (rounds 1-3) */
  int32_t mujoco_actuators;
  int32_t pad_params;
  /* armature of the actuated joints (prismatic, revolute, palm, base): the motors'
   * reflected inertia the absent MJCF would carry (invented; DESIGN.md "Model spec") */
  double  actuator_armature[4];
} gm_model_params;

typedef struct gm_model {
  int32_t nbody, njnt, nq, nv, ngeom, npair, nlock, n_seg;
  /* bodies (parent always has a lower index) */
  int32_t body_parent[GM_MAX_BODY];
  int32_t body_jnt[GM_MAX_BODY];      /* -1 = welded to parent             */
  int32_t body_group[GM_MAX_BODY];    /* GM_GRP_*                          */
  double  body_pos[GM_MAX_BODY][3];   /* in parent frame                   */
  double  body_quat[GM_MAX_BODY][4];  /* w,x,y,z in parent frame           */
  double  body_mass[GM_MAX_BODY];
  double  body_ipos[GM_MAX_BODY][3];  /* centre of mass, body frame        */
  double  body_inertia[GM_MAX_BODY][3]; /* principal, body-frame aligned   */
  /* joints: at most one per body */
  int32_t jnt_type[GM_MAX_BODY];
  int32_t jnt_body[GM_MAX_BODY];
  int32_t jnt_qposadr[GM_MAX_BODY];
  int32_t jnt_dofadr[GM_MAX_BODY];
  double  jnt_pos[GM_MAX_BODY][3];    /* anchor, body frame                */
  double  jnt_axis[GM_MAX_BODY][3];   /* body frame, unit                  */
  double  jnt_stiffness[GM_MAX_BODY];
  double  jnt_damping[GM_MAX_BODY];
  double  jnt_armature[GM_MAX_BODY];
  /* dofs */
  int32_t dof_parent[GM_MAX_DOF];
  int32_t dof_body[GM_MAX_DOF];
  int32_t dof_group[GM_MAX_DOF];      /* GM_GRP_* of the owning chain       */
  int32_t dof_slot[GM_MAX_DOF];       /* index inside the compact group block */
  /* geoms */
  int32_t geom_type[GM_MAX_GEOM];
  int32_t geom_body[GM_MAX_GEOM];
  int32_t geom_class[GM_MAX_GEOM];
  double  geom_pos[GM_MAX_GEOM][3];
  double  geom_quat[GM_MAX_GEOM][4];
  double  geom_size[GM_MAX_GEOM][3];
  double  geom_friction[GM_MAX_GEOM];
  double  geom_rbound[GM_MAX_GEOM];
  /* candidate pairs (object pairs first; unordered: canonical order per env) */
  int32_t pair_a[GM_MAX_PAIR];
  int32_t pair_b[GM_MAX_PAIR];
  /* motor locks (reference weld constraints on 1-DoF motors) */
  int32_t lock_dof[GM_MAX_LOCK];
  int32_t lock_kind[GM_MAX_LOCK];     /* 0 prismatic, 2 palm               */
  /* keyframe "initial pose" (myfunctions.cpp:171) */
  double  qpos0[GM_MAX_QPOS];
  /* mj_setConst at qpos0: body_invweight0 (translation, rotation: the mean diagonal of
   * J M^-1 J^T at the body's centre of mass) and dof_invweight0 (M^-1 diagonal); they set
   * the constraint regulariser R = (1 - d) / d * diagApprox (mj_diagApprox).  Derived by
   * gm_build_model / gm_model_from_mjcf; the live object's are per env. */
  double  body_invweight0[GM_MAX_BODY][2];
  double  dof_invweight0[GM_MAX_DOF];
  /* named indices */
  int32_t dof_base, dof_palm, dof_obj;
  int32_t dof_pris[3], dof_rev[3], dof_seg[3];   /* first segment dof per finger */
  int32_t body_base, body_finger[3], body_palm, body_obj, geom_obj, geom_ground;
  /* physics options */
  double  timestep;
  double  gravity[3];
  double  solref[2];                  /* timeconst, dampratio              */
  double  solimp[5];                  /* dmin, dmax, width, midpoint, power */
  int32_t pgs_iterations;             /* sweeps of the oracle's PGS cross-check (the engine: Newton) */
  double  mpr_tolerance;
  int32_t mpr_iterations;
  /* gripper dimensions used by the env logic (JointSettings::Dim) */
  double  finger_length, finger_width, finger_thickness, finger_E, finger_EI;
  double  segment_length, hook_length, hook_angle_degrees, fingertip_clearance;
  double  yield_stress;
  int32_t fixed_first_segment;
  /* PD gains (JointSettings::ctrl, myfunctions.cpp:273-296) */
  double  kp_gripper[3], kd_gripper[3], kp_base[3], kd_base[3];
  double  time_per_step;              /* stepper chunk: num_steps / pulses_per_s */
  int32_t stepper_num_steps;
  /* gauge (JointSettings::gauge, myfunctions.cpp:264-270) */
  double  gauge_xpos;
  int32_t gauge_order;
  /* tip loading for the gauge calibration (get_segment_matrices / apply_segment_force,
   * myfunctions.cpp:1521-1610, 1660-1727): the last link of each finger and the finger's
   * bending direction at the keyframe (world frame, radially outward) */
  int32_t body_tip[3];
  double  tip_dir[3][3];
  /* gm_model_params.mujoco_actuators */
  int32_t mujoco_actuators;
  /* Newton iterations per constraint solve (0: GM_NEWTON_MAXIT): a test knob that makes
   * capped solves happen (their qacc is no optimum; mj_Euler then integrates qfrc_smooth +
   * J^T efc, not M qacc, see euler_damping) */
  int32_t newton_maxit;
} gm_model;

/* one graspable object (a synthetic object-set entry) */
typedef struct gm_object {
  int32_t type;                       /* GM_GEOM_BOX / _CYLINDER / _SPHERE  */
  double  size[3];                    /* MuJoCo geom size semantics (half sizes) */
  double  mass;
  double  friction;
} gm_object;

/* per-env spawn request: MjClass::spawn_object(index, x, y, zrot) (mjclass.cpp:2352-2420) */
typedef struct gm_spawn {
  int32_t object_index;
  double  x, y, zrot;
} gm_spawn;

/* spawn search request: MjType::SpawnParams (mjclass.h:916-931), defaults as there
 * (gm_default_spawn_params).  The xy grid holds at most GM_SPAWN_MAX_XY points and the
 * rotation grid GM_SPAWN_MAX_ROT (gm_spawn_into_scene rejects larger grids). */
typedef struct gm_spawn_params {
  int32_t index;
  int32_t pad;
  double  x, y, zrot;
  double  xrange, yrange, rotrange;
  double  xmin, xmax, ymin, ymax;
  double  smallest_gap;
  double  xy_increment, rot_increment;
} gm_spawn_params;
#define GM_SPAWN_MAX_XY  1024
#define GM_SPAWN_MAX_ROT 256

/* ------------------------------------------------------------ C ABI */
typedef struct gm_ctx gm_ctx;

/* library / build information */
const char* gm_version(void);
int  gm_device_count(void);
/* sizes of the interface structs (0 settings, 1 model, 2 config, 3 object, 4 spawn,
 * 5 model params, 6 spawn params, 7 calibration) so bindings can verify their layouts */
int64_t gm_struct_size(int which);
/* model summary: nq, nv, nbody, ngeom, npair, n_seg, dof_base, dof_palm, dof_obj,
 * dof_pris[3], dof_rev[3], dof_seg[3], nlock, nM (tree-sparse M nonzeros)  (20 int32) */
void gm_model_info(const gm_model* m, int32_t* out);
/* derived config summary: n_obs, n_actions, sim_steps_per_action, sensor_fcn, state_fcn */
void gm_config_info(const gm_config* c, int32_t* out);

/* Model builder: the MJCF the reference loads with mj_loadXML
 * (mjclass.cpp:377-409) is unavailable (empty `description` submodule), so the
 * gripper is compiled from its numeric parameters instead. */
void gm_default_model_params(gm_model_params* p);
int  gm_build_model(const gm_model_params* p, gm_model* out);

/* MJCF.  The reference compiles its task MJCF with mj_loadXML
 * (mjclass.cpp:377-409), finds everything by the JointSettings / ObjectHandler names
 * (myfunctions.cpp:176-196, 719-787; objecthandler.cpp:22-133) and reads the gripper
 * numerics from <custom><numeric> (read_gripper_dimensions, myfunctions.cpp:836-953).
 * gm_model_to_mjcf writes a model as MJCF with those names (returns the text length;
 * writes it, NUL-terminated, when cap > length); gm_model_from_mjcf compiles the MJCF
 * subset it uses (option, default geom solref/solimp, custom numerics, body / joint
 * slide|hinge|free / inertial / geom plane|sphere|cylinder|box|capsule, contact pairs,
 * equality joint locks, the "initial pose" keyframe) into a gm_model.  A written model
 * reads back identical bit for bit.  err (optional): a message on failure. */
int64_t gm_model_to_mjcf(const gm_model* m, char* buf, int64_t cap);
int  gm_model_from_mjcf(const char* xml, gm_model* out, char* err, int err_cap);

/* Settings defaults (simsettings.h) and derived configuration
 * (MjClass::configure_settings, mjclass.cpp:97-314). */
void gm_default_settings(gm_settings* s);
int  gm_configure(const gm_settings* s, const gm_model* m, gm_config* out);

/* MjClass::set_base_XYZ_limits / set_base_yaw_limit (mjclass.cpp:3847-3859 ->
 * luke::set_base_XYZ_limits / set_base_yaw_limit, myfunctions.cpp:2309-2333): symmetric
 * base operating limits [-x, x], [-y, y], [-z, z] (m) and, when yaw >= 0, [-yaw, yaw]
 * (rad) in a configuration; push it to a context with gm_update_config. */
int  gm_config_set_base_limits(gm_config* cfg, double x, double y, double z, double yaw);

/* Synthetic object sets (the reference's set6/set9 MJCF sets are unavailable). */
int  gm_make_object_set(const char* name, uint64_t seed, gm_object* out, int max_objects);

/* The automatic settings of MjClass::configure_settings (mjclass.cpp:241-308), found by
 * simulation: find_highest_stable_timestep (mjclass.cpp:4745-4854) and
 * calibrate_simulated_sensors (4643-4676, tip load via validate_curve_under_force
 * 4023-4105).  Timesteps keep the reference's float arithmetic. */
typedef struct gm_calibration {
  double  timestep;                   /* s_.mujoco_timestep after the search (and any 0.8x
                                         gauge-run retries, mjclass.cpp:4080)            */
  int32_t sim_steps_per_action;       /* ceil(time_for_action / timestep) (mjclass.cpp:306) */
  int32_t n_tested;                   /* candidate timesteps simulated by the search      */
  double  search_timestep;            /* highest stable timestep found (before the factor) */
  double  yield_load;                 /* calc_yield_point_load (myfunctions.cpp:3587-3595), N */
  double  bend_gauge_normalise;       /* saturation_yield_factor * yield_load (mjclass.cpp:278) */
  float   bending_normalise;          /* gauge reading under that tip load (mjclass.cpp:4666) */
  float   sim_gauge_raw_to_N_factor;  /* mjclass.cpp:281                                   */
  float   wrist_Z_offset;             /* mjclass.cpp:4659: userdata[2] is never written, 0  */
  int32_t gauge_retries;              /* 0.8x timestep retries of the tip-load run          */
} gm_calibration;
/* calibrate_reset's first-call settle as the reference scopes it (myfunctions.cpp:1441-1519:
 * a function-static first_call, so the 400-substep settle runs once per PROCESS and later
 * models with the same joint count reuse its equilibrium even when their timestep or finger
 * stiffness differ).  on = 1: contexts created from now on share one settle (the first one
 * made after the call); 0 (default): every context settles its own model. */
void gm_set_settle_cache(int on);

#define GM_CAL_TIMESTEP 1
#define GM_CAL_GAUGES   2
/* validate_curve_under_force's retry as the reference runs it (mjclass.cpp:4073-4090): on
 * instability the timestep drops to 0.8x, reset() wipes the tip load, and `continue` resumes
 * the step loop -- the remaining steps run unloaded from the reset pose.  Without the flag
 * the whole loaded settle is rerun at the reduced step (the engine's default). */
#define GM_CAL_REFERENCE_RETRY 4
#define GM_CAL_MAX_TRACE 256

/* Batched calibration on `device`: every candidate timestep of the search is simulated
 * for 1 s as its own env in one launch (per-env timestep, mjWARN_BADQACC-style
 * instability flag), and the search replays the reference's coarse/fine sequence over the
 * results, so the answer equals the sequential search.  The gauge run is one env under
 * the saturation tip load for 50 s of simulated time.  `what`: GM_CAL_TIMESTEP |
 * GM_CAL_GAUGES (the gauge run uses model->timestep when the search is off).  trace_dt /
 * trace_unstable (optional, max_trace entries): the search's candidates in order.
 * Sensor and base-position noise are off during calibration. */
int  gm_calibrate(const gm_model* model, const gm_config* cfg, const gm_object* objects, int n_objects,
                  int device, int what, gm_calibration* out, double* trace_dt, uint8_t* trace_unstable,
                  int max_trace);

/* Context lifetime: MjClass() + load() + init() (bind.cpp:46-52, mjclass.cpp:8-95) */
int  gm_create(const gm_model* model, const gm_config* cfg, const gm_object* objects,
               int n_objects, int n_envs, int env_offset, int device, uint64_t seed,
               gm_ctx** out);
void gm_destroy(gm_ctx* ctx);
const char* gm_last_error(const gm_ctx* ctx);
int  gm_n_envs(const gm_ctx* ctx);
int  gm_n_obs(const gm_ctx* ctx);        /* MjClass::get_n_obs     (bind.cpp:157) */
int  gm_n_actions(const gm_ctx* ctx);    /* MjClass::get_n_actions (bind.cpp:156) */
int  gm_update_config(gm_ctx* ctx, const gm_config* cfg);  /* mj.set.* writes */

/* MjClass::reset() (mjclass.cpp:434-486) for envs with mask[e] != 0 (NULL = all),
 * followed by spawn_object(spawn[e]) (mjclass.cpp:2352-2420).  Host arrays. */
int  gm_reset(gm_ctx* ctx, const uint8_t* mask, const gm_spawn* spawn);
/* MjClass::spawn_object(idx, x, y, zrot) alone (mjclass.cpp:2352-2420; bind.cpp:98-105):
 * replaces the live object of masked envs; consumes no RNG draws.  Host arrays. */
int  gm_spawn_object(gm_ctx* ctx, const uint8_t* mask, const gm_spawn* spawn);
/* MjType::SpawnParams defaults (mjclass.h:916-931). */
void gm_default_spawn_params(gm_spawn_params* p);
/* MjClass::spawn_into_scene(SpawnParams) (mjclass.cpp:2475-2654; bind.cpp:100-103) on the
 * device for envs with mask[e] != 0 (NULL = all): the xy and rotation grids are shuffled
 * with std::shuffle semantics on the env's RNG stream, every candidate pose is tested with
 * the Box2d SAT rules (customtypes.h:35-172) against the scene bounds and the initial
 * fingertip boxes (Env::reset, mjclass.h:895-904, from get_finger_hook_locations,
 * myfunctions.cpp:3717-3761), and the object is spawned at the first free pose
 * (spawn_object).  params: n_params == 1 (shared) or n_envs entries.  ok[e] = 1 when
 * spawned, 0 when no pose is free (state unchanged apart from the RNG draws, as in the
 * reference); ok may be NULL.  Host arrays.  The device env holds one live object, so
 * the reference's loop over objects already in the scene is empty (MjEnv._spawn_object
 * spawns one object per reset). */
int  gm_spawn_into_scene(gm_ctx* ctx, const uint8_t* mask, const gm_spawn_params* params, int n_params,
                         uint8_t* ok);
/* Make gm_reset / gm_autoreset place each reset env's object the way MjEnv._spawn_object
 * does (MjEnv.py:1177-1267): spawn_into_scene(spawn[e].object_index) with *params, up to
 * max_tries attempts, falling back to spawn_object(spawn[e]) (MjEnv's "old method").
 * params == NULL restores plain spawn_object(spawn[e]). */
int  gm_set_scene_spawn(gm_ctx* ctx, const gm_spawn_params* params, int max_tries);

/* MjEnv._spawn_object's Python-side draws (MjEnv.py:1177-1267) made per reset on the
 * device: with enable != 0, gm_reset / gm_autoreset called without a spawn table draw each
 * reset env's object index uniformly over the set and its fallback ("old method") pose
 * -- integer-mm x, y in [-position_noise_mm, position_noise_mm], z rotation one of
 * {0, 60, 120} deg plus integer-degree noise in [-rotation_noise_deg, rotation_noise_deg]
 * -- from splitmix64(seed, global env id, episode, draw) (gm_state.h gm_spawn_int), so
 * every episode gets a fresh object, results do not depend on how envs are sharded, and
 * the reference's C++ RNG stream is not consumed.  With gm_set_scene_spawn the drawn index
 * goes to spawn_into_scene first, as MjEnv does. */
int  gm_set_random_spawn(gm_ctx* ctx, int enable, uint64_t seed, int position_noise_mm, int rotation_noise_deg);

/* MjClass::set_motor_target(x, y, z) (bind.cpp:82; mjclass.cpp:1359-1364 ->
 * luke::set_gripper_target_m, myfunctions.cpp:2347-2355 -> Gripper::set_xyz_m, gripper.h:152):
 * the gripper's motor-position target in metres for envs with mask[e] != 0 (NULL = all);
 * the stepper walks toward it over the following action_step()s.  xyz: 3 doubles shared
 * (n_xyz == 1) or 3 per env (n_xyz == n_envs), host array.  in_limits[e] (may be NULL) is
 * the reference's return value: 0 when a motor limit clamped the target.  Used by the
 * reference's force-measurement programs (mysimulate.cpp:2720-2811). */
int  gm_set_motor_target(gm_ctx* ctx, const uint8_t* mask, const double* xyz, int n_xyz, uint8_t* in_limits);
/* MjClass::sim_sensors_SI_ (mjclass.cpp:741-898, read through SensorData::read_finger1_gauge
 * etc., bind.cpp:1149-1151): the latest SI reading of every env, out[e * 5 + k] for k =
 * finger 1..3 bending gauge (N, the raw gauge times sim_gauge_raw_to_N_factor), palm (N),
 * wrist Z (N).  Host array [n_envs x 5]. */
int  gm_get_sensor_si(gm_ctx* ctx, float* out);

/* Synthetic driver for benchmarks and parity tests (not a reference interface): the
 * scripted grasp mix -- per env and episode, phase lengths from splitmix64(seed, global
 * env id, episode); close the fingers, squeeze, press the palm, lift the base, indexed by
 * the env's episode step, plus uniform jitter -- written as continuous action fractions
 * [n_envs x n_actions] to `out` (a device pointer when on_device; feed it to
 * gm_set_action).  Runs on the context's stream after whatever reset came before it. */
int  gm_scripted_actions(gm_ctx* ctx, uint64_t seed, float jitter, float* out, int on_device);
/* Synthetic driver (not a reference interface): uniform random action fractions U[-1, 1)
 * per env and action from a counter-based hash of (seed, global env id, episode, episode
 * step, action index) -- the north star's "synthetic random-action rollouts" -- written like
 * gm_scripted_actions. */
int  gm_random_actions(gm_ctx* ctx, uint64_t seed, float* out, int on_device);
/* Synthetic driver (not a reference interface): the grasp-lift-hold program (mode 3) or the
 * benchmark mix (mode 4: the program in 1 episode of 4 per env -- draw 21 of the episode's
 * counter-based hash -- the scripted grasp mix with `jitter` otherwise) for the current
 * state of every env, written like gm_scripted_actions.  The program is closed-loop and
 * stateless (gm_state.h gm_program_fraction): close, squeeze, lift the base, lower the palm
 * onto the object and hold the palm reading in the stable band -- the reference's success
 * chain (mjclass.cpp:1148-1210, 1295-1322).  GM_E_ARG for another mode. */
int  gm_program_actions(gm_ctx* ctx, uint64_t seed, float jitter, int mode, float* out, int on_device);

/* MjClass::set_continous_action for every action index i in order
 * (mjclass.cpp:1517-1630; called per index by MjEnv._set_action, MjEnv.py:591-594).
 * actions: [n_envs x n_actions] float32.  Host actions are copied into a pinned staging
 * buffer before the call returns (the caller may reuse its array at once); the upload and
 * the action kernel run asynchronously on the context's stream. */
int  gm_set_action(gm_ctx* ctx, const float* actions, int on_device);
/* MjClass::set_discrete_action (mjclass.cpp:1510-1515). actions: [n_envs] int32. */
int  gm_set_discrete_action(gm_ctx* ctx, const int32_t* actions, int on_device);

/* MjClass::action_step() (mjclass.cpp:1483-1508) + get_observation (1700-1959)
 * + is_done (1632-1698) + reward (3000-3049), fused in one device launch,
 * evaluated in the order MjEnv.step uses them (obs, done, reward). */
int  gm_step(gm_ctx* ctx);

int  gm_get_obs(gm_ctx* ctx, float* out, int on_device);                 /* [n_envs x n_obs] */
int  gm_get_reward_done(gm_ctx* ctx, float* reward, uint8_t* done, int on_device);
/* The three at once into host buffers, one stream synchronisation (the facade's
 * get_observation_numpy / is_done / reward of one transition). */
int  gm_get_outputs(gm_ctx* ctx, float* obs, float* reward, uint8_t* done);
/* EventTrack rows: [n_envs x (GM_N_BINARY + GM_N_LINEAR)] int32 `row`, and
 * `abs` counters; MjClass::get_event_state / EventTrack (bind.cpp:525-590). */
int  gm_get_event_rows(gm_ctx* ctx, int32_t* rows, int32_t* abs_counts, float* last_values);
/* raw state readback (testing / checkpoint), fp64 like mjData's qpos / qvel:
 * qpos [n_envs x nq], qvel [n_envs x nv], time [n_envs] (MjClass::get_state-style access
 * the reference's tests use through mjData) */
int  gm_get_state(gm_ctx* ctx, double* qpos, double* qvel, double* time);
int  gm_set_state(gm_ctx* ctx, const double* qpos, const double* qvel);
/* The whole per-env state (everything an MjClass carries between action_step() calls:
 * mjData qpos/qvel/time, target_ stepper state, sensor windows, event tracks, RNG,
 * function-static flags), fp64 where the reference is: gm_env_state_size() bytes per env,
 * [n_envs] records.  Checkpoint / resume, and the hand-off the parity tests use to run
 * the CPU oracle from exactly the device's state.  Host buffers. */
int64_t gm_env_state_size(void);
int  gm_get_env_states(gm_ctx* ctx, void* out);
int  gm_set_env_states(gm_ctx* ctx, const void* in);
/* target (stepper) state: [n_envs x 8] = end x,y,z,th (m/rad) then step x,y,z and base z */
int  gm_get_target(gm_ctx* ctx, double* end_xyzth, int32_t* end_steps, int32_t* next_steps,
                   double* base_xyz);
/* number of envs whose contact list overflowed GM_MAX_CON in the last gm_step */
int  gm_get_overflow(gm_ctx* ctx, int32_t* counts);

/* device pointers for zero-copy (torch.from_blob-style) access */
void* gm_device_obs(gm_ctx* ctx);
void* gm_device_reward(gm_ctx* ctx);
void* gm_device_done(gm_ctx* ctx);
void* gm_device_actions(gm_ctx* ctx);
void* gm_stream(gm_ctx* ctx);
/* route every later launch of ctx to `stream` (a hipStream_t, e.g. torch's current
   stream) so device-pointer I/O is ordered with the caller's work; NULL restores
   the ctx's own stream.  Synchronises the previous stream first. */
int  gm_set_stream(gm_ctx* ctx, void* stream);
/* MjEnv's episode-boundary handling done on the device (MjEnv.py:616-637 then
 * MjEnv.reset, MjEnv.py:2222-2263): every env with done != 0 from the last gm_step,
 * or num_action_steps >= max_episode_steps (<= 0 disables truncation), writes its
 * cumulative reward to returns[e] (NaN for envs that continue; returns may be NULL),
 * is flagged in gm_device_reset_mask, and is reset + respawned from spawn[e].
 * spawn: host array unless spawn_on_device; NULL spawns object 0 at the origin. */
int  gm_autoreset(gm_ctx* ctx, int max_episode_steps, const gm_spawn* spawn, int spawn_on_device,
                  float* returns);
void* gm_device_reset_mask(gm_ctx* ctx);   /* uint8 [n_envs], written by gm_autoreset */
/* The episode-end record north_star's RCCL all-gather carries: per env, the
 * episode return (MjEnv's cumulative reward, MjEnv.py:616-637), its length in env-steps
 * (MjClass::env_.num_action_steps) and success -- the reference's successful_grasp metric
 * (mjclass.cpp:1295-1322: a +1-reward, done-setting binary event triggered this step).  Envs
 * whose episode continues hold {NaN, 0, 0}.  12 bytes, so a [n_envs] array is a plain
 * [n_envs x 3] 4-byte tensor for the collective. */
typedef struct gm_episode_end {
  float   ret;
  int32_t length;
  uint8_t success;
  uint8_t pad[3];
} gm_episode_end;
/* gm_autoreset that also writes the episode-end record of every env (device array
 * [n_envs], may be NULL) -- returns may be NULL too. */
int  gm_autoreset_episodes(gm_ctx* ctx, int max_episode_steps, const gm_spawn* spawn, int spawn_on_device,
                           float* returns, gm_episode_end* episodes);

/* A fused batched rollout (the env-step hot path with its synthetic driver on the device):
 * n_steps repetitions, for every env, of exactly the per-step API's sequence
 *   gm_scripted_actions (action_mode 0, seed, jitter), gm_random_actions (1, seed) or
 *   gm_program_actions (3: the grasp program, 4: the benchmark's program / scripted mix)
 *   -> gm_set_action -> gm_step -> gm_autoreset_episodes(max_episode_steps, spawn = NULL,
 *      records + k * n_envs)
 * -- the same code on the same state, so the results are bit for bit those of the n_steps
 * per-step calls -- but as ONE persistent launch: an env that finishes env-step k starts k + 1
 * at once on its wave (actions, the termination lift's extra substeps, the episode-end record
 * and MjEnv.reset's reset + spawn included) while the work queue balances envs at substep
 * granularity, so the launch's tail is paid once per n_steps env-steps instead of every step.
 * records: device array [n_steps x n_envs] (or NULL); obs / reward / done buffers hold the last
 * env-step's (the reset observation for envs reset at its end), as after the per-step calls. */
typedef struct gm_rollout_params {
  int32_t  action_mode;        /* 0: scripted grasp mix, 1: uniform random, 3: grasp program,
                                  4: program in 1 episode of 4, scripted mix otherwise */
  int32_t  max_episode_steps;  /* MjEnv truncation; <= 0 disables it */
  uint64_t seed;
  float    jitter;             /* scripted mode only */
  int32_t  pad;
} gm_rollout_params;
int  gm_rollout(gm_ctx* ctx, int n_steps, const gm_rollout_params* params, gm_episode_end* records);

/* Timing of the last env-step kernel launch (HIP events on the context's stream): a gm_step
 * (one env-step per env) or a gm_rollout / gm_policy_rollout launch of n_steps env-steps per
 * env -- gm_dispatch_info out[3] says which; divide by it for a per-env-step figure.
 * gm_chunk_stats and gm_chunk_timeline likewise describe that last launch. */
int  gm_last_step_ms(gm_ctx* ctx, float* ms);
/* The last gm_step's work queue (chunked dispatch): out[0] envs started,
 * out[1] envs finished, out[2] yields (an env handed back to its XCD's queue because an
 * unstarted env had more work left), out[3] resumptions; out[4] substeps between
 * preemption tests (0: the one-shot kernel ran), out[5] resident workgroups, out[6] the
 * resumptions by a wave of another XCD than the yielding one's.  times (may
 * be NULL; 100 MHz constant-clock ticks): [0] first pick, [1] first pick that found no
 * unstarted env, [2] last env finished, [3] sum of wave-busy time, [4] sum of wave polling.
 * Synchronises the context's stream. */
int  gm_chunk_stats(gm_ctx* ctx, uint32_t* out7, uint64_t* times5);
/* The last chunked launch's claim waits: out[0] claims of a yielded env's ring slot that found
 * the slot still empty (its producer between the tail increment and the entry store), out[1]
 * the polls those claims made.  A claimed slot always has a producer in flight
 * (claim_bucket's invariant), so the polls per waiting claim stay small; a claim parked on a
 * slot only a future yield would fill shows as a run of polls.  Synchronises the stream. */
int  gm_chunk_claim_waits(gm_ctx* ctx, uint32_t* out2);
/* The last chunked launch's jobs, per env (arrays of n_envs, either may be NULL): clk[e] the
 * shader clocks / 64 (s_memtime) env e's job ran for, summed over its chunks; yields[e] how
 * often the job was handed back to the queue.  Set when a job finishes (an env the launch
 * did not reach keeps the previous value).  Synchronises the context's stream.  Diagnostics:
 * a job's work against its life (gm_chunk_timeline). */
int  gm_chunk_job_stats(gm_ctx* ctx, uint32_t* clk, int32_t* yields);
/* How gm_step / gm_rollout dispatch this context (fixed at gm_create): out[0] substeps
 * between preemption tests (0: the one-shot kernel), out[1] workgroups of the chunked
 * grid, out[2] waves per env (1; 2 = DUO workgroups, whose second wave runs the collider
 * concurrently -- chosen when every env's two waves fit resident, GM_DUO=0/1 forces it),
 * out[3] env-steps per env of the last launch (1 after gm_step, n_steps after a rollout:
 * the unit of gm_last_step_ms / gm_chunk_stats / gm_chunk_timeline). */
int  gm_dispatch_info(const gm_ctx* ctx, int32_t* out4);
/* The last chunked launch's per-workgroup end of work: when workgroup w finished the last
 * env (or env chunk) it ran, before it polled out the rest of the launch (100 MHz constant
 * clock, the clock of gm_chunk_stats' times, in the low 60 bits; the workgroup's XCD in
 * the top 4): out[w] for w < G = out[1] of gm_dispatch_info; then, per env e, when it was first
 * picked and when its job finished: out[G + 2 e], out[G + 2 e + 1] (up to max_out words).  Returns the count written (>= 0) or a negative error.  Synchronises
 * the context's stream.  Diagnostics: the shape of the launch's tail. */
int  gm_chunk_timeline(gm_ctx* ctx, uint64_t* out, int max_out);

/* ---- single-substep stage hooks for parity testing (GPU vs oracle) ---- */
/* Runs exactly one MjClass::step (mj_step1 + control + mj_step2 + mj_rnePostConstraint
 * equivalent, then update_all and monitor_sensors; mjclass.cpp:504-530) on every env,
 * from the current state, and copies out fp64 diagnostics (any pointer may be NULL):
 * ncon[n_envs], contact [n_envs x GM_MAX_CON x 16] (dist, pos3, frame9, g1, g2, mu),
 * efc_force [n_envs x GM_MAX_EFC], qacc [n_envs x GM_MAX_DOF], nefc [n_envs], and
 * obj_wrench [n_envs x 6]: the live object's cfrc_ext as
 * ObjectHandler::get_object_net_force_faster returns it (objecthandler.cpp:543-565),
 * [force; torque about its centre of mass]. */
int  gm_debug_substep(gm_ctx* ctx, int32_t* ncon, double* contact, double* efc_force,
                      double* qacc, int32_t* nefc, double* obj_wrench);
/* diagnostic: one gm_step with per-phase shader-clock cycle counters, lane-0 view,
   summed over substeps: out[n_envs][32]; columns 0-27 are clocks (names in gmx.env
   BatchedGripperEnv.PHASES: kinematics, crb_rne, mass+forces, collision, newton_solve,
   integrate, update_all, monitor_sensors, the Newton sub-phases, the env-step epilogue),
   28 = constraint rows summed, 29 = substeps that ran MPR, 30 = Newton iterations,
   31 = line-search evaluations */
int  gm_step_profiled(gm_ctx* ctx, uint64_t* phase_cycles);

/* ---- on-device DQN policy ----
 * VariableNetwork.forward (rl/networks.py:7-41: Linear+ReLU hidden layers, final Linear,
 * Softmax(dim=1)) on every env's current observation, then Agent_DQN.select_action
 * (rl/agents/DQN.py:184-209): argmax of the network output, or with probability eps a
 * uniform random action.  The chosen discrete actions are applied to the envs on the
 * device (MjClass::set_discrete_action), so a rollout needs no host round trip.
 * sizes: n_sizes layer widths [n_obs, hidden..., n_actions] (<= 8 layers, widths <= 256);
 * params: torch state_dict order, f32 -- W0 [sizes[1] x sizes[0]] row-major, b0
 * [sizes[1]], W1, b1, ...  (host pointer). */
typedef struct gm_policy gm_policy;
int  gm_policy_create(gm_ctx* ctx, const int32_t* sizes, int n_sizes, const float* params,
                      gm_policy** out);
void gm_policy_destroy(gm_policy* p);
/* Host-side repack of params into the device layout (MFMA B-fragment order, zero
 * padded); returns the packed float count, writes `out` when non-NULL.  Exposed so the
 * layout is testable without a GPU. */
int64_t gm_policy_pack(const int32_t* sizes, int n_sizes, const float* params, float* out);
/* select (eps-greedy, counter-based per-env draws from (seed, global env id, decision))
 * and apply actions for every env; eps = eps_threshold of select_action */
int  gm_policy_act(gm_policy* p, float eps, uint64_t seed, uint64_t decision);
/* last selected actions [n_envs] int32 and softmax outputs [n_envs x n_actions] f32
 * (either may be NULL); host copies */
int  gm_policy_read(gm_policy* p, int32_t* actions, float* q);
/* A fused on-device DQN rollout: n_steps repetitions, for every env, of
 *   gm_policy_act(p, eps[k], seed, decision0 + k) -> gm_step
 *   -> gm_autoreset_episodes(max_episode_steps, spawn = NULL, records + k * n_envs)
 * as ONE persistent launch of gm_rollout's kind: each env's own wave runs select_action on
 * its observation (the batched kernel's MFMA tiles with the env in row 0 -- rows are
 * independent, so the action is bit for bit the batched kernel's) before each env-step.
 * Results (state, observations, records) equal the per-step sequence's bit for bit.
 * eps: host array [n_steps] (copied before the call returns); records: device array
 * [n_steps x n_envs] or NULL.  gm_policy_read's buffers are not written by the fused
 * launch (they are under GM_CHUNK_SUBSTEPS=0, which runs the per-step sequence). */
int  gm_policy_rollout(gm_policy* p, int n_steps, const float* eps, uint64_t seed, uint64_t decision0,
                       int max_episode_steps, gm_episode_end* records);

#ifdef __cplusplus
}
#endif

#endif /* GRIPPER_MI355X_H_ */
