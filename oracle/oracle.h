/* oracle.h -- CPU fp64 restatement of the reference env-step hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker /
 * CPU baseline -- never as the thing measured or shipped.  The product path
 * (gripper-mujoco_amd/) never links or calls it.
 *
 * One or_env is one reference MjClass: single env, single thread, fp64.
 * Each function cites the reference code it restates (paths relative to the
 * reference checkout).  Parity status is recorded in DESIGN.md section "Oracle":
 * pinned by the reference's own compilable code (src/gripper.cpp,
 * src/slidingwindow.h via oracle/_ref), the test.cpp:293-311 known answer and
 * numpy.polyfit; MuJoCo 2.1.5 itself is absent, so the physics restatement is pinned
 * by the MuJoCo outputs the reference kept as data (the force curves of its
 * measure-constrict / measure-tilt programs, rl/juypter/thesis_plots/sim_vs_real_forces*.csv,
 * tests/test_force_curves.py; the stable timesteps of mujoco_timesteps.csv at inertia x50)
 * and by independent restatements of MuJoCo's published algorithms
 * (tests/test_physics_independent.py).
 */
#ifndef GM_ORACLE_H_
#define GM_ORACLE_H_

#include <stdint.h>
#include <stddef.h>
#include "../include/gripper_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_env or_env;

/* create one env; runs the one-time 400-substep settle of calibrate_reset()
 * (myfunctions.cpp:1470-1505) once, shared semantics with the product */
or_env* or_create(const gm_model* m, const gm_config* c, const gm_object* objects,
                  int n_objects, int64_t env_id);
void    or_destroy(or_env* e);
size_t  or_sizeof(void);

void  or_reset(or_env* e, const gm_spawn* spawn);
void  or_spawn(or_env* e, const gm_spawn* spawn);                  /* MjClass::spawn_object alone */
int   or_spawn_into_scene(or_env* e, const gm_spawn_params* p);    /* MjClass::spawn_into_scene */
void  or_set_action(or_env* e, const float* actions);              /* set_continous_action x n_actions */
void  or_set_discrete_action(or_env* e, int32_t action);           /* set_discrete_action */
void  or_driver_actions(const or_env* e, int mode, uint64_t seed, float jitter, int64_t gid,
                        float* out);   /* the rollout drivers (scripted / random / grasp program) */
void  or_step(or_env* e);                                          /* action_step */
int   or_get_obs(or_env* e, float* out);                           /* get_observation */
int   or_is_done(or_env* e);                                       /* is_done */
float or_reward(or_env* e);                                        /* reward */
void  or_get_state(const or_env* e, double* qpos, double* qvel, double* time);
void  or_set_state(or_env* e, const double* qpos, const double* qvel);
void  or_get_target(const or_env* e, double* end_xyzth, int32_t* end_steps, int32_t* next_steps,
                    double* base_xyz);
void  or_get_event_rows(const or_env* e, int32_t* rows, int32_t* abs_counts, float* last_values);
int   or_overflow(const or_env* e);
void  or_get_eq(const or_env* e, double* eq_qpos);                 /* settled equilibrium */
void  or_set_settle_cache(int on);            /* calibrate_reset's process-wide first_call settle */
int   or_set_motor_target(or_env* e, double x, double y, double z);   /* MjClass::set_motor_target */
void  or_want_forces(or_env* e, int on);    /* record each substep's qfrc_smooth / J^T efc (dense) */
void  or_last_forces(const or_env* e, double* qfrc_smooth, double* qfrc_constraint);
void  or_get_sensor_si(const or_env* e, float* out5);   /* sim_sensors_SI_: gauges 1..3, palm, wrist Z */

/* one physics substep, with diagnostics (same layout as gm_debug_substep, fp64);
 * obj_wrench: the live object's cfrc_ext [force; torque about its centre of mass] */
void  or_debug_substep(or_env* e, int32_t* ncon, double* contact, double* efc_force, double* qacc,
                       double* obj_wrench);
void  or_object_net_wrench(const or_env* e, double* out);
/* independent-check hooks: kinematics / H~ / bias at the current state, one narrowphase call */
void  or_dynamics(or_env* e, double* xpos, double* xquat, double* H, double* add, double* bias);
int   or_collide(int type1, const double* size1, const double* c1, const double* R1, int type2,
                 const double* size2, const double* c2, const double* R2, double mpr_tol, int mpr_it,
                 double* out);

/* fp64 state hand-off with the device's GmEnvState (gripper-mujoco_amd/csrc/gm_state.h) */
size_t or_state_size(void);
int   or_import_state(or_env* e, const void* gm_env_state);   /* 0 ok, <0 not a step boundary */
void  or_export_state(const or_env* e, void* gm_env_state);
/* n envs x one env-step from device-format states (updated in place), threaded */
int   or_batch_step(const gm_model* m, const gm_config* c, const gm_object* objects, int n_objects, int n,
                    void* states, const float* cont_actions, const int32_t* disc_actions, float* obs,
                    float* reward, uint8_t* done, int n_threads);
/* n envs x one substep with diagnostics from device-format states (updated in place) */
int   or_batch_substep(const gm_model* m, const gm_config* c, const gm_object* objects, int n_objects, int n,
                       void* states, int32_t* ncon, int32_t* nefc, double* contact, double* efc_force,
                       double* qacc, double* obj_wrench, int n_threads);

/* standalone pieces used by the golden-vector tests */
float  or_gauge_reading(const gm_model* m, const double* finger_q);   /* read_armadillo_gauge */
double or_minstd_next_canonical_float(uint32_t* state);               /* generate_canonical<float> */
double or_minstd_next_canonical_double(uint32_t* state);              /* generate_canonical<double> */
float  or_polyfit_eval(const double* X, const double* Y, int P, int order, double x);
void   or_gauge_points(const gm_model* m, const double* q, double* X, double* Y);
void   or_ring_trace(const float* adds, int n_adds, int n_reads, float* out);
uint32_t or_std_shuffle(uint32_t seed, int n, int32_t* out);     /* std::shuffle, minstd_rand0 */
int    or_box2d_overlaps(const double* a5, const double* b5, double gap);   /* Box2d::overlapsWith */
int    or_grip_step_sequence(const double* cmds, int n, double* out);  /* Gripper golden driver */
int    or_sample(int mode, const float* window_recent_first, int n_avail, int prev_steps,
                 int readings_per_step, float* out);                  /* Sensor::*_sample */
/* automatic calibration (find_highest_stable_timestep + calibrate_simulated_sensors) */
int    or_calibrate(const gm_model* m, const gm_config* c, const gm_object* objects, int n_objects, int what,
                    gm_calibration* out, double* trace_dt, uint8_t* trace_unstable, int max_trace);
/* time one bounded CPU sample: n_envs envs x n_steps env-steps of the benchmark workload
 * (mode 1: scripted grasp mix, 0: random actions; resets at done / max_episode_steps) */
double or_bench(const gm_model* m, const gm_config* c, const gm_object* objects, int n_objects,
                int n_envs, int n_steps, uint64_t seed, int n_threads, int mode, int max_episode_steps);

#ifdef __cplusplus
}
#endif
#endif
