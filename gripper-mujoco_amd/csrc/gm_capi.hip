// gm_capi.hip -- C ABI (include/gripper_mi355x.h) over the device kernels.
//
// Replaces the pybind11 MjClass boundary (src/bind.cpp:43-205).  A context owns
// one HIP stream and the device buffers of n_envs envs; every call is
// asynchronous on that stream except the host-buffer getters, which copy and
// synchronise.  No C++ exception crosses the ABI: failures return GM_E_* and
// leave a message for gm_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdlib>
#include <cstdio>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>
#include <mutex>

#include "gm_kernels.hip"
#include "gm_policy.hip"

// calibration translation unit (gm_calib.hip)
hipError_t gm_cal_launch_step(int n_seg, int n_envs, hipStream_t st, GmEnvState* states, const gm_model* m,
                              const gm_config* C, const GmTopo* T);
hipError_t gm_cal_launch_setup(hipStream_t st, GmEnvState* states, const double* dt, const int32_t* steps, double tip,
                               int n);
hipError_t gm_cal_launch_read(hipStream_t st, const GmEnvState* states, uint8_t* bad, int n);
hipError_t gm_cal_launch_gauge(int n_seg, hipStream_t st, const GmEnvState* states, const gm_model* m, const GmTopo* T,
                               int env, float* out);

struct gm_ctx {
  int device = 0;
  int n_envs = 0;
  long long env_offset = 0;
  int n_objects = 0;
  hipStream_t stream = nullptr;        // stream every launch of this ctx goes to
  hipStream_t own_stream = nullptr;    // the one gm_create made (destroyed with the ctx)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  bool timed = false;
  int last_launch_steps = 1;           // env-steps per env of the last timed launch
  gm_model model;
  gm_config cfg;
  GmTopo topo;
  // device buffers
  GmEnvState* d_state = nullptr;
  gm_model* d_model = nullptr;
  gm_config* d_cfg = nullptr;
  GmTopo* d_topo = nullptr;
  gm_object* d_objs = nullptr;
  double* d_eq = nullptr;
  float* d_obs = nullptr;              // d_obs, d_rew, d_done: one allocation (d_out), read back
  float* d_rew = nullptr;              // by gm_get_outputs in one copy through h_out (pinned)
  uint8_t* d_done = nullptr;
  void* d_out = nullptr;
  void* h_out = nullptr;
  size_t out_bytes = 0;
  float* d_act = nullptr;
  // host actions are staged through a pinned buffer so gm_set_action / gm_set_discrete_action
  // return without a stream synchronisation (stage_ev: the previous staging copy is done)
  void* h_stage = nullptr;
  size_t stage_bytes = 0;
  hipEvent_t stage_ev = nullptr;
  int32_t* d_dact = nullptr;
  uint8_t* d_mask = nullptr;
  // scratch of the force-measurement calls (gm_set_motor_target's targets and flags,
  // gm_get_sensor_si's readings): allocated once with the context, no per-call hipMalloc /
  // hipFree (a hipFree synchronises the whole device)
  void* d_scratch = nullptr;
  gm_spawn* d_spawn = nullptr;
  int32_t* d_order = nullptr;          // workgroup -> env dispatch order (cost-sorted)
  uint32_t* d_cost = nullptr;          // per-env cost of the last env-step (clocks / 64)
  // chunked env-step (gm_step_chunked_kernel): queue counters, per-XCD continuation rings,
  // per-env carry; chunk = substeps per chunk (0: the one-shot kernel)
  uint32_t* d_chunk_ctr = nullptr;
  uint64_t* d_chunk_ring = nullptr;
  GmChunkCarry* d_chunk_carry = nullptr;
  unsigned long long* d_chunk_st = nullptr;
  int chunk = 0, chunk_grid = 0, chunk_cap = 0, chunk_margin = 50, chunk_yields = 20, chunk_cmargin = 50;
  int chunk_steal = 1;                 // idle waves resume yielded envs of other XCDs (GM_CHUNK_STEAL=0: off)
  int chunk_prio = 1;                  // issue priority by predicted work left (GM_CHUNK_PRIO=0: off)
  // DUO workgroups (gm_step_kernel<CL, false, true>): two waves per env, the second running
  // the collider concurrently -- for batches small enough that wave slots are spare
  bool duo = false;
  gm_spawn_params* d_scene = nullptr;  // gm_set_scene_spawn parameters (NULL: plain spawn_object)
  int scene_tries = 0;
  GmSpawnRand spawn_rand{};            // gm_set_random_spawn (enable = 0: spawn tables)
  std::string err;
};

namespace {

int fail(gm_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}
#define HIPCHK(ctx, x)                                                               \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess)                                                            \
      return fail(ctx, GM_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_));    \
  } while (0)

bool nseg_supported(int n) {
  switch (n) {
#define X(N) case N:
    GM_NSEG_LIST
#undef X
    return true;
    default: return false;
  }
}
struct RolloutArgs {
  int steps, act_mode;
  uint64_t act_seed;
  float jitter;
  int max_ep;
  gm_episode_end* rec;
  // act_mode 2 (gm_policy_rollout): the packed network, its layout, eps per env-step
  const float* pparams = nullptr;
  GpNet pnet{};
  const float* peps = nullptr;
  uint64_t pdecision = 0;
};
hipError_t launch_step(gm_ctx* c, int grid, int n_envs, int mode, DebugOut dbg, const RolloutArgs* roll = nullptr) {
  // the full env-step (mode 0) runs in cost-sorted order and records each env's cost
  const int32_t* order = (mode == 0 && grid == c->n_envs) ? c->d_order : nullptr;
  uint32_t* cost = (mode == 0 && grid == c->n_envs) ? c->d_cost : nullptr;
  // the chunked work queue (gm_kernels.hip chunked_env_steps): one workgroup per resident
  // wave slot, each pulling env chunks until every env has finished
  const bool chunked = order && c->chunk > 0 && c->chunk_grid > 0 && dbg.phase == nullptr;
  GmChunkQ q{c->d_chunk_ctr, c->d_chunk_ring, c->d_chunk_carry, c->chunk_cap, chunked ? c->chunk : 0,
             c->chunk_margin, c->chunk_yields, c->chunk_cmargin, c->d_chunk_st};
  q.steal = c->chunk_steal;
  q.prio = c->chunk_prio;
  q.steps = 1;
  q.act_mode = -1;   // gm_step: one plain env-step per env (gm_rollout sets the rollout fields)
  if (roll && chunked) {
    q.steps = roll->steps;
    q.act_mode = roll->act_mode;
    q.act_seed = roll->act_seed;
    q.jitter = roll->jitter;
    q.max_ep = roll->max_ep;
    q.rec = roll->rec;
    q.eq = c->d_eq;
    q.objs = c->d_objs;
    q.n_objects = c->n_objects;
    q.scene = c->d_scene;
    q.scene_tries = c->scene_tries;
    q.sr = c->spawn_rand;
    q.sr.env_offset = c->env_offset;   // (the driver's global env ids even without random spawns)
    q.pparams = roll->pparams;
    q.pnet = roll->pnet;
    q.peps = roll->peps;
    q.pseed = roll->act_seed;
    q.pdecision = roll->pdecision;
  }
  if (chunked) grid = c->chunk_grid;
  // the env-step proper (not the settle, a diagnostic substep or a profiled step) on DUO
  // workgroups when the context chose them; the chunked grid was sized for that kernel
  const bool duo = c->duo && mode == 0;   // (a profiled step too: the owner wave's phase clocks)
  switch (c->model.n_seg) {
#define X(N)                                                                                                 \
  case N:                                                                                                    \
    if (duo)                                                                                                 \
      hipLaunchKernelGGL((gm_step_kernel<N + 2, false, true>), dim3(grid), dim3(2 * NT), 0, c->stream,        \
                         c->d_state, c->d_model, c->d_cfg, c->d_topo, c->d_obs, c->d_rew, c->d_done, n_envs,   \
                         mode, dbg, order, cost, q);                                                           \
    else                                                                                                     \
      hipLaunchKernelGGL((gm_step_kernel<N + 2, false>), dim3(grid), dim3(NT), 0, c->stream, c->d_state,      \
                         c->d_model, c->d_cfg, c->d_topo, c->d_obs, c->d_rew, c->d_done, n_envs, mode, dbg,    \
                         order, cost, q);                                                                      \
    return hipGetLastError();
    GM_NSEG_LIST
#undef X
    default: return hipErrorInvalidValue;
  }
}


int build_topo(const gm_model& m, GmTopo& T, std::string& err) {
  std::memset(&T, 0, sizeof(T));
  T.N = m.n_seg;
  T.CL = m.n_seg + 2;
  T.nbody = m.nbody; T.nv = m.nv; T.nq = m.nq; T.ngeom = m.ngeom; T.npair = m.npair; T.nlock = m.nlock;
  T.body_base = m.body_base; T.dof_base = m.dof_base;
  for (int f = 0; f < 3; f++) {
    T.dof_f0[f] = m.dof_pris[f];
    T.body_f0[f] = m.dof_body[m.dof_pris[f]];
    T.body_finger[f] = m.body_finger[f];
  }
  T.body_palm = m.body_palm; T.dof_palm = m.dof_palm;
  T.body_obj = m.body_obj; T.dof_obj = m.dof_obj; T.geom_obj = m.geom_obj;
  T.qadr_obj = m.jnt_qposadr[m.body_jnt[m.body_obj]];
  // verify the canonical tree layout the kernels index arithmetically
  for (int f = 0; f < 3; f++)
    for (int p = 1; p <= T.CL; p++) {
      int d = T.dof_f0[f] + p - 1, b = T.body_f0[f] + p - 1;
      if (m.dof_body[d] != b || m.body_group[b] != f) { err = "model is not the canonical gripper tree"; return GM_E_ARG; }
      int par = (p == 1) ? m.dof_base : d - 1;
      if (m.dof_parent[d] != par) { err = "unexpected dof parent"; return GM_E_ARG; }
    }
  if (m.npair > GM_MAX_PAIR || m.npair > NT * gm_pair_batches(T.CL) || m.nv > GM_MAX_DOF || T.qadr_obj != m.dof_obj) {
    err = "model exceeds kernel limits";
    return GM_E_RANGE;
  }
  for (int b = 0; b < GM_MAX_BODY; b++) { T.body_group[b] = -1; T.body_cpos[b] = 0; }
  for (int b = 0; b < m.nbody; b++) {
    T.body_group[b] = m.body_group[b];
    if (m.body_group[b] >= 0 && m.body_group[b] < 3) T.body_cpos[b] = b - T.body_f0[m.body_group[b]] + 1;
    else if (m.body_group[b] == GM_GRP_PALM) T.body_cpos[b] = 1;
  }
  for (int l = 0; l < 64; l++) T.lane_body[l] = -1;
  if (T.CL > 15) { err = "finger chain longer than a 16-lane DPP row"; return GM_E_RANGE; }
  for (int f = 0; f < 3; f++)
    for (int p = 1; p <= T.CL; p++) T.lane_body[16 * f + p] = T.body_f0[f] + p - 1;
  T.lane_base = 48;
  T.lane_body[48] = T.body_base;
  T.lane_body[49] = T.body_palm;
  T.lane_body[50] = T.body_obj;
  // per-dof constants: the engine-spec H~ diagonal additions and PD gains
  // (mj_step2 implicit damping / PD terms and luke::control gains, oracle.c ctrl_gains / step2)
  for (int d = 0; d < m.nv; d++) {
    const int b = m.dof_body[d], j = m.body_jnt[b];
    T.dof_body[d] = b;
    T.dof_grp[d] = m.body_group[b];
    T.dof_p[d] = (m.body_group[b] == GM_GRP_OBJECT) ? d - m.dof_obj : T.body_cpos[b];
    double kp = 0, kd = 0;
    int tgt = 0;
    for (int f = 0; f < 3; f++) {
      if (d == m.dof_pris[f]) { kp = m.kp_gripper[0]; kd = m.kd_gripper[0]; tgt = 1; }
      if (d == m.dof_rev[f]) { kp = m.kp_gripper[1]; kd = m.kd_gripper[1]; tgt = 2; }
    }
    if (d == m.dof_palm) { kp = m.kp_gripper[2]; kd = m.kd_gripper[2]; tgt = 3; }
    if (d == m.dof_base) { kp = m.kp_base[2]; kd = m.kd_base[2]; tgt = 4; }
    const bool free = m.jnt_type[j] == GM_JNT_FREE;
    // the constraint solve's matrix: M + armature under MuJoCo's actuator order (the PD
    // forces explicit, the joint damping implicit in the Euler step, integrate); with the
    // folded scheme also h (damping + kd) + h^2 kp.  Joint springs are explicit either way.
    const bool mj = m.mujoco_actuators != 0;
    double add = m.jnt_armature[j] + (mj ? 0.0 : m.timestep * (m.jnt_damping[j] + kd));
    if (!free && !mj) add += m.timestep * m.timestep * kp;
    T.dof_add[d] = add;
    T.dof_arm[d] = m.jnt_armature[j];
    T.dof_dsum[d] = mj ? 0.0 : m.jnt_damping[j] + kd;
    T.dof_ksum[d] = (free || mj) ? 0.0 : kp;
    T.dof_stiff[d] = free ? 0.0 : m.jnt_stiffness[j];
    T.dof_damp[d] = m.jnt_damping[j];
    T.dof_kp[d] = kp; T.dof_kd[d] = kd; T.dof_target[d] = tgt;
  }
  for (int g = 0; g < m.ngeom; g++) {
    int b = m.geom_body[g];
    T.geom_group[g] = (b == 0) ? -1 : T.body_group[b];
    if (T.geom_group[g] == GM_GRP_BASE) T.geom_group[g] = -1;
    T.geom_cpos[g] = T.body_cpos[b];
  }
  // flattened per-lane constants (GmTopo kl_* / dof_* / pr_* / lock_*): the same values
  // the kernels read through the model's index chains, resolved here once
  for (int l = 0; l < 64; l++) {
    const int b = T.lane_body[l];
    T.kl_type[l] = -1; T.kl_qadr[l] = 0;
    T.kl_grp[l] = (b >= 0) ? T.body_group[b] : -1;
    const bool chain = T.kl_grp[l] >= 0 && T.kl_grp[l] <= 3;
    T.kl_cpos[l] = chain ? T.body_cpos[b] : 0;
    for (int k = 0; k < 3; k++) { T.kl_pos[l][k] = 0; T.kl_axis[l][k] = 0; }
    T.kl_quat[l][0] = 1; T.kl_quat[l][1] = T.kl_quat[l][2] = T.kl_quat[l][3] = 0;
    if (b > 0) {
      for (int k = 0; k < 3; k++) T.kl_pos[l][k] = m.body_pos[b][k];
      for (int k = 0; k < 4; k++) T.kl_quat[l][k] = m.body_quat[b][k];
      const int j = m.body_jnt[b];
      if (j >= 0) {
        T.kl_type[l] = m.jnt_type[j];
        T.kl_qadr[l] = m.jnt_qposadr[j];
        for (int k = 0; k < 3; k++) T.kl_axis[l][k] = m.jnt_axis[j][k];
      }
    }
  }
  for (int d = 0; d < m.nv; d++) {
    const int j = m.body_jnt[m.dof_body[d]];
    T.dof_jtype[d] = m.jnt_type[j];
    T.dof_k[d] = d - m.jnt_dofadr[j];
    for (int k = 0; k < 3; k++) T.dof_axis[d][k] = m.jnt_axis[j][k];
  }
  for (int p = 0; p < m.npair; p++) {
    const int gs[2] = {m.pair_a[p], m.pair_b[p]};
    for (int s = 0; s < 2; s++) {
      const int g = gs[s];
      T.pr_g[p][s] = g;
      T.pr_type[p][s] = (g == m.geom_obj) ? -1 : m.geom_type[g];
      T.pr_body[p][s] = m.geom_body[g];
      for (int k = 0; k < 3; k++) { T.pr_pos[p][s][k] = m.geom_pos[g][k]; T.pr_size[p][s][k] = m.geom_size[g][k]; }
      for (int k = 0; k < 4; k++) T.pr_quat[p][s][k] = m.geom_quat[g][k];
      T.pr_rbound[p][s] = m.geom_rbound[g];
      T.pr_fric[p][s] = m.geom_friction[g];
    }
  }
  for (int k = 0; k < m.nlock; k++) {
    const int b = m.dof_body[m.lock_dof[k]];
    T.lock_grp[k] = T.body_group[b];
    T.lock_cpos[k] = T.body_cpos[b];
    T.lock_tran[k] = m.body_invweight0[b][0] + m.body_invweight0[m.body_parent[b]][0];
  }
  // per scan lane: the lane body's pairs with the object / the ground (oracle topo_init)
  T.lane_obj = 50;
  T.pair_gobj = -1;
  for (int l = 0; l < 64; l++)
    for (int s = 0; s < 2; s++) { T.lane_opair[l][s] = -1; T.lane_gpair[l][s] = -1; }
  for (int pr = 0; pr < m.npair; pr++) {
    const int a = m.pair_a[pr], bg = m.pair_b[pr];
    const bool with_obj = a == m.geom_obj || bg == m.geom_obj;
    const bool with_gnd = a == m.geom_ground || bg == m.geom_ground;
    if (with_obj && with_gnd) {
      if (T.pair_gobj >= 0) { err = "more than one object-ground pair"; return GM_E_RANGE; }
      T.pair_gobj = pr;
      continue;
    }
    if (!with_obj && !with_gnd) { err = "gripper self-collision pairs are not supported"; return GM_E_RANGE; }
    const int g = with_obj ? (a == m.geom_obj ? bg : a) : (a == m.geom_ground ? bg : a);
    const int b = m.geom_body[g];
    bool assigned = false;
    for (int l = 0; l < 64; l++) {
      if (T.lane_body[l] != b || l == T.lane_obj) continue;
      int32_t* slot = with_obj ? T.lane_opair[l] : T.lane_gpair[l];
      if (slot[0] < 0) slot[0] = pr;
      else if (slot[1] < 0) slot[1] = pr;
      else { err = "a body has more than two object (or ground) pairs"; return GM_E_RANGE; }
      assigned = true;
    }
    // the Newton Hessian composites reach a contact only through its gripper body's scan
    // lane: a pair on a body without one would be solved with an inconsistent Hessian
    if (!assigned) {
      err = "contact pair " + std::to_string(pr) + " is on body " + std::to_string(b) +
            ", which has no scan lane (fingers, palm); the solver cannot take it";
      return GM_E_RANGE;
    }
  }
  return GM_OK;
}

}  // namespace

namespace {
// the process-wide settle cache of gm_set_settle_cache (calibrate_reset's first_call)
std::mutex g_settle_mu;
bool g_settle_cache_on = false, g_settle_valid = false;
int g_settle_nseg = -1;
double g_settle_eq[GM_MAX_QPOS];
}  // namespace

extern "C" {

const char* gm_version(void) { return "gripper-mi355x 0.1 (gfx950, one-wave-per-env fused env-step)"; }

int gm_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int gm_create(const gm_model* model, const gm_config* cfg, const gm_object* objects, int n_objects,
              int n_envs, int env_offset, int device, uint64_t seed, gm_ctx** out) {
  if (!model || !cfg || !objects || !out || n_envs <= 0 || n_objects <= 0) return GM_E_ARG;
  *out = nullptr;
  gm_ctx* c = new gm_ctx();
  c->device = device;
  c->n_envs = n_envs;
  c->env_offset = env_offset;
  c->n_objects = n_objects;
  c->model = *model;
  c->cfg = *cfg;
  std::string err;
  int rc = build_topo(c->model, c->topo, err);
  if (rc != GM_OK) { fprintf(stderr, "gm_create: %s\n", err.c_str()); delete c; return rc; }
  if (!nseg_supported(c->model.n_seg)) {
    fprintf(stderr, "gm_create: n_seg=%d has no compiled step kernel (GM_NSEG_LIST)\n", c->model.n_seg);
    delete c;
    return GM_E_RANGE;
  }
  {
    const int CLm = c->model.n_seg + 2;
    if (c->model.nbody != 3 * CLm + 4 || c->model.nv != 3 * CLm + 8 || c->model.nq != c->model.nv + 1) {
      fprintf(stderr, "gm_create: model sizes (nbody %d, nv %d, nq %d) do not match the canonical tree for n_seg=%d\n",
              c->model.nbody, c->model.nv, c->model.nq, c->model.n_seg);
      delete c;
      return GM_E_RANGE;
    }
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device) {
    fprintf(stderr, "gm_create: no HIP device %d (found %d)\n", device, ndev);
    delete c;
    return GM_E_NOEXT;
  }
  *out = c;
  HIPCHK(c, hipSetDevice(device));
  HIPCHK(c, hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
  c->stream = c->own_stream;
  HIPCHK(c, hipEventCreate(&c->ev0));
  HIPCHK(c, hipEventCreate(&c->ev1));
  HIPCHK(c, hipEventCreateWithFlags(&c->stage_ev, hipEventDisableTiming));
  c->stage_bytes = std::max(sizeof(float) * (size_t)n_envs * GM_ACTION_CODE_COUNT, sizeof(int32_t) * (size_t)n_envs);
  HIPCHK(c, hipHostMalloc(&c->h_stage, c->stage_bytes, hipHostMallocDefault));
  HIPCHK(c, hipMalloc(&c->d_state, sizeof(GmEnvState) * (size_t)n_envs));
  HIPCHK(c, hipMalloc(&c->d_scratch, std::max(sizeof(double) * 3 * (size_t)n_envs + (size_t)n_envs + 16,
                                              sizeof(float) * 5 * (size_t)n_envs)));
  HIPCHK(c, hipMalloc(&c->d_model, sizeof(gm_model)));
  HIPCHK(c, hipMalloc(&c->d_cfg, sizeof(gm_config)));
  HIPCHK(c, hipMalloc(&c->d_topo, sizeof(GmTopo)));
  HIPCHK(c, hipMalloc(&c->d_objs, sizeof(gm_object) * (size_t)n_objects));
  HIPCHK(c, hipMalloc(&c->d_eq, sizeof(double) * GM_MAX_QPOS));
  {
    const size_t obs_b = sizeof(float) * (size_t)n_envs * (cfg->n_obs > 0 ? cfg->n_obs : 1);
    const size_t rew_b = sizeof(float) * (size_t)n_envs;
    c->out_bytes = obs_b + rew_b + (size_t)n_envs;
    HIPCHK(c, hipMalloc(&c->d_out, c->out_bytes));
    HIPCHK(c, hipHostMalloc(&c->h_out, c->out_bytes, hipHostMallocDefault));
    c->d_obs = static_cast<float*>(c->d_out);
    c->d_rew = reinterpret_cast<float*>(static_cast<char*>(c->d_out) + obs_b);
    c->d_done = reinterpret_cast<uint8_t*>(static_cast<char*>(c->d_out) + obs_b + rew_b);
  }
  HIPCHK(c, hipMalloc(&c->d_act, sizeof(float) * (size_t)n_envs * GM_ACTION_CODE_COUNT));
  HIPCHK(c, hipMalloc(&c->d_dact, sizeof(int32_t) * (size_t)n_envs));
  HIPCHK(c, hipMalloc(&c->d_mask, (size_t)n_envs));
  HIPCHK(c, hipMalloc(&c->d_spawn, sizeof(gm_spawn) * (size_t)n_envs));
  HIPCHK(c, hipMalloc(&c->d_order, sizeof(int32_t) * (size_t)n_envs));
  // two halves: [0, n) the costs the current launch is ordered and scheduled by (read-only
  // during it), [n, 2n) the costs it records; gm_dispatch_order_kernel moves them over
  HIPCHK(c, hipMalloc(&c->d_cost, sizeof(uint32_t) * 2 * (size_t)n_envs));
  HIPCHK(c, hipMemsetAsync(c->d_cost, 0, sizeof(uint32_t) * 2 * (size_t)n_envs, c->stream));
  {
    // chunked env-step: as many workgroups as wave slots are resident (occupancy query),
    // GM_CHUNK_SUBSTEPS substeps per preemption test (default 16; 0 selects the one-shot
    // kernel).  r05 sweep on the C3 workload (tools/rollout_probe.py): 8 / 16 / 24 / 32 give
    // 5.28 / 5.22 / 5.35 / 5.21 ms per env-step for 10-step rollouts, the per-step API the same
    // 5.74-5.76 ms at 8 and 16
    const char* ev = std::getenv("GM_CHUNK_SUBSTEPS");
    c->chunk = ev ? std::atoi(ev) : 16;
    if (const char* e2 = std::getenv("GM_CHUNK_MARGIN")) c->chunk_margin = std::atoi(e2);
    if (const char* e3 = std::getenv("GM_CHUNK_YIELDS")) c->chunk_yields = std::atoi(e3);
    if (const char* e4 = std::getenv("GM_CHUNK_CMARGIN")) c->chunk_cmargin = std::atoi(e4);
    if (const char* e6 = std::getenv("GM_CHUNK_STEAL")) c->chunk_steal = std::atoi(e6) != 0;
    if (const char* e7 = std::getenv("GM_CHUNK_PRIO")) c->chunk_prio = std::atoi(e7);
    int per_cu = 0, per_cu_duo = 0, n_cu = 0;
    switch (c->model.n_seg) {
#define X(N)                                                                                              \
  case N:                                                                                                 \
    HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, gm_step_kernel<N + 2, false>, NT, 0)); \
    HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_duo, (gm_step_kernel<N + 2, false, true>), \
                                                           2 * NT, 0));                                   \
    break;
      GM_NSEG_LIST
#undef X
      default: break;
    }
    HIPCHK(c, hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device));
    // DUO when every env gets its two waves resident at once (GM_DUO = 0 / 1 forces it off
    // / on): the helper wave then costs no env a slot
    const char* ed = std::getenv("GM_DUO");
    c->duo = ed ? std::atoi(ed) != 0 : (per_cu_duo > 0 && n_envs <= per_cu_duo * n_cu);
    c->chunk_grid = std::min(n_envs, (c->duo ? per_cu_duo : per_cu) * n_cu);
    // GM_CHUNK_GRID caps the persistent grid (tests: a small batch on fewer workgroups than
    // envs, so the work queue hands envs off between waves)
    if (const char* e5 = std::getenv("GM_CHUNK_GRID")) c->chunk_grid = std::max(1, std::min(c->chunk_grid, std::atoi(e5)));
    c->chunk_cap = n_envs + c->chunk_grid;
    HIPCHK(c, hipMalloc(&c->d_chunk_ctr, sizeof(uint32_t) * GM_CQ_ALLOC));
    HIPCHK(c, hipMemsetAsync(c->d_chunk_ctr, 0, sizeof(uint32_t) * GM_CQ_ALLOC, c->stream));
    // [0, 16) launch stats, then per workgroup its end of work, then per env its start and finish
    const size_t st_words = 16 + (size_t)c->chunk_grid + 2 * (size_t)n_envs;
    HIPCHK(c, hipMalloc(&c->d_chunk_st, sizeof(unsigned long long) * st_words));
    HIPCHK(c, hipMemsetAsync(c->d_chunk_st, 0, sizeof(unsigned long long) * st_words, c->stream));
    HIPCHK(c, hipMalloc(&c->d_chunk_ring, sizeof(uint64_t) * 8 * GM_CQ_NB * (size_t)c->chunk_cap));
    HIPCHK(c, hipMalloc(&c->d_chunk_carry, sizeof(GmChunkCarry) * (size_t)n_envs));
    HIPCHK(c, hipMemsetAsync(c->d_chunk_ring, 0, sizeof(uint64_t) * 8 * GM_CQ_NB * (size_t)c->chunk_cap, c->stream));
  }
  hipLaunchKernelGGL(gm_dispatch_order_kernel, dim3(1), dim3(1024), 0, c->stream, c->d_cost, c->d_order, n_envs,
                     c->d_chunk_ctr, c->d_chunk_st);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemsetAsync(c->d_state, 0, sizeof(GmEnvState) * (size_t)n_envs, c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_obs, 0, sizeof(float) * (size_t)n_envs * (cfg->n_obs > 0 ? cfg->n_obs : 1), c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_rew, 0, sizeof(float) * (size_t)n_envs, c->stream));
  HIPCHK(c, hipMemsetAsync(c->d_done, 0, (size_t)n_envs, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_model, &c->model, sizeof(gm_model), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_cfg, &c->cfg, sizeof(gm_config), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_topo, &c->topo, sizeof(GmTopo), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(c->d_objs, objects, sizeof(gm_object) * (size_t)n_objects, hipMemcpyHostToDevice, c->stream));
  // one-time calibrate_reset settle (myfunctions.cpp:1470-1505) on env 0 -- per context, or,
  // with gm_set_settle_cache(1), once per process as the reference's function-static
  // first_call does (myfunctions.cpp:1447): later contexts with the same joint count reuse
  // the cached settle's equilibrium whatever else changed; a context whose joint count
  // differs settles again and replaces the cache (the reference's changed-joint-count
  // check sets first_call = true and keeps the new settle, myfunctions.cpp:1453-1468)
  bool from_cache = false;
  {
    std::lock_guard<std::mutex> lk(g_settle_mu);
    if (g_settle_cache_on && g_settle_valid && g_settle_nseg == c->model.n_seg) {
      HIPCHK(c, hipMemcpyAsync(c->d_eq, g_settle_eq, sizeof(double) * GM_MAX_QPOS, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      from_cache = true;
    }
  }
  if (!from_cache) {
    hipLaunchKernelGGL(gm_settle_init_kernel, dim3(1), dim3(1), 0, c->stream, c->d_state, c->d_model, c->d_topo, c->d_objs);
    DebugOut dbg{nullptr, nullptr, nullptr, nullptr, nullptr};
    HIPCHK(c, launch_step(c, 1, 1, 1, dbg));
    HIPCHK(c, hipMemcpyAsync(c->d_eq, reinterpret_cast<char*>(c->d_state) + offsetof(GmEnvHot, qpos), sizeof(double) * GM_MAX_QPOS, hipMemcpyDeviceToDevice, c->stream));
    std::lock_guard<std::mutex> lk(g_settle_mu);
    if (g_settle_cache_on && (!g_settle_valid || g_settle_nseg != c->model.n_seg)) {
      HIPCHK(c, hipMemcpyAsync(g_settle_eq, c->d_eq, sizeof(double) * GM_MAX_QPOS, hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      g_settle_valid = true;
      g_settle_nseg = c->model.n_seg;
    }
  }
  int threads = 256, blocks = (n_envs + threads - 1) / threads;
  hipLaunchKernelGGL(gm_init_envs_kernel, dim3(blocks), dim3(threads), 0, c->stream, c->d_state, cfg->s.random_seed,
                     (long long)env_offset, n_envs, c->model.timestep);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GM_OK;
}

void gm_destroy(gm_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  (void)hipFree(c->d_state); (void)hipFree(c->d_model); (void)hipFree(c->d_cfg); (void)hipFree(c->d_topo); (void)hipFree(c->d_objs);
  if (c->h_stage) (void)hipHostFree(c->h_stage);
  if (c->h_out) (void)hipHostFree(c->h_out);
  if (c->stage_ev) (void)hipEventDestroy(c->stage_ev);
  (void)hipFree(c->d_eq); (void)hipFree(c->d_out); (void)hipFree(c->d_act);
  (void)hipFree(c->d_dact); (void)hipFree(c->d_mask); (void)hipFree(c->d_spawn); (void)hipFree(c->d_scratch);
  (void)hipFree(c->d_order); (void)hipFree(c->d_cost); (void)hipFree(c->d_scene);
  (void)hipFree(c->d_chunk_ctr); (void)hipFree(c->d_chunk_ring); (void)hipFree(c->d_chunk_carry);
  (void)hipFree(c->d_chunk_st);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

const char* gm_last_error(const gm_ctx* c) { return c ? c->err.c_str() : "null context"; }
int gm_n_envs(const gm_ctx* c) { return c ? c->n_envs : 0; }
int gm_n_obs(const gm_ctx* c) { return c ? c->cfg.n_obs : 0; }
int gm_n_actions(const gm_ctx* c) { return c ? c->cfg.n_actions : 0; }

int gm_update_config(gm_ctx* c, const gm_config* cfg) {
  if (!c || !cfg) return GM_E_ARG;
  if (cfg->n_obs != c->cfg.n_obs) return fail(c, GM_E_STATE, "n_obs changed: recreate the context");
  c->cfg = *cfg;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMemcpyAsync(c->d_cfg, &c->cfg, sizeof(gm_config), hipMemcpyHostToDevice, c->stream));
  return GM_OK;
}

int gm_reset(gm_ctx* c, const uint8_t* mask, const gm_spawn* spawn) {
  if (!c) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const uint8_t* dm = nullptr;
  const gm_spawn* ds = nullptr;
  if (mask) { HIPCHK(c, hipMemcpyAsync(c->d_mask, mask, (size_t)c->n_envs, hipMemcpyHostToDevice, c->stream)); dm = c->d_mask; }
  if (spawn) {
    HIPCHK(c, hipMemcpyAsync(c->d_spawn, spawn, sizeof(gm_spawn) * (size_t)c->n_envs, hipMemcpyHostToDevice, c->stream));
    ds = c->d_spawn;
  }
  // gm_reset_kernel: one 64-lane workgroup per env
  hipLaunchKernelGGL(gm_reset_kernel, dim3(c->n_envs), dim3(64), 0, c->stream, c->d_state, c->d_model, c->d_cfg,
                     c->d_topo, c->d_eq, dm, ds, c->d_objs, c->n_objects, c->n_envs, c->d_scene, c->scene_tries,
                     c->d_obs, c->spawn_rand);
  HIPCHK(c, hipGetLastError());
  if (mask || spawn) HIPCHK(c, hipStreamSynchronize(c->stream));   // host buffers may be reused
  return GM_OK;
}

int gm_spawn_object(gm_ctx* c, const uint8_t* mask, const gm_spawn* spawn) {
  if (!c || !spawn) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const uint8_t* dm = nullptr;
  if (mask) { HIPCHK(c, hipMemcpyAsync(c->d_mask, mask, (size_t)c->n_envs, hipMemcpyHostToDevice, c->stream)); dm = c->d_mask; }
  HIPCHK(c, hipMemcpyAsync(c->d_spawn, spawn, sizeof(gm_spawn) * (size_t)c->n_envs, hipMemcpyHostToDevice, c->stream));
  int threads = 64, blocks = (c->n_envs + threads - 1) / threads;
  hipLaunchKernelGGL(gm_spawn_kernel, dim3(blocks), dim3(threads), 0, c->stream, c->d_state, c->d_topo, dm,
                     c->d_spawn, c->d_objs, c->n_objects, c->n_envs);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GM_OK;
}

int gm_set_motor_target(gm_ctx* c, const uint8_t* mask, const double* xyz, int n_xyz, uint8_t* in_limits) {
  if (!c || !xyz || (n_xyz != 1 && n_xyz != c->n_envs)) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t n = (size_t)c->n_envs;
  const uint8_t* dm = nullptr;
  if (mask) { HIPCHK(c, hipMemcpyAsync(c->d_mask, mask, n, hipMemcpyHostToDevice, c->stream)); dm = c->d_mask; }
  double* d_xyz = static_cast<double*>(c->d_scratch);
  uint8_t* d_ok = reinterpret_cast<uint8_t*>(d_xyz + 3 * n);
  HIPCHK(c, hipMemcpyAsync(d_xyz, xyz, sizeof(double) * 3 * (size_t)n_xyz, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(d_ok, 1, n, c->stream));
  int threads = 64, blocks = (c->n_envs + threads - 1) / threads;
  hipLaunchKernelGGL(gm_motor_target_kernel, dim3(blocks), dim3(threads), 0, c->stream, c->d_state, dm, d_xyz,
                     n_xyz == c->n_envs ? 1 : 0, d_ok, c->n_envs);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && in_limits) e = hipMemcpyAsync(in_limits, d_ok, n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);   // xyz / in_limits: host arrays
  HIPCHK(c, e);
  return GM_OK;
}

int gm_get_sensor_si(gm_ctx* c, float* out) {
  if (!c || !out) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const size_t n = (size_t)c->n_envs;
  float* d_out = static_cast<float*>(c->d_scratch);
  int threads = 64, blocks = (c->n_envs + threads - 1) / threads;
  hipLaunchKernelGGL(gm_sensor_si_kernel, dim3(blocks), dim3(threads), 0, c->stream, c->d_state, d_out, c->n_envs);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, sizeof(float) * 5 * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  HIPCHK(c, e);
  return GM_OK;
}

int gm_set_action(gm_ctx* c, const float* actions, int on_device) {
  if (!c || !actions) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const float* da = actions;
  if (!on_device) {
    const size_t bytes = sizeof(float) * (size_t)c->n_envs * c->cfg.n_actions;
    HIPCHK(c, hipEventSynchronize(c->stage_ev));   // the last staging copy has left the buffer
    std::memcpy(c->h_stage, actions, bytes);
    HIPCHK(c, hipMemcpyAsync(c->d_act, c->h_stage, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipEventRecord(c->stage_ev, c->stream));
    da = c->d_act;
  }
  int threads = 64, blocks = (c->n_envs + threads - 1) / threads;
  hipLaunchKernelGGL(gm_action_kernel, dim3(blocks), dim3(threads), 0, c->stream, c->d_state, c->d_model, c->d_cfg,
                     da, (const int32_t*)nullptr, c->n_envs);
  HIPCHK(c, hipGetLastError());
  return GM_OK;
}

int gm_set_discrete_action(gm_ctx* c, const int32_t* actions, int on_device) {
  if (!c || !actions) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const int32_t* da = actions;
  if (!on_device) {
    const size_t bytes = sizeof(int32_t) * (size_t)c->n_envs;
    HIPCHK(c, hipEventSynchronize(c->stage_ev));
    std::memcpy(c->h_stage, actions, bytes);
    HIPCHK(c, hipMemcpyAsync(c->d_dact, c->h_stage, bytes, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipEventRecord(c->stage_ev, c->stream));
    da = c->d_dact;
  }
  int threads = 64, blocks = (c->n_envs + threads - 1) / threads;
  hipLaunchKernelGGL(gm_action_kernel, dim3(blocks), dim3(threads), 0, c->stream, c->d_state, c->d_model, c->d_cfg,
                     (const float*)nullptr, da, c->n_envs);
  HIPCHK(c, hipGetLastError());
  return GM_OK;
}

static bool spawn_grid_ok(const gm_spawn_params& p) {
  if (!(p.xy_increment > 0) || !(p.rot_increment > 0) || p.xrange < 0 || p.yrange < 0 || p.rotrange < 0) return false;
  const double nx = ((2 * p.xrange) / p.xy_increment) + 1, ny = ((2 * p.yrange) / p.xy_increment) + 1;
  const double nr = ((2 * p.rotrange) / p.rot_increment) + 1;
  return nx * ny < GM_SPAWN_MAX_XY + 1 && (int)nx * (int)ny <= GM_SPAWN_MAX_XY && nr < GM_SPAWN_MAX_ROT + 1;
}

int gm_spawn_into_scene(gm_ctx* c, const uint8_t* mask, const gm_spawn_params* params, int n_params, uint8_t* ok) {
  if (!c || !params || (n_params != 1 && n_params != c->n_envs)) return fail(c, GM_E_ARG, "gm_spawn_into_scene: params must hold 1 or n_envs entries");
  for (int i = 0; i < n_params; i++)
    if (!spawn_grid_ok(params[i]))
      return fail(c, GM_E_ARG, "gm_spawn_into_scene: spawn grid empty or larger than GM_SPAWN_MAX_XY / GM_SPAWN_MAX_ROT");
  HIPCHK(c, hipSetDevice(c->device));
  gm_spawn_params* dp = nullptr;
  uint8_t* dok = nullptr;
  HIPCHK(c, hipMalloc(&dp, sizeof(gm_spawn_params) * (size_t)n_params));
  HIPCHK(c, hipMalloc(&dok, (size_t)c->n_envs));
  HIPCHK(c, hipMemcpyAsync(dp, params, sizeof(gm_spawn_params) * (size_t)n_params, hipMemcpyHostToDevice, c->stream));
  const uint8_t* dm = nullptr;
  if (mask) { HIPCHK(c, hipMemcpyAsync(c->d_mask, mask, (size_t)c->n_envs, hipMemcpyHostToDevice, c->stream)); dm = c->d_mask; }
  int threads = 64, blocks = (c->n_envs + threads - 1) / threads;
  hipLaunchKernelGGL(gm_spawn_into_scene_kernel, dim3(blocks), dim3(threads), 0, c->stream, c->d_state, c->d_model,
                     c->d_topo, c->d_objs, c->n_objects, dm, dp, n_params, dok, c->n_envs);
  HIPCHK(c, hipGetLastError());
  if (ok) HIPCHK(c, hipMemcpyAsync(ok, dok, (size_t)c->n_envs, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  (void)hipFree(dp);
  (void)hipFree(dok);
  return GM_OK;
}

int gm_set_scene_spawn(gm_ctx* c, const gm_spawn_params* params, int max_tries) {
  if (!c) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  if (!params) { c->scene_tries = 0; HIPCHK(c, hipStreamSynchronize(c->stream)); (void)hipFree(c->d_scene); c->d_scene = nullptr; return GM_OK; }
  if (max_tries < 1 || !spawn_grid_ok(*params)) return fail(c, GM_E_ARG, "gm_set_scene_spawn: max_tries < 1 or bad spawn grid");
  if (!c->d_scene) HIPCHK(c, hipMalloc(&c->d_scene, sizeof(gm_spawn_params)));
  HIPCHK(c, hipMemcpyAsync(c->d_scene, params, sizeof(gm_spawn_params), hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->scene_tries = max_tries;
  return GM_OK;
}

int gm_scripted_actions(gm_ctx* c, uint64_t seed, float jitter, float* out, int on_device) {
  if (!c || !out) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  float* d = on_device ? out : c->d_act;
  int threads = 64, blocks = (c->n_envs + threads - 1) / threads;
  hipLaunchKernelGGL(gm_scripted_action_kernel, dim3(blocks), dim3(threads), 0, c->stream, c->d_state, c->d_cfg, d,
                     c->n_envs, seed, (long long)c->env_offset, jitter);
  HIPCHK(c, hipGetLastError());
  if (!on_device) {
    HIPCHK(c, hipMemcpyAsync(out, d, sizeof(float) * (size_t)c->n_envs * c->cfg.n_actions, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return GM_OK;
}

int gm_program_actions(gm_ctx* c, uint64_t seed, float jitter, int mode, float* out, int on_device) {
  if (!c || !out || (mode != 3 && mode != 4)) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  float* d = on_device ? out : c->d_act;
  int threads = 64, blocks = (c->n_envs + threads - 1) / threads;
  hipLaunchKernelGGL(gm_program_action_kernel, dim3(blocks), dim3(threads), 0, c->stream, c->d_state, c->d_model,
                     c->d_cfg, d, c->n_envs, seed, (long long)c->env_offset, jitter, mode);
  HIPCHK(c, hipGetLastError());
  if (!on_device) {
    HIPCHK(c, hipMemcpyAsync(out, d, sizeof(float) * (size_t)c->n_envs * c->cfg.n_actions, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return GM_OK;
}

int gm_random_actions(gm_ctx* c, uint64_t seed, float* out, int on_device) {
  if (!c || !out) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  float* d = on_device ? out : c->d_act;
  int threads = 64, blocks = (c->n_envs + threads - 1) / threads;
  hipLaunchKernelGGL(gm_random_action_kernel, dim3(blocks), dim3(threads), 0, c->stream, c->d_state, c->d_cfg, d,
                     c->n_envs, seed, (long long)c->env_offset);
  HIPCHK(c, hipGetLastError());
  if (!on_device) {
    HIPCHK(c, hipMemcpyAsync(out, d, sizeof(float) * (size_t)c->n_envs * c->cfg.n_actions, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  return GM_OK;
}

// the persistent rollout launch (gm_rollout, gm_policy_rollout) and the next launch's order
static int rollout_launch(gm_ctx* c, const RolloutArgs& ra) {
  DebugOut dbg{nullptr, nullptr, nullptr, nullptr, nullptr};
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  HIPCHK(c, launch_step(c, c->n_envs, c->n_envs, 0, dbg, &ra));
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  hipLaunchKernelGGL(gm_dispatch_order_kernel, dim3(1), dim3(1024), 0, c->stream, c->d_cost, c->d_order, c->n_envs,
                     c->d_chunk_ctr, c->d_chunk_st);
  HIPCHK(c, hipGetLastError());
  c->timed = true;
  c->last_launch_steps = ra.steps;
  return GM_OK;
}

int gm_rollout(gm_ctx* c, int n_steps, const gm_rollout_params* p, gm_episode_end* records) {
  if (!c || !p || n_steps < 1 ||
      (p->action_mode != 0 && p->action_mode != 1 && p->action_mode != 3 && p->action_mode != 4))
    return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  if (c->chunk > 0 && c->chunk_grid > 0) {
    // one persistent launch: every env runs its n_steps env-steps back to back
    const RolloutArgs ra{n_steps, p->action_mode, p->seed, p->jitter, p->max_episode_steps, records};
    return rollout_launch(c, ra);
  }
  // the one-shot kernel (GM_CHUNK_SUBSTEPS=0): the same sequence as per-step launches
  for (int k = 0; k < n_steps; k++) {
    int rc = p->action_mode == 0 ? gm_scripted_actions(c, p->seed, p->jitter, c->d_act, 1)
             : p->action_mode == 1 ? gm_random_actions(c, p->seed, c->d_act, 1)
                                   : gm_program_actions(c, p->seed, p->jitter, p->action_mode, c->d_act, 1);
    if (rc == GM_OK) rc = gm_set_action(c, c->d_act, 1);
    if (rc == GM_OK) rc = gm_step(c);
    if (rc == GM_OK) rc = gm_autoreset_episodes(c, p->max_episode_steps, nullptr, 1, nullptr,
                                                records ? records + (size_t)k * c->n_envs : nullptr);
    if (rc != GM_OK) return rc;
  }
  return GM_OK;
}

int gm_set_random_spawn(gm_ctx* c, int enable, uint64_t seed, int position_noise_mm, int rotation_noise_deg) {
  if (!c) return GM_E_ARG;
  if (position_noise_mm < 0 || rotation_noise_deg < 0) return fail(c, GM_E_ARG, "gm_set_random_spawn: negative noise");
  c->spawn_rand.enable = enable ? 1 : 0;
  c->spawn_rand.seed = seed;
  c->spawn_rand.position_noise_mm = position_noise_mm;
  c->spawn_rand.rotation_noise_deg = rotation_noise_deg;
  c->spawn_rand.env_offset = c->env_offset;
  return GM_OK;
}

void gm_set_settle_cache(int on) {
  std::lock_guard<std::mutex> lk(g_settle_mu);
  g_settle_cache_on = on != 0;
  g_settle_valid = false;        // first_call = true: the next context settles and is kept
}

// ---------------------------------------------------------------- calibration
namespace {
uint32_t fbits(float x) { uint32_t u; std::memcpy(&u, &x, 4); return u; }

// calc_yield_point_load (myfunctions.cpp:3587-3595), float where the reference is float
float yield_point_load(const gm_model& m) {
  const double I = (m.finger_width * std::pow(m.finger_thickness, 3)) / 12.0;
  const float M_max = (m.yield_stress * I) / (0.5 * m.finger_thickness);
  const float F_max = M_max / m.finger_length;
  return F_max;
}

struct CalCtx {
  gm_ctx* c = nullptr;
  int nb = 0;
  double* d_dt = nullptr;
  int32_t* d_steps = nullptr;
  uint8_t* d_bad = nullptr;
  float* d_gauge = nullptr;
  std::vector<gm_spawn> spawn;
  ~CalCtx() {
    if (c) { (void)hipFree(d_dt); (void)hipFree(d_steps); (void)hipFree(d_bad); (void)hipFree(d_gauge); gm_destroy(c); }
  }
  // reset the first n envs (object 0 at the origin, as MjClass::reset leaves the scene),
  // give env i timestep dt[i], steps[i] substeps and the tip load, run them, read BADQACC
  int run(const std::vector<double>& dt, const std::vector<int32_t>& steps, double tip, std::vector<uint8_t>& bad,
          bool reset = true, int32_t* ran0 = nullptr) {
    const int n = (int)dt.size();
    if (n == 0) return GM_OK;
    if (reset) {
      std::vector<uint8_t> mask(nb, 0);
      for (int i = 0; i < n; i++) mask[i] = 1;
      int rc = gm_reset(c, mask.data(), spawn.data());
      if (rc != GM_OK) return rc;
    }
    HIPCHK(c, hipMemcpyAsync(d_dt, dt.data(), sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipMemcpyAsync(d_steps, steps.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, gm_cal_launch_setup(c->stream, c->d_state, d_dt, d_steps, tip, n));
    HIPCHK(c, gm_cal_launch_step(c->model.n_seg, n, c->stream, c->d_state, c->d_model, c->d_cfg, c->d_topo));
    HIPCHK(c, gm_cal_launch_read(c->stream, c->d_state, d_bad, n));
    bad.assign(n, 0);
    HIPCHK(c, hipMemcpyAsync(bad.data(), d_bad, n, hipMemcpyDeviceToHost, c->stream));
    if (ran0)   // substeps env 0 made (GmEnvState::cal_steps after the run)
      HIPCHK(c, hipMemcpyAsync(ran0, reinterpret_cast<char*>(c->d_state) + offsetof(GmEnvHot, cal_steps), sizeof(int32_t),
                               hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return GM_OK;
  }
};
}  // namespace

int gm_calibrate(const gm_model* model, const gm_config* cfg, const gm_object* objects, int n_objects, int device,
                 int what, gm_calibration* out, double* trace_dt, uint8_t* trace_unstable, int max_trace) {
  if (!model || !cfg || !objects || !out || n_objects <= 0) return GM_E_ARG;
  std::memset(out, 0, sizeof(*out));
  gm_config cc = *cfg;
  cc.s.base_position_noise = 0;          // calibration runs from the same reset pose
  CalCtx k;
  k.nb = 64;
  int rc = gm_create(model, &cc, objects, n_objects, k.nb, 0, device, 0, &k.c);
  if (rc != GM_OK) return rc;
  gm_ctx* c = k.c;
  HIPCHK(c, hipMalloc(&k.d_dt, sizeof(double) * k.nb));
  HIPCHK(c, hipMalloc(&k.d_steps, sizeof(int32_t) * k.nb));
  HIPCHK(c, hipMalloc(&k.d_bad, k.nb));
  HIPCHK(c, hipMalloc(&k.d_gauge, sizeof(float)));
  k.spawn.assign(k.nb, gm_spawn{0, 0.0, 0.0, 0.0});

  double timestep = model->timestep;
  if (what & GM_CAL_TIMESTEP) {
    // find_highest_stable_timestep (mjclass.cpp:4745-4854) replayed over batched results:
    // unknown candidates along the predicted path (coarse: stable, fine: unstable) are
    // simulated together, one env each, then the reference's sequence is replayed
    const float coarse_increment = 0.5e-3f, fine_increment = 50e-6f, start_value = 1.0e-3f;
    const float test_time = 1.0f, max_allowable_timestep = 20.0e-3f, tune_param = 1.0f;
    std::map<uint32_t, uint8_t> memo;
    std::vector<std::pair<float, uint8_t>> trace;
    float found = 0;
    for (int round = 0; round < 1000; round++) {
      std::vector<float> unknown;
      trace.clear();
      float next = start_value;
      bool coarse_pass = true;
      int status = 1;   // 0 done, -1 no stable timestep, 1 need evaluations
      for (int guard = 0; guard < 100000; guard++) {
        uint8_t unstable;
        auto it = memo.find(fbits(next));
        if (it != memo.end()) unstable = it->second;
        else {
          unknown.push_back(next);
          if ((int)unknown.size() >= k.nb) break;
          unstable = coarse_pass ? 0 : 1;
        }
        trace.push_back({next, unstable});
        if (unstable) { if (coarse_pass) coarse_pass = false; next -= fine_increment; }
        else { if (coarse_pass) next += coarse_increment; else { status = 0; found = next; break; } }
        if (next < fine_increment) { status = -1; break; }
        if (next > max_allowable_timestep) { next = max_allowable_timestep; coarse_pass = false; }
      }
      if (unknown.empty()) {
        if (status == -1) {
          fprintf(stderr, "gm_calibrate: no stable timestep found for the simulation\n");
          return GM_E_RANGE;
        }
        if (status == 0) break;
      }
      std::vector<double> dts(unknown.size());
      std::vector<int32_t> steps(unknown.size());
      for (size_t i = 0; i < unknown.size(); i++) {
        dts[i] = unknown[i];
        steps[i] = (int32_t)((test_time / unknown[i]) + 1);
      }
      std::vector<uint8_t> bad;
      rc = k.run(dts, steps, 0.0, bad);
      if (rc != GM_OK) return rc;
      for (size_t i = 0; i < unknown.size(); i++) memo[fbits(unknown[i])] = bad[i];
    }
    float factor;
    if (found <= 3.0e-3) factor = tune_param * 0.8;
    else if (found < 5.0e-3) factor = tune_param * 0.75;
    else if (found < 10.0e-3) factor = tune_param * 0.65;
    else factor = tune_param * 0.65;
    float final_timestep = found * factor;
    final_timestep = (float)((int)(final_timestep * 1e6) * 1e-6);
    out->search_timestep = found;
    out->n_tested = (int32_t)trace.size();
    for (int i = 0; i < (int)trace.size() && i < max_trace; i++) {
      if (trace_dt) trace_dt[i] = trace[i].first;
      if (trace_unstable) trace_unstable[i] = trace[i].second;
    }
    timestep = final_timestep;
  }
  out->timestep = timestep;
  if (what & GM_CAL_GAUGES) {
    // calibrate_simulated_sensors (mjclass.cpp:4643-4676): 0.3 s settle (wrist Z offset
    // from userdata[2], never written: 0), then validate_curve_under_force
    // (mjclass.cpp:4023-4105) with the saturation tip load for 50 s, 0.8x timestep retries
    const float yield = yield_point_load(*model);
    const float bend_gauge_normalise = cc.s.saturation_yield_factor * yield;
    double tsd = timestep;                 // s_.mujoco_timestep (double in simsettings.h:29)
    const float settle_time = 0.3f;
    std::vector<uint8_t> bad;
    rc = k.run({tsd}, {(int32_t)(settle_time / tsd)}, 0.0, bad);
    if (rc != GM_OK) return rc;
    const float time_to_settle = 50;
    const int steps_to_make = (int)(time_to_settle / tsd);
    int repeats_done = 1;
    bool first = true;
    const bool ref_retry = (what & GM_CAL_REFERENCE_RETRY) != 0;
    int left = steps_to_make;            // the reference's loop index resumes after a retry
    double tip = (double)bend_gauge_normalise;
    while (true) {
      int32_t ran = 0;
      rc = k.run({tsd}, {ref_retry ? left : steps_to_make}, tip, bad, !first, &ran);
      if (rc != GM_OK) return rc;
      first = false;
      if (bad[0]) {
        tsd *= 0.8;
        repeats_done += 1;
        if (repeats_done > 5) {
          fprintf(stderr, "gm_calibrate: curve validation unstable\n");
          return GM_E_RANGE;
        }
        if (ref_retry) {
          // reset() wiped the segment forces; `continue` resumes the step loop after the
          // unstable step, at the new timestep, unloaded
          tip = 0.0;
          left -= ran;
          if (left <= 0) {   // the unstable step was the last: only the reset remains
            rc = k.run({tsd}, {0}, 0.0, bad, true);
            if (rc != GM_OK) return rc;
            break;
          }
        }
        continue;
      }
      break;
    }
    HIPCHK(c, gm_cal_launch_gauge(c->model.n_seg, c->stream, c->d_state, c->d_model, c->d_topo, 0, k.d_gauge));
    float normalise = 0;
    HIPCHK(c, hipMemcpyAsync(&normalise, k.d_gauge, sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    out->yield_load = yield;
    out->bend_gauge_normalise = bend_gauge_normalise;
    out->bending_normalise = normalise;
    out->sim_gauge_raw_to_N_factor = bend_gauge_normalise / normalise;
    out->wrist_Z_offset = 0.0f;
    out->gauge_retries = repeats_done - 1;
    out->timestep = tsd;
  }
  out->sim_steps_per_action = (int32_t)std::ceil(cc.s.time_for_action / out->timestep);
  return GM_OK;
}

int gm_step(gm_ctx* c) {
  if (!c) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  DebugOut dbg{nullptr, nullptr, nullptr, nullptr, nullptr};
  HIPCHK(c, hipEventRecord(c->ev0, c->stream));
  HIPCHK(c, launch_step(c, c->n_envs, c->n_envs, 0, dbg));
  HIPCHK(c, hipEventRecord(c->ev1, c->stream));
  hipLaunchKernelGGL(gm_dispatch_order_kernel, dim3(1), dim3(1024), 0, c->stream, c->d_cost, c->d_order, c->n_envs,
                     c->d_chunk_ctr, c->d_chunk_st);
  HIPCHK(c, hipGetLastError());
  c->timed = true;
  c->last_launch_steps = 1;
  return GM_OK;
}

int gm_chunk_claim_waits(gm_ctx* c, uint32_t* out2) {
  if (!c || !out2) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  uint32_t w[2];
  HIPCHK(c, hipMemcpyAsync(w, c->d_chunk_ctr + GM_CQ_LAST + 37, sizeof(w), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  out2[0] = w[0]; out2[1] = w[1];
  return GM_OK;
}

int gm_chunk_job_stats(gm_ctx* c, uint32_t* clk, int32_t* yields) {
  if (!c || (!clk && !yields)) return GM_E_ARG;
  if (!c->d_chunk_carry) return GM_E_STATE;
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<GmChunkCarry> h((size_t)c->n_envs);
  HIPCHK(c, hipMemcpyAsync(h.data(), c->d_chunk_carry, sizeof(GmChunkCarry) * h.size(), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int e = 0; e < c->n_envs; e++) {
    if (clk) clk[e] = h[(size_t)e].clk;
    if (yields) yields[e] = h[(size_t)e].job_yields;
  }
  return GM_OK;
}

int gm_chunk_stats(gm_ctx* c, uint32_t* out, uint64_t* times) {
  if (!c || !out) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  uint32_t w[37];
  HIPCHK(c, hipMemcpyAsync(w, c->d_chunk_ctr + GM_CQ_LAST, sizeof(w), hipMemcpyDeviceToHost, c->stream));
  if (times) HIPCHK(c, hipMemcpyAsync(times, c->d_chunk_st + 8, sizeof(uint64_t) * 5, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  out[0] = std::min<uint32_t>(w[0], (uint32_t)c->n_envs);
  out[1] = w[32]; out[2] = w[33]; out[3] = w[34];
  out[4] = (uint32_t)c->chunk; out[5] = (uint32_t)c->chunk_grid;
  out[6] = w[36];
  return GM_OK;
}

int gm_chunk_timeline(gm_ctx* c, uint64_t* out, int max_out) {
  if (!c || !out || max_out < 0) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const int n = std::min(max_out, c->chunk_grid + 2 * c->n_envs);
  HIPCHK(c, hipMemcpyAsync(out, c->d_chunk_st + 16, sizeof(uint64_t) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return n;
}

int gm_dispatch_info(const gm_ctx* c, int32_t* out) {
  if (!c || !out) return GM_E_ARG;
  out[0] = c->chunk; out[1] = c->chunk_grid; out[2] = c->duo ? 2 : 1; out[3] = c->last_launch_steps;
  return GM_OK;
}

int gm_last_step_ms(gm_ctx* c, float* ms) {
  if (!c || !ms || !c->timed) return GM_E_STATE;
  HIPCHK(c, hipEventSynchronize(c->ev1));
  HIPCHK(c, hipEventElapsedTime(ms, c->ev0, c->ev1));
  return GM_OK;
}

int gm_get_obs(gm_ctx* c, float* out, int on_device) {
  if (!c || !out) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  size_t bytes = sizeof(float) * (size_t)c->n_envs * c->cfg.n_obs;
  HIPCHK(c, hipMemcpyAsync(out, c->d_obs, bytes, on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GM_OK;
}

int gm_get_outputs(gm_ctx* c, float* obs, float* reward, uint8_t* done) {
  if (!c || !obs || !reward || !done) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  // one copy of the contiguous obs / reward / done block into pinned memory (one DMA, no
  // pageable staging), then the three host copies
  HIPCHK(c, hipMemcpyAsync(c->h_out, c->d_out, c->out_bytes, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const char* h = static_cast<const char*>(c->h_out);
  const size_t obs_b = sizeof(float) * (size_t)c->n_envs * c->cfg.n_obs;
  const size_t off_rew = reinterpret_cast<const char*>(c->d_rew) - static_cast<const char*>(c->d_out);
  const size_t off_done = reinterpret_cast<const char*>(c->d_done) - static_cast<const char*>(c->d_out);
  std::memcpy(obs, h, obs_b);
  std::memcpy(reward, h + off_rew, sizeof(float) * (size_t)c->n_envs);
  std::memcpy(done, h + off_done, (size_t)c->n_envs);
  return GM_OK;
}

int gm_get_reward_done(gm_ctx* c, float* reward, uint8_t* done, int on_device) {
  if (!c) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  hipMemcpyKind k = on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  if (reward) HIPCHK(c, hipMemcpyAsync(reward, c->d_rew, sizeof(float) * (size_t)c->n_envs, k, c->stream));
  if (done) HIPCHK(c, hipMemcpyAsync(done, c->d_done, (size_t)c->n_envs, k, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GM_OK;
}

static int fetch_states(gm_ctx* c, std::vector<GmEnvState>& h) {
  h.resize(c->n_envs);
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMemcpyAsync(h.data(), c->d_state, sizeof(GmEnvState) * (size_t)c->n_envs, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GM_OK;
}

int gm_get_event_rows(gm_ctx* c, int32_t* rows, int32_t* absc, float* lastv) {
  if (!c) return GM_E_ARG;
  std::vector<GmEnvState> h;
  int rc = fetch_states(c, h);
  if (rc) return rc;
  const int W = GM_N_BINARY + GM_N_LINEAR;
  for (int e = 0; e < c->n_envs; e++) {
    for (int k = 0; k < GM_N_BINARY; k++) {
      if (rows) rows[e * W + k] = h[e].bev_row[k];
      if (absc) absc[e * W + k] = h[e].bev_abs[k];
      if (lastv) lastv[e * W + k] = (float)h[e].bev_last[k];
    }
    for (int k = 0; k < GM_N_LINEAR; k++) {
      if (rows) rows[e * W + GM_N_BINARY + k] = h[e].lev_row[k];
      if (absc) absc[e * W + GM_N_BINARY + k] = h[e].lev_abs[k];
      if (lastv) lastv[e * W + GM_N_BINARY + k] = h[e].lev_last[k];
    }
  }
  return GM_OK;
}

int gm_get_state(gm_ctx* c, double* qpos, double* qvel, double* time) {
  if (!c) return GM_E_ARG;
  std::vector<GmEnvState> h;
  int rc = fetch_states(c, h);
  if (rc) return rc;
  for (int e = 0; e < c->n_envs; e++) {
    if (qpos) for (int i = 0; i < c->model.nq; i++) qpos[(size_t)e * c->model.nq + i] = h[e].qpos[i];
    if (qvel) for (int i = 0; i < c->model.nv; i++) qvel[(size_t)e * c->model.nv + i] = h[e].qvel[i];
    if (time) time[e] = h[e].time;
  }
  return GM_OK;
}

int gm_set_state(gm_ctx* c, const double* qpos, const double* qvel) {
  if (!c) return GM_E_ARG;
  std::vector<GmEnvState> h;
  int rc = fetch_states(c, h);
  if (rc) return rc;
  for (int e = 0; e < c->n_envs; e++) {
    if (qpos) for (int i = 0; i < c->model.nq; i++) h[e].qpos[i] = qpos[(size_t)e * c->model.nq + i];
    if (qvel) for (int i = 0; i < c->model.nv; i++) h[e].qvel[i] = qvel[(size_t)e * c->model.nv + i];
  }
  HIPCHK(c, hipMemcpyAsync(c->d_state, h.data(), sizeof(GmEnvState) * (size_t)c->n_envs, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GM_OK;
}

int64_t gm_env_state_size(void) { return (int64_t)sizeof(GmEnvState); }

int gm_get_env_states(gm_ctx* c, void* out) {
  if (!c || !out) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMemcpyAsync(out, c->d_state, sizeof(GmEnvState) * (size_t)c->n_envs, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GM_OK;
}

int gm_set_env_states(gm_ctx* c, const void* in) {
  if (!c || !in) return GM_E_ARG;
  const GmEnvState* h = (const GmEnvState*)in;
  // every field the kernels use as an index or a flag (a bad ring index would address
  // outside the env's sensor windows)
  for (int e = 0; e < c->n_envs; e++) {
    const GmEnvState& r = h[e];
    bool ok = r.obj_index >= 0 && r.obj_index < c->n_objects && r.extra_substeps >= 0 && r.cal_steps >= 0 &&
              r.num_action_steps >= 0 && (r.done == 0 || r.done == 1) &&
              (r.obj_type == GM_GEOM_BOX || r.obj_type == GM_GEOM_CYLINDER || r.obj_type == GM_GEOM_SPHERE);
    for (int st = 0; st < GM_NSTREAM; st++) ok = ok && r.ring_i[st] >= -1 && r.ring_i[st] < GM_RING;
    for (int k = 0; k < GM_MAX_LOCK; k++) ok = ok && (r.lock_active[k] == 0 || r.lock_active[k] == 1);
    if (!ok) return fail(c, GM_E_ARG, "gm_set_env_states: env " + std::to_string(e) + " is not a valid state");
  }
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMemcpyAsync(c->d_state, in, sizeof(GmEnvState) * (size_t)c->n_envs, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GM_OK;
}

int gm_get_target(gm_ctx* c, double* end_xyzth, int32_t* es, int32_t* ns, double* base_xyz) {
  if (!c) return GM_E_ARG;
  std::vector<GmEnvState> h;
  int rc = fetch_states(c, h);
  if (rc) return rc;
  for (int e = 0; e < c->n_envs; e++) {
    if (end_xyzth) { end_xyzth[4 * e] = h[e].end.x; end_xyzth[4 * e + 1] = h[e].end.y; end_xyzth[4 * e + 2] = h[e].end.z; end_xyzth[4 * e + 3] = h[e].end.th; }
    if (es) { es[3 * e] = h[e].end.sx; es[3 * e + 1] = h[e].end.sy; es[3 * e + 2] = h[e].end.sz; }
    if (ns) { ns[3 * e] = h[e].next.sx; ns[3 * e + 1] = h[e].next.sy; ns[3 * e + 2] = h[e].next.sz; }
    if (base_xyz) { base_xyz[3 * e] = h[e].base[0]; base_xyz[3 * e + 1] = h[e].base[1]; base_xyz[3 * e + 2] = h[e].base[2]; }
  }
  return GM_OK;
}

int gm_get_overflow(gm_ctx* c, int32_t* counts) {
  if (!c || !counts) return GM_E_ARG;
  std::vector<GmEnvState> h;
  int rc = fetch_states(c, h);
  if (rc) return rc;
  for (int e = 0; e < c->n_envs; e++) counts[e] = h[e].overflow;
  return GM_OK;
}

void* gm_device_obs(gm_ctx* c) { return c ? c->d_obs : nullptr; }
void* gm_device_reward(gm_ctx* c) { return c ? c->d_rew : nullptr; }
void* gm_device_done(gm_ctx* c) { return c ? c->d_done : nullptr; }
void* gm_device_actions(gm_ctx* c) { return c ? c->d_act : nullptr; }
void* gm_stream(gm_ctx* c) { return c ? (void*)c->stream : nullptr; }

int gm_debug_substep(gm_ctx* c, int32_t* ncon, double* contact, double* efc_force, double* qacc, int32_t* nefc,
                     double* obj_wrench) {
  if (!c) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  int32_t *d_ncon, *d_nefc; double *d_con, *d_f, *d_q, *d_w;
  size_t n = (size_t)c->n_envs;
  HIPCHK(c, hipMalloc(&d_ncon, sizeof(int32_t) * n));
  HIPCHK(c, hipMalloc(&d_nefc, sizeof(int32_t) * n));
  HIPCHK(c, hipMalloc(&d_con, sizeof(double) * n * GM_MAX_CON * 16));
  HIPCHK(c, hipMalloc(&d_f, sizeof(double) * n * GM_MAX_EFC));
  HIPCHK(c, hipMalloc(&d_q, sizeof(double) * n * GM_MAX_DOF));
  HIPCHK(c, hipMalloc(&d_w, sizeof(double) * n * 6));
  DebugOut dbg{d_ncon, d_con, d_f, d_q, nullptr, d_nefc, d_w};
  HIPCHK(c, launch_step(c, c->n_envs, c->n_envs, 2, dbg));
  if (ncon) HIPCHK(c, hipMemcpyAsync(ncon, d_ncon, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  if (nefc) HIPCHK(c, hipMemcpyAsync(nefc, d_nefc, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
  if (contact) HIPCHK(c, hipMemcpyAsync(contact, d_con, sizeof(double) * n * GM_MAX_CON * 16, hipMemcpyDeviceToHost, c->stream));
  if (efc_force) HIPCHK(c, hipMemcpyAsync(efc_force, d_f, sizeof(double) * n * GM_MAX_EFC, hipMemcpyDeviceToHost, c->stream));
  if (qacc) HIPCHK(c, hipMemcpyAsync(qacc, d_q, sizeof(double) * n * GM_MAX_DOF, hipMemcpyDeviceToHost, c->stream));
  if (obj_wrench) HIPCHK(c, hipMemcpyAsync(obj_wrench, d_w, sizeof(double) * n * 6, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  (void)hipFree(d_ncon); (void)hipFree(d_nefc); (void)hipFree(d_con); (void)hipFree(d_f); (void)hipFree(d_q);
  (void)hipFree(d_w);
  return GM_OK;
}

int gm_set_stream(gm_ctx* c, void* stream) {
  if (!c) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->stream = stream ? (hipStream_t)stream : c->own_stream;
  return GM_OK;
}

int gm_autoreset(gm_ctx* c, int max_episode_steps, const gm_spawn* spawn, int spawn_on_device, float* returns) {
  return gm_autoreset_episodes(c, max_episode_steps, spawn, spawn_on_device, returns, nullptr);
}

int gm_autoreset_episodes(gm_ctx* c, int max_episode_steps, const gm_spawn* spawn, int spawn_on_device,
                          float* returns, gm_episode_end* episodes) {
  static_assert(sizeof(gm_episode_end) == 12, "episode-end record is 3 x 4 bytes");
  if (!c) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  const gm_spawn* ds = nullptr;
  if (spawn && !spawn_on_device) {
    HIPCHK(c, hipMemcpyAsync(c->d_spawn, spawn, sizeof(gm_spawn) * (size_t)c->n_envs, hipMemcpyHostToDevice, c->stream));
    ds = c->d_spawn;
  } else if (spawn) {
    ds = spawn;
  }
  int threads = 64, blocks = (c->n_envs + threads - 1) / threads;
  hipLaunchKernelGGL(gm_autoreset_mask_kernel, dim3(blocks), dim3(threads), 0, c->stream, c->d_state, c->d_done,
                     max_episode_steps, c->d_mask, returns, episodes, c->n_envs);
  HIPCHK(c, hipGetLastError());
  hipLaunchKernelGGL(gm_reset_kernel, dim3(c->n_envs), dim3(64), 0, c->stream, c->d_state, c->d_model, c->d_cfg,
                     c->d_topo, c->d_eq, c->d_mask, ds, c->d_objs, c->n_objects, c->n_envs, c->d_scene,
                     c->scene_tries, c->d_obs, c->spawn_rand);
  HIPCHK(c, hipGetLastError());
  if (spawn && !spawn_on_device) HIPCHK(c, hipStreamSynchronize(c->stream));
  return GM_OK;
}

void* gm_device_reset_mask(gm_ctx* c) { return c ? (void*)c->d_mask : nullptr; }

int gm_step_profiled(gm_ctx* c, uint64_t* phase_cycles) {
  if (!c || !phase_cycles) return GM_E_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  size_t n = (size_t)c->n_envs;
  unsigned long long* d_ph;
  HIPCHK(c, hipMalloc(&d_ph, sizeof(unsigned long long) * n * GM_NPHASE));
  DebugOut dbg{nullptr, nullptr, nullptr, nullptr, d_ph};
  HIPCHK(c, launch_step(c, c->n_envs, c->n_envs, 0, dbg));
  HIPCHK(c, hipMemcpyAsync(phase_cycles, d_ph, sizeof(unsigned long long) * n * GM_NPHASE, hipMemcpyDeviceToHost,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  (void)hipFree(d_ph);
  return GM_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- on-device DQN policy
struct gm_policy {
  gm_ctx* ctx = nullptr;
  GpNet net{};
  float* d_params = nullptr;
  int32_t* d_actions = nullptr;
  float* d_q = nullptr;
  float* d_eps = nullptr;      // gm_policy_rollout's exploration thresholds, one per env-step
  int eps_cap = 0;
};

static int64_t policy_layout(const int32_t* sizes, int n_sizes, GpNet* net) {
  if (!sizes || n_sizes < 2 || n_sizes - 1 > GP_MAX_LAYERS) return -1;
  GpNet P{};
  P.n_layers = n_sizes - 1;
  long long off = 0;
  for (int l = 0; l < n_sizes; l++) {
    if (sizes[l] < 1 || sizes[l] > GP_MAX_WIDTH) return -1;
    P.width[l] = sizes[l];
  }
  for (int l = 0; l < P.n_layers; l++) {
    P.kpad[l] = (P.width[l] + 3) & ~3;
    P.tiles[l] = (P.width[l + 1] + 15) / 16;
    P.woff[l] = off;
    off += (long long)P.tiles[l] * (P.kpad[l] / 4) * 64;
    P.boff[l] = off;
    off += (long long)P.tiles[l] * 16;
  }
  if (net) *net = P;
  return off;
}

extern "C" {

int64_t gm_policy_pack(const int32_t* sizes, int n_sizes, const float* params, float* out) {
  GpNet P;
  const int64_t total = policy_layout(sizes, n_sizes, &P);
  if (total < 0 || !out) return total;
  if (!params) return GM_E_ARG;
  std::memset(out, 0, sizeof(float) * (size_t)total);
  const float* src = params;
  for (int l = 0; l < P.n_layers; l++) {
    const int in = P.width[l], outw = P.width[l + 1], ks = P.kpad[l] / 4;
    const float* W = src;            // [outw x in] row-major (torch nn.Linear.weight)
    const float* b = src + (size_t)outw * in;
    for (int t = 0; t < P.tiles[l]; t++)
      for (int s4 = 0; s4 < ks; s4++)
        for (int lane = 0; lane < 64; lane++) {
          const int j = 16 * t + (lane & 15), k = 4 * s4 + (lane >> 4);
          out[P.woff[l] + ((int64_t)t * ks + s4) * 64 + lane] = (j < outw && k < in) ? W[(size_t)j * in + k] : 0.0f;
        }
    for (int j = 0; j < outw; j++) out[P.boff[l] + j] = b[j];
    src = b + outw;
  }
  return total;
}

int gm_policy_create(gm_ctx* c, const int32_t* sizes, int n_sizes, const float* params, gm_policy** out) {
  if (!c || !sizes || !params || !out) return GM_E_ARG;
  GpNet P;
  const int64_t total = policy_layout(sizes, n_sizes, &P);
  if (total < 0) return fail(c, GM_E_RANGE, "gm_policy_create: <= 8 layers of width 1..256 expected");
  if (P.width[0] != c->cfg.n_obs || P.width[P.n_layers] != c->cfg.n_actions)
    return fail(c, GM_E_ARG, "gm_policy_create: network must map n_obs (" + std::to_string(c->cfg.n_obs) +
                                 ") to n_actions (" + std::to_string(c->cfg.n_actions) + ")");
  if (c->cfg.s.continous_actions)
    return fail(c, GM_E_ARG, "gm_policy_create: the DQN policy needs discrete actions (continous_actions = 0)");
  std::vector<float> packed((size_t)total);
  gm_policy_pack(sizes, n_sizes, params, packed.data());
  gm_policy* p = new gm_policy;
  p->ctx = c;
  p->net = P;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipMalloc(&p->d_params, sizeof(float) * (size_t)total));
  HIPCHK(c, hipMalloc(&p->d_actions, sizeof(int32_t) * (size_t)c->n_envs));
  HIPCHK(c, hipMalloc(&p->d_q, sizeof(float) * (size_t)c->n_envs * c->cfg.n_actions));
  HIPCHK(c, hipMemcpyAsync(p->d_params, packed.data(), sizeof(float) * (size_t)total, hipMemcpyHostToDevice,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  *out = p;
  return GM_OK;
}

void gm_policy_destroy(gm_policy* p) {
  if (!p) return;
  if (p->ctx) (void)hipSetDevice(p->ctx->device);
  (void)hipFree(p->d_params);
  (void)hipFree(p->d_actions);
  (void)hipFree(p->d_q);
  (void)hipFree(p->d_eps);
  delete p;
}

int gm_policy_act(gm_policy* p, float eps, uint64_t seed, uint64_t decision) {
  if (!p || !p->ctx) return GM_E_ARG;
  gm_ctx* c = p->ctx;
  HIPCHK(c, hipSetDevice(c->device));
  const int blocks = (c->n_envs + GP_TILE - 1) / GP_TILE;
  hipLaunchKernelGGL(gm_policy_kernel, dim3(blocks), dim3(64), 0, c->stream, c->d_obs, c->n_envs,
                     (long long)c->env_offset, p->d_params, p->net, eps, seed, decision, p->d_actions, p->d_q);
  HIPCHK(c, hipGetLastError());
  return gm_set_discrete_action(c, p->d_actions, 1);
}

int gm_policy_rollout(gm_policy* p, int n_steps, const float* eps, uint64_t seed, uint64_t decision0,
                      int max_episode_steps, gm_episode_end* records) {
  if (!p || !p->ctx || !eps || n_steps < 1) return GM_E_ARG;
  gm_ctx* c = p->ctx;
  HIPCHK(c, hipSetDevice(c->device));
  if (c->chunk > 0 && c->chunk_grid > 0) {
    if (n_steps > p->eps_cap) {
      // (the stream may still read the old buffer: wait before freeing it)
      HIPCHK(c, hipStreamSynchronize(c->stream));
      (void)hipFree(p->d_eps);
      p->d_eps = nullptr;
      p->eps_cap = 0;
      HIPCHK(c, hipMalloc(&p->d_eps, sizeof(float) * (size_t)n_steps));
      p->eps_cap = n_steps;
    }
    // eps is the caller's (pageable) array: stage it through the ctx's pinned buffer so the
    // copy owns its bytes before the call returns (stage_ev: the previous staging copy has
    // left the buffer), or copy and wait when it does not fit
    const size_t eb = sizeof(float) * (size_t)n_steps;
    if (eb <= c->stage_bytes) {
      HIPCHK(c, hipEventSynchronize(c->stage_ev));
      std::memcpy(c->h_stage, eps, eb);
      HIPCHK(c, hipMemcpyAsync(p->d_eps, c->h_stage, eb, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipEventRecord(c->stage_ev, c->stream));
    } else {
      HIPCHK(c, hipMemcpyAsync(p->d_eps, eps, eb, hipMemcpyHostToDevice, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
    }
    RolloutArgs ra{n_steps, 2, seed, 0.0f, max_episode_steps, records};
    ra.pparams = p->d_params;
    ra.pnet = p->net;
    ra.peps = p->d_eps;
    ra.pdecision = decision0;
    return rollout_launch(c, ra);
  }
  // the one-shot kernel (GM_CHUNK_SUBSTEPS=0): the per-step sequence it fuses
  for (int k = 0; k < n_steps; k++) {
    int rc = gm_policy_act(p, eps[k], seed, decision0 + (uint64_t)k);
    if (rc == GM_OK) rc = gm_step(c);
    if (rc == GM_OK) rc = gm_autoreset_episodes(c, max_episode_steps, nullptr, 1, nullptr,
                                                records ? records + (size_t)k * c->n_envs : nullptr);
    if (rc != GM_OK) return rc;
  }
  return GM_OK;
}

int gm_policy_read(gm_policy* p, int32_t* actions, float* q) {
  if (!p || !p->ctx) return GM_E_ARG;
  gm_ctx* c = p->ctx;
  HIPCHK(c, hipSetDevice(c->device));
  if (actions)
    HIPCHK(c, hipMemcpyAsync(actions, p->d_actions, sizeof(int32_t) * (size_t)c->n_envs, hipMemcpyDeviceToHost,
                             c->stream));
  if (q)
    HIPCHK(c, hipMemcpyAsync(q, p->d_q, sizeof(float) * (size_t)c->n_envs * c->cfg.n_actions,
                             hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return GM_OK;
}

}  // extern "C"
