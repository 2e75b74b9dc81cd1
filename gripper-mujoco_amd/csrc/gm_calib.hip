// gm_calib.hip -- the calibration variant of the env-step kernel (gm_step_kernel<CL,
// true>: per-env timestep, tip load, mjWARN_BADQACC) and its helper kernels, compiled as
// a translation unit of its own.  Co-compiling these instantiations with the env-step
// kernel perturbed the env-step kernel's code generation (measured 7% slower on one
// box, A/B in one gpurun call); in their own module they leave it untouched.
// Reference: MjClass::configure_settings' automatic settings (mjclass.cpp:241-308),
// find_highest_stable_timestep (4745-4854), calibrate_simulated_sensors (4643-4676),
// validate_curve_under_force (4023-4105); the host side is gm_calibrate in gm_capi.hip.
#define GM_CAL_TU
#include "gm_kernels.hip"

// per-env timestep / substep count / tip load for a calibration launch
__global__ void gm_cal_setup_kernel(GmEnvState* __restrict__ states, const double* __restrict__ dt,
                                    const int32_t* __restrict__ steps, double tip_force, int n) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  states[e].dt = dt[e];
  states[e].cal_steps = steps[e];
  states[e].tip_force = tip_force;
  states[e].badqacc = 0;
}
__global__ void gm_cal_read_kernel(const GmEnvState* __restrict__ states, uint8_t* __restrict__ bad, int n) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  bad[e] = (uint8_t)(states[e].badqacc != 0);
}
// read_armadillo_gauge(data, finger 0) of one env (mjclass.cpp:4666)
template <int CL>
__global__ void gm_gauge_read_kernel(const GmEnvState* __restrict__ states, const gm_model* __restrict__ m,
                                     const GmTopo* __restrict__ T, int env, float* __restrict__ out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  out[0] = gauge_reading<CL - 2>(m, &states[env].qpos[T->dof_f0[0] + 2]);
}

// host launchers (C++ linkage, called by gm_calibrate)
hipError_t gm_cal_launch_step(int n_seg, int n_envs, hipStream_t st, GmEnvState* states, const gm_model* m,
                              const gm_config* C, const GmTopo* T) {
  DebugOut dbg{nullptr, nullptr, nullptr, nullptr, nullptr};
  switch (n_seg) {
#define X(N)                                                                                               \
  case N:                                                                                                  \
    hipLaunchKernelGGL((gm_step_kernel<N + 2, true>), dim3(n_envs), dim3(NT), 0, st, states, m, C, T,      \
                       (float*)nullptr, (float*)nullptr, (uint8_t*)nullptr, n_envs, 3, dbg,                \
                       (const int32_t*)nullptr, (uint32_t*)nullptr, GmChunkQ{});                           \
    return hipGetLastError();
    GM_NSEG_LIST
#undef X
    default: return hipErrorInvalidValue;
  }
}
hipError_t gm_cal_launch_setup(hipStream_t st, GmEnvState* states, const double* dt, const int32_t* steps, double tip,
                               int n) {
  hipLaunchKernelGGL(gm_cal_setup_kernel, dim3((n + 63) / 64), dim3(64), 0, st, states, dt, steps, tip, n);
  return hipGetLastError();
}
hipError_t gm_cal_launch_read(hipStream_t st, const GmEnvState* states, uint8_t* bad, int n) {
  hipLaunchKernelGGL(gm_cal_read_kernel, dim3((n + 63) / 64), dim3(64), 0, st, states, bad, n);
  return hipGetLastError();
}
hipError_t gm_cal_launch_gauge(int n_seg, hipStream_t st, const GmEnvState* states, const gm_model* m, const GmTopo* T,
                               int env, float* out) {
  switch (n_seg) {
#define X(N)                                                                                               \
  case N:                                                                                                  \
    hipLaunchKernelGGL((gm_gauge_read_kernel<N + 2>), dim3(1), dim3(64), 0, st, states, m, T, env, out);   \
    return hipGetLastError();
    GM_NSEG_LIST
#undef X
    default: return hipErrorInvalidValue;
  }
}
