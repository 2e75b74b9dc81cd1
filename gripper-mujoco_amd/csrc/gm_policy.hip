// gm_policy.hip -- the batched select_action kernel; network layout, MFMA forward and the
// selection are in gm_policy_net.h (shared with gm_rollout's per-env policy driver).
#pragma once
#include "gm_policy_net.h"

__global__ __launch_bounds__(64) void gm_policy_kernel(const float* __restrict__ obs, int n_envs, long long env_offset,
                                                       const float* __restrict__ params, GpNet P, float eps,
                                                       uint64_t seed, uint64_t decision, int32_t* __restrict__ actions,
                                                       float* __restrict__ qout) {
  __shared__ float act[2][GP_TILE][GP_MAX_WIDTH + 4];
  const int lane = threadIdx.x;
  const int e0 = blockIdx.x * GP_TILE;
  const int n_obs = P.width[0];
  const int k0 = P.kpad[0];
  for (int i = lane; i < GP_TILE * k0; i += 64) {
    const int r = i / k0, k = i - r * k0;
    act[0][r][k] = (e0 + r < n_envs && k < n_obs) ? obs[(size_t)(e0 + r) * n_obs + k] : 0.0f;
  }
  __syncthreads();
  int cur = 0;
  for (int l = 0; l < P.n_layers; l++) {
    const float* __restrict__ W = params + P.woff[l];
    const float* __restrict__ Bv = params + P.boff[l];
    const int ksteps = P.kpad[l] >> 2;
    const bool last = (l == P.n_layers - 1);
    const int outw = P.width[l + 1];
    for (int t = 0; t < P.tiles[l]; t++) {
      gp_f32x4 c = {0.0f, 0.0f, 0.0f, 0.0f};
      const float* Wt = W + (size_t)t * ksteps * 64;
      for (int s = 0; s < ksteps; s++) {
        const float a = act[cur][lane & 15][4 * s + (lane >> 4)];
        const float b = Wt[s * 64 + lane];
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
      }
      // D fragment: output column j = 16 t + (lane & 15), env row (lane >> 4) * 4 + r
      const int j = t * 16 + (lane & 15);
      const float bias = Bv[j];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        float v = c[r] + bias;
        if (!last) v = fmaxf(v, 0.0f);
        act[cur ^ 1][(lane >> 4) * 4 + r][j] = (j < outw) ? v : 0.0f;
      }
    }
    __syncthreads();
    cur ^= 1;
  }
  // softmax over the logits (nn.Softmax(dim=1)), then select_action (gp_choose)
  if (lane < GP_TILE && e0 + lane < n_envs) {
    const size_t env = (size_t)(e0 + lane);
    const int n_out = P.width[P.n_layers];
    actions[env] = gp_choose(act[cur][lane], n_out, eps, seed, decision, (uint64_t)(env_offset + (long long)env),
                             qout ? qout + env * n_out : nullptr);
  }
}
