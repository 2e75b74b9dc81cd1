// gm_policy_net.h -- on-device DQN action selection (shared by gm_policy.hip and the rollout driver) for the batched env (SURVEY.md 8f,
// rank 1: "fused on-device DQN inference").
//
// Reference: rl/networks.py:7-41 VariableNetwork.forward (Linear + ReLU per hidden
// layer, a final Linear, Softmax over dim 1) and rl/agents/DQN.py:184-209
// Agent_DQN.select_action (a uniform random action with probability eps_threshold,
// otherwise policy_net(state).max(1)[1]).  The canonical network is
// [n_obs = 63, 150, 100, 50, n_actions = 8] (launch_training.py:850-857).
//
// f32 throughout (torch's default dtype).  The layer products run on the f32-input MFMA
// v_mfma_f32_16x16x4_f32, whose result is bit-for-bit a k-ordered fmaf chain.  One wave
// handles a tile of 16 envs: activations live in LDS as [16 envs][width] f32 (ping-pong
// between layers); weights are repacked on the host into B-fragment order -- for each
// 16-output tile and 4-wide k step, 64 floats in lane order (lane l holds
// W[16 t + (l & 15)][4 s + (l >> 4)]) -- so every MFMA's B operand is one coalesced
// 256-byte load from L2 (the canonical network is 119 KB).  Zero padding in k and in
// the output tiles keeps every lane's arithmetic defined.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#define GP_MAX_LAYERS 8
#define GP_MAX_WIDTH 256
#define GP_TILE 16

struct GpNet {
  int n_layers;                   // Linear layers
  int width[GP_MAX_LAYERS + 1];   // layer sizes: width[0] = n_obs, width[n_layers] = n_actions
  int kpad[GP_MAX_LAYERS];        // width[l] rounded up to 4 (MFMA k step)
  int tiles[GP_MAX_LAYERS];       // ceil(width[l + 1] / 16)
  long long woff[GP_MAX_LAYERS];  // float offset of layer l's packed weights
  long long boff[GP_MAX_LAYERS];  // float offset of layer l's bias (padded to tiles * 16)
};

typedef float gp_f32x4 __attribute__((ext_vector_type(4)));

// counter-based uniform in [0, 1) and integer draws for epsilon-greedy: splitmix64 of
// (seed, global env id, decision index) -- one independent stream per env, so actions do
// not depend on how envs are sharded (the reference draws from one numpy Generator per
// agent, which a batched device policy cannot reproduce draw for draw)
__device__ __forceinline__ uint64_t gp_mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}


// softmax over the logits (nn.Softmax(dim=1)), then Agent_DQN.select_action: argmax (first
// maximum, like torch's max on CPU) or, with probability eps, a uniform random action from
// the env's own counter-based stream.  One lane, one env; q (may be NULL) gets the softmax.
__device__ __forceinline__ int gp_choose(const float* x, int n_out, float eps, uint64_t seed, uint64_t decision,
                                         uint64_t gid, float* q_out) {
  float m = x[0];
  for (int j = 1; j < n_out; j++) m = fmaxf(m, x[j]);
  float sum = 0.0f;
  for (int j = 0; j < n_out; j++) sum += expf(x[j] - m);
  int best = 0;
  float qbest = -1.0f;
  for (int j = 0; j < n_out; j++) {
    const float q = expf(x[j] - m) / sum;
    if (q_out) q_out[j] = q;
    if (q > qbest) { qbest = q; best = j; }
  }
  const uint64_t h1 = gp_mix(seed ^ gp_mix(gid * 0x100000001B3ull + decision));
  const uint64_t h2 = gp_mix(h1);
  const float u = (float)((h1 >> 40) * (1.0 / 16777216.0));   // 24-bit uniform in [0, 1)
  if (u < eps) best = (int)(h2 % (uint64_t)n_out);
  return best;
}

// select_action for ONE env on its own wave (gm_rollout's policy driver, gm_kernels.hip
// chunked_env_steps): the batched kernel's MFMA tiles with this env in row 0 and zero rows
// below it.  MFMA rows are independent, so every logit is bit for bit the batched kernel's
// for the same observation.  obs: the env's observation (read with agent-scope loads, past
// this CU's L1: the env-step epilogue or a reset on another CU may have written it); act:
// 2 x (GP_MAX_WIDTH + 4) floats of LDS scratch.  Returns the action on every lane.
__device__ __forceinline__ int gp_select_one(const float* obs, const float* __restrict__ params, const GpNet& P,
                                             float eps, uint64_t seed, uint64_t decision, uint64_t gid, float* act,
                                             int lane) {
  constexpr int W = GP_MAX_WIDTH + 4;
  const int n_obs = P.width[0];
  const int k0 = P.kpad[0];
  // this wave's own stores of the observation (the previous env-step's epilogue or reset,
  // other lanes) have reached L2 before the loads below go there
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (int k = lane; k < k0; k += 64)
    act[k] = k < n_obs ? __hip_atomic_load(obs + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.0f;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  int cur = 0;
  for (int l = 0; l < P.n_layers; l++) {
    const float* __restrict__ Wl = params + P.woff[l];
    const float* __restrict__ Bv = params + P.boff[l];
    const int ksteps = P.kpad[l] >> 2;
    const bool last = (l == P.n_layers - 1);
    const int outw = P.width[l + 1];
    const float* src = act + cur * W;
    float* dst = act + (cur ^ 1) * W;
    for (int t = 0; t < P.tiles[l]; t++) {
      gp_f32x4 c = {0.0f, 0.0f, 0.0f, 0.0f};
      const float* Wt = Wl + (size_t)t * ksteps * 64;
      for (int s = 0; s < ksteps; s++) {
        const float a = (lane & 15) == 0 ? src[4 * s + (lane >> 4)] : 0.0f;
        const float b = Wt[s * 64 + lane];
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
      }
      // row 0 of the D fragment: lanes 0..15, element 0; column j = 16 t + lane
      const int j = t * 16 + (lane & 15);
      if (lane < 16) {
        float v = c[0] + Bv[j];
        if (!last) v = fmaxf(v, 0.0f);
        dst[j] = (j < outw) ? v : 0.0f;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    cur ^= 1;
  }
  int best = 0;
  if (lane == 0) best = gp_choose(act + cur * W, P.width[P.n_layers], eps, seed, decision, gid, nullptr);
  return __builtin_amdgcn_readfirstlane(best);
}
