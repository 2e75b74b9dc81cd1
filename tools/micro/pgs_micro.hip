// Developer micro-benchmark: cycles per PGS row update for the lane-per-row /
// v_readlane broadcast formulation used in gm_step_kernel (fp64).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double real;

template <int MODE>
__global__ __launch_bounds__(64) void pgs(const double* Ain, const double* bin, double* fout, int nefc, int iters,
                                          unsigned long long* cyc) {
  int lane = threadIdx.x;
  real A[64];
#pragma unroll
  for (int i = 0; i < 64; i++) A[i] = Ain[i * 64 + lane];
  real R = 1e-3, arinv = 1.0 / (A[lane & 63] + 1.0 + R);
  real res = bin[lane], f = 0;
  const real lb = (lane & 3) ? 0.0 : -__builtin_inf();
  const int nefc_s = __builtin_amdgcn_readfirstlane(nefc);
  unsigned long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 64; r++) {
      if (r >= nefc_s) continue;
      real g, fn;
      if (MODE == 0) {
        g = fma(R, f, res);
        fn = fmax(fma(-g, arinv, f), lb);
      } else {
        g = res + R * f;
        fn = f - g * arinv;
        if (lb == 0.0 && fn < 0) fn = 0;
      }
      const real dl = fn - f;
      const long long bits = __double_as_longlong(dl);
      const int lo = __builtin_amdgcn_readlane((int)bits, r);
      const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), r);
      const real delta = __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
      res = fma(A[r], delta, res);
      if (lane == r) f = fn;
    }
  }
  unsigned long long t1 = clock64();
  fout[blockIdx.x * 64 + lane] = f;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int nb = 4096, nefc = 18, iters = 24;
  std::vector<double> A(64 * 64), b(64);
  for (int i = 0; i < 64; i++) for (int j = 0; j < 64; j++) A[i * 64 + j] = (i == j) ? 2.0 : 0.01 * ((i + j) % 7);
  for (int i = 0; i < 64; i++) b[i] = -0.1 * (i % 5);
  double *dA, *db, *df; unsigned long long* dc;
  hipMalloc(&dA, A.size() * 8); hipMalloc(&db, 64 * 8); hipMalloc(&df, nb * 64 * 8); hipMalloc(&dc, nb * 8);
  hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice); hipMemcpy(db, b.data(), 64 * 8, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; mode++) {
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int rep = 0; rep < 2; rep++) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(pgs<0>, dim3(nb), dim3(64), 0, 0, dA, db, df, nefc, iters, dc);
      else hipLaunchKernelGGL(pgs<1>, dim3(nb), dim3(64), 0, 0, dA, db, df, nefc, iters, dc);
      hipEventRecord(e1); hipEventSynchronize(e1);
    }
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(nb); hipMemcpy(c.data(), dc, nb * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (auto x : c) avg += x; avg /= nb;
    printf("mode %d: %.3f ms for %d envs, %.0f cycles per env (lane0), %.1f cycles per row update\n", mode, ms, nb, avg,
           avg / (iters * nefc));
  }
  return 0;
}
