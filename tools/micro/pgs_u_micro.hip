// Developer micro-benchmark: shader cycles per PGS row for the u-formulation used in
// gm_step_kernel (lane per row, v_readlane broadcast), at the kernel's occupancy
// (19 KB LDS per workgroup -> 8 workgroups per CU, 2 waves per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int MODE, typename T>
__global__ __launch_bounds__(64, 2) void pgs(const double* Ain, const double* bin, double* fout, int nefc, int iters,
                                             unsigned long long* cyc) {
  extern __shared__ double lds_pad[];
  const int lane = threadIdx.x;
  T A[64];
#pragma unroll
  for (int i = 0; i < 64; i++) A[i] = (T)Ain[i * 64 + lane];
  const T lb = (lane & 3) ? (T)0 : -(T)__builtin_inf();
  T u = (T)bin[lane], f = 0;
  const int nchunk = (__builtin_amdgcn_readfirstlane(nefc) + 3) >> 2;
  if (lane == 0) lds_pad[0] = 0;
  unsigned long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < 16; c++) {
      if (c >= nchunk) continue;
#pragma unroll
      for (int rr = 0; rr < 4; rr++) {
        const int r = c * 4 + rr;
        const T fn = u > lb ? u : lb;
        const T dl = fn - f;
        T delta;
        if constexpr (sizeof(T) == 8) {
          const long long bits = __double_as_longlong(dl);
          const int lo = __builtin_amdgcn_readlane((int)bits, r);
          const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), r);
          delta = __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
        } else {
          delta = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dl), r));
        }
        if (MODE == 1) delta = (T)1e-9;   // no broadcast: chain without the readlane
        u = u - A[r] * delta;
        unsigned long long onehot;
        asm volatile("s_bfm_b64 %0, 1, %1" : "=s"(onehot) : "i"(r));
        f = __builtin_amdgcn_inverse_ballot_w64(onehot) ? fn : f;
      }
    }
  }
  unsigned long long t1 = clock64();
  fout[blockIdx.x * 64 + lane] = (double)(f + u);
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, typename T>
void run(const char* name, double* dA, double* db, double* df, unsigned long long* dc, int nb, int nefc, int iters,
         size_t lds) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  pgs<MODE, T><<<nb, 64, lds>>>(dA, db, df, nefc, iters, dc);
  hipEventRecord(e0);
  pgs<MODE, T><<<nb, 64, lds>>>(dA, db, df, nefc, iters, dc);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> c(nb);
  hipMemcpy(c.data(), dc, nb * 8, hipMemcpyDeviceToHost);
  double m = 0; for (auto x : c) m += x; m /= nb;
  const int rows = ((nefc + 3) / 4) * 4 * iters;
  printf("%-28s lds %6zu  %.1f cyc/row (wave clock)  kernel %.3f ms  %.2f ns/row/env (throughput)\n", name, lds, m / rows, ms,
         ms * 1e6 / ((double)rows * nb));
}

int main() {
  const int nefc = 20, iters = 24;
  std::vector<double> A(64 * 64), b(64);
  for (int i = 0; i < 64; i++) for (int j = 0; j < 64; j++) A[i * 64 + j] = (i == j) ? 0.0 : 0.01 * ((i + j) % 7) / 2.0;
  for (int i = 0; i < 64; i++) b[i] = (i < nefc) ? 0.1 * ((i % 5) - 2) : 0.0;
  double *dA, *db, *df; unsigned long long* dc;
  const int nbmax = 4096 * 4;
  hipMalloc(&dA, 64 * 64 * 8); hipMalloc(&db, 64 * 8); hipMalloc(&df, nbmax * 64 * 8); hipMalloc(&dc, nbmax * 8);
  hipMemcpy(dA, A.data(), 64 * 64 * 8, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), 64 * 8, hipMemcpyHostToDevice);
  for (size_t lds : {(size_t)19200, (size_t)38400, (size_t)9600}) {
    run<0, double>("fp64 u-form", dA, db, df, dc, 4096, nefc, iters, lds);
    run<1, double>("fp64 u-form no readlane", dA, db, df, dc, 4096, nefc, iters, lds);
    run<0, float>("fp32 u-form", dA, db, df, dc, 4096, nefc, iters, lds);
  }
  return 0;
}
