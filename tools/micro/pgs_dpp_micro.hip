// Developer micro-benchmark: shader cycles per PGS row, v_readlane broadcast (general
// path) vs the replicated DPP-row layout (v_fmac_f64_dpp row_newbcast) of gm_step_kernel,
// at the kernel's occupancy (2 waves per SIMD) and at 1 wave per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ double vmax(double a, double b) {
  double r;
  asm volatile("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
template <int P>
__device__ __forceinline__ void fmac_bc(double& u, double d, double nb) {
  asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
               : "+v"(u) : "v"(d), "v"(nb), "i"(P));
}
__device__ __forceinline__ void movm(double& f, double fn, unsigned long long mask) {
  unsigned long long save;
  asm volatile("s_mov_b64 %1, exec\n\ts_mov_b64 exec, %2\n\tv_mov_b64 %0, %3\n\ts_mov_b64 exec, %1"
               : "+v"(f), "=&s"(save) : "s"(mask), "v"(fn));
}

template <int C> __device__ __forceinline__ double bc64(double x) { return __builtin_amdgcn_update_dpp(0.0, x, C, 0xF, 0xF, true); }
__device__ __forceinline__ double bcast(double x, int r) {
  switch (r) {
    case 0: return bc64<0x150>(x); case 1: return bc64<0x151>(x); case 2: return bc64<0x152>(x);
    case 3: return bc64<0x153>(x); case 4: return bc64<0x154>(x); case 5: return bc64<0x155>(x);
    case 6: return bc64<0x156>(x); case 7: return bc64<0x157>(x); case 8: return bc64<0x158>(x);
    case 9: return bc64<0x159>(x); case 10: return bc64<0x15A>(x); case 11: return bc64<0x15B>(x);
    case 12: return bc64<0x15C>(x); case 13: return bc64<0x15D>(x); case 14: return bc64<0x15E>(x);
    default: return bc64<0x15F>(x);
  }
}

template <int R, int MODE>
__device__ __forceinline__ void row(double& u, double& f, double& f2, double lb, const double* B) {
  if constexpr (MODE == 0) {          // general path: lane per row, readlane broadcast
    const double fn = fmax(u, lb);
    const double dl = fn - f;
    const long long bits = __double_as_longlong(dl);
    const int lo = __builtin_amdgcn_readlane((int)bits, R);
    const int hi = __builtin_amdgcn_readlane((int)(bits >> 32), R);
    const double delta = __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
    u = fma(-B[R], delta, u);
    unsigned long long onehot;
    asm volatile("s_bfm_b64 %0, 1, %1" : "=s"(onehot) : "i"(R));
    f = __builtin_amdgcn_inverse_ballot_w64(onehot) ? fn : f;
  } else if constexpr (MODE == 1) {   // DPP row broadcast, masked move
    const double fn = vmax(u, lb);
    const double dl = fn - f;
    fmac_bc<R & 15>(u, dl, B[R]);
    movm(f, fn, 0x0001000100010001ull << (R & 15));
  } else if constexpr (MODE == 2) {   // DPP chain only (no f bookkeeping)
    const double fn = vmax(u, lb);
    fmac_bc<R & 15>(u, fn, B[R]);
  } else if constexpr (MODE == 4) {   // DPP row broadcast, cndmask select
    const double fn = vmax(u, lb);
    const double dl = fn - f;
    fmac_bc<R & 15>(u, dl, B[R]);
    f = __builtin_amdgcn_inverse_ballot_w64(0x0001000100010001ull << (R & 15)) ? fn : f;
  } else if constexpr (MODE == 5) {   // v_mov_b64_dpp to a temporary, plain fma, cndmask
    const double fn = vmax(u, lb);
    const double dl = fn - f;
    const double bd = __builtin_amdgcn_update_dpp(0.0, dl, 0x150 + (R & 15), 0xF, 0xF, true);
    u = fma(B[R], bd, u);
    f = __builtin_amdgcn_inverse_ballot_w64(0x0001000100010001ull << (R & 15)) ? fn : f;
  } else if constexpr (MODE == 6) {   // as 4, two sets (second FMA off the chain)
    const double fn = vmax(u, lb);
    const double dl = fn - f;
    fmac_bc<R & 15>(u, dl, B[R]);
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(f2) : "v"(dl), "v"(B[(R + 1) & 15]), "i"(R & 15));
    f = __builtin_amdgcn_inverse_ballot_w64(0x0001000100010001ull << (R & 15)) ? fn : f;
  } else {                            // plain dependent chain: max, add, fma
    const double fn = vmax(u, lb);
    const double dl = fn - f;
    u = fma(B[R], dl, u);
  }
}

template <int MODE, int OCC>
__global__ __launch_bounds__(64, OCC) void pgs(const double* Ain, const double* bin, double* fout, int iters,
                                               unsigned long long* cyc) {
  const int lane = threadIdx.x;
  double B[16];
#pragma unroll
  for (int i = 0; i < 16; i++) B[i] = Ain[i * 64 + lane];
  const double lb = (lane & 3) ? 0.0 : -__builtin_inf();
  double u = bin[lane], f = 0, f2 = 0;
  unsigned long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
    row<0, MODE>(u, f, f2, lb, B); row<1, MODE>(u, f, f2, lb, B); row<2, MODE>(u, f, f2, lb, B); row<3, MODE>(u, f, f2, lb, B);
    row<4, MODE>(u, f, f2, lb, B); row<5, MODE>(u, f, f2, lb, B); row<6, MODE>(u, f, f2, lb, B); row<7, MODE>(u, f, f2, lb, B);
    row<8, MODE>(u, f, f2, lb, B); row<9, MODE>(u, f, f2, lb, B); row<10, MODE>(u, f, f2, lb, B); row<11, MODE>(u, f, f2, lb, B);
    row<12, MODE>(u, f, f2, lb, B); row<13, MODE>(u, f, f2, lb, B); row<14, MODE>(u, f, f2, lb, B); row<15, MODE>(u, f, f2, lb, B);
  }
  unsigned long long t1 = clock64();
  fout[blockIdx.x * 64 + lane] = f + u + f2;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int OCC>
void run(const char* name, double* dA, double* db, double* df, unsigned long long* dc, int nb, int iters, size_t lds) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  pgs<MODE, OCC><<<nb, 64, lds>>>(dA, db, df, iters, dc);
  hipEventRecord(e0);
  pgs<MODE, OCC><<<nb, 64, lds>>>(dA, db, df, iters, dc);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> c(nb);
  hipMemcpy(c.data(), dc, nb * 8, hipMemcpyDeviceToHost);
  double m = 0; for (auto x : c) m += x; m /= nb;
  const double rows = 16.0 * iters;
  printf("%-34s lds %6zu  %6.1f cyc/row (wave clock)  kernel %.3f ms  %.3f ns/row/env\n", name, lds, m / rows, ms,
         ms * 1e6 / (rows * nb));
}

// FN registers: each row's last max(u, lb) kept in its own register, so f_r needs no
// per-row select (lane p0 of FN[r] is f_r); BUF=2 double-buffers FN across sweep pairs
template <int BUF, int OCC>
__global__ __launch_bounds__(64, OCC) void pgs_fn(const double* Ain, const double* bin, double* fout, int iters,
                                                  unsigned long long* cyc) {
  const int lane = threadIdx.x;
  double B[16], FN[16], FM[16];
#pragma unroll
  for (int i = 0; i < 16; i++) { B[i] = Ain[i * 64 + lane]; FN[i] = 0; FM[i] = 0; }
  const double lb = (lane & 3) ? 0.0 : -__builtin_inf();
  double u = bin[lane];
  unsigned long long t0 = clock64();
  for (int it = 0; it < iters; it += BUF) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
      const double fn = vmax(u, lb);
      const double dl = fn - FN[r];
      if (BUF == 1) FN[r] = fn; else FM[r] = fn;
      const double bd = bcast(dl, r & 15);
      u = fma(B[r], bd, u);
    }
    if (BUF == 2) {
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const double fn = vmax(u, lb);
        const double dl = fn - FM[r];
        FN[r] = fn;
        const double bd = bcast(dl, r & 15);
        u = fma(B[r], bd, u);
      }
    }
  }
  unsigned long long t1 = clock64();
  double f = 0;
#pragma unroll
  for (int r = 0; r < 16; r++) f = ((lane & 15) == r) ? FN[r] : f;
  fout[blockIdx.x * 64 + lane] = f + u;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int BUF, int OCC>
void run_fn(const char* name, double* dA, double* db, double* df, unsigned long long* dc, int nb, int iters, size_t lds) {
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  pgs_fn<BUF, OCC><<<nb, 64, lds>>>(dA, db, df, iters, dc);
  hipEventRecord(e0);
  pgs_fn<BUF, OCC><<<nb, 64, lds>>>(dA, db, df, iters, dc);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> c(nb);
  hipMemcpy(c.data(), dc, nb * 8, hipMemcpyDeviceToHost);
  double m = 0; for (auto x : c) m += x; m /= nb;
  const double rows = 16.0 * iters;
  printf("%-34s lds %6zu  %6.1f cyc/row (wave clock)  kernel %.3f ms  %.3f ns/row/env\n", name, lds, m / rows, ms,
         ms * 1e6 / (rows * nb));
}

int main() {
  const int iters = 2000, nb = 2048;
  std::vector<double> A(16 * 64), b(64);
  for (int i = 0; i < 16; i++) for (int j = 0; j < 64; j++) A[i * 64 + j] = ((i == (j & 15)) ? 0.0 : -0.01 * ((i + j) % 7) / 2.0);
  for (int i = 0; i < 64; i++) b[i] = 0.1 * ((i % 5) - 2);
  double *dA, *db, *df; unsigned long long* dc;
  hipMalloc(&dA, 16 * 64 * 8); hipMalloc(&db, 64 * 8); hipMalloc(&df, nb * 64 * 8); hipMalloc(&dc, nb * 8);
  hipMemcpy(dA, A.data(), 16 * 64 * 8, hipMemcpyHostToDevice);
  hipMemcpy(db, b.data(), 64 * 8, hipMemcpyHostToDevice);
  for (size_t lds : {(size_t)19200, (size_t)38400}) {   // 8 / 4 workgroups per CU = 2 / 1 waves per SIMD
    run<0, 2>("readlane (general path)", dA, db, df, dc, nb, iters, lds);
    run<1, 2>("dpp row bcast + masked mov", dA, db, df, dc, nb, iters, lds);
    run<2, 2>("dpp chain only (max, fmac_dpp)", dA, db, df, dc, nb, iters, lds);
    run<3, 2>("plain chain (max, add, fma)", dA, db, df, dc, nb, iters, lds);
    run<4, 2>("dpp fmac + cndmask", dA, db, df, dc, nb, iters, lds);
    run<5, 2>("mov_b64_dpp + fma + cndmask", dA, db, df, dc, nb, iters, lds);
    run<6, 2>("dpp fmac x2 + cndmask (two sets)", dA, db, df, dc, nb, iters, lds);
    run_fn<1, 2>("FN regs, mov_dpp + fma", dA, db, df, dc, nb, iters, lds);
    run_fn<2, 2>("FN regs x2 buffers, mov_dpp + fma", dA, db, df, dc, nb, iters, lds);
  }
  return 0;
}
