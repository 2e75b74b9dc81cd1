// Developer micro-benchmark: dependent-chain latency and independent issue rate of
// fp64 / fp32 VALU ops on one wave (shader clock via clock64 and wall time).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int KIND, int NCH>
__global__ __launch_bounds__(64) void k(double* out, int n, unsigned long long* cyc) {
  const int lane = threadIdx.x;
  double x[NCH]; float y[NCH];
#pragma unroll
  for (int c = 0; c < NCH; c++) { x[c] = lane * 1e-3 + c; y[c] = lane * 1e-3f + c; }
  const double a = out[0] + 0.999, b = out[1] + 1e-7;
  const float af = (float)a, bf = (float)b;
  unsigned long long t0 = clock64();
  for (int i = 0; i < n; i++) {
#pragma unroll
    for (int j = 0; j < 16; j++) {
#pragma unroll
      for (int c = 0; c < NCH; c++) {
        if (KIND == 0) x[c] = fma(x[c], a, b);
        if (KIND == 1) y[c] = fmaf(y[c], af, bf);
        if (KIND == 2) x[c] = fmax(x[c], b) - a;      // max + add chain
        if (KIND == 3) { unsigned long long m; asm volatile("s_bfm_b64 %0, 1, %1" : "=s"(m) : "i"(j)); x[c] = __builtin_amdgcn_inverse_ballot_w64(m) ? x[c] * a : x[c]; }
      }
    }
  }
  unsigned long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int c = 0; c < NCH; c++) s += x[c] + y[c];
  out[2 + blockIdx.x * 64 + lane] = s;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND, int NCH>
void run(const char* nm, double* d, unsigned long long* c, int nb) {
  const int n = 1000;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  k<KIND, NCH><<<nb, 64>>>(d, n, c);
  (void)hipEventRecord(e0);
  k<KIND, NCH><<<nb, 64>>>(d, n, c);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h; (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  const double ops = (double)n * 16 * NCH;
  printf("%-22s chains %2d blocks %5d: %6.2f clk64/op per wave, %6.3f ns/op per wave (wall)\n", nm, NCH, nb, h / ops,
         ms * 1e6 / ops);
}

int main() {
  double* d; unsigned long long* c;
  (void)hipMalloc(&d, (2 + 4096 * 64) * 8); (void)hipMalloc(&c, 4096 * 8);
  (void)hipMemset(d, 0, 16);
  for (int nb : {1, 1024, 2048}) {
    run<0, 1>("fp64 fma", d, c, nb); run<0, 4>("fp64 fma", d, c, nb); run<0, 8>("fp64 fma", d, c, nb);
    run<1, 1>("fp32 fma", d, c, nb); run<1, 4>("fp32 fma", d, c, nb); run<1, 8>("fp32 fma", d, c, nb);
    run<2, 1>("fp64 max+add", d, c, nb); run<2, 4>("fp64 max+add", d, c, nb);
    run<3, 1>("fp64 mul+cndmask", d, c, nb); run<3, 4>("fp64 mul+cndmask", d, c, nb);
  }
  return 0;
}
