// Developer microbenchmark: accuracy of v_rcp_f64 / v_rsq_f64 (and one Newton step) against
// the correctly rounded 1 / x and 1 / sqrt(x), in ulps, over log-uniform random x.
// build: hipcc --offload-arch=gfx950 -O3 tools/micro/rcp_rsq_acc.hip -o /tmp/rcp_rsq_acc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <cmath>
#include <vector>
#include <random>

__global__ void k(const double* x, double* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double v = x[i];
  const double r0 = __builtin_amdgcn_rcp(v);
  const double e = fma(-v, r0, 1.0);
  const double r1 = fma(r0, e, r0);
  const double s0 = __builtin_amdgcn_rsq(v);
  const double hx = 0.5 * v;
  const double f = fma(-hx * s0, s0, 0.5);
  const double s1 = fma(s0, f, s0);
  out[4 * i + 0] = r0; out[4 * i + 1] = r1; out[4 * i + 2] = s0; out[4 * i + 3] = s1;
}
static double ulps(double a, double b) {   // |a - b| in ulps of b
  int64_t ia, ib; std::memcpy(&ia, &a, 8); std::memcpy(&ib, &b, 8);
  return (double)std::llabs(ia - ib);
}
int main() {
  const int n = 1 << 20;
  std::vector<double> x(n), o(4 * (size_t)n);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(-20.0, 20.0);
  for (int i = 0; i < n; i++) x[i] = std::exp(u(g));
  double *dx, *dout;
  hipMalloc(&dx, 8 * (size_t)n); hipMalloc(&dout, 32 * (size_t)n);
  hipMemcpy(dx, x.data(), 8 * (size_t)n, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, dout, n);
  hipMemcpy(o.data(), dout, 32 * (size_t)n, hipMemcpyDeviceToHost);
  double m[4] = {0, 0, 0, 0};
  long cnt[4] = {0, 0, 0, 0};
  for (int i = 0; i < n; i++) {
    const double rc = 1.0 / x[i], sc = 1.0 / std::sqrt(x[i]);
    const double ref[4] = {rc, rc, sc, sc};
    for (int j = 0; j < 4; j++) { const double d = ulps(o[4 * (size_t)i + j], ref[j]); m[j] = d > m[j] ? d : m[j]; cnt[j] += d != 0; }
  }
  printf("max ulps vs correctly rounded: rcp %.0f (%ld differ), rcp+1NR %.0f (%ld), rsq %.0f (%ld), rsq+1NR %.0f (%ld) of %d\n",
         m[0], cnt[0], m[1], cnt[1], m[2], cnt[2], m[3], cnt[3], n);
  return 0;
}
