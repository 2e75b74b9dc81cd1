// rng_golden.cpp -- golden draws of the reference's RNG stack, produced by libstdc++
// itself: std::default_random_engine (= minstd_rand0 in libstdc++) consumed through
// std::uniform_real_distribution<float>{0,1} (mjclass.cpp:1567, mjclass.h:137-210) and
// std::uniform_real_distribution<double>(-size, size) (mjclass.cpp:1415, 1428), and
// std::shuffle of the spawn grids (mjclass.cpp:2533-2536) on the same engine.
// TEST INFRASTRUCTURE ONLY: pins oracle/oracle.c's restatement of these draws.
// Output lines: seed kind value...
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>

int main() {
  const unsigned seeds[] = {1u, 5u, 1234u, 1000004u, 2147483646u};
  for (unsigned s : seeds) {
    std::default_random_engine g(s);
    std::uniform_real_distribution<float> uf{0.0, 1.0};
    std::printf("%u float", s);
    for (int i = 0; i < 16; i++) std::printf(" %.9g", (double)uf(g));
    std::printf("\n");
    std::default_random_engine g2(s);
    std::uniform_real_distribution<double> ud(-0.01, 0.01);
    std::printf("%u double_pm0.01", s);
    for (int i = 0; i < 16; i++) std::printf(" %.17g", ud(g2));
    std::printf("\n");
    std::default_random_engine g3(s);
    std::printf("%u raw", s);
    for (int i = 0; i < 16; i++) std::printf(" %u", (unsigned)g3());
    std::printf("\n");
    for (int n : {1, 2, 3, 4, 11, 30, 31, 121, 441, 1024}) {
      std::default_random_engine g4(s);
      std::vector<int> v(n);
      for (int i = 0; i < n; i++) v[i] = i;
      std::shuffle(std::begin(v), std::end(v), g4);
      std::printf("%u shuffle%d", s, n);
      for (int x : v) std::printf(" %d", x);
      std::printf("\n%u shuffle%d_next %u\n", s, n, (unsigned)g4());   // engine position after it
    }
  }
  return 0;
}
