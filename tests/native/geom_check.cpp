// Host-side check of the implicit-GEMM geometry helpers (csrc/conv_geom.h), built with
// AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_host_sanitizers.py.
// The device code divides pixel indices by the GEMM grid sizes with
//   q = (umulhi(n, mul) + n) >> shr        (32-bit, n < 2^31)
// — this program checks that formula against n / d for every divisor the kernels use
// (1..4096) on edge values and a pseudo-random sweep, and checks geom_finalize on the
// ResNet-18 layer grids.
#include <cstdint>
#include <cstdio>

#include "../../csrc/conv_geom.h"

static inline unsigned umulhi(unsigned a, unsigned b) {
  return (unsigned)(((unsigned long long)a * b) >> 32);
}

int main() {
  unsigned long long checked = 0;
  unsigned x = 12345u;
  for (unsigned d = 1; d <= 4096; ++d) {
    unsigned mul, shr;
    dm::fastdiv_init(d, mul, shr);
    const unsigned edge[] = {0u, 1u, d - 1, d, d + 1, 2 * d - 1, 2 * d, 0x7fffffffu,
                             0x7fffffffu - d, (0x7fffffffu / d) * d, (0x7fffffffu / d) * d - 1};
    for (unsigned n : edge) {
      if (n > 0x7fffffffu) continue;
      const unsigned q = (umulhi(n, mul) + n) >> shr;
      if (q != n / d) {
        std::printf("fastdiv mismatch d=%u n=%u q=%u\n", d, n, q);
        return 1;
      }
      ++checked;
    }
    for (int i = 0; i < 2000; ++i) {
      x = x * 1664525u + 1013904223u;
      const unsigned n = x & 0x7fffffffu;
      const unsigned q = (umulhi(n, mul) + n) >> shr;
      if (q != n / d) {
        std::printf("fastdiv mismatch d=%u n=%u q=%u\n", d, n, q);
        return 1;
      }
      ++checked;
    }
  }
  // ResNet-18 grids: m = (n*Hg + y)*Wg + x decomposed back exactly
  const int grids[][2] = {{112, 112}, {56, 56}, {28, 28}, {14, 14}, {7, 7}, {56, 28}};
  for (auto& gr : grids) {
    dm::ConvGeom g{};
    g.Hg = gr[0];
    g.Wg = gr[1];
    dm::geom_finalize(g);
    for (unsigned m = 0; m < 256u * g.Hg * g.Wg; m += 97) {
      const unsigned t = (umulhi(m, g.wg_mul) + m) >> g.wg_shr;
      const unsigned xx = m - t * g.Wg;
      const unsigned n = (umulhi(t, g.hg_mul) + t) >> g.hg_shr;
      const unsigned y = t - n * g.Hg;
      if (xx >= (unsigned)g.Wg || y >= (unsigned)g.Hg || (n * g.Hg + y) * g.Wg + xx != m) {
        std::printf("decompose mismatch grid %dx%d m=%u\n", g.Hg, g.Wg, m);
        return 1;
      }
      ++checked;
    }
  }
  std::printf("ok %llu\n", checked);
  return 0;
}
