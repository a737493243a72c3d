// asan_host.cpp -- TEST INFRASTRUCTURE ONLY: the host builds of the kernel's
// headers under AddressSanitizer + UndefinedBehaviorSanitizer.
//
// np_math.h (the reference NumPy's sin/cos/tan/power, as npmath.cpp builds it
// for tests/test_np_math.py) and nproots.h (np.roots restated, as
// tests/test_nproots.py builds it) run over random, edge and special inputs;
// the sanitizers abort on any out-of-bounds table read, overflow or undefined
// shift.  The values are checked elsewhere (bitwise vs NumPy); this driver
// only prints a checksum so the calls are not optimised away.
//
// Build: make -C oracle asan  ->  oracle/_devmath/asan_host; run by
// tests/test_sanitizers.py.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <random>

static inline double fma_rz(double a, double b, double c) {
  asm("vfmadd213sd %{rz-sae%}, %2, %1, %0" : "+x"(a) : "x"(b), "x"(c));
  return a;
}
static inline double mul_rz(double a, double b) {
  asm("vmulsd %{rz-sae%}, %1, %0, %0" : "+x"(a) : "x"(b));
  return a;
}
static inline double add_rz(double a, double b) {
  asm("vaddsd %{rz-sae%}, %1, %0, %0" : "+x"(a) : "x"(b));
  return a;
}
static inline double add_rd(double a, double b) {
  asm("vaddsd %{rd-sae%}, %1, %0, %0" : "+x"(a) : "x"(b));
  return a;
}
#define NM_FN static inline
#define NM_CONST static constexpr
#define NM_TABLE static const
#define NM_FMA_RZ(a, b, c) fma_rz((a), (b), (c))
#define NM_MUL_RZ(a, b) mul_rz((a), (b))
#define NM_ADD_RZ(a, b) add_rz((a), (b))
#define NM_ADD_RD(a, b) add_rd((a), (b))
#define NM_FALLBACK_SIN(x) std::sin(x)
#define NM_FALLBACK_COS(x) std::cos(x)
#define NM_FALLBACK_TAN(x) std::tan(x)
#define NM_FALLBACK_POW(x, y) std::pow((x), (y))
#include "np_math.h"
#include <math.h>
#define RWRT_HD
#include "nproots.h"

static uint64_t bits(double x) {
  uint64_t u;
  std::memcpy(&u, &x, 8);
  return u;
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? std::atol(argv[1]) : 200000;
  std::mt19937_64 rng(7);
  std::uniform_real_distribution<double> U(-1.0, 1.0);
  const double inf = std::numeric_limits<double>::infinity(), nan = std::nan("");
  const double specials[] = {0.0, -0.0, inf, -inf, nan, 1e-310, -1e-310, 5e-324, 1e308, -1e308,
                             0.85546875, 2.426265, 105414350.0, 65536.0, 1.0, -1.0, 3.141592653589793,
                             1.5707963267948966, 2.0, 0.5};
  uint64_t h = 0;
  auto mix = [&](double v) { h = h * 1099511628211ull ^ bits(v); };
  for (long i = 0; i < n; ++i) {
    // arguments over many scales, and every special value now and then
    double x = U(rng) * std::pow(10.0, (int)(rng() % 40) - 20);
    double y = U(rng) * std::pow(10.0, (int)(rng() % 8) - 4);
    if (i % 97 == 0) x = specials[(i / 97) % 20];
    if (i % 89 == 0) y = specials[(i / 89) % 20];
    mix(np_math::nm_sin(x));
    mix(np_math::nm_cos(x));
    mix(np_math::nm_tan(x));
    double s, c, t;
    np_math::nm_sincostan(x, s, c, t);
    mix(s + c + t);
    mix(np_math::nm_pow(std::fabs(x), y));
    mix(np_math::nm_pow(x, y));
    // np.roots of degree 1..3, highest coefficient first
    double p[4];
    const int deg = 1 + (int)(rng() % 3);
    for (int q = 0; q <= deg; ++q) p[q] = U(rng) * std::pow(10.0, (int)(rng() % 12) - 6);
    if (i % 53 == 0) p[rng() % (deg + 1)] = specials[(i / 53) % 20];
    if (i % 59 == 0) p[deg] = 0.0;
    nproots::cx r[3] = {{nan, nan}, {nan, nan}, {nan, nan}};
    const bool finite = std::isfinite(p[0]) && std::isfinite(p[1]) && (deg < 2 || std::isfinite(p[2])) &&
                        (deg < 3 || std::isfinite(p[3]));
    if (finite && p[0] != 0.0) {
      nproots::np_roots(p, deg, r);
      for (int q = 0; q < 3; ++q) mix(r[q].re + r[q].im);
    }
  }
  std::printf("asan_host ok: %ld cases, checksum %016llx\n", n, (unsigned long long)h);
  return 0;
}
