// devmath.cpp -- TEST INFRASTRUCTURE ONLY (see oracle/rwrt_oracle.py's header).
//
// The device's transcendental functions for the HOST: the same source the
// kernel runs (rossby-wave-ray-tracing_amd/csrc/rwrt_math.h: sin/cos/tan with
// one reduction and pow, ocml's f64 algorithms restated), compiled with gcc.
// rwrt_oracle.device_math() swaps these in for NumPy's sin/cos/tan/power so
// the oracle computes exactly what the GPU computes, transcendental for
// transcendental; trajectories then compare bit for bit over any horizon
// (tests/test_gpu_devmath.py).  Never linked into the product.
//
// Build: oracle/Makefile -> oracle/_devmath/libdevmath.so
#include <cmath>
#include <cstdint>

#define RM_FN static inline
#define RM_FMA3(a, b, c) std::fma((a), (b), (c))
#define RM_RECIP2(b) (1.0 / (b))
using std::fabs;
using std::fma;
using std::fmax;
using std::fmin;
using std::frexp;
using std::ldexp;
using std::rint;
using std::trunc;
using std::copysign;
#include "rwrt_math.h"

using namespace rwrt_math;

// np.sin / np.cos / np.tan replacements: |x| >= 2^30, inf and NaN use glibc
// (the device uses its library there too; no such argument reaches the
// kernel's reduced path)
static inline void sct(double x, double& s, double& c, double& t) {
  if (!(std::fabs(x) < 0x1p30)) {
    s = std::sin(x);
    c = std::cos(x);
    t = std::tan(x);
    return;
  }
  rm_sincostan_small(x, s, c, t);
}

extern "C" {

void dm_sin(const double* x, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) { double s, c, t; sct(x[i], s, c, t); out[i] = s; }
}
void dm_cos(const double* x, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) { double s, c, t; sct(x[i], s, c, t); out[i] = c; }
}
void dm_tan(const double* x, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) { double s, c, t; sct(x[i], s, c, t); out[i] = t; }
}
// x ** y element-wise (y broadcast when ystride == 0)
void dm_pow(const double* x, const double* y, int64_t ystride, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = rm_pow(x[i], y[i * ystride]);
}
void dm_exp(const double* x, double* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = rm_exp(x[i]);
}

}  // extern "C"
