// rwrt.hip -- fused RK45 Rossby-wave ray integrator for MI355X (gfx950).
//
// One lane owns one ray for a whole time chunk: Dormand-Prince 5(4) stages,
// the dispersion-relation RHS (bilinear gather of the basic state, Mercator
// conversion, group velocity, wavenumber/amplitude tendencies), per-ray
// adaptive step control, the per-interval masks and the output rows all run
// in registers.  Lanes pull rays from a device work queue so that a lane whose
// ray finishes early immediately starts another one (the 4.6x spread of steps
// per ray would otherwise idle most of every wavefront).
//
// Numerics follow the reference operation by operation (built with
// -ffp-contract=off, IEEE division and sqrt): every expression keeps the
// reference's evaluation order.  Reference file:line in each comment.

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <type_traits>

#include "rwrt.h"
#include "nproots.h"

// RARE(c): the condition of a rarely taken branch.  The static analysis build
// (-DRWRT_ANALYZE_HOT, tools/hot_count.py; never loaded) compiles those branches
// away so that the run kernel's loop is its common path, straight-line, and
// its static instruction count is the dynamic count of an attempt.
#ifdef RWRT_ANALYZE_HOT
// (the condition is still computed: its lane mask is consumed by an empty asm)
__device__ __forceinline__ bool rwrt_rare_sink(bool c) {
  asm volatile("; rare %0" ::"s"(__builtin_amdgcn_ballot_w64(c)));
  return false;
}
#define RARE(c) rwrt_rare_sink(c)
#else
#define RARE(c) (c)
#endif
// MARK(name): a named point in the analysis build's assembly (tools/hot_count.py
// --marks counts the instructions between consecutive marks); nothing otherwise
#ifdef RWRT_ANALYZE_MARK
#define MARK(name) do { __builtin_amdgcn_sched_barrier(0); asm volatile("; @MARK " name); __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define MARK(name)
#endif

namespace rwrt {

// constants.py:13-16
constexpr double kPi = 3.14159265358979323846;
constexpr double kHalfPi = 0.5 * kPi;  // "0.5 * pi"  wr.py:508, bs.py:787
constexpr double kTwoPi = 2.0 * kPi;   // "2 * pi"    bs.py:519, interpolation.py:80
constexpr double kREarth = 6.3712e6;
constexpr double kOmega = 7.2921e-5;   // constants.py omega

// x / R (wr.py:80-82), IEEE
__device__ __forceinline__ double div_rearth(double x) { return x / kREarth; }
constexpr double kNaN = __builtin_nan("");

// Output rows are written once and never read back by the kernels.  The ray
// loops store a ray's 64-B row with plain (write-back) stores: the L2 merges
// the four 16-B pieces -- and a ray's next row, the other half of the 128-B
// line -- before writing back, so HBM sees the row bytes (1.16x).  Marked
// non-temporal they streamed past the L2 as partial writes, 2.4x the row
// bytes, and the step was 1 % slower (round 5, profiles/r5/rows/).
// (RWRT_ROW_NT=1: non-temporal row stores, A/B build.)  frozen_fill_kernel's
// coalesced full-line stores stay non-temporal.
#ifndef RWRT_ROW_NT
#define RWRT_ROW_NT 0
#endif
typedef double v2f64 __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ void store_row16(double2* o, double2 v) {
  if (NT) {
    v2f64 w;
    w.x = v.x;
    w.y = v.y;
    __builtin_nontemporal_store(w, reinterpret_cast<v2f64*>(o));
  } else {
    *o = v;
  }
}

// Two IEEE f64 divisions qa = a1 / b1, qb = a2 / b2 with the compiler's own
// instruction sequence (v_div_scale, v_rcp, two Newton steps, v_div_fmas,
// v_div_fixup: correctly rounded for every input), interleaved by hand.  The
// compiler emits each division as a dependent chain that waits on the
// v_rcp result and on VCC before v_div_fmas (an s_nop each, 2 of 13 issue
// slots); two chains fill each other's waits.  VCC carries the numerator's
// scale flag from v_div_scale to v_div_fmas, so the two flag windows are
// sequential: A's flag is written early (it only needs the inputs) and read
// 5 instructions later; B's is written after A's v_div_fmas and read after
// 3 instructions + 1 wait state (4 are required).
__device__ __forceinline__ void div2(double a1, double b1, double a2, double b2, double& qa,
                                     double& qb) {
  double dA, dB, rA, rB, eA, eB, nA, nB;
  asm(
      "v_div_scale_f64 %[dA], vcc, %[bA], %[bA], %[aA]\n\t"
      "v_div_scale_f64 %[dB], vcc, %[bB], %[bB], %[aB]\n\t"
      "v_rcp_f64 %[rA], %[dA]\n\t"
      "v_rcp_f64 %[rB], %[dB]\n\t"
      "v_fma_f64 %[eA], -%[dA], %[rA], 1.0\n\t"
      "v_fma_f64 %[eB], -%[dB], %[rB], 1.0\n\t"
      "v_fma_f64 %[rA], %[rA], %[eA], %[rA]\n\t"
      "v_fma_f64 %[rB], %[rB], %[eB], %[rB]\n\t"
      "v_fma_f64 %[eA], -%[dA], %[rA], 1.0\n\t"
      "v_div_scale_f64 %[nA], vcc, %[aA], %[bA], %[aA]\n\t"
      "v_fma_f64 %[eB], -%[dB], %[rB], 1.0\n\t"
      "v_fma_f64 %[rA], %[rA], %[eA], %[rA]\n\t"
      "v_fma_f64 %[rB], %[rB], %[eB], %[rB]\n\t"
      "v_mul_f64 %[qA], %[nA], %[rA]\n\t"
      "v_fma_f64 %[eA], -%[dA], %[qA], %[nA]\n\t"
      "v_div_fmas_f64 %[qA], %[eA], %[rA], %[qA]\n\t"
      "v_div_scale_f64 %[nB], vcc, %[aB], %[bB], %[aB]\n\t"
      "v_mul_f64 %[qB], %[nB], %[rB]\n\t"
      "v_fma_f64 %[eB], -%[dB], %[qB], %[nB]\n\t"
      "v_div_fixup_f64 %[qA], %[qA], %[bA], %[aA]\n\t"
      "s_nop 0\n\t"
      "v_div_fmas_f64 %[qB], %[eB], %[rB], %[qB]\n\t"
      "v_div_fixup_f64 %[qB], %[qB], %[bB], %[aB]"
      : [qA] "=&v"(qa), [qB] "=&v"(qb), [dA] "=&v"(dA), [dB] "=&v"(dB), [rA] "=&v"(rA),
        [rB] "=&v"(rB), [eA] "=&v"(eA), [eB] "=&v"(eB), [nA] "=&v"(nA), [nB] "=&v"(nB)
      : [aA] "v"(a1), [bA] "v"(b1), [aB] "v"(a2), [bB] "v"(b2)
      : "vcc");
}

// rkf45.py:604-615 (Dormand-Prince 5(4)); C++ constant division is IEEE
// correctly rounded, like Python's.
constexpr double kC[6] = {0.0, 1.0 / 5, 3.0 / 10, 4.0 / 5, 8.0 / 9, 1.0};
constexpr double kA[6][5] = {
    {0, 0, 0, 0, 0},
    {1.0 / 5, 0, 0, 0, 0},
    {3.0 / 40, 9.0 / 40, 0, 0, 0},
    {44.0 / 45, -56.0 / 15, 32.0 / 9, 0, 0},
    {19372.0 / 6561, -25360.0 / 2187, 64448.0 / 6561, -212.0 / 729, 0},
    {9017.0 / 3168, -355.0 / 33, 46732.0 / 5247, 49.0 / 176, -5103.0 / 18656}};
constexpr double kB[6] = {35.0 / 384, 0, 500.0 / 1113, 125.0 / 192, -2187.0 / 6784, 11.0 / 84};
constexpr double kE[7] = {-71.0 / 57600, 0, 71.0 / 16695, -71.0 / 1920,
                          17253.0 / 339200, -22.0 / 525, 1.0 / 40};
constexpr double kSafety = 0.9, kMinFactor = 0.2, kMaxFactor = 10.0;  // rkf45.py:363-366
constexpr double kErrExp = -0.2;  // -1 / (error_estimator_order + 1)   rkf45.py:360

// x.shape[0] ** 0.5 in rkf45.norm (rkf45.py:31), per number of variables.
template <int NV> struct RootN;
template <> struct RootN<1> { static constexpr double v = 1.0; };
template <> struct RootN<3> { static constexpr double v = 1.7320508075688772; };
template <> struct RootN<5> { static constexpr double v = 2.23606797749979; };

// ---------------------------------------------------------------------------
// NumPy element semantics
// ---------------------------------------------------------------------------
// np.maximum / np.minimum: NaN-propagating.
__device__ __forceinline__ double np_max(double a, double b) {
  return (a >= b || a != a) ? a : b;
}
__device__ __forceinline__ double np_min(double a, double b) {
  return (a <= b || a != a) ? a : b;
}
// fmod(a, b) for b > 0, exact (fmod is always exactly representable): for
// |a| < 2^40 the integer quotient n = trunc(|a|/b) is off by at most one.  The
// remainder r = |a| - n b is a multiple of ulp(b) (or |a| itself), exact from
// one FMA when it lies in (-b, b); a quotient one too large shows as r < 0 and
// r + b is then the exact remainder; one too small as r >= b (possibly
// rounded), recomputed with n + 1.  Branch-free apart from the library call
// for huge, infinite or NaN |a|.  binv (optional) ~ 1/b replaces the
// division: its quotient is off by at most one too (relative error ~2^-52 of
// a quotient below 2^40), which the same correction absorbs.
__device__ __forceinline__ double fmod_pos(double a, double b, double binv = 0.0) {
  const double x = fabs(a);
  const double n = trunc(binv != 0.0 ? x * binv : x / b);
  double r = fma(-n, b, x);
  const double lo = r + b, hi = fma(-(n + 1.0), b, x);
  r = (r < 0.0) ? lo : ((r >= b) ? hi : r);
  if (RARE(!(x < 0x1p40))) {
    asm volatile("");   // NaN, inf, huge: library routine (rare branch)
    r = fabs(fmod(a, b));
  }
  return copysign(r, a);
}

// Python/NumPy floor modulo for float64 (npy_remainder): fmod, then move a
// remainder whose sign differs from b into [0, b); exact zero gets b's sign.
__device__ __forceinline__ double py_mod(double a, double b, double binv = 0.0) {
  double m = fmod_pos(a, b, binv);
  if (m != 0.0) {
    if ((b < 0.0) != (m < 0.0)) m += b;
  } else {
    m = copysign(0.0, b);
  }
  return m;
}
// x % (2 * pi) (bs.py:519, interpolation.py:80)
constexpr double kInvTwoPi = 1.0 / kTwoPi;
__device__ __forceinline__ double py_mod_2pi(double a) { return py_mod(a, kTwoPi, kInvTwoPi); }
// py_mod_2pi(m) for m = py_mod_2pi(x), which lies in [0, 2 pi] or is NaN: the
// identity, except that a remainder that rounded up to 2 pi itself becomes +0.
__device__ __forceinline__ double py_mod_2pi_again(double m) { return (m >= kTwoPi) ? 0.0 : m; }

// np.floor(x).astype('int32') on x86-64 (cvttsd2si): out-of-range and NaN give
// INT32_MIN.  v_cvt_i32_f64 saturates (INT32_MIN below the range, as x86) and
// maps NaN to 0; above the range x86's INT32_MIN is restored.  (NaN -> 0 only
// moves the x1/y1 corner of a lookup whose weights are NaN: same NaN result.)
__device__ __forceinline__ int floor_i32(double x) {
  const double f = floor(x);
  const int i = __double2int_rz(f);
  return (f > 2147483647.0) ? INT32_MIN : i;
}
// x0 + 1 on an int32 array: wraps (NumPy integer arithmetic is modular)
__device__ __forceinline__ int inc_i32(int v) { return (int)((unsigned)v + 1u); }
// np.clip(v, 0, hi) -> v_med3_i32
__device__ __forceinline__ int clip(int v, int hi) { return ::max(0, ::min(v, hi)); }

// a / b with the reciprocal rb of b precomputed by recip_hw(b): the same
// operations as the compiler's IEEE f64 division (v_div_scale, v_rcp_f64, two
// Newton steps, q = a*r, rem = fma(-b, q, a), q' = fma(rem, r, q),
// v_div_fixup) minus the scaling and special-case steps, which are the
// identity when nothing is near the exponent limits: b in [2^-100, 2^100]
// (else recip_hw returns 0 and every quotient takes the IEEE division), a in
// {0} U [2^-900, 2^600] (else, or non-finite, the IEEE division).  The sign of
// a zero quotient comes from q = a * r.  Bit-identical to a / b
// (tests/test_gpu_parity.py::test_device_math_exactness).
__device__ __forceinline__ double recip_hw(double b) {
  const double ab = fabs(b);
  double r = __builtin_amdgcn_rcp(b);
  double e = fma(-b, r, 1.0);
  r = fma(r, e, r);
  e = fma(-b, r, 1.0);
  r = fma(r, e, r);
  return (ab >= 0x1p-100 && ab <= 0x1p100) ? r : 0.0;
}
__device__ __forceinline__ double div_hw(double a, double b, double rb) {
  const double q = a * rb;
  const double rem = fma(-b, q, a);
  double r = copysign(fma(rem, rb, q), q);
  const double aa = fabs(a);
  const bool bad = !(aa < 0x1p600) | ((aa < 0x1p-900) & (aa != 0.0)) | (rb == 0.0);
  if (RARE(bad)) {
    asm volatile("");   // keep the IEEE division on its (rarely taken) branch
    r = a / b;
  }
  return r;
}

// ---------------------------------------------------------------------------
// Basic state: packed [W][H][12] fp64, the 11 hot fields of BS.fields
// ---------------------------------------------------------------------------
enum { F_U = 0, F_V, F_UX, F_UY, F_VX, F_VY, F_QX, F_QY, F_QXX, F_QXY, F_QYY, F_PAD };
constexpr int kNF = RWRT_NFIELD_PACK;
// slot -> index in the reference 18-field stack (bs.py:349-368); qyx (10) and
// the six third derivatives are never read on the hot path.
__constant__ int kRefIndex[11] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 11};

struct Field {
  const double* __restrict__ P;
  int W, H;
  double lon0, dlon, lat0, dlat;
};

// Bilinear corner set + weights of batch_linint2_metpy/bilinear_interpolation_
// (interpolation.py:77-85, 103-135) for one in-range point.
struct Corners {
  const double* a;  // F[x0, y1]
  const double* b;  // F[x1, y1]
  const double* c;  // F[x0, y0]
  const double* d;  // F[x1, y0]
  double wa, wb, wc, wd;
  unsigned key_x, key_y;   // x0 | x1 << 16, y0 | y1 << 16 (W, H < 2^16)
  unsigned pa, pb, pc, pd; // grid-point indices x * H + y of a, b, c, d
  unsigned oa, ob, oc, od; // element offsets of a, b, c, d from F.P
};

__device__ __forceinline__ Corners corners(const Field& F, double lon, double lat) {
  // lon arrives already reduced once (bs.py:519); interpolation.py:80 reduces again.
  const double lons = py_mod_2pi_again(lon);
  double x, y;
  div2(lons - F.lon0, F.dlon, lat - F.lat0, F.dlat, x, y);
  const int ix = floor_i32(x), iy = floor_i32(y);
  const int x0 = clip(ix, F.W - 1), x1 = clip(inc_i32(ix), F.W - 1);
  const int y0 = clip(iy, F.H - 1), y1 = clip(inc_i32(iy), F.H - 1);
  const double sx = x - (double)x0, sy = y - (double)y0;
  // 32-bit element offsets (a packed state holds < 2^31 doubles; checked on the host)
  // (W, H < 2^24: 24-bit multiplies)
  const unsigned c0 = __umul24(x0, F.H), c1 = __umul24(x1, F.H);
  Corners k;
  k.pa = c0 + y1;
  k.pb = c1 + y1;
  k.pc = c0 + y0;
  k.pd = c1 + y0;
  k.oa = __umul24(k.pa, kNF);
  k.ob = __umul24(k.pb, kNF);
  k.oc = __umul24(k.pc, kNF);
  k.od = __umul24(k.pd, kNF);
  k.a = F.P + k.oa;
  k.b = F.P + k.ob;
  k.c = F.P + k.oc;
  k.d = F.P + k.od;
  k.wa = (1.0 - sx) * sy;
  k.wb = sx * sy;
  k.wc = (1.0 - sx) * (1.0 - sy);
  k.wd = sx * (1.0 - sy);
  k.key_x = (unsigned)x0 | ((unsigned)x1 << 16);
  k.key_y = (unsigned)y0 | ((unsigned)y1 << 16);
  return k;
}

// a*wa + b*wb + c*wc + d*wd, left to right (interpolation.py:132-133)
__device__ __forceinline__ double blend(const Corners& k, double a, double b, double c, double d) {
  return ((a * k.wa + b * k.wb) + c * k.wc) + d * k.wd;
}

// Interpolate all 11 hot fields (NaN outside |lat| <= pi/2, bs.py:787,822-836).
__device__ __forceinline__ void interp11(const Field& F, double lon, double lat, double g[11]) {
  if (!(fabs(lat) <= kHalfPi)) {
#pragma unroll
    for (int i = 0; i < 11; ++i) g[i] = kNaN;
    return;
  }
  const Corners k = corners(F, lon, lat);
  const double2* pa = reinterpret_cast<const double2*>(k.a);
  const double2* pb = reinterpret_cast<const double2*>(k.b);
  const double2* pc = reinterpret_cast<const double2*>(k.c);
  const double2* pd = reinterpret_cast<const double2*>(k.d);
  // Three groups of 2 records x 4 corners: bounds the registers held by
  // in-flight loads (the lookup is L2-resident; occupancy hides the latency).
#pragma unroll
  for (int q0 = 0; q0 < 6; q0 += 2) {
#pragma unroll
    for (int q = q0; q < q0 + 2; ++q) {
      const double2 va = pa[q], vb = pb[q], vc = pc[q], vd = pd[q];
      g[2 * q] = blend(k, va.x, vb.x, vc.x, vd.x);
      if (2 * q + 1 < 11) g[2 * q + 1] = blend(k, va.y, vb.y, vc.y, vd.y);
    }
    if (q0 + 2 < 6) __builtin_amdgcn_sched_barrier(0);
  }
}

// Only u, v, qx, qy (what cal_ugvg needs, wr.py:856-865).
__device__ __forceinline__ void interp4(const Field& F, double lon, double lat,
                                        double& fu, double& fv, double& fqx, double& fqy) {
  if (!(fabs(lat) <= kHalfPi)) {
    fu = fv = fqx = fqy = kNaN;
    return;
  }
  const Corners k = corners(F, lon, lat);
  const double2 a0 = *reinterpret_cast<const double2*>(k.a + F_U);
  const double2 b0 = *reinterpret_cast<const double2*>(k.b + F_U);
  const double2 c0 = *reinterpret_cast<const double2*>(k.c + F_U);
  const double2 d0 = *reinterpret_cast<const double2*>(k.d + F_U);
  const double2 a1 = *reinterpret_cast<const double2*>(k.a + F_QX);
  const double2 b1 = *reinterpret_cast<const double2*>(k.b + F_QX);
  const double2 c1 = *reinterpret_cast<const double2*>(k.c + F_QX);
  const double2 d1 = *reinterpret_cast<const double2*>(k.d + F_QX);
  fu = blend(k, a0.x, b0.x, c0.x, d0.x);
  fv = blend(k, a0.y, b0.y, c0.y, d0.y);
  fqx = blend(k, a1.x, b1.x, c1.x, d1.x);
  fqy = blend(k, a1.y, b1.y, c1.y, d1.y);
}

// ---------------------------------------------------------------------------
// Backgrounds the RHS reads.  StaticBG is the reference's (one basic state,
// fun ignores t: wr.py:784-789).  VaryingBG<T> is this framework's extension
// for time-varying flows (BASELINE configs[4]): nlev
// packed levels at t0 + j*dt, each interpolated bilinearly in space exactly
// like the static state, then linearly in time,
//   s = (t - t0)/dt, j = clip(floor(s), 0, nlev-2), w = clip(s - j, 0, 1),
//   g = g_j (1 - w) + g_{j+1} w                       (per hot field).
// T = float stores the levels in fp32 (half the gather bytes; arithmetic
// stays fp64).  A one-level background never takes this path.
// ---------------------------------------------------------------------------
struct StaticBG {
  static constexpr bool kTimeVarying = false;
  Field F;
  const char* img = nullptr;   // cache image of F (cache_image_kernel; the run kernels' refills)
  __device__ __forceinline__ void interp11(double lon, double lat, double, double g[11]) const {
    rwrt::interp11(F, py_mod_2pi(lon), lat, g);
  }
  __device__ __forceinline__ void interp4(double lon, double lat, double, double& fu, double& fv,
                                          double& fqx, double& fqy) const {
    rwrt::interp4(F, py_mod_2pi(lon), lat, fu, fv, fqx, fqy);
  }
};

// Lookups in two halves, begin() and end(): the RHS issues a lookup, computes
// what does not depend on it (sin, cos, tan of lat), then collects it.  For
// the plain backgrounds begin() only records the point.
struct PendingPoint {
  double lon, lat, t;
};
template <class BG>
__device__ __forceinline__ PendingPoint lookup_begin(const BG&, double lon, double lat, double t) {
  return PendingPoint{lon, lat, t};
}
template <class BG>
__device__ __forceinline__ void lookup_end(const BG& B, const PendingPoint& p, double g[11]) {
  B.interp11(p.lon, p.lat, p.t, g);
}

// StaticBG with a per-lane cache of the last cell's four corner records (the
// 11 hot fields of F[x0,y1], F[x1,y1], F[x0,y0], F[x1,y0]) in LDS.  The six
// stage evaluations of an attempt lie within a fraction of a 2.5-degree cell
// (C3: ~0.3 cell changes per 2-h interval against ~10 RHS evaluations), so a
// lookup is usually 24 conflict-free ds_read_b128 instead of 24 scattered
// 16-B global gathers.  A lane whose cell changed refills its slice by LDS-DMA
// (global_load_lds_dwordx4: no VGPRs, no ds_write), issued in begin() so that
// the fill's latency overlaps the trigonometry; end() waits for it.  Same
// values, same blend: results are unchanged.
//
// Slice layout (LDS-DMA writes wave base + lane * 16 B): per wave, chunk
// (corner j, record q) of all 64 lanes at wave_base + (j * 6 + q) * 1 KiB --
// a refill is 24 LDS-DMA instructions for the wave.  (A lane-major layout with
// one LDS-DMA per missing lane measured 0.91x on C3: every ray a lane pulls
// starts with a miss, so several lanes of a wave miss together;
// profiles/r2/ab/lane_slice.txt.)
constexpr int kCacheChunks = 4 * 6;                        // 4 corners x 6 x 16 B
constexpr int kCacheBytesPerWave = kCacheChunks * 64 * 16;  // 24 KiB
typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef __attribute__((address_space(1))) const void* global_void_ptr;

// The LDS destination (M0) of LDS-DMA chunk k of a refill: the wave's slice
// base passed through an opaque SGPR copy, so that the compiler rebuilds the
// 24 destinations with one s_add each instead of keeping 24 loop-invariant
// M0 values live (they spill to VGPR lanes: v_readlane + s_mov per load).
__device__ __forceinline__ char* lds_slice_base(char* wave_base) {
  typedef __attribute__((address_space(3))) char lds_char;
  unsigned b = (unsigned)(size_t)(lds_char*)wave_base;
  asm volatile("" : "+s"(b));
  return (char*)(lds_char*)(size_t)b;
}

// Before end() reads a slice: wait for the refill's LDS-DMA.  Explicit,
// because the compiler's own wait is not reliable once a kernel holds more
// than one LDS variable (the NumPy-math tables): its LDS reads then carry
// alias scopes, and a scoped read is only checked against LDS-DMA stores
// that carry scopes too -- which these (through lds_slice_base) do not.
__device__ __forceinline__ void lds_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The static cached lookup reads its cell's LDS slice software-pipelined by
// chunk (4 reads, 16 VGPRs each): chunk q is blended while chunk q + 1 is in
// flight, and chunk q + 2 is issued once q's registers are free.  All 24
// reads in flight at once (96 VGPRs) spilled 158 VGPRs to AGPRs; round 3's
// two groups of 12 (48 VGPRs) removed the spills (+2.3 %,
// profiles/r3/sched/pass_ee_cache_read_groups.txt) but left the second
// group's latency exposed; one chunk ahead: +1.5 % over the two groups, two
// chunks ahead +0.0 % (profiles/r4/sched/cache_pipe.txt).  The refill is
// ordered to match (CachedStaticBG::refill): chunks 0-3 of every corner
// first, so the first reads wait for part of it only.
constexpr int kCacheAhead = 1;
// end() reads chunks 0..kCacheAhead after waiting for the refill's first 16
// loads only (chunks 0-3, vmcnt(8)); the wait for all 24 sits before the
// read of chunk 4 -- a read-ahead of 4 or more would read chunk 4 early
static_assert(kCacheAhead >= 0 && kCacheAhead < 4, "end() prologue waits for chunks 0-3 only");

// The cache image of the static state: the records of 64 consecutive grid
// points stored chunk-major, so that a corner's six 16-B chunks lie 1 KiB
// apart in global memory exactly as in the LDS slice (where one LDS-DMA
// instruction writes its 64 lanes' 16 B as 1 KiB):
//   chunk q of point p at (p >> 6) * 6 KiB + q * 1 KiB + (p & 63) * 16 B.
// A refill then addresses each corner ONCE (a 32-bit offset from the image
// base) and its chunks by the instruction's immediate offset, which the
// hardware adds to the global and to the LDS address alike: per refill 4
// corner offsets and 8 M0 values instead of 24 64-bit addresses and 24 M0
// values.  Built per launch from the packed state (cache_image_kernel, ~1 MB
// at 2.5 degrees, the context's scratch).
constexpr unsigned kImgTile = 6 * 1024;
inline size_t cache_image_bytes(int64_t npts) { return (size_t)((npts + 63) / 64) * kImgTile; }
// (= p * 16 + (p >> 6) * 5 KiB: a shift, a 24-bit multiply, a shift-add)
__device__ __forceinline__ unsigned img_offset(unsigned p) { return __umul24(p >> 6, kImgTile - 1024u) + p * 16u; }

__global__ void cache_image_kernel(Field F, char* __restrict__ img) {
  const int64_t n = (int64_t)F.W * F.H * 6;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const unsigned p = (unsigned)(i / 6), q = (unsigned)(i - (int64_t)p * 6);
    const double2 v = reinterpret_cast<const double2*>(F.P + (size_t)p * kNF)[q];
    *reinterpret_cast<double2*>(img + img_offset(p) + q * 1024u) = v;
  }
}

struct CachedStaticBG {
  static constexpr bool kTimeVarying = false;
  Field F;
  const char* img;                // cache image of F (global)
  char* wave_base;                // this wave's slice area (wave-uniform)
  const char* img_hi;             // img + 4 KiB, kept in its own SGPR pair (the refill's chunks 4-5)
  unsigned lane16;                // lane * 16
  mutable unsigned key_x, key_y;  // cell held in the slice (~0u: none)

  struct Pending {
    double wa, wb, wc, wd;
  };
  __device__ __forceinline__ const double2& chunk(int j, int q) const {
    return *reinterpret_cast<const double2*>(wave_base + (j * 6 + q) * 1024 + lane16);
  }
  // The 24 LDS-DMA loads of a refill (corner j's chunks from image offset oj
  // into the slice at j * 6 KiB), in ONE asm statement that sets M0 itself
  // (M0 is compiler-reserved: saved and restored here).  Issued behind the
  // compiler's back on purpose: an LDS-DMA the compiler knows of makes it
  // wait for EVERY outstanding LDS read (lgkmcnt(0)) before the first use of
  // any -- the cell cache's reads in end() would all have to land before the
  // first blend; unaware of the DMA it waits per read (lgkmcnt(N)).  end()
  // waits for the DMA explicitly (lds_dma_wait), as before.
  __device__ __forceinline__ void refill(unsigned o0, unsigned o1, unsigned o2, unsigned o3) const {
    typedef __attribute__((address_space(3))) char lds_char;
    const unsigned l = (unsigned)(size_t)(lds_char*)wave_base;
    unsigned keep;
#define RWRT_REFILL_LO(O, LOFF)                                                  \
    "s_add_u32 m0, %[l], " #LOFF "\n\t"                                          \
    "s_nop 0\n\t"                                                               \
    "global_load_lds_dwordx4 %[" #O "], %[g0]\n\t"                              \
    "global_load_lds_dwordx4 %[" #O "], %[g0] offset:1024\n\t"                  \
    "global_load_lds_dwordx4 %[" #O "], %[g0] offset:2048\n\t"                  \
    "global_load_lds_dwordx4 %[" #O "], %[g0] offset:3072\n\t"
#define RWRT_REFILL_HI(O, LOFF4)                                                 \
    "s_add_u32 m0, %[l], " #LOFF4 "\n\t"                                         \
    "s_nop 0\n\t"                                                               \
    "global_load_lds_dwordx4 %[" #O "], %[g1]\n\t"                              \
    "global_load_lds_dwordx4 %[" #O "], %[g1] offset:1024\n\t"
    // chunks 0-3 of every corner first (16 loads), then chunks 4-5 (8): the
    // reads of chunks 0-3 wait for the first 16 only (vmcnt(8), end())
    asm volatile("s_mov_b32 %[keep], m0\n\t"
                 RWRT_REFILL_LO(o0, 0)
                 RWRT_REFILL_LO(o1, 6144)
                 RWRT_REFILL_LO(o2, 12288)
                 RWRT_REFILL_LO(o3, 18432)
                 RWRT_REFILL_HI(o0, 4096)
                 RWRT_REFILL_HI(o1, 10240)
                 RWRT_REFILL_HI(o2, 16384)
                 RWRT_REFILL_HI(o3, 22528)
                 "s_mov_b32 m0, %[keep]"
                 : [keep] "=&s"(keep)
                 : [g0] "s"(img), [g1] "s"(img_hi), [o0] "v"(o0), [o1] "v"(o1), [o2] "v"(o2),
                   [o3] "v"(o3), [l] "s"(l)
                 : "memory");
#undef RWRT_REFILL_LO
#undef RWRT_REFILL_HI
  }
  // Latency mode (quad_rays): the four lanes of a quad hold one ray, and lane
  // role r blends only records ra = r and rb = r + 4 (roles 2, 3: rb = r) of
  // the four corners (quad_lookup_end), so each lane loads just those two
  // chunks per corner into slots (j, 0) and (j, 1) of its slice: 8 LDS-DMA
  // loads per refill instead of 24.  qa = ra KiB, qb = (rb - 1) KiB: slot 1
  // is read with the instruction offset 1 KiB, which also moves the source.
  __device__ __forceinline__ void quad_refill(unsigned o0, unsigned o1, unsigned o2, unsigned o3, unsigned qa,
                                              unsigned qb) const {
    typedef __attribute__((address_space(3))) char lds_char;
    const unsigned l = (unsigned)(size_t)(lds_char*)wave_base;
    unsigned keep;
#define RWRT_QUAD_CORNER(O, LOFF)                                                 \
    "v_add_u32 %[ta], %[" #O "], %[qa]\n\t"                                       \
    "v_add_u32 %[tb], %[" #O "], %[qb]\n\t"                                       \
    "s_add_u32 m0, %[l], " #LOFF "\n\t"                                          \
    "s_nop 0\n\t"                                                               \
    "global_load_lds_dwordx4 %[ta], %[g0]\n\t"                                  \
    "global_load_lds_dwordx4 %[tb], %[g0] offset:1024\n\t"
    unsigned ta, tb;
    asm volatile("s_mov_b32 %[keep], m0\n\t"
                 RWRT_QUAD_CORNER(o0, 0)
                 RWRT_QUAD_CORNER(o1, 2048)
                 RWRT_QUAD_CORNER(o2, 4096)
                 RWRT_QUAD_CORNER(o3, 6144)
                 "s_mov_b32 m0, %[keep]"
                 : [keep] "=&s"(keep), [ta] "=&v"(ta), [tb] "=&v"(tb)
                 : [g0] "s"(img), [o0] "v"(o0), [o1] "v"(o1), [o2] "v"(o2), [o3] "v"(o3), [qa] "v"(qa),
                   [qb] "v"(qb), [l] "s"(l)
                 : "memory");
#undef RWRT_QUAD_CORNER
  }
  __device__ __forceinline__ Pending quad_begin(double lon, double lat, unsigned qa, unsigned qb) const {
    const Corners k = corners(F, py_mod_2pi(lon), lat);
    if (k.key_x != key_x || k.key_y != key_y) {
      quad_refill(img_offset(k.pa), img_offset(k.pb), img_offset(k.pc), img_offset(k.pd), qa, qb);
      key_x = k.key_x;
      key_y = k.key_y;
    }
    return Pending{k.wa, k.wb, k.wc, k.wd};
  }
  __device__ __forceinline__ Pending begin(double lon, double lat) const {
    const Corners k = corners(F, py_mod_2pi(lon), lat);
    const bool miss = k.key_x != key_x || k.key_y != key_y;
    if (miss) {   // miss: refill the slice by LDS-DMA from the cache image
      refill(img_offset(k.pa), img_offset(k.pb), img_offset(k.pc), img_offset(k.pd));
      key_x = k.key_x;
      key_y = k.key_y;
    }
    return Pending{k.wa, k.wb, k.wc, k.wd};
  }
  // fill(): independent work placed between the first reads and the first
  // blend (the reads' latency; nothing else is in flight there)
  template <class Fill>
  __device__ __forceinline__ void end(const Pending& p, double g[11], Fill&& fill) const {
    // the refill's first 16 loads (chunks 0-3) have landed once at most its
    // last 8 are outstanding: loads complete in order (chunk 4's reads wait
    // for them all)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    Corners k;
    k.wa = p.wa;
    k.wb = p.wb;
    k.wc = p.wc;
    k.wd = p.wd;
    constexpr int kAhead = kCacheAhead;
    double2 v[6][4];
#pragma unroll
    for (int q = 0; q <= kAhead; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[q][j] = chunk(j, q);
    fill();
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int f = 2 * q;
      g[f] = blend(k, v[q][0].x, v[q][1].x, v[q][2].x, v[q][3].x);
      if (f + 1 < 11) g[f + 1] = blend(k, v[q][0].y, v[q][1].y, v[q][2].y, v[q][3].y);
      __builtin_amdgcn_sched_barrier(0);
      const int n = q + kAhead + 1;
      if (n < 6) {
        if (n == 4) lds_dma_wait();
#pragma unroll
        for (int j = 0; j < 4; ++j) v[n][j] = chunk(j, n);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // Only the RHS looks up through the cache: a lane with |lat| > pi/2 is
  // masked there (its l is NaN, so are its derivatives), a NaN lat gives NaN
  // weights; the clipped cell keeps every access in bounds either way.
  __device__ __forceinline__ void interp4(double lon, double lat, double, double& fu, double& fv,
                                          double& fqx, double& fqy) const {
    rwrt::interp4(F, py_mod_2pi(lon), lat, fu, fv, fqx, fqy);
  }
};
__device__ __forceinline__ CachedStaticBG::Pending lookup_begin(const CachedStaticBG& B, double lon,
                                                                double lat, double) {
  return B.begin(lon, lat);
}
__device__ __forceinline__ void lookup_end(const CachedStaticBG& B,
                                           const CachedStaticBG::Pending& p, double g[11]) {
  B.end(p, g, [] {});
}
template <class Fill>
__device__ __forceinline__ void lookup_end(const CachedStaticBG& B, const CachedStaticBG::Pending& p,
                                           double g[11], Fill&& fill) {
  B.end(p, g, fill);
}
// (the other backgrounds: the independent work first)
template <class BG, class Fill>
__device__ __forceinline__ void lookup_end(const BG& B, const typename std::decay<decltype(lookup_begin(
                                                            B, 0.0, 0.0, 0.0))>::type& p,
                                           double g[11], Fill&& fill) {
  fill();
  lookup_end(B, p, g);
}

template <class T>
struct VaryingBG {
  static constexpr bool kTimeVarying = true;
  const T* __restrict__ P;   // [nlev][W][H][12]
  int W, H, nlev;
  int half;                  // fp64 ray loop at 32 rays per wave, both levels cached (rwrt_ctx_set_tv_lanes)
  int64_t lev_stride;        // W * H * 12
  double lon0, dlon, lat0, dlat, t0, dt;

  // cell corners and weights: the arithmetic of corners() (interpolation.py:77-135)
  __device__ __forceinline__ void cell(double lon, double lat, unsigned o[4], double w[4]) const {
    unsigned kx, ky;
    cell(lon, lat, o, w, kx, ky);
  }
  __device__ __forceinline__ void cell(double lon, double lat, unsigned o[4], double w[4],
                                       unsigned& key_x, unsigned& key_y) const {
    const double lons = py_mod_2pi_again(py_mod_2pi(lon));
    double x, y;
    div2(lons - lon0, dlon, lat - lat0, dlat, x, y);
    const int ix = floor_i32(x), iy = floor_i32(y);
    const int x0 = clip(ix, W - 1), x1 = clip(inc_i32(ix), W - 1);
    const int y0 = clip(iy, H - 1), y1 = clip(inc_i32(iy), H - 1);
    const double sx = x - (double)x0, sy = y - (double)y0;
    const unsigned c0 = __umul24(x0, H), c1 = __umul24(x1, H);
    o[0] = __umul24(c0 + y1, kNF);   // a = F[x0, y1]
    o[1] = __umul24(c1 + y1, kNF);   // b = F[x1, y1]
    o[2] = __umul24(c0 + y0, kNF);   // c = F[x0, y0]
    o[3] = __umul24(c1 + y0, kNF);   // d = F[x1, y0]
    w[0] = (1.0 - sx) * sy;
    w[1] = sx * sy;
    w[2] = (1.0 - sx) * (1.0 - sy);
    w[3] = sx * (1.0 - sy);
    key_x = (unsigned)x0 | ((unsigned)x1 << 16);
    key_y = (unsigned)y0 | ((unsigned)y1 << 16);
  }
  // level index and weight of time t
  __device__ __forceinline__ const T* level(double t, double& wt) const {
    int j;
    return level(t, wt, j);
  }
  __device__ __forceinline__ const T* level(double t, double& wt, int& jlev) const {
    const double s = (t - t0) / dt;
    const int64_t j = (nlev > 1) ? (int64_t)clip(floor_i32(s), nlev - 2) : 0;
    wt = np_min(np_max(s - (double)j, 0.0), 1.0);
    jlev = (int)j;
    return P + j * lev_stride;
  }
  __device__ __forceinline__ static double bl(const double w[4], double a, double b, double c,
                                              double d) {
    return ((a * w[0] + b * w[1]) + c * w[2]) + d * w[3];
  }
  // fields [f0, f0 + n) of one level at the corners
  template <int N>
  __device__ __forceinline__ void blend_level(const T* L, const unsigned o[4], const double w[4],
                                              int f0, double* g) const {
#pragma unroll
    for (int q = 0; q < N; ++q)
      g[q] = bl(w, (double)L[o[0] + f0 + q], (double)L[o[1] + f0 + q], (double)L[o[2] + f0 + q],
                (double)L[o[3] + f0 + q]);
  }
  __device__ __forceinline__ void interp11(double lon, double lat, double t, double g[11]) const {
    if (!(fabs(lat) <= kHalfPi)) {
#pragma unroll
      for (int i = 0; i < 11; ++i) g[i] = kNaN;
      return;
    }
    unsigned o[4];
    double w[4], wt;
    cell(lon, lat, o, w);
    const T* A = level(t, wt);
    const T* B = A + (nlev > 1 ? lev_stride : 0);
    double ga[11], gb[11];
    blend_level<11>(A, o, w, 0, ga);
    blend_level<11>(B, o, w, 0, gb);
#pragma unroll
    for (int i = 0; i < 11; ++i) g[i] = ga[i] * (1.0 - wt) + gb[i] * wt;
  }
  __device__ __forceinline__ void interp4(double lon, double lat, double t, double& fu, double& fv,
                                          double& fqx, double& fqy) const {
    if (!(fabs(lat) <= kHalfPi)) {
      fu = fv = fqx = fqy = kNaN;
      return;
    }
    unsigned o[4];
    double w[4], wt;
    cell(lon, lat, o, w);
    const T* A = level(t, wt);
    const T* B = A + (nlev > 1 ? lev_stride : 0);
    double a[2], b[2], c[2], d[2];
    blend_level<2>(A, o, w, F_U, a);
    blend_level<2>(B, o, w, F_U, b);
    blend_level<2>(A, o, w, F_QX, c);
    blend_level<2>(B, o, w, F_QX, d);
    fu = a[0] * (1.0 - wt) + b[0] * wt;
    fv = a[1] * (1.0 - wt) + b[1] * wt;
    fqx = c[0] * (1.0 - wt) + d[0] * wt;
    fqy = c[1] * (1.0 - wt) + d[1] * wt;
  }
};

// fp32 levels with an fp32 RHS (rwrt_background.fp32 == 2): the fields'
// blends, the time interpolation, the trigonometry, Mercator, group velocity
// and tendencies in fp32 (ray_rhs overload below); positions, the cell and
// level indices, time and the stepper stay fp64.  Not the reference's
// arithmetic: the fp32-vs-fp64 comparison of BASELINE configs[4].
struct VaryingBGA32 : VaryingBG<float> {};

// VaryingBG<float> with the same per-lane LDS cache, keyed by (cell, level
// pair): both bracketing levels' four fp32 corner records (2 x 4 x 48 B = 24
// chunks of 16 B, the same 24 KiB per wave as the static cache).  A lane
// refills when its cell or its level pair changes (every dt of ray time).
// fp64 levels would need twice the LDS and stay on plain gathers.
struct CachedVaryingBG32 {
  static constexpr bool kTimeVarying = true;
  VaryingBG<float> V;
  char* wave_base;
  unsigned lane16;
  mutable unsigned key_x, key_y;
  mutable int key_j;

  struct Pending {
    double w[4];
    double wt;
  };
  __device__ __forceinline__ float4 chunk(int lev, int j, int q) const {
    return *reinterpret_cast<const float4*>(wave_base + ((lev * 4 + j) * 3 + q) * 1024 + lane16);
  }
  __device__ __forceinline__ Pending begin(double lon, double lat, double t) const {
    Pending p;
    unsigned o[4], kx, ky;
    int jl;
    V.cell(lon, lat, o, p.w, kx, ky);
    const float* A = V.level(t, p.wt, jl);
    if (kx != key_x || ky != key_y || jl != key_j) {   // miss: refill by LDS-DMA
      const float* L[2] = {A, A + (V.nlev > 1 ? V.lev_stride : 0)};
      char* const base = lds_slice_base(wave_base);
#pragma unroll
      for (int lev = 0; lev < 2; ++lev)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int q = 0; q < 3; ++q)
            __builtin_amdgcn_global_load_lds((global_void_ptr)(L[lev] + o[j] + 4 * q),
                                             (lds_void_ptr)(base + ((lev * 4 + j) * 3 + q) * 1024),
                                             16, 0, 0);
      key_x = kx;
      key_y = ky;
      key_j = jl;
    }
    return p;
  }
  __device__ __forceinline__ void end(const Pending& p, double g[11]) const {
    lds_dma_wait();
    float4 v[2][4][3];
#pragma unroll
    for (int lev = 0; lev < 2; ++lev)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q) v[lev][j][q] = chunk(lev, j, q);
    __builtin_amdgcn_sched_barrier(0);
    double ga[11], gb[11];
#pragma unroll
    for (int f = 0; f < 11; ++f) {
      const int q = f >> 2, e = f & 3;
      auto el = [&](int lev, int j) -> double {
        const float4& c = v[lev][j][q];
        return (double)(e == 0 ? c.x : e == 1 ? c.y : e == 2 ? c.z : c.w);
      };
      ga[f] = VaryingBG<float>::bl(p.w, el(0, 0), el(0, 1), el(0, 2), el(0, 3));
      gb[f] = VaryingBG<float>::bl(p.w, el(1, 0), el(1, 1), el(1, 2), el(1, 3));
    }
#pragma unroll
    for (int i = 0; i < 11; ++i) g[i] = ga[i] * (1.0 - p.wt) + gb[i] * p.wt;
  }
  __device__ __forceinline__ void interp4(double lon, double lat, double t, double& fu, double& fv,
                                          double& fqx, double& fqy) const {
    V.interp4(lon, lat, t, fu, fv, fqx, fqy);
  }
};
__device__ __forceinline__ CachedVaryingBG32::Pending lookup_begin(const CachedVaryingBG32& B, double lon,
                                                                   double lat, double t) {
  return B.begin(lon, lat, t);
}
__device__ __forceinline__ void lookup_end(const CachedVaryingBG32& B,
                                           const CachedVaryingBG32::Pending& p, double g[11]) {
  B.end(p, g);
}

// VaryingBGA32 through CachedVaryingBG32's cache (the same LDS-DMA refills),
// blended in fp32 (endf)
struct CachedVaryingBGA32 : CachedVaryingBG32 {
  __device__ __forceinline__ void endf(const Pending& p, float g[11]) const {
    lds_dma_wait();
    float4 v[2][4][3];
#pragma unroll
    for (int lev = 0; lev < 2; ++lev)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 3; ++q) v[lev][j][q] = chunk(lev, j, q);
    __builtin_amdgcn_sched_barrier(0);
    const float w0 = (float)p.w[0], w1 = (float)p.w[1], w2 = (float)p.w[2], w3 = (float)p.w[3];
    const float wt = (float)p.wt;
#pragma unroll
    for (int f = 0; f < 11; ++f) {
      const int q = f >> 2, e = f & 3;
      auto el = [&](int lev, int j) -> float {
        const float4& c = v[lev][j][q];
        return e == 0 ? c.x : e == 1 ? c.y : e == 2 ? c.z : c.w;
      };
      const float ga = ((el(0, 0) * w0 + el(0, 1) * w1) + el(0, 2) * w2) + el(0, 3) * w3;
      const float gb = ((el(1, 0) * w0 + el(1, 1) * w1) + el(1, 2) * w2) + el(1, 3) * w3;
      g[f] = ga * (1.0f - wt) + gb * wt;
    }
  }
};

// VaryingBG<double> with the per-lane LDS cache holding ONE level: the lower
// bracketing level's four fp64 corner records (4 x 96 B = the static cache's
// 24 chunks), keyed by (cell, level pair); the upper level is gathered from
// global memory in end().  Both levels of fp64 corners (768 B per lane) would
// not fit next to the stages; caching one halves the gathers of every
// evaluation that stays in its cell.  Same values, same blend as
// VaryingBG<double>::interp11.
struct CachedVaryingBG64 {
  static constexpr bool kTimeVarying = true;
  VaryingBG<double> V;
  char* wave_base;
  unsigned lane16;
  mutable unsigned key_x, key_y;
  mutable int key_j;

  struct Pending {
    double w[4];
    double wt;
    unsigned o[4];
    const double* B;
  };
  __device__ __forceinline__ const double2& chunk(int j, int q) const {
    return *reinterpret_cast<const double2*>(wave_base + (j * 6 + q) * 1024 + lane16);
  }
  __device__ __forceinline__ Pending begin(double lon, double lat, double t) const {
    Pending p;
    unsigned kx, ky;
    int jl;
    V.cell(lon, lat, p.o, p.w, kx, ky);
    const double* A = V.level(t, p.wt, jl);
    p.B = A + (V.nlev > 1 ? V.lev_stride : 0);
    if (kx != key_x || ky != key_y || jl != key_j) {   // miss: refill by LDS-DMA
      char* const base = lds_slice_base(wave_base);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 6; ++q)
          __builtin_amdgcn_global_load_lds((global_void_ptr)(A + p.o[j] + 2 * q),
                                           (lds_void_ptr)(base + (j * 6 + q) * 1024), 16, 0, 0);
      if (V.half) {   // (wave-uniform) the upper level into lanes 32-63's slots
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int q = 0; q < 6; ++q)
            __builtin_amdgcn_global_load_lds((global_void_ptr)(p.B + p.o[j] + 2 * q),
                                             (lds_void_ptr)(base + (j * 6 + q) * 1024 + 512), 16, 0, 0);
      }
      key_x = kx;
      key_y = ky;
      key_j = jl;
    }
    return p;
  }
  // the eleven blends of one level from the slice (lv 1: the upper level,
  // half density only)
  __device__ __forceinline__ void cached11(int lv, const double w[4], double g[11]) const {
    double2 v[4][6];
#pragma unroll
    for (int q = 0; q < 6; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[j][q] = *reinterpret_cast<const double2*>(wave_base + (j * 6 + q) * 1024 + lv * 512 + lane16);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      g[2 * q] = VaryingBG<double>::bl(w, v[0][q].x, v[1][q].x, v[2][q].x, v[3][q].x);
      if (2 * q + 1 < 11) g[2 * q + 1] = VaryingBG<double>::bl(w, v[0][q].y, v[1][q].y, v[2][q].y, v[3][q].y);
    }
  }
  __device__ __forceinline__ void end(const Pending& p, double g[11]) const {
    lds_dma_wait();
    double gb[11];
    if (V.half) {
      double ga[11];
      cached11(0, p.w, ga);
      cached11(1, p.w, gb);
#pragma unroll
      for (int i = 0; i < 11; ++i) g[i] = ga[i] * (1.0 - p.wt) + gb[i] * p.wt;
      return;
    }
    V.blend_level<11>(p.B, p.o, p.w, 0, gb);
    double2 v[4][6];
#pragma unroll
    for (int q = 0; q < 6; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j][q] = chunk(j, q);
    __builtin_amdgcn_sched_barrier(0);
    double ga[11];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      ga[2 * q] = VaryingBG<double>::bl(p.w, v[0][q].x, v[1][q].x, v[2][q].x, v[3][q].x);
      if (2 * q + 1 < 11) ga[2 * q + 1] = VaryingBG<double>::bl(p.w, v[0][q].y, v[1][q].y, v[2][q].y, v[3][q].y);
    }
#pragma unroll
    for (int i = 0; i < 11; ++i) g[i] = ga[i] * (1.0 - p.wt) + gb[i] * p.wt;
  }
  __device__ __forceinline__ void interp4(double lon, double lat, double t, double& fu, double& fv,
                                          double& fqx, double& fqy) const {
    V.interp4(lon, lat, t, fu, fv, fqx, fqy);
  }
};
__device__ __forceinline__ CachedVaryingBG64::Pending lookup_begin(const CachedVaryingBG64& B, double lon,
                                                                   double lat, double t) {
  return B.begin(lon, lat, t);
}
__device__ __forceinline__ void lookup_end(const CachedVaryingBG64& B,
                                           const CachedVaryingBG64::Pending& p, double g[11]) {
  B.end(p, g);
}

// fp64 levels at 32 rays per wave (rwrt_ctx_set_tv_lanes 32), lane pairs
// (round 5): lanes L and L + 32 hold the same ray (the same state, the same
// operations -- run_rays<.., kPair>), and each caches ONE bracketing level in
// its own slice column: lane L the lower level, lane L + 32 the upper, at the
// LDS addresses the single-lane layout used (the upper level in lane L + 32's
// column).  A refill is then 24 LDS-DMA instructions for the wave with both
// halves active instead of 48 with one half, and each lane blends 11 fields
// instead of 22; v_permlane32_swap hands every lane both levels' blends
// (lanes 0-31's in one register, lanes 32-63's in the other), so the time
// interpolation g_A (1 - w) + g_B w is the same operation on the same values
// as VaryingBG<double>::interp11 -- bit for bit.
struct PairVaryingBG64 {
  static constexpr bool kTimeVarying = true;
  VaryingBG<double> V;
  char* wave_base;
  unsigned lane16;   // this lane's slice column (lane * 16)
  bool upper;        // lanes 32-63: the upper bracketing level
  mutable unsigned key_x, key_y;
  mutable int key_j;

  struct Pending {
    double w[4];
    double wt;
  };
  __device__ __forceinline__ Pending begin(double lon, double lat, double t) const {
    Pending p;
    unsigned o[4], kx, ky;
    int jl;
    V.cell(lon, lat, o, p.w, kx, ky);
    const double* A = V.level(t, p.wt, jl);
    if (kx != key_x || ky != key_y || jl != key_j) {   // miss (both lanes of the pair): refill by LDS-DMA
      const double* L = (upper && V.nlev > 1) ? A + V.lev_stride : A;
      char* const base = lds_slice_base(wave_base);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 6; ++q)
          __builtin_amdgcn_global_load_lds((global_void_ptr)(L + o[j] + 2 * q),
                                           (lds_void_ptr)(base + (j * 6 + q) * 1024), 16, 0, 0);
      key_x = kx;
      key_y = ky;
      key_j = jl;
    }
    return p;
  }
  // both lanes' values of x: (lanes 0-31's, lanes 32-63's) on every lane
  __device__ __forceinline__ static void both(double x, double& a, double& b) {
    const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    a = __hiloint2double((int)h[0], (int)l[0]);
    b = __hiloint2double((int)h[1], (int)l[1]);
  }
  __device__ __forceinline__ void end(const Pending& p, double g[11]) const {
    lds_dma_wait();
    double2 v[4][6];
#pragma unroll
    for (int q = 0; q < 6; ++q)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[j][q] = *reinterpret_cast<const double2*>(wave_base + (j * 6 + q) * 1024 + lane16);
    __builtin_amdgcn_sched_barrier(0);
    double go[11];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      go[2 * q] = VaryingBG<double>::bl(p.w, v[0][q].x, v[1][q].x, v[2][q].x, v[3][q].x);
      if (2 * q + 1 < 11) go[2 * q + 1] = VaryingBG<double>::bl(p.w, v[0][q].y, v[1][q].y, v[2][q].y, v[3][q].y);
    }
    MARK("p_blend");
    // g = g_A (1 - w) + g_B w: each lane forms its own level's product, the
    // swap hands both products to every lane, one add -- the same operations
    // on the same operands (4 instructions per field instead of 5)
    const double f = upper ? p.wt : 1.0 - p.wt;
#pragma unroll
    for (int i = 0; i < 11; ++i) {
      double pa, pb;
      both(go[i] * f, pa, pb);
      g[i] = pa + pb;
    }
  }
  __device__ __forceinline__ void interp4(double lon, double lat, double t, double& fu, double& fv,
                                          double& fqx, double& fqy) const {
    V.interp4(lon, lat, t, fu, fv, fqx, fqy);
  }
  __device__ static PairVaryingBG64 make(const VaryingBG<double>& B, char* lds) {
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    return PairVaryingBG64{B, lds + wave * kCacheBytesPerWave, (threadIdx.x & 63u) * 16u,
                           (threadIdx.x & 63u) >= 32u, ~0u, ~0u, -1};
  }
};
__device__ __forceinline__ PairVaryingBG64::Pending lookup_begin(const PairVaryingBG64& B, double lon, double lat,
                                                                 double t) {
  return B.begin(lon, lat, t);
}
__device__ __forceinline__ void lookup_end(const PairVaryingBG64& B, const PairVaryingBG64::Pending& p,
                                           double g[11]) {
  B.end(p, g);
}

// Latency mode of the time-varying ray loops (rk45_run_kernel's first
// heavy_blocks blocks, run_rays<.., kReplica>): ONE ray per wavefront,
// replicated on all 64 lanes (the same state and the same operations on every
// lane, so the wave never diverges), whose lookups read a block of kP x kP
// grid points (kP - 1 cells a side) of BOTH bracketing levels held in the
// wave's 24 KiB of LDS.  The per-lane cell cache refills whenever a stage
// leaves its cell or level pair -- 1.7-2.3 refills per attempt of the
// heaviest C5 rays at 0.25 degrees (tools/c5_misses.py,
// profiles/r5/c5lat/misses.json), each an HBM round trip in a dependent
// chain; here a ray moves kP / 2 - 1 cells or more before the block is
// reloaded, and a reload is kLoads wave-wide LDS-DMA instructions (64 lanes x
// 16 B each) instead of 48 single-lane ones.  Records are contiguous in the
// block: level lv, point (i, j) at ((lv * kP + i) * kP + j) * kRec bytes.  The
// corner values are the level arrays' own (the same doubles or floats), the
// blends and the time interpolation those of VaryingBG<T>::interp11: results
// are the run kernel's bit for bit.
template <class T>
struct BlockVaryingBG {
  static constexpr bool kTimeVarying = true;
  static constexpr int kP = 8;                                  // grid points per side
  static constexpr int kRec = 12 * (int)sizeof(T);              // one record: 96 B (fp64) / 48 B (fp32)
  static constexpr int kCh = kRec / 16;                         // 16-B chunks per record
  static constexpr int kChunks = 2 * kP * kP * kCh;             // chunks of a reload
  static constexpr int kLoads = (kChunks + 63) / 64;            // wave-wide LDS-DMA instructions
  static_assert(kChunks * 16 <= kCacheBytesPerWave, "block must fit the wave's LDS");
  VaryingBG<T> V;
  char* wave_base;
  mutable int bx, by, bj;   // block origin (grid point) and level pair held (bj = -1: none)

  struct Pending {
    double w[4];
    double wt;
    unsigned o[4];   // LDS byte offsets of corners a, b, c, d in level A's block
  };
  __device__ __forceinline__ Pending begin(double lon, double lat, double t) const {
    Pending p;
    unsigned og[4], kx, ky;
    int jl;
    V.cell(lon, lat, og, p.w, kx, ky);
    const T* A = V.level(t, p.wt, jl);
    const int x0 = (int)(kx & 0xffffu), x1 = (int)(kx >> 16), y0 = (int)(ky & 0xffffu), y1 = (int)(ky >> 16);
    if (!(jl == bj && x0 >= bx && x1 < bx + kP && y0 >= by && y1 < by + kP)) {
      // reload (wave-uniform: every lane holds the same ray): the cell near
      // the block's centre, the block inside the grid where it fits
      bx = min(max(x0 - (kP / 2 - 1), 0), max(V.W - kP, 0));
      by = min(max(y0 - (kP / 2 - 1), 0), max(V.H - kP, 0));
      bj = jl;
      const T* L[2] = {A, A + (V.nlev > 1 ? V.lev_stride : 0)};
      char* const base = lds_slice_base(wave_base);
      const int lane = (int)(threadIdx.x & 63u);
#pragma unroll
      for (int k = 0; k < kLoads; ++k) {
        const int c = k * 64 + lane;   // chunk q of record r = (lv, i, j)
        if (kChunks % 64 == 0 || c < kChunks) {
          const int r = c / kCh, q = c - r * kCh;
          const int lv = r / (kP * kP), pt = r - lv * (kP * kP);
          const int i = pt / kP, j = pt - i * kP;
          const int gx = min(bx + i, V.W - 1), gy = min(by + j, V.H - 1);
          const T* src = L[lv] + (size_t)__umul24(__umul24(gx, V.H) + gy, kNF) + q * (16 / (int)sizeof(T));
          __builtin_amdgcn_global_load_lds((global_void_ptr)src, (lds_void_ptr)(base + k * 1024), 16, 0, 0);
        }
      }
    }
    const unsigned xa = (unsigned)(x0 - bx), xb = (unsigned)(x1 - bx), ya = (unsigned)(y0 - by),
                   yb = (unsigned)(y1 - by);
    p.o[0] = (xa * kP + yb) * kRec;   // a = F[x0, y1]
    p.o[1] = (xb * kP + yb) * kRec;   // b = F[x1, y1]
    p.o[2] = (xa * kP + ya) * kRec;   // c = F[x0, y0]
    p.o[3] = (xb * kP + ya) * kRec;   // d = F[x1, y0]
    return p;
  }
  __device__ __forceinline__ double el(unsigned off, int f) const {
    return (double)*reinterpret_cast<const T*>(wave_base + off + f * (int)sizeof(T));
  }
  __device__ __forceinline__ void end(const Pending& p, double g[11]) const {
    lds_dma_wait();
    double ga[11], gb[11];
    constexpr unsigned kLev = kP * kP * kRec;
#pragma unroll
    for (int f = 0; f < 11; ++f)
      ga[f] = VaryingBG<T>::bl(p.w, el(p.o[0], f), el(p.o[1], f), el(p.o[2], f), el(p.o[3], f));
#pragma unroll
    for (int f = 0; f < 11; ++f)
      gb[f] = VaryingBG<T>::bl(p.w, el(p.o[0] + kLev, f), el(p.o[1] + kLev, f), el(p.o[2] + kLev, f),
                               el(p.o[3] + kLev, f));
#pragma unroll
    for (int i = 0; i < 11; ++i) g[i] = ga[i] * (1.0 - p.wt) + gb[i] * p.wt;
  }
  __device__ __forceinline__ void interp4(double lon, double lat, double t, double& fu, double& fv,
                                          double& fqx, double& fqy) const {
    V.interp4(lon, lat, t, fu, fv, fqx, fqy);
  }
  __device__ static BlockVaryingBG make(const VaryingBG<T>& B, char* lds) {
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    return BlockVaryingBG{B, lds + wave * kCacheBytesPerWave, 0, 0, -1};
  }
};
template <class T>
__device__ __forceinline__ typename BlockVaryingBG<T>::Pending lookup_begin(const BlockVaryingBG<T>& B, double lon,
                                                                            double lat, double t) {
  return B.begin(lon, lat, t);
}
template <class T>
__device__ __forceinline__ void lookup_end(const BlockVaryingBG<T>& B, const typename BlockVaryingBG<T>::Pending& p,
                                           double g[11]) {
  B.end(p, g);
}

// The background a persistent lane integrates with: the cached lookup for the
// static state (kernel-owned LDS), the plain one otherwise.
template <class BG>
struct LaneBG {
  using type = BG;
  static constexpr int kLdsBytes = 0;
  __device__ static BG make(const BG& B, char*) { return B; }
};
template <>
struct LaneBG<StaticBG> {
  using type = CachedStaticBG;
  static constexpr int kLdsBytes = 4 * kCacheBytesPerWave;   // 256-thread blocks
  __device__ static CachedStaticBG make(const StaticBG& B, char* lds) {
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    uint64_t hi = (uint64_t)(uintptr_t)(B.img + 4096);
    asm volatile("" : "+s"(hi));   // a second base pair: chunks 4-5 address like chunks 0-3
    return CachedStaticBG{B.F, B.img, lds + wave * kCacheBytesPerWave, (const char*)(uintptr_t)hi,
                          (threadIdx.x & 63u) * 16u, ~0u, ~0u};
  }
};
template <>
struct LaneBG<VaryingBG<float>> {
  using type = CachedVaryingBG32;
  static constexpr int kLdsBytes = 4 * kCacheBytesPerWave;
  __device__ static CachedVaryingBG32 make(const VaryingBG<float>& B, char* lds) {
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    return CachedVaryingBG32{B, lds + wave * kCacheBytesPerWave, (threadIdx.x & 63u) * 16u, ~0u, ~0u, -1};
  }
};
template <>
struct LaneBG<VaryingBGA32> {
  using type = CachedVaryingBGA32;
  static constexpr int kLdsBytes = 4 * kCacheBytesPerWave;
  __device__ static CachedVaryingBGA32 make(const VaryingBGA32& B, char* lds) {
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    CachedVaryingBGA32 c;
    c.V = B;
    c.wave_base = lds + wave * kCacheBytesPerWave;
    c.lane16 = (threadIdx.x & 63u) * 16u;
    c.key_x = c.key_y = ~0u;
    c.key_j = -1;
    return c;
  }
};
template <>
struct LaneBG<VaryingBG<double>> {
  using type = CachedVaryingBG64;
  static constexpr int kLdsBytes = 4 * kCacheBytesPerWave;
  __device__ static CachedVaryingBG64 make(const VaryingBG<double>& B, char* lds) {
    const unsigned wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    return CachedVaryingBG64{B, lds + wave * kCacheBytesPerWave, (threadIdx.x & 63u) * 16u, ~0u, ~0u, -1};
  }
};

}  // namespace rwrt

// ---------------------------------------------------------------------------
// The reference NumPy's own transcendentals (np_math.h: glibc 2.35
// __sin_fma/__cos_fma, SVML __svml_tan8_ha/__svml_pow8_ha), bitwise equal to
// np.sin/np.cos/np.tan/np.power on the reference's AVX-512 hosts
// (tests/test_np_math.py on the host, tests/test_gpu_np_math.py here).
// SVML pow's round-toward-zero / -infinity steps set the f64 round mode for
// one instruction each (MODE.FP_ROUND[3:2]: 3 toward zero, 2 toward -inf),
// inline: the device library's rounded operations are out-of-line calls,
// and a call waits for every outstanding memory operation at its entry.
// The s_nops cover the VALU -> s_setreg(MODE) hazard both ways.
// ---------------------------------------------------------------------------
#define RWRT_F64_RM_ASM(op, mode)                                                  \
  "s_nop 1\n\ts_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), " #mode "\n\t" op       \
  "\n\ts_nop 1\n\ts_setreg_imm32_b32 hwreg(HW_REG_MODE, 2, 2), 0\n\ts_nop 1"
namespace rwrt {
__device__ __forceinline__ double fma_rz(double a, double b, double c) {
  double r;
  asm(RWRT_F64_RM_ASM("v_fma_f64 %0, %1, %2, %3", 3) : "=&v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ double mul_rz(double a, double b) {
  double r;
  asm(RWRT_F64_RM_ASM("v_mul_f64 %0, %1, %2", 3) : "=&v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double add_rz(double a, double b) {
  double r;
  asm(RWRT_F64_RM_ASM("v_add_f64 %0, %1, %2", 3) : "=&v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ double add_rd(double a, double b) {
  double r;
  asm(RWRT_F64_RM_ASM("v_add_f64 %0, %1, %2", 2) : "=&v"(r) : "v"(a), "v"(b));
  return r;
}
}  // namespace rwrt
#define NM_FN __device__ __forceinline__
#define NM_CONST constexpr
#define NM_TABLE constexpr
#define NM_FMA_RZ(a, b, c) ::rwrt::fma_rz((a), (b), (c))
#define NM_MUL_RZ(a, b) ::rwrt::mul_rz((a), (b))
#define NM_ADD_RZ(a, b) ::rwrt::add_rz((a), (b))
#define NM_ADD_RD(a, b) ::rwrt::add_rd((a), (b))
#define NM_ISSUE_FENCE() __builtin_amdgcn_sched_barrier(0)
#define NM_RARE(c) RARE(c)
#define NM_RARE_ANY(c) RARE(__builtin_amdgcn_ballot_w64(c) != 0)
#define NM_FALLBACK_SIN(x) ::sin(x)
#define NM_FALLBACK_COS(x) ::cos(x)
#define NM_FALLBACK_TAN(x) ::tan(x)
#define NM_FALLBACK_POW(x, y) ::pow((x), (y))
// The tables live in LDS inside the kernels (staged at kernel entry by
// nm_stage): per-lane table reads from global memory would share vmcnt with
// the cell cache's LDS-DMA refills, so every read would also wait for the
// refill the RHS issued before its trigonometry.  Stored interleaved, so
// that each pair of values read together is one 16-B read (one 8-B read for
// the reciprocal's knots): the sin/cos table as two arrays of (sn, ssn) and
// (cs, ccs) pairs -- a lane's pair j sits in 16-B bank slot j mod 16 of its
// array, where the flat table put the pairs of the 64 lanes' lane-random
// reads in 8 slots -- tan's, log's and exp's (head, tail) pairs, the knots'
// (A, N) pairs.  Same values, so the same results.
__shared__ __attribute__((aligned(16))) double2 nm_lds_sc_s[110];    // kG_SINCOSTAB[4j], [4j + 1]
__shared__ __attribute__((aligned(16))) double2 nm_lds_sc_c[110];    // kG_SINCOSTAB[4j + 2], [4j + 3]
__shared__ __attribute__((aligned(16))) double2 nm_lds_tan[16];      // kT_TAN_HI[j], kT_TAN_LO[j]
__shared__ __attribute__((aligned(16))) double2 nm_lds_log[32];      // kP_LOG_HI[f], kP_LOG_LO[f]
__shared__ __attribute__((aligned(16))) double2 nm_lds_exp[16];      // kP_EXP_HI[j], kP_EXP_LO[j]
__shared__ __attribute__((aligned(8))) uint2 nm_lds_knot[64];        // kRCP14_KNOT[2i], [2i + 1]
#define NM_SINCOS4(k, a, b, c, d)                        \
  do {                                                   \
    const double2 nm_s_ = nm_lds_sc_s[(k) >> 2];         \
    const double2 nm_c_ = nm_lds_sc_c[(k) >> 2];         \
    a = nm_s_.x;                                         \
    b = nm_s_.y;                                         \
    c = nm_c_.x;                                         \
    d = nm_c_.y;                                         \
  } while (0)
#define NM_PAIR_(arr, i, hi, lo)       \
  do {                                 \
    const double2 nm_p_ = arr[i];      \
    hi = nm_p_.x;                      \
    lo = nm_p_.y;                      \
  } while (0)
#define NM_TAN2(j, hi, lo) NM_PAIR_(nm_lds_tan, j, hi, lo)
#define NM_LOG2(f, hi, lo) NM_PAIR_(nm_lds_log, f, hi, lo)
#define NM_EXP2(j, hi, lo) NM_PAIR_(nm_lds_exp, j, hi, lo)
#define NM_KNOT2(k, a, n)                    \
  do {                                       \
    const uint2 nm_k_ = nm_lds_knot[(k) >> 1]; \
    a = nm_k_.x;                             \
    n = nm_k_.y;                             \
  } while (0)
#define NM_LD(t, i) NM_LD_unused_##t
// (The polynomial constants stay s_mov_b32 pairs: as scalar loads they share
// lgkmcnt with the LDS reads, 0.99x; from LDS the round trip lands on the
// polynomial chains, 0.91x -- profiles/r2/ab/const_lds.txt.)
#include "np_math.h"

namespace rwrt {
// Copies the tables a kernel's math reads into its LDS (every thread of the
// block must call it, before any other use): NM_SINCOS = glibc's sin/cos
// table, NM_TAN = SVML tan's tables, NM_POW = SVML pow's (both with the
// VRCP14 knots).
enum { NM_SINCOS = 1, NM_TAN = 2, NM_POW = 4, NM_ALL = 7 };
template <int MASK>
__device__ __forceinline__ void nm_stage() {
  const int t = threadIdx.x, nt = blockDim.x;
  auto d = [](unsigned long long u) { return __builtin_bit_cast(double, u); };
  if (MASK & NM_SINCOS)
    for (int i = t; i < 110; i += nt) {
      nm_lds_sc_s[i] = make_double2(d(np_math::kG_SINCOSTAB[4 * i]), d(np_math::kG_SINCOSTAB[4 * i + 1]));
      nm_lds_sc_c[i] = make_double2(d(np_math::kG_SINCOSTAB[4 * i + 2]), d(np_math::kG_SINCOSTAB[4 * i + 3]));
    }
  if (MASK & NM_TAN)
    for (int i = t; i < 16; i += nt) nm_lds_tan[i] = make_double2(d(np_math::kT_TAN_HI[i]), d(np_math::kT_TAN_LO[i]));
  if (MASK & NM_POW)
    for (int i = t; i < 32; i += nt) {
      nm_lds_log[i] = make_double2(d(np_math::kP_LOG_HI[i]), d(np_math::kP_LOG_LO[i]));
      if (i < 16) nm_lds_exp[i] = make_double2(d(np_math::kP_EXP_HI[i]), d(np_math::kP_EXP_LO[i]));
    }
  if (MASK & (NM_TAN | NM_POW))
    for (int i = t; i < 64; i += nt) nm_lds_knot[i] = make_uint2(np_math::kRCP14_KNOT[2 * i], np_math::kRCP14_KNOT[2 * i + 1]);
  __syncthreads();
}

// The kernels' transcendentals: the reference NumPy's.
__device__ __forceinline__ double k_sin(double x) {
  return np_math::nm_sin(x);
}
__device__ __forceinline__ double k_cos(double x) {
  return np_math::nm_cos(x);
}
__device__ __forceinline__ double k_tan(double x) {
  return np_math::nm_tan(x);
}
__device__ __forceinline__ double k_pow(double x, double y) {
  return np_math::nm_pow(x, y);
}
// sin, cos, tan of a latitude (the RHS): the same values as k_sin/k_cos/k_tan
__device__ __forceinline__ void k_sincostan(double x, double& s, double& c, double& t) {
  np_math::nm_sincostan(x, s, c, t);
}

// Mercator factors of cal_bs_mercator_point (bs.py:856-860).
struct Merc {
  double c, s, m, cp;
};
__device__ __forceinline__ Merc merc_factors(double lat, double c, double s) {
  Merc r;
  r.c = c;
  r.s = s;
  r.m = (fabs(c) <= 0.0175) ? 0.0 : 1.0;
  r.cp = c * r.m + (1.0 - r.m) * 1e-6;
  return r;
}

// The 12 Mercator outputs the hot path uses (bs.py:862-883), in the order of
// the returned stack: fmu fmv fmux fmuy fmvx fmvy fmqx fmqy fmqxx fmqxy fmqyx fmqyy.
__device__ __forceinline__ void mercator12_masked(const double g[11], const Merc& M, double t,
                                                  double o[12]) {
  const double m = M.m, cp = M.cp;
  const double fu = g[F_U], fv = g[F_V];
  o[0] = (fu / cp) * m;                                      // fmu
  o[1] = (fv / cp) * m;                                      // fmv
  o[2] = (g[F_UX] / cp) * m;                                 // fmux
  o[3] = (g[F_UY] + t * fu) * m;                             // fmuy
  o[4] = (g[F_VX] / cp) * m;                                 // fmvx
  o[5] = (g[F_VY] + t * fv) * m;                             // fmvy
  o[6] = g[F_QX] * m;                                        // fmqx
  o[7] = (g[F_QY] * cp) * m;                                 // fmqy
  o[8] = g[F_QXX] * m;                                       // fmqxx
  o[10] = (g[F_QXY] * cp) * m;                               // fmqyx
  o[9] = o[10] * m;                                          // fmqxy = fmqyx * mask
  o[11] = (((g[F_QYY] * cp) - (g[F_QY] * M.s)) * cp) * m;    // fmqyy
}
// Away from the pole mask (m == 1, cp == c: x * 1.0 and c * 1.0 + 0.0 * 1e-6
// are the identity, NaN included) the multiplications by the mask drop out;
// the rare masked lanes (|cos(lat)| <= 0.0175) redo the full expressions.
__device__ __forceinline__ void mercator12(const double g[11], const Merc& M, double t, double o[12]) {
  const double cp = M.c;
  const double fu = g[F_U], fv = g[F_V];
  div2(fu, cp, fv, cp, o[0], o[1]);
  div2(g[F_UX], cp, g[F_VX], cp, o[2], o[4]);
  o[3] = g[F_UY] + t * fu;
  o[5] = g[F_VY] + t * fv;
  o[6] = g[F_QX];
  o[7] = g[F_QY] * cp;
  o[8] = g[F_QXX];
  o[10] = g[F_QXY] * cp;
  o[9] = o[10];
  o[11] = ((g[F_QYY] * cp) - (g[F_QY] * M.s)) * cp;
  if (RARE(M.m != 1.0)) {
    asm volatile("");   // keep the masked recomputation on its (rarely taken) branch
    mercator12_masked(g, M, t, o);
  }
}

// The wavenumber terms of cal_ugvg and core_diffun: they depend on k and l
// only, so the RHS forms them beside the trigonometry and the lookup.
//   kap = l / k, kap^2, 1 + kap^2, k^2 (1 + kap^2), k^2 (1 + kap^2)^2
// (wn.py:276-281; core_diffun's kap, kap2, kap1, kk and kk * kap1 are the same
// operations on the same operands, wr.py:53-60).
struct KapTerms {
  double kap, kap2, kap1, kk, denom;
};
__device__ __forceinline__ KapTerms kap_terms(double k, double l) {
  KapTerms w;
  w.kap = l / k;
  w.kap2 = w.kap * w.kap;
  w.kap1 = 1.0 + w.kap2;
  w.kk = (k * k) * w.kap1;
  w.denom = w.kk * w.kap1;
  return w;
}
// cal_ugvg(mode='extent') -> core_cal_ugvg_extent (wn.py:266-294)
__device__ __forceinline__ void ugvg(double fu, double fv, double fqx, double fqy,
                                     const KapTerms& w, double& ug, double& vg) {
  const double kap = w.kap, kap2 = w.kap2, denom = w.denom;
  double qu, qv;
  div2(((1.0 - kap2) * fqy) - ((2.0 * kap) * fqx), denom,
       ((2.0 * kap) * fqy) + ((1.0 - kap2) * fqx), denom, qu, qv);
  ug = fu + qu;
  vg = fv + qv;
}
__device__ __forceinline__ void ugvg(double fu, double fv, double fqx, double fqy,
                                     double k, double l, double& ug, double& vg) {
  ugvg(fu, fv, fqx, fqy, kap_terms(k, l), ug, vg);
}

// ---------------------------------------------------------------------------
// Shared-reciprocal division.  The RHS divides 16 times by five distinct
// divisors (cos(lat) four times, k (1 + kap^2)^2 three times, k (1 + kap^2)
// twice, R five times).  The hardware's IEEE f64 division (the compiler's
// sequence, div2 above) is: v_div_scale both operands, v_rcp_f64 + two
// Newton steps on the divisor, q = n r, one FMA remainder correction
// (v_div_fmas), v_div_fixup.  v_div_scale is the identity unless an operand
// is near the exponent limits, and then the reciprocal part depends on the
// divisor alone: formed once (rcp2), shared by its numerators (qdiv: four
// instructions instead of eleven, and a four-deep chain instead of eleven).
// qdiv(n, d, rcp2(d)) == n / d bit for bit when the numerator's frexp
// exponent is in [-899, 600] (|n| in [2^-900, 2^600)) or n is 0, inf or NaN
// (v_div_fixup's cases, frexp exponent 0), and the divisor's in [-99, 100]
// (tests/test_gpu_parity.py::test_device_math_exactness, kinds 34-35).
// DivGuard collects those exponents; a lane outside the range recomputes the
// RHS tail with IEEE divisions (rhs_tail<false>, a rarely taken branch).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double rcp2(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}
__device__ __forceinline__ double qdiv(double n, double d, double r) {
  const double q = n * r;
  const double e = fma(-d, q, n);
  return __builtin_amdgcn_div_fixup(fma(e, r, q), d, n);
}
struct DivGuard {
  int nlo = 0, nhi = 0, dlo = 0, dhi = 0;   // exponent range seen (0: neutral)
  __device__ __forceinline__ void num(double n) {
    const int e = __builtin_amdgcn_frexp_exp(n);
    nlo = ::min(nlo, e);
    nhi = ::max(nhi, e);
  }
  __device__ __forceinline__ void den(double d) {
    const int e = __builtin_amdgcn_frexp_exp(d);
    dlo = ::min(dlo, e);
    dhi = ::max(dhi, e);
  }
  __device__ __forceinline__ bool ok() const {
    return (nlo >= -899) & (nhi <= 600) & (dlo >= -99) & (dhi <= 100);
  }
};
__device__ __forceinline__ double qdiv(double n, double d, double r, DivGuard& G) {
  G.num(n);
  return qdiv(n, d, r);
}

// kap_terms with kap = l / k through the shared-reciprocal division, and the
// reciprocals of the three divisors it forms (guarded: G)
struct KapTermsR : KapTerms {
  double rkk, rk1, rden;   // rcp2 of kk, kap1, denom
};
__device__ __forceinline__ KapTermsR kap_terms_r(double k, double l, DivGuard& G) {
  KapTermsR w;
  G.den(k);
  w.kap = qdiv(l, k, rcp2(k), G);
  w.kap2 = w.kap * w.kap;
  w.kap1 = 1.0 + w.kap2;
  w.kk = (k * k) * w.kap1;
  w.denom = w.kk * w.kap1;
  G.den(w.kap1);
  G.den(w.kk);
  G.den(w.denom);
  w.rkk = rcp2(w.kk);
  w.rk1 = rcp2(w.kap1);
  w.rden = rcp2(w.denom);
  return w;
}

// ---------------------------------------------------------------------------
// The RHS: WR.diffun_numpy (wr.py:492-556) + core_diffun (wr.py:44-82)
// ---------------------------------------------------------------------------
// Everything after the lookup and the trigonometry: Mercator (bs.py:856-883),
// cal_ugvg (wn.py:266-294), core_diffun (wr.py:53-78; freq only feeds the
// dead ps/up terms) and the / R of wr.py:80-82, with IEEE divisions.
__device__ __forceinline__ void rhs_tail_ieee(const double g[11], const Merc& M, double s, double c,
                                              double tn, double kx, double ky, double amp, double* dy,
                                              double& ug, double& vg) {
  const KapTerms kw = kap_terms(kx, ky);
  double o[12];
  mercator12(g, M, tn, o);
  const double fmu = o[0], fmv = o[1], fmux = o[2], fmuy = o[3], fmvx = o[4], fmvy = o[5];
  const double fmqx = o[6], fmqy = o[7], fmqxx = o[8], fmqxy = o[9], fmqyx = o[10], fmqyy = o[11];
  ugvg(fmu, fmv, fmqx, fmqy, kw, ug, vg);
  const double kap = kw.kap, kap2 = kw.kap2, kap1 = kw.kap1, kk = kw.kk;
  double qk, ql;
  div2(kap * fmqxx - fmqyx, kk, kap * fmqxy - fmqyy, kk, qk, ql);
  const double dzwn = (-kx) * ((fmux + kap * fmvx) + qk);
  const double dmwn = (-kx) * ((fmuy + kap * fmvy) + ql);
  double damp1, damp2;
  div2(2.0 * ((fmux + fmvy) + kap * (fmvx + fmuy)), kap1,
       2.0 * (kap * (fmqxx - fmqyy) + (kap2 - 1.0) * fmqxy), kw.denom, damp1, damp2);
  const double damp3 = (-2.0 * s) * fmv;
  const double damp = (damp1 + damp2) + damp3;
  div2(ug, kREarth, vg * c, kREarth, dy[0], dy[1]);     // x / R, x / R
  div2(dzwn, kREarth, dmwn, kREarth, dy[2], dy[3]);
  dy[4] = div_rearth(damp * amp);
}
// The same operations on the same operands with the shared-reciprocal
// division; false when a lane must redo them with rhs_tail_ieee (an operand
// outside qdiv's exact range, or the Mercator pole band).
__device__ __forceinline__ bool rhs_tail_fast(const double g[11], const Merc& M, double s, double c,
                                              double tn, double kx, const KapTermsR& kw, DivGuard G,
                                              double amp, double* dy, double& ug, double& vg) {
  // Mercator off the pole band (M.m == 1, M.cp == c; mercator12)
  const double fu = g[F_U], fv = g[F_V];
  const double rc = rcp2(c);
  const double fmu = qdiv(fu, c, rc, G), fmv = qdiv(fv, c, rc, G);
  const double fmux = qdiv(g[F_UX], c, rc, G), fmvx = qdiv(g[F_VX], c, rc, G);
  const double fmuy = g[F_UY] + tn * fu, fmvy = g[F_VY] + tn * fv;
  const double fmqx = g[F_QX], fmqy = g[F_QY] * c, fmqxx = g[F_QXX];
  const double fmqyx = g[F_QXY] * c, fmqxy = fmqyx;
  const double fmqyy = ((g[F_QYY] * c) - (g[F_QY] * s)) * c;
  // cal_ugvg
  const double kap = kw.kap, kap2 = kw.kap2;
  ug = fmu + qdiv(((1.0 - kap2) * fmqy) - ((2.0 * kap) * fmqx), kw.denom, kw.rden, G);
  vg = fmv + qdiv(((2.0 * kap) * fmqy) + ((1.0 - kap2) * fmqx), kw.denom, kw.rden, G);
  // core_diffun
  const double qk = qdiv(kap * fmqxx - fmqyx, kw.kk, kw.rkk, G);
  const double ql = qdiv(kap * fmqxy - fmqyy, kw.kk, kw.rkk, G);
  const double dzwn = (-kx) * ((fmux + kap * fmvx) + qk);
  const double dmwn = (-kx) * ((fmuy + kap * fmvy) + ql);
  const double damp1 = qdiv(2.0 * ((fmux + fmvy) + kap * (fmvx + fmuy)), kw.kap1, kw.rk1, G);
  const double damp2 = qdiv(2.0 * (kap * (fmqxx - fmqyy) + (kap2 - 1.0) * fmqxy), kw.denom, kw.rden, G);
  const double damp3 = (-2.0 * s) * fmv;
  const double damp = (damp1 + damp2) + damp3;
  const double rR = rcp2(kREarth);   // (loop-invariant)
  dy[0] = qdiv(ug, kREarth, rR, G);
  dy[1] = qdiv(vg * c, kREarth, rR, G);
  dy[2] = qdiv(dzwn, kREarth, rR, G);
  dy[3] = qdiv(dmwn, kREarth, rR, G);
  dy[4] = qdiv(damp * amp, kREarth, rR, G);
  return G.ok() & (M.m == 1.0);
}

// rhs_tail_fast for a lane pair's split outputs: the same operations, but
// each lane divides only the numerators of its own variables by R -- the
// lower lane dy0, dy2, the upper one dy1, dy3 (the same operation shape on
// the other operand), both dy4 -- returned as (dA, dB, dC) (pair_attempt)
// (The quotients that need no other quotient -- fu | fv, ux | vx over cos,
// ug's | vg's and qk | ql -- one of each pair per lane measured no gain
// statically: -36 VALU per attempt but +56 moves, each exchange being two
// copies and two v_permlane32_swap per double.)
__device__ __forceinline__ bool rhs_tail_fast_pair(const double g[11], const Merc& M, double s, double c,
                                                   double tn, double kx, const KapTermsR& kw, DivGuard G,
                                                   double amp, bool up, double& dA, double& dB, double& dC,
                                                   double& ug, double& vg) {
  const double fu = g[F_U], fv = g[F_V];
  const double rc = rcp2(c);
  const double fmuy = g[F_UY] + tn * fu, fmvy = g[F_VY] + tn * fv;
  const double fmqx = g[F_QX], fmqy = g[F_QY] * c, fmqxx = g[F_QXX];
  const double fmqyx = g[F_QXY] * c, fmqxy = fmqyx;
  const double fmqyy = ((g[F_QYY] * c) - (g[F_QY] * s)) * c;
  const double kap = kw.kap, kap2 = kw.kap2;
  const double fmu = qdiv(fu, c, rc, G), fmv = qdiv(fv, c, rc, G);
  const double fmux = qdiv(g[F_UX], c, rc, G), fmvx = qdiv(g[F_VX], c, rc, G);
  ug = fmu + qdiv(((1.0 - kap2) * fmqy) - ((2.0 * kap) * fmqx), kw.denom, kw.rden, G);
  vg = fmv + qdiv(((2.0 * kap) * fmqy) + ((1.0 - kap2) * fmqx), kw.denom, kw.rden, G);
  const double qk = qdiv(kap * fmqxx - fmqyx, kw.kk, kw.rkk, G);
  const double ql = qdiv(kap * fmqxy - fmqyy, kw.kk, kw.rkk, G);
  const double dzwn = (-kx) * ((fmux + kap * fmvx) + qk);
  const double dmwn = (-kx) * ((fmuy + kap * fmvy) + ql);
  const double damp1 = qdiv(2.0 * ((fmux + fmvy) + kap * (fmvx + fmuy)), kw.kap1, kw.rk1, G);
  const double damp2 = qdiv(2.0 * (kap * (fmqxx - fmqyy) + (kap2 - 1.0) * fmqxy), kw.denom, kw.rden, G);
  const double damp3 = (-2.0 * s) * fmv;
  const double damp = (damp1 + damp2) + damp3;
  const double rR = rcp2(kREarth);   // (loop-invariant)
  const double vgc = vg * c;
  dA = qdiv(up ? vgc : ug, kREarth, rR, G);
  dB = qdiv(up ? dmwn : dzwn, kREarth, rR, G);
  dC = qdiv(damp * amp, kREarth, rR, G);
  return G.ok() & (M.m == 1.0);
}

// aux (optional) receives {ug, vg, cos(lat)} of this evaluation -- exactly what
// the per-interval post-processing recomputes at the same position
// (wr.py:844, 856-865) -- or NaN for a masked ray (no values computed).
template <class BG>
__device__ __forceinline__ void ray_rhs(const BG& B, double t, const double* y, double* dy,
                                        double* aux = nullptr) {
  const double lon = y[0], lat = y[1], kx = y[2];
  // wr.py:508-514: a masked ray's l is NaN; every derivative of it is then NaN
  // (each one depends on kap = l / k), as the reference's NaN fill
  // (wr.py:552-553) makes them -- no branch.
  const bool bad = fabs(lat) >= kHalfPi || fabs(y[3]) >= 100.0;
  const double ky = bad ? kNaN : y[3], amp = y[4];
  double g[11];
  // the trigonometry's table reads and tan polynomial beside the lookup's cell
  // arithmetic (one scheduling region: the refill below is a branch)
  MARK("r_entry");
  const auto trig = np_math::nm_sincostan_begin(lat);
  MARK("r_trig_begin");
  double s, c;
  DivGuard G;
  KapTermsR kw;
  const auto pending = lookup_begin(B, lon, lat, t);   // the lookup's fill overlaps the trig
  MARK("r_lookup_begin");
  double tn;
  np_math::nm_sincostan_end(lat, trig, s, c, tn);   // == k_sincostan(lat, s, c, tn)
  MARK("r_trig_end");
  __builtin_amdgcn_sched_barrier(0);
  // the wavenumber terms (k, l only) under the cell cache's first reads (+0.3 %, r4e)
  lookup_end(B, pending, g, [&] { kw = kap_terms_r(kx, ky, G); MARK("r_kap"); });
  MARK("r_lookup_end");
  const Merc M = merc_factors(lat, c, s);
  double ug, vg;
  if (RARE(!rhs_tail_fast(g, M, s, c, tn, kx, kw, G, amp, dy, ug, vg))) {
    asm volatile("");   // an operand outside qdiv's exact range, or the pole band (rare branch)
    rhs_tail_ieee(g, M, s, c, tn, kx, ky, amp, dy, ug, vg);
  }
  MARK("r_tail");
  if (aux) {
    aux[0] = ug;
    aux[1] = vg;
    aux[2] = bad ? kNaN : c;
  }
}

// ray_rhs for a lane pair (PairVaryingBG64: lanes L and L + 32 hold one ray):
// the lower lane evaluates sin(lat), the upper one cos(lat) -- one do_sin /
// do_cos stream and one table point per lane (np_math.h nm_sinorcos_fin) --
// exchanged by v_permlane32_swap; everything else as ray_rhs.
// (A lane pair could evaluate sin on its lower lane and cos on its upper one
// (np_math.h nm_sinorcos_fin, as quad_rhs does): 1.2 % slower on C5 fp64,
// profiles/r6/sinorcos_ab.txt -- the operand selects cost what the second
// evaluation did, and the exchange adds its latency to the serial chain.)
#ifndef RWRT_TEAM_SINORCOS
#define RWRT_TEAM_SINORCOS 1
#endif

// ray_rhs with fp32 arithmetic on fp32 levels (VaryingBGA32): the same
// expressions as ray_rhs / mercator12 / ugvg / core_diffun in float, the
// device library's sinf/cosf/tanf; dy and aux are returned in fp64.
// lookup(g) fills the eleven fields (fp32 blends of fp32 levels).
template <class Lookup>
__device__ __forceinline__ void ray_rhs_f32(Lookup&& lookup, const double* y, double* dy, double* aux) {
  const double lat = y[1];
  const bool bad = fabs(lat) >= kHalfPi || fabs(y[3]) >= 100.0;
  const float fnan = __builtin_nanf("");
  const float kx = (float)y[2], ky = bad ? fnan : (float)y[3], amp = (float)y[4];
  float g[11];
  lookup(g);
  if (!(fabs(lat) <= kHalfPi)) {
#pragma unroll
    for (int i = 0; i < 11; ++i) g[i] = fnan;
  }
  const float latf = (float)lat;
  float s, c;
  sincosf(latf, &s, &c);
  const float tn = tanf(latf);
  const float m = (fabsf(c) <= 0.0175f) ? 0.0f : 1.0f;
  const float cp = c * m + (1.0f - m) * 1e-6f;
  const float fu = g[F_U], fv = g[F_V];
  const float fmu = (fu / cp) * m, fmv = (fv / cp) * m;
  const float fmux = (g[F_UX] / cp) * m, fmuy = (g[F_UY] + tn * fu) * m;
  const float fmvx = (g[F_VX] / cp) * m, fmvy = (g[F_VY] + tn * fv) * m;
  const float fmqx = g[F_QX] * m, fmqy = (g[F_QY] * cp) * m, fmqxx = g[F_QXX] * m;
  const float fmqyx = (g[F_QXY] * cp) * m, fmqxy = fmqyx * m;
  const float fmqyy = (((g[F_QYY] * cp) - (g[F_QY] * s)) * cp) * m;
  const float kap = ky / kx, kap2 = kap * kap, kap1 = 1.0f + kap2;
  const float kk = (kx * kx) * kap1, denom = kk * kap1;
  const float ug = fmu + (((1.0f - kap2) * fmqy) - ((2.0f * kap) * fmqx)) / denom;
  const float vg = fmv + (((2.0f * kap) * fmqy) + ((1.0f - kap2) * fmqx)) / denom;
  const float qk = (kap * fmqxx - fmqyx) / kk, ql = (kap * fmqxy - fmqyy) / kk;
  const float dzwn = (-kx) * ((fmux + kap * fmvx) + qk);
  const float dmwn = (-kx) * ((fmuy + kap * fmvy) + ql);
  const float damp1 = (2.0f * ((fmux + fmvy) + kap * (fmvx + fmuy))) / kap1;
  const float damp2 = (2.0f * (kap * (fmqxx - fmqyy) + (kap2 - 1.0f) * fmqxy)) / denom;
  const float damp = (damp1 + damp2) + (-2.0f * s) * fmv;
  const float rinv = (float)(1.0 / kREarth);
  dy[0] = (double)(ug * rinv);
  dy[1] = (double)((vg * c) * rinv);
  dy[2] = (double)(dzwn * rinv);
  dy[3] = (double)(dmwn * rinv);
  dy[4] = (double)((damp * amp) * rinv);
  if (aux) {
    aux[0] = ug;
    aux[1] = vg;
    aux[2] = bad ? kNaN : (double)c;
  }
}
// plain gathers (rwrt_rhs_tv, the initial step)
__device__ __forceinline__ void ray_rhs(const VaryingBGA32& B, double t, const double* y, double* dy,
                                        double* aux = nullptr) {
  ray_rhs_f32(
      [&](float g[11]) {
        unsigned o[4];
        double wd[4], wtd;
        B.cell(y[0], y[1], o, wd);
        const float* A = B.level(t, wtd);
        const float* L1 = A + (B.nlev > 1 ? B.lev_stride : 0);
        const float w0 = (float)wd[0], w1 = (float)wd[1], w2 = (float)wd[2], w3 = (float)wd[3];
        const float wt = (float)wtd;
#pragma unroll
        for (int q = 0; q < 11; ++q) {
          const float ga = ((A[o[0] + q] * w0 + A[o[1] + q] * w1) + A[o[2] + q] * w2) + A[o[3] + q] * w3;
          const float gb = ((L1[o[0] + q] * w0 + L1[o[1] + q] * w1) + L1[o[2] + q] * w2) + L1[o[3] + q] * w3;
          g[q] = ga * (1.0f - wt) + gb * wt;
        }
      },
      y, dy, aux);
}
// through the ray loop's per-lane LDS cache (rk45_run_kernel)
__device__ __forceinline__ void ray_rhs(const CachedVaryingBGA32& B, double t, const double* y, double* dy,
                                        double* aux = nullptr) {
  ray_rhs_f32(
      [&](float g[11]) {
        const auto p = B.begin(y[0], y[1], t);
        B.endf(p, g);
      },
      y, dy, aux);
}

// group velocity at a stored position (wr.py:856-865): no |l| mask here
template <class BG>
__device__ __forceinline__ void ugvg_at(const BG& B, double t, double lon, double lat, double k,
                                        double l, double& ug, double& vg) {
  double fu, fv, fqx, fqy;
  B.interp4(lon, lat, t, fu, fv, fqx, fqy);
  const double c = k_cos(lat);
  const double m = (fabs(c) <= 0.0175) ? 0.0 : 1.0;
  const double cp = c * m + (1.0 - m) * 1e-6;
  ugvg((fu / cp) * m, (fv / cp) * m, fqx * m, (fqy * cp) * m, k, l, ug, vg);
}

// cal_dis (wr.py:97-112): haversine between consecutive stored positions
__device__ __forceinline__ double cal_dis(double lon_c, double lat_c, double lon_p, double lat_p) {
  const double sd = k_sin((lat_c - lat_p) / 2.0);
  const double sl = k_sin((lon_c - lon_p) / 2.0);
  const double a = sd * sd + (k_cos(lat_p) * k_cos(lat_c)) * (sl * sl);
  return fabs(2.0 * atan2(sqrt(a), sqrt(1.0 - a)));
}
// the same with cos(lat_p), cos(lat_c) supplied by the caller
__device__ __forceinline__ double cal_dis_c(double lon_c, double lat_c, double lon_p, double lat_p,
                                            double cos_c, double cos_p) {
  const double sd = k_sin((lat_c - lat_p) / 2.0);
  const double sl = k_sin((lon_c - lon_p) / 2.0);
  const double a = sd * sd + (cos_p * cos_c) * (sl * sl);
  return fabs(2.0 * atan2(sqrt(a), sqrt(1.0 - a)));
}
// cal_dis_c(...) >= cut_off, with the atan2 skipped when the haversine
// argument is certainly below the threshold (cut_a: haversine_cut on the host)
// sin() of two arguments through the one-reduction routine (== sin() for
// |x| < 2^30), with one shared fallback branch to the library for the rest
__device__ __forceinline__ void sin2(double a, double b, double& sa, double& sb) {
  sa = k_sin(a);
  sb = k_sin(b);
}
// cos() of an argument known to be below pi/2 in magnitude or NaN
__device__ __forceinline__ double cos_small(double x) {
  return k_cos(x);
}
// sin(x) for |x| <= 1/16 by its Taylor series to x^7: relative error below
// 1e-15 there (the x^9 term: 2^-36 / 9! ~ 4e-17, plus rounding)
__device__ __forceinline__ double sin_small(double x) {
  const double x2 = x * x;
  double p = fma(x2, -1.0 / 5040.0, 1.0 / 120.0);
  p = fma(x2, p, -1.0 / 6.0);
  return fma(x * x2, p, x);
}
template <bool kFast = true>
__device__ __forceinline__ bool cal_dis_reaches(double lon_c, double lat_c, double lon_p,
                                                double lat_p, double cos_c, double cos_p,
                                                double cut_off, double cut_a) {
  if (kFast) {
    // a from the polynomial sines is within ~1e-14 relative of the reference's
    // a (NumPy sines), so a_poly < cut_a (1 - 1e-12) proves a < cut_a -- the
    // "no jump" verdict below, bit for bit -- without the table sines; any
    // other lane (larger steps, near the threshold, NaN) takes the exact path.
    // C3 +1.2 % zonal, +2.1 % non-zonal (profiles/r4/sched/ab_round4.txt).
    // quad_dis_reaches repeats these operations; tests/test_gpu_parity.py
    // (selftest kinds 36/37) checks the verdict with and without them on
    // steps straddling the threshold.
    const double x1 = (lat_c - lat_p) / 2.0, x2 = (lon_c - lon_p) / 2.0;
    const double s1 = sin_small(x1), s2 = sin_small(x2);
    const double ap = s1 * s1 + (cos_p * cos_c) * (s2 * s2);
    if (fabs(x1) <= 0.0625 && fabs(x2) <= 0.0625 && ap < cut_a * (1.0 - 1e-12)) return false;
  }
  double sd, sl;
  sin2((lat_c - lat_p) / 2.0, (lon_c - lon_p) / 2.0, sd, sl);
  const double a = sd * sd + (cos_p * cos_c) * (sl * sl);
  bool r = false;
  if (RARE(!(a < cut_a))) {
    asm volatile("");   // rare: near or past the threshold, or NaN
    r = fabs(2.0 * atan2(sqrt(a), sqrt(1.0 - a))) >= cut_off;
  }
  return r;
}

// ---------------------------------------------------------------------------
// Problems the stepper integrates
// ---------------------------------------------------------------------------
// The step control reuses K6 as the next step's f (FSAL) for both
// backgrounds: the reference recomputes f = fun(t, y) (rkf45.py:378), which is
// K6 bit for bit when fun ignores t; for a time-varying flow K6 = fun(t + h,
// y_new) is scipy's RK45 convention (the reference has no time-varying mode).
template <class BG>
struct RayProblemT {
  static constexpr int NV = 5;
  static constexpr int NAUX = 3;             // ug, vg, cos(lat) of the evaluation
  static constexpr bool kAutonomous = true;  // FSAL (see above)
  BG B;
  __device__ __forceinline__ void operator()(double t, const double* y, double* dy,
                                             double* aux = nullptr) const {
    ray_rhs(B, t, y, dy, aux);
  }
};
using RayProblem = RayProblemT<StaticBG>;

// rkf45.py demo ODEs (rkf45.py:775-782, 839-841, 861-863)
struct KatLinear {
  static constexpr int NV = 1;
  static constexpr int NAUX = 0;
  static constexpr bool kAutonomous = false;
  __device__ void operator()(double t, const double* y, double* dy, double* = nullptr) const {
    dy[0] = 2.0 * t + y[0] * 0.0;
  }
};
struct KatExp {
  static constexpr int NV = 1;
  static constexpr int NAUX = 0;
  static constexpr bool kAutonomous = false;
  __device__ void operator()(double t, const double* y, double* dy, double* = nullptr) const {
    dy[0] = k_pow(2.718281828459045, 0.1 * t) + y[0] * 0.0;  // np.e ** (0.1 * t)
  }
};
struct KatLorenz {
  static constexpr int NV = 3;
  static constexpr int NAUX = 0;
  static constexpr bool kAutonomous = false;
  __device__ void operator()(double, const double* u, double* d, double* = nullptr) const {
    const double p = 10.0, b = 8.0 / 3, r = 28.0;
    const double x = u[0], y = u[1], z = u[2];
    d[0] = (-p) * x + p * y;
    d[1] = ((-x) * z + r * x) - y;
    d[2] = x * y - b * z;
  }
};

// ---------------------------------------------------------------------------
// Dormand-Prince 5(4) attempt, rk_step (rkf45.py:259-321) + error norm
// ---------------------------------------------------------------------------
// Stage weights: row s = 1..5 is A[s][0..4] (stage inputs), row 6 is B[0..5]
// (y_new); the time offset of stage 6 is c = 1 (K6 = fun(t + h, y_new)).
// Only ever indexed by compile-time stage numbers (stage_input<S>), so the
// weights are instruction immediates, not loads.
constexpr double kW[7][6] = {
    {0, 0, 0, 0, 0, 0},
    {kA[1][0], 0, 0, 0, 0, 0},
    {kA[2][0], kA[2][1], 0, 0, 0, 0},
    {kA[3][0], kA[3][1], kA[3][2], 0, 0, 0},
    {kA[4][0], kA[4][1], kA[4][2], kA[4][3], 0, 0},
    {kA[5][0], kA[5][1], kA[5][2], kA[5][3], kA[5][4], 0},
    {kB[0], kB[1], kB[2], kB[3], kB[4], kB[5]}};
constexpr double kCs[7] = {0.0, kC[1], kC[2], kC[3], kC[4], kC[5], 1.0};

// Storage of the stages K1..K5 of one attempt, per lane: in registers, or in a
// per-thread slice of LDS (frees 50 VGPRs of the ray kernel for occupancy).
template <int NV>
struct KRegs {
  double k[6][NV];
  __device__ __forceinline__ double get(int j, int v) const { return k[j][v]; }
  // stage index s is wave-uniform; select the register row statically
  __device__ __forceinline__ void put_stage(int s, const double* r) {
#pragma unroll
    for (int j = 0; j < 6; ++j)
      if (j == s) {
#pragma unroll
        for (int v = 0; v < NV; ++v) k[j][v] = r[v];
      }
  }
};

// K1..K5 only (K0 is the step's f, in registers).
template <int NV>
struct KShared {
  double* p;   // this lane's slice: element (j, v) at p[((j - 1) * NV + v) * stride]
  int stride;  // threads per block
  __device__ __forceinline__ double get(int j, int v) const { return p[((j - 1) * NV + v) * stride]; }
  __device__ __forceinline__ void put_stage(int s, const double* r) {
#pragma unroll
    for (int v = 0; v < NV; ++v) p[((s - 1) * NV + v) * stride] = r[v];
  }
};

// np.einsum('snf,s->nf', K[:S], w) in NumPy's order for stage S: sequential
// in j for more than one variable; for one variable einsum's 2-lane SIMD dot
// product sums even and odd terms separately (oracle/rwrt_oracle.py wsum).
// K0 is the step's f (registers); K1..K5 come from KS.  Zero weights (B[1])
// are kept: NumPy multiplies them too (NaN/inf propagate).
template <int S, int NV, class KS>
__device__ __forceinline__ double wsum(const KS& K, const double* f, int v) {
  if constexpr (NV == 1) {
    double even = 0.0, odd = 0.0;
#pragma unroll
    for (int j = 0; j < S; ++j) {
      const double kj = (j == 0) ? f[v] : K.get(j, v);
      if (j % 2 == 0) even = even + kj * kW[S][j];
      else odd = odd + kj * kW[S][j];
    }
    return even + odd;
  } else {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < S; ++j) acc = acc + ((j == 0) ? f[v] : K.get(j, v)) * kW[S][j];
    return acc;
  }
}

// Input (t_s, y_s) of stage S (rkf45.py:300-306).
template <int S, int NV, class KS>
__device__ __forceinline__ double stage_input(const KS& K, double t, const double* y,
                                              const double* f, double h, double* ys) {
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    ys[v] = y[v] + wsum<S, NV>(K, f, v) * h;
  }
  return t + kCs[S] * h;
}

// The first J terms of wsum<S> (J < S) for every variable, in wsum's order
// (more than one variable: sequential in j).
template <int S, int J, int NV, class KS>
__device__ __forceinline__ void stage_part(const KS& K, const double* f, double* part) {
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    double acc = 0.0;
#pragma unroll
    for (int j = 0; j < J; ++j) acc = acc + ((j == 0) ? f[v] : K.get(j, v)) * kW[S][j];
    part[v] = acc;
  }
}
// The error estimate's terms K0..K5 (dp54_attempt's es without "+ K6 * E6").
template <int NV, class KS>
__device__ __forceinline__ void error_part(const KS& K, const double* f, double* part) {
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    double es = 0.0;
#pragma unroll
    for (int j = 0; j < 6; ++j) es = es + ((j == 0) ? f[v] : K.get(j, v)) * kE[j];
    part[v] = es;
  }
}

// One DP5(4) attempt: rk_step (rkf45.py:259-321) + _estimate_error_norm
// (rkf45.py:368-373).  The six stage evaluations are unrolled (six inlined RHS
// copies: fits the instruction cache; one copy in a wave-uniform stage loop
// measured 0.92x).  Returns the error norm (NaN kept); fills y_new,
// K6, if aux is given the problem's side outputs of the K6 evaluation (at
// y_new), and if Kout is given all seven stages.
template <class P, class KS>
__device__ __forceinline__ double dp54_attempt(const P& fun, KS& K, double t, const double* y,
                                               const double* f, double h, double rtol,
                                               double atol, double* ynew, double* k6,
                                               double* Kout = nullptr, int64_t kstride = 0,
                                               double* aux = nullptr) {
  constexpr int NV = P::NV;
  double ys[NV], r[NV];
  if constexpr (NV > 1) {
    // Each stage's weighted sum is sequential in j and its newest stage comes
    // last: the terms of the older stages are summed while the current RHS
    // runs (their LDS reads and dependent adds off the critical path), and
    // only "+ K_s * w" follows the RHS.  The same operations in the same order
    // as wsum: bit for bit.
    double part[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) ys[v] = y[v] + wsum<1, NV>(K, f, v) * h;
    double ts = t + kCs[1] * h;
#pragma unroll
    for (int s = 1; s <= 6; ++s) {
      double w = 0.0, cn = 0.0;   // the newest term's weight and the time offset of stage s + 1
      switch (s) {   // wave-uniform (compile-time when unrolled)
        case 1: stage_part<2, 1, NV>(K, f, part); w = kW[2][1]; cn = kCs[2]; break;
        case 2: stage_part<3, 2, NV>(K, f, part); w = kW[3][2]; cn = kCs[3]; break;
        case 3: stage_part<4, 3, NV>(K, f, part); w = kW[4][3]; cn = kCs[4]; break;
        case 4: stage_part<5, 4, NV>(K, f, part); w = kW[5][4]; cn = kCs[5]; break;
        case 5: stage_part<6, 5, NV>(K, f, part); w = kW[6][5]; cn = kCs[6]; break;
        default: error_part<NV>(K, f, part); break;
      }
      MARK("a_stage_part");
      fun(ts, ys, r, aux);
      if (s < 6) {
        K.put_stage(s, r);
#pragma unroll
        for (int v = 0; v < NV; ++v) ys[v] = y[v] + (part[v] + r[v] * w) * h;
        ts = t + cn * h;
      }
      MARK("a_stage_sum");
    }
    double ss = 0.0;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      ynew[v] = ys[v];
      k6[v] = r[v];
      const double e = h * (part[v] + r[v] * kE[6]);
      const double sc = atol + np_max(fabs(y[v]), fabs(ys[v])) * rtol;
      const double x = e / sc;
      ss = (v == 0) ? x * x : ss + x * x;
    }
    if (Kout) {
#pragma unroll
      for (int j = 0; j < 6; ++j)
#pragma unroll
        for (int v = 0; v < NV; ++v) Kout[(j * NV + v) * kstride] = (j == 0) ? f[v] : K.get(j, v);
#pragma unroll
      for (int v = 0; v < NV; ++v) Kout[(6 * NV + v) * kstride] = r[v];
    }
    return sqrt(ss) / RootN<NV>::v;
  }
  // one variable (the stepper KATs): einsum's even/odd sums (wsum)
#pragma unroll
  for (int s = 1; s <= 6; ++s) {
    double ts;
    switch (s) {   // wave-uniform: one straight-line combination per stage
      case 1: ts = stage_input<1, NV>(K, t, y, f, h, ys); break;
      case 2: ts = stage_input<2, NV>(K, t, y, f, h, ys); break;
      case 3: ts = stage_input<3, NV>(K, t, y, f, h, ys); break;
      case 4: ts = stage_input<4, NV>(K, t, y, f, h, ys); break;
      case 5: ts = stage_input<5, NV>(K, t, y, f, h, ys); break;
      default: ts = stage_input<6, NV>(K, t, y, f, h, ys); break;
    }
    fun(ts, ys, r, aux);
    if (s < 6) K.put_stage(s, r);
  }
  // after the loop: ys = y + h*(B . K[:6]) = y_new, r = K6
  double ss = 0.0;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    ynew[v] = ys[v];
    k6[v] = r[v];
    double es;
    if constexpr (NV == 1) {
      double even = 0.0, odd = 0.0;
#pragma unroll
      for (int j = 0; j < 6; ++j) {
        const double kj = (j == 0) ? f[v] : K.get(j, v);
        if (j % 2 == 0) even = even + kj * kE[j];
        else odd = odd + kj * kE[j];
      }
      even = even + r[v] * kE[6];
      es = even + odd;
    } else {
      es = 0.0;
#pragma unroll
      for (int j = 0; j < 6; ++j) es = es + ((j == 0) ? f[v] : K.get(j, v)) * kE[j];
      es = es + r[v] * kE[6];
    }
    const double e = h * es;
    const double sc = atol + np_max(fabs(y[v]), fabs(ys[v])) * rtol;
    const double x = e / sc;
    ss = (v == 0) ? x * x : ss + x * x;
  }
  if (Kout) {
#pragma unroll
    for (int j = 0; j < 6; ++j)
#pragma unroll
      for (int v = 0; v < NV; ++v) Kout[(j * NV + v) * kstride] = (j == 0) ? f[v] : K.get(j, v);
#pragma unroll
    for (int v = 0; v < NV; ++v) Kout[(6 * NV + v) * kstride] = r[v];
  }
  return sqrt(ss) / RootN<NV>::v;
}

// ---------------------------------------------------------------------------
// Lane pairs (fp64 time-varying loop, PairVaryingBG64): lanes L and L + 32
// hold one ray.  Besides the two levels' blends (PairVaryingBG64::end), the
// work that is the same operation on other operands is dealt out over the
// pair instead of done twice: the lower lane owns variables 0 and 2, the
// upper one 1 and 3, both 4 -- the RHS's final divisions by R (dy0 = ug / R
// | dy1 = vg cos / R, dy2 = dzwn / R | dy3 = dmwn / R), the stage sums and
// stage values K1..K5 (three per lane in LDS instead of five), the error
// estimate's quotients -- and exchanged by v_permlane32_swap (both()).  Every
// value is the same operation on the same operands as in ray_rhs /
// dp54_attempt: results are bit for bit the 64-lane loop's.
// ---------------------------------------------------------------------------
// ray_rhs for a pair: (dA, dB, dC) = this lane's (dy0 | dy1, dy2 | dy3, dy4)
__device__ __forceinline__ void pair_rhs(const PairVaryingBG64& B, double t, const double* y, double& dA,
                                         double& dB, double& dC, double* aux) {
  const double lon = y[0], lat = y[1], kx = y[2];
  const bool bad = fabs(lat) >= kHalfPi || fabs(y[3]) >= 100.0;
  const double ky = bad ? kNaN : y[3], amp = y[4];
  double g[11];
  const auto trig = np_math::nm_sincostan_begin(lat);
  double s, c;
  DivGuard G;
  KapTermsR kw;
  const auto pending = lookup_begin(B, lon, lat, t);
  double tn;
  np_math::nm_sincostan_end(lat, trig, s, c, tn);
  __builtin_amdgcn_sched_barrier(0);
  lookup_end(B, pending, g, [&] { kw = kap_terms_r(kx, ky, G); });
  const Merc M = merc_factors(lat, c, s);
  double ug, vg;
  if (RARE(!rhs_tail_fast_pair(g, M, s, c, tn, kx, kw, G, amp, B.upper, dA, dB, dC, ug, vg))) {
    asm volatile("");   // an operand outside qdiv's exact range, or the pole band (rare branch)
    double dy[5];
    rhs_tail_ieee(g, M, s, c, tn, kx, ky, amp, dy, ug, vg);
    dA = B.upper ? dy[1] : dy[0];
    dB = B.upper ? dy[3] : dy[2];
    dC = dy[4];
  }
  aux[0] = ug;
  aux[1] = vg;
  aux[2] = bad ? kNaN : c;
}

// the first J terms of wsum<S> for this lane's three variables (K0 = f)
template <int S, int J>
__device__ __forceinline__ void pair_part(const KShared<3>& K, double fA, double fB, double fC, double& pA,
                                          double& pB, double& pC) {
  double a = 0.0, b = 0.0, c = 0.0;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    a = a + ((j == 0) ? fA : K.get(j, 0)) * kW[S][j];
    b = b + ((j == 0) ? fB : K.get(j, 1)) * kW[S][j];
    c = c + ((j == 0) ? fC : K.get(j, 2)) * kW[S][j];
  }
  pA = a;
  pB = b;
  pC = c;
}
__device__ __forceinline__ void pair_epart(const KShared<3>& K, double fA, double fB, double fC, double& pA,
                                           double& pB, double& pC) {
  double a = 0.0, b = 0.0, c = 0.0;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    a = a + ((j == 0) ? fA : K.get(j, 0)) * kE[j];
    b = b + ((j == 0) ? fB : K.get(j, 1)) * kE[j];
    c = c + ((j == 0) ? fC : K.get(j, 2)) * kE[j];
  }
  pA = a;
  pB = b;
  pC = c;
}

// dp54_attempt (rkf45.py:259-321, 368-373) for a pair's ray: y, f, ynew and
// k6 whole on both lanes; the stage values in this lane's slice of the stage
// area (K5's, three variables of it)
__device__ __forceinline__ double pair_attempt(const PairVaryingBG64& B, const KShared<5>& K5, double t,
                                               const double* y, const double* f, double h, double rtol,
                                               double atol, double* ynew, double* k6, double* aux) {
  const bool up = B.upper;
  KShared<3> K{K5.p, K5.stride};
  const double yA = up ? y[1] : y[0], yB = up ? y[3] : y[2], yC = y[4];
  const double fA = up ? f[1] : f[0], fB = up ? f[3] : f[2], fC = f[4];
  double ys[5];
#pragma unroll
  for (int v = 0; v < 5; ++v) ys[v] = y[v] + wsum<1, 5>(K5, f, v) * h;   // (K unused for stage 1)
  double ts = t + kCs[1] * h;
  double ysA = 0.0, ysB = 0.0, ysC = 0.0, rA = 0.0, rB = 0.0, rC = 0.0, pA = 0.0, pB = 0.0, pC = 0.0;
#pragma unroll
  for (int s = 1; s <= 6; ++s) {
    double w = 0.0, cn = 0.0;
    switch (s) {
      case 1: pair_part<2, 1>(K, fA, fB, fC, pA, pB, pC); w = kW[2][1]; cn = kCs[2]; break;
      case 2: pair_part<3, 2>(K, fA, fB, fC, pA, pB, pC); w = kW[3][2]; cn = kCs[3]; break;
      case 3: pair_part<4, 3>(K, fA, fB, fC, pA, pB, pC); w = kW[4][3]; cn = kCs[4]; break;
      case 4: pair_part<5, 4>(K, fA, fB, fC, pA, pB, pC); w = kW[5][4]; cn = kCs[5]; break;
      case 5: pair_part<6, 5>(K, fA, fB, fC, pA, pB, pC); w = kW[6][5]; cn = kCs[6]; break;
      default: pair_epart(K, fA, fB, fC, pA, pB, pC); break;
    }
    pair_rhs(B, ts, ys, rA, rB, rC, aux);
    if (s < 6) {
      const double r3[3] = {rA, rB, rC};
      K.put_stage(s, r3);
      ysA = yA + (pA + rA * w) * h;
      ysB = yB + (pB + rB * w) * h;
      ysC = yC + (pC + rC * w) * h;
      PairVaryingBG64::both(ysA, ys[0], ys[1]);
      PairVaryingBG64::both(ysB, ys[2], ys[3]);
      ys[4] = ysC;
      ts = t + cn * h;
    }
  }
  // ys = y_new, (rA, rB, rC) = K6; the error estimate of the owned variables
#pragma unroll
  for (int v = 0; v < 5; ++v) ynew[v] = ys[v];
  PairVaryingBG64::both(rA, k6[0], k6[1]);
  PairVaryingBG64::both(rB, k6[2], k6[3]);
  k6[4] = rC;
  const double eA = h * (pA + rA * kE[6]), eB = h * (pB + rB * kE[6]), eC = h * (pC + rC * kE[6]);
  const double scA = atol + np_max(fabs(yA), fabs(ysA)) * rtol;
  const double scB = atol + np_max(fabs(yB), fabs(ysB)) * rtol;
  const double scC = atol + np_max(fabs(yC), fabs(ysC)) * rtol;
  double xA, xB;
  div2(eA, scA, eB, scB, xA, xB);
  const double xC = eC / scC;
  double x0, x1, x2, x3;
  PairVaryingBG64::both(xA, x0, x1);
  PairVaryingBG64::both(xB, x2, x3);
  double ss = x0 * x0;
  ss = ss + x1 * x1;
  ss = ss + x2 * x2;
  ss = ss + x3 * x3;
  ss = ss + xC * xC;
  return sqrt(ss) / RootN<5>::v;
}
template <class P>
struct IsPair : std::false_type {};
template <>
struct IsPair<RayProblemT<PairVaryingBG64>> : std::true_type {};

// select_initial_step (rkf45.py:34-99), direction = +1
template <class P>
__device__ __forceinline__ double initial_step(const P& fun, double t0, const double* y0,
                                               const double* f0, double rtol, double atol) {
  constexpr int NV = P::NV;
  double sc[NV], y1[NV], f1[NV];
  double s0 = 0.0, s1 = 0.0;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    sc[v] = atol + fabs(y0[v]) * rtol;
    const double a = y0[v] / sc[v], b = f0[v] / sc[v];
    s0 = (v == 0) ? a * a : s0 + a * a;
    s1 = (v == 0) ? b * b : s1 + b * b;
  }
  const double d0 = sqrt(s0) / RootN<NV>::v, d1 = sqrt(s1) / RootN<NV>::v;
  double h0 = (0.01 * d0) / d1;
  if (d0 < 1e-5) h0 = 1e-6;
  if (d1 < 1e-5) h0 = 1e-6;
#pragma unroll
  for (int v = 0; v < NV; ++v) y1[v] = y0[v] + h0 * f0[v];
  fun(t0 + h0, y1, f1);
  double s2 = 0.0;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const double a = (f1[v] - f0[v]) / sc[v];
    s2 = (v == 0) ? a * a : s2 + a * a;
  }
  const double d2 = (sqrt(s2) / RootN<NV>::v) / h0;
  double h1;
  if (!(d1 > 1e-15) && !(d2 > 1e-15)) {
    h1 = np_max(1e-6, h0 * 1e-3);
  } else {
    const double dm = (d1 != d1) ? d2 : ((d2 != d2) ? d1 : (d1 >= d2 ? d1 : d2));  // nanmax
    h1 = k_pow(0.01 / dm, 0.2);
  }
  return np_min(100.0 * h0, h1);
}

// One lane's solver: the per-column part of OdeSolver.step / _step_impl
// (rkf45.py:222-253, 375-514).  iterate() runs at most ONE attempt and
// reports whether the column reached t_bound.
template <class P, class KS>
struct Lane {
  static constexpr int NV = P::NV;
  KS K;
  double y[NV], f[NV];
  // side outputs of the last evaluation at y (valid after an accepted step;
  // the caller sets aux[NAUX-1] = NaN whenever y changes otherwise)
  double aux[P::NAUX > 0 ? P::NAUX : 1];
  double t, habs, hs;
  double tk6 = 0.0;   // the time of the last accepted step's K6 evaluation (t_old + h), aux's time
  bool in_step, rejected;

  // Returns kStep (attempt made, interval not finished), kReached (t == t_bound)
  // or kFrozen (NaN mean at step start: t := t_bound, y never changes again).
  enum { kStep = 0, kReached = 1, kFrozen = 2 };

  __device__ __forceinline__ int iterate(const P& fun, double tb, double min_step, double rtol,
                                         double atol, int64_t& nacc, int64_t& nrej) {
    if (!in_step) {
      double sum = y[0];
#pragma unroll
      for (int v = 1; v < NV; ++v) sum = sum + y[v];
      // NaN mean: frozen, t := t_bound (rkf45.py:400-403); sum / NV is NaN
      // exactly when sum is (inf / NV = inf, a finite sum stays finite)
      if (isnan(sum)) {
        t = tb;
        return kFrozen;
      }
      if (t == tb) return kReached;
      if constexpr (!P::kAutonomous) fun(t, y, f);   // rkf45.py:378 (equal to K6 if autonomous)
      hs = np_max(habs, min_step);         // rkf45.py:383-387
      rejected = false;
      in_step = true;
    }
    double h = hs;                          // h_abs * direction
    double tn = t + h;
    if (tn - tb > 0.0) tn = tb;             // rkf45.py:429
    h = tn - t;
    const double ha = fabs(h);
    double yn[NV], k6[NV];
    double en;
    if constexpr (IsPair<P>::value)   // (lane pairs: the split attempt)
      en = pair_attempt(fun.B, K, t, y, f, h, rtol, atol, yn, k6, aux);
    else
      en = dp54_attempt(fun, K, t, y, f, h, rtol, atol, yn, k6, nullptr, 0, P::NAUX > 0 ? aux : nullptr);
    MARK("a_error_norm");
    if (en != en) en = 0.0;                 // rkf45.py:446
    // SAFETY * error_norm ** (-1/5), shared by the accept (rkf45.py:453-469) and
    // reject (rkf45.py:471-475) factors: one pow per attempt even when the
    // wave's lanes split between the two outcomes
    const double sp = kSafety * k_pow(en, kErrExp);
    // Accept / reject as selects: the lanes of a wave usually disagree, and
    // a branch pair would execute both sides anyway.
    const bool acc = en < 1.0;
    double fac = np_min(kMaxFactor, sp);
    if (en == 0.0) fac = kMaxFactor;
    if (rejected) fac = np_min(1.0, fac);
    const double tnew = (tn != tn) ? tb : tn;              // rkf45.py:503
    habs = acc ? ha * fac : habs;
    hs = acc ? hs : ha * np_max(kMinFactor, sp);
    tk6 = acc ? t + h : tk6;                                // (dp54_attempt's last stage time)
    t = acc ? tnew : t;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      y[v] = acc ? yn[v] : y[v];
      f[v] = acc ? k6[v] : f[v];
    }
    in_step = !acc;
    rejected = rejected || !acc;
    nacc += acc ? 1 : 0;
    nrej += acc ? 0 : 1;
    return (acc && t - tb >= 0.0) ? kReached : kStep;   // rkf45.py:250
  }
};

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------
__global__ void pack_fields_kernel(const double* __restrict__ ref, double* __restrict__ out,
                                   int64_t npts) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= npts) return;
  const double* src = ref + i * RWRT_NFIELD_REF;
  double* dst = out + i * kNF;
#pragma unroll
  for (int q = 0; q < 11; ++q) dst[q] = src[kRefIndex[q]];
  dst[F_PAD] = 0.0;
}

__global__ void mercator_kernel(Field F, int64_t n, const double* __restrict__ lon,
                                const double* __restrict__ lat, double* __restrict__ out) {
  nm_stage<NM_SINCOS | NM_TAN>();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double la = lat[i];
    double g[11], o[12];
    interp11(F, py_mod_2pi(lon[i]), la, g);
    const Merc M = merc_factors(la, k_cos(la), k_sin(la));
    mercator12(g, M, k_tan(la), o);
#pragma unroll
    for (int q = 0; q < 12; ++q) out[q * n + i] = o[q];
  }
}

__global__ void rhs_kernel(Field F, int64_t n, const double* __restrict__ y,
                           double* __restrict__ dydt) {
  nm_stage<NM_SINCOS | NM_TAN>();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double yy[5], d[5];
#pragma unroll
    for (int v = 0; v < 5; ++v) yy[v] = y[v * n + i];
    ray_rhs(StaticBG{F}, 0.0, yy, d);
#pragma unroll
    for (int v = 0; v < 5; ++v) dydt[v * n + i] = d[v];
  }
}

__global__ void attempt_kernel(Field F, int64_t n, const double* __restrict__ y,
                               const double* __restrict__ f, const double* __restrict__ h,
                               double rtol, double atol, double* __restrict__ Kout,
                               double* __restrict__ ynew, double* __restrict__ err) {
  nm_stage<NM_SINCOS | NM_TAN>();
  const RayProblem P{StaticBG{F}};
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double yy[5], ff[5], yn[5], k6[5];
#pragma unroll
    for (int v = 0; v < 5; ++v) {
      yy[v] = y[v * n + i];
      ff[v] = f[v * n + i];
    }
    KRegs<5> K;
    err[i] = dp54_attempt(P, K, 0.0, yy, ff, h[i], rtol, atol, yn, k6, Kout + i, n);
#pragma unroll
    for (int v = 0; v < 5; ++v) ynew[v * n + i] = yn[v];
  }
}

template <class BG>
struct InitArgs {
  BG B;
  int64_t nray;
  const double* y0;
  double rtol, atol;
  int32_t nt;
  double* state;
  int64_t* count;
  int32_t* nanrow;
  int32_t* live;
  int64_t* summary;
};

template <class BG>
__global__ void rk45_init_kernel(InitArgs<BG> a) {
  nm_stage<NM_ALL>();
  const RayProblemT<BG> P{a.B};
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < a.nray;
       i += (int64_t)gridDim.x * blockDim.x) {
    double y[5], f[5];
#pragma unroll
    for (int v = 0; v < 5; ++v) y[v] = a.y0[v * a.nray + i];
    P(0.0, y, f);                                   // RungeKutta.__init__: f = fun(t, y)
    const double habs = initial_step(P, 0.0, y, f, a.rtol, a.atol);
#pragma unroll
    for (int v = 0; v < 5; ++v) {
      a.state[v * a.nray + i] = y[v];
      a.state[(5 + v) * a.nray + i] = f[v];
    }
    a.state[10 * a.nray + i] = 0.0;
    a.state[11 * a.nray + i] = habs;
    a.count[2 * i] = 0;
    a.count[2 * i + 1] = 0;
    a.nanrow[i] = a.nt;
    const double mean = ((((y[0] + y[1]) + y[2]) + y[3]) + y[4]) / 5.0;
    const bool live = !isnan(mean);
    a.live[i] = live ? 1 : 0;
    if (live) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&a.summary[0]), 1ull);
      if (!isnan(habs)) atomicAdd(reinterpret_cast<unsigned long long*>(&a.summary[1]), 1ull);
    }
  }
}

template <class BG>
struct RunArgs {
  BG B;
  int64_t nray;
  double rtol, atol, min_step, cut_off;
  int32_t nt, it_begin, it_end;
  const double* tbound;
  const int64_t* order;
  double* state;
  int64_t* count;
  int32_t* nanrow;
  double* out;
  int32_t* queue;       // [1]: the work queue's head; [0]: rays handed off (drain-time hand-off)
  int64_t n_heavy;      // order[0, n_heavy): rays in latency mode (quad_rays); the queue is the rest
  int32_t heavy_blocks; // blocks [0, heavy_blocks) run order[0, n_heavy) in latency mode (quad_rays)
  double cut_a;         // haversine argument certainly below cut_off (cal_dis_below)
  const uint8_t* frozen;  // rays frozen at the launch start (NULL: none skipped), see frozen_fill_kernel
  int32_t quad_per_wave = 16;  // latency mode: rays per wave (1..16; fewer = less divergence per ray)
  int64_t* trace = nullptr;    // diagnostic ray trace (rwrt_ctx_set_trace), positions < trace_cap
  int64_t trace_cap = 0;
  // ABI 4 (rwrt_rk45_run_slots): the row block of ray j in out is
  // row_slot[j] (the rays live at the call's start, numbered in ray order by
  // rwrt_row_slots; -1 for a frozen ray, whose rows are its tail); NULL: j
  const int32_t* row_slot = nullptr;
  // drain-time hand-off (run_rays, static state): once the queue is drained,
  // a wave with at most this many rays left continues them in the latency
  // mode's quad layout (0: off; rwrt_ctx_set_handoff, default 16)
  int32_t handoff = 16;
};

// The first output row of ray `ray` in this call's row buffer (NULL when the
// ray has no row block: frozen at the call's start, so never stepped here)
template <class BG>
__device__ __forceinline__ double* row_block(const RunArgs<BG>& a, int64_t ray) {
  const int64_t slot = a.row_slot ? (int64_t)a.row_slot[ray] : ray;
  return slot < 0 ? nullptr : a.out + (size_t)slot * (size_t)(a.it_end - a.it_begin) * RWRT_NOUT;
}


// A frozen ray's rows are all one row (rkf45.py:400-403: its state never
// changes again): with tails, that row is stored once per ray instead
__device__ __forceinline__ void store_tail(double* tail_row, int64_t ray, double2 r0, double2 r1, double2 r2,
                                           double2 r3) {
  double2* o = reinterpret_cast<double2*>(tail_row + (size_t)ray * RWRT_NOUT);
  o[0] = r0;
  o[1] = r1;
  o[2] = r2;
  o[3] = r3;
}

// rwrt_ctx_set_trace: where (HW_ID, XCC) and when a traced ray ran
constexpr int kTraceWords = 10;
__device__ __forceinline__ void trace_start(int64_t* tr, int64_t w) {
  tr[w * kTraceWords + 3] = (int64_t)__builtin_amdgcn_s_memrealtime();
  tr[w * kTraceWords + 8] = (int64_t)__builtin_amdgcn_s_memtime();
}
__device__ __forceinline__ void trace_ray(int64_t* tr, int64_t w, int64_t ray, int64_t attempts, bool latency) {
  const unsigned hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID, 32 bits
  const unsigned xcc = __builtin_amdgcn_s_getreg(20 | (15 << 11));  // HW_REG_XCC_ID
  int64_t* r = tr + w * kTraceWords;
  r[0] = ray;
  r[1] = hw;
  r[2] = xcc;
  r[4] = (int64_t)__builtin_amdgcn_s_memrealtime();   // (r[3], r[8]: trace_start)
  r[5] = attempts;
  r[6] = latency ? 1 : 0;
  r[7] = blockIdx.x;
  r[9] = (int64_t)__builtin_amdgcn_s_memtime();       // shader clock: r[9]-r[8] cycles over r[4]-r[3]
}

// Haversine threshold: d = 2 atan2(sqrt(a), sqrt(1 - a)) increases with a, so
// a < sin^2(cut_off / 2) (1 - 1e-9) proves d < cut_off for the computed d too
// (its error is ~1e-15 relative) -- the common "no jump" verdict of wr.py:844-850
// without the atan2 and the two square roots.  Any other a (near or above the
// threshold, > 1, NaN) takes the full cal_dis.  -1 disables the shortcut.
inline double haversine_cut(double cut_off) {
  if (!(cut_off > 0.0 && cut_off <= 3.0)) return -1.0;
  const double s = std::sin(0.5 * cut_off);
  return s * s * (1.0 - 1e-9);
}

// ---------------------------------------------------------------------------
// Latency mode, v2 (quad_rays, in rk45_run_kernel's first blocks).  Four lanes of one wavefront per ray
// (a DPP quad, 16 rays per wave): the quad's lanes hold the ray's state
// replicated and compute the serial parts -- trigonometry, cell arithmetic,
// lookup, Mercator products, pow, step control -- identically (free on a
// SIMD), while the parts that are the same instructions on different
// operands are dealt out over the four lanes (role = lane & 3) and exchanged
// with quad_perm DPP moves (no LDS, no barrier):
//   * the RHS's 16 IEEE divisions become two divisions pairs and one
//     division per lane:
//       slot 1   role 0: fu/cp, fv/cp       role 1: ux/cp, vx/cp
//                role 2: cal_ugvg's qu, qv  role 3: core_diffun's qk, ql
//       slot 2   role 0: damp1, damp2       role 1: dy0, dy1 (ug/R, vg c/R)
//                role 2: dy2, dy3           (role 3: a copy of role 2)
//       then     damp * amp / R on every lane;
//   * the stage sums and the error estimate: lane `role` owns variable `role`
//     (and every lane variable 4): two sums per lane instead of five, its
//     stage values K_s (two per stage) in its LDS slice;
//   * the error norm's five quotients: one pair per lane.
// Every value is the same operation on the same operands as in ray_rhs /
// dp54_attempt, so results are the run kernel's bit for bit.  A wave of 16
// heavy rays also diverges less often (interval ends, cell refills) than one
// of 64.
// ---------------------------------------------------------------------------

// x of lane (quad base + P[role]) for every lane of the quad (DPP quad_perm;
// every lane of a quad is active whenever one is: they share the ray)
template <int P0, int P1, int P2, int P3>
__device__ __forceinline__ double qperm(double x) {
  constexpr int ctrl = P0 | (P1 << 2) | (P2 << 4) | (P3 << 6);
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), ctrl, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), ctrl, 0xf, 0xf, true);
  return __hiloint2double(hi, lo);
}
template <int J>
__device__ __forceinline__ double qbcast(double x) { return qperm<J, J, J, J>(x); }

struct QuadRole {
  int role;
  bool odd, high;   // role & 1, role & 2
  __device__ __forceinline__ double sel(double a, double b, double c, double d) const {
    const double ab = odd ? b : a, cd = odd ? d : c;
    return high ? cd : ab;
  }
};

// lookup_end for a quad: the eleven blends dealt out by record (role r blends
// records r and r + 4, roles 2 and 3 record r only: u v qxx qxy | ux uy qyy |
// vx vy | qx qy), 8 LDS reads per lane instead of 24, then broadcast; each
// field is the same blend of the same corner values (bit for bit).
__device__ __forceinline__ void quad_lookup_end(const CachedStaticBG& B, const QuadRole& R,
                                                const CachedStaticBG::Pending& p, double g[11]) {
  lds_dma_wait();
  Corners k;
  k.wa = p.wa;
  k.wb = p.wb;
  k.wc = p.wc;
  k.wd = p.wd;
  // records ra = role and rb = role + 4 (roles 2, 3: role again) of corner j
  // sit in this lane's slots (j, 0) and (j, 1) (CachedStaticBG::quad_refill)
  const char* base = B.wave_base + B.lane16;
  double2 va[4], vb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    va[j] = *reinterpret_cast<const double2*>(base + (j * 2) * 1024);
    vb[j] = *reinterpret_cast<const double2*>(base + (j * 2 + 1) * 1024);
  }
  const double ax = blend(k, va[0].x, va[1].x, va[2].x, va[3].x);
  const double ay = blend(k, va[0].y, va[1].y, va[2].y, va[3].y);
  const double bx = blend(k, vb[0].x, vb[1].x, vb[2].x, vb[3].x);
  const double by = blend(k, vb[0].y, vb[1].y, vb[2].y, vb[3].y);
  g[F_U] = qbcast<0>(ax);
  g[F_V] = qbcast<0>(ay);
  g[F_UX] = qbcast<1>(ax);
  g[F_UY] = qbcast<1>(ay);
  g[F_VX] = qbcast<2>(ax);
  g[F_VY] = qbcast<2>(ay);
  g[F_QX] = qbcast<3>(ax);
  g[F_QY] = qbcast<3>(ay);
  g[F_QXX] = qbcast<0>(bx);
  g[F_QXY] = qbcast<0>(by);
  g[F_QYY] = qbcast<1>(bx);
}

// ray_rhs (wr.py:492-556) for one ray per quad: returns dy[role] (rA) and
// dy[4] (rB); aux as in ray_rhs (every lane).
__device__ __forceinline__ void quad_rhs(const CachedStaticBG& B, const QuadRole& R, const double* y,
                                         double& rA, double& rB, double* aux) {
  MARK("rhs");
  const double lon = y[0], lat = y[1], kx = y[2];
  const bool bad = fabs(lat) >= kHalfPi || fabs(y[3]) >= 100.0;
  const double ky = bad ? kNaN : y[3], amp = y[4];
  double g[11];
  // sin on roles 0 and 2, cos on roles 1 and 3: one do_sin / do_cos stream
  // and one table point per lane (np_math.h nm_sinorcos_fin), then broadcast
#if RWRT_TEAM_SINORCOS
  const auto trig = np_math::nm_sinorcostan_begin(lat, R.odd);
#else
  const auto trig = np_math::nm_sincostan_begin(lat);
#endif
  MARK("trig_begin_done");
  const KapTerms kw = kap_terms(kx, ky);
  MARK("kap_done");
  const int rb = R.high ? R.role : R.role + 4;
  const auto pending = B.quad_begin(lon, lat, (unsigned)R.role * 1024u, (unsigned)(rb - 1) * 1024u);
  MARK("cell_done");
#if RWRT_TEAM_SINORCOS
  double sc, tn;
  np_math::nm_sinorcostan_end(lat, R.odd, trig, sc, tn);
  const double s = qbcast<0>(sc), c = qbcast<1>(sc);
#else
  double s, c, tn;
  np_math::nm_sincostan_end(lat, trig, s, c, tn);
#endif
  MARK("trig_end_done");
  __builtin_amdgcn_sched_barrier(0);
  quad_lookup_end(B, R, pending, g);
  MARK("lookup_done");
  // Mercator (bs.py:856-883): M.cp == c off the pole band; there every
  // output takes mercator12_masked's extra factor m
  const Merc M = merc_factors(lat, c, s);
  const double cp = M.cp, m = M.m;
  const bool mk = m != 1.0;
  const double fu = g[F_U], fv = g[F_V];
  // (the mask's factor on a branch, not as selects: 24 v_cndmask per RHS
  // on the common path otherwise)
  double fmuy = g[F_UY] + tn * fu, fmvy = g[F_VY] + tn * fv;
  double fmqx = g[F_QX], fmqy = g[F_QY] * cp, fmqxx = g[F_QXX], fmqyx = g[F_QXY] * cp;
  double fmqxy = fmqyx, fmqyy = ((g[F_QYY] * cp) - (g[F_QY] * M.s)) * cp;
  if (RARE(mk)) {
    asm volatile("");   // the pole band (rare branch)
    fmuy = fmuy * m;
    fmvy = fmvy * m;
    fmqx = fmqx * m;
    fmqy = fmqy * m;
    fmqxx = fmqxx * m;
    fmqyx = fmqyx * m;
    fmqxy = fmqyx * m;
    fmqyy = fmqyy * m;
  }
  const double kap = kw.kap, kap2 = kw.kap2;
  MARK("merc_done");
  // slot 1: the quotients that need no other quotient
  double q1, q2;
  {
    const double n1 = R.sel(fu, g[F_UX], ((1.0 - kap2) * fmqy) - ((2.0 * kap) * fmqx), kap * fmqxx - fmqyx);
    const double n2 = R.sel(fv, g[F_VX], ((2.0 * kap) * fmqy) + ((1.0 - kap2) * fmqx), kap * fmqxy - fmqyy);
    const double d = R.sel(cp, cp, kw.denom, kw.kk);
    div2(n1, d, n2, d, q1, q2);
  }
  const double du = qbcast<0>(q1), dv = qbcast<0>(q2), dux = qbcast<1>(q1), dvx = qbcast<1>(q2);
  const double qu = qbcast<2>(q1), qv = qbcast<2>(q2), qk = qbcast<3>(q1), ql = qbcast<3>(q2);
  double fmu = du, fmv = dv, fmux = dux, fmvx = dvx;
  if (RARE(mk)) {
    asm volatile("");   // the pole band (rare branch)
    fmu = du * m;
    fmv = dv * m;
    fmux = dux * m;
    fmvx = dvx * m;
  }
  const double ug = fmu + qu, vg = fmv + qv;                       // cal_ugvg (wn.py:266-294)
  const double dzwn = (-kx) * ((fmux + kap * fmvx) + qk);          // core_diffun (wr.py:53-78)
  const double dmwn = (-kx) * ((fmuy + kap * fmvy) + ql);
  MARK("slot1_done");
  // slot 2
  double p1, p2;
  {
    const double a1 = 2.0 * ((fmux + fmvy) + kap * (fmvx + fmuy));
    const double a2 = 2.0 * (kap * (fmqxx - fmqyy) + (kap2 - 1.0) * fmqxy);
    const double n1 = R.sel(a1, ug, dzwn, dzwn);
    const double n2 = R.sel(a2, vg * c, dmwn, dmwn);
    const bool r0 = !R.odd && !R.high;
    div2(n1, r0 ? kw.kap1 : kREarth, n2, r0 ? kw.denom : kREarth, p1, p2);
  }
  const double damp1 = qbcast<0>(p1), damp2 = qbcast<0>(p2);
  const double damp = (damp1 + damp2) + (-2.0 * s) * fmv;
  rB = div_rearth(damp * amp);
  // dy[role]: dy0, dy1 on role 1, dy2, dy3 on role 2
  const double a = qperm<1, 1, 2, 2>(p1), b = qperm<1, 1, 2, 2>(p2);
  rA = R.odd ? b : a;
  aux[0] = ug;
  aux[1] = vg;
  aux[2] = bad ? kNaN : c;
  MARK("slot2_done");
}

// The stage values K1..K5 this lane owns (variables `role` and 4), in its
// slice of LDS: element (stage j, slot) at p[((j - 1) * 2 + slot) * 256]
struct KQuad {
  double* p;
  __device__ __forceinline__ double get(int j, int slot) const { return p[((j - 1) * 2 + slot) * 256]; }
  __device__ __forceinline__ void put(int s, double a, double b) {
    p[((s - 1) * 2 + 0) * 256] = a;
    p[((s - 1) * 2 + 1) * 256] = b;
  }
};
// wsum's first J terms of stage S for the owned variables (K0 = fA, fB)
template <int S, int J>
__device__ __forceinline__ void quad_part(const KQuad& K, double fA, double fB, double& pA, double& pB) {
  double a = 0.0, b = 0.0;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    a = a + ((j == 0) ? fA : K.get(j, 0)) * kW[S][j];
    b = b + ((j == 0) ? fB : K.get(j, 1)) * kW[S][j];
  }
  pA = a;
  pB = b;
}
__device__ __forceinline__ void quad_epart(const KQuad& K, double fA, double fB, double& pA, double& pB) {
  double a = 0.0, b = 0.0;
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    a = a + ((j == 0) ? fA : K.get(j, 0)) * kE[j];
    b = b + ((j == 0) ? fB : K.get(j, 1)) * kE[j];
  }
  pA = a;
  pB = b;
}

// dp54_attempt (rkf45.py:259-321, 368-373) for the quad's ray: fills y_new
// and K6 (every lane), returns the error norm (every lane)
__device__ __forceinline__ double quad_attempt(const CachedStaticBG& B, const QuadRole& R, KQuad& K,
                                               const double* y, const double* f, double h,
                                               double rtol, double atol, double* ynew, double* k6,
                                               double* aux) {
  const double yA = R.sel(y[0], y[1], y[2], y[3]), fA = R.sel(f[0], f[1], f[2], f[3]);
  const double yB = y[4], fB = f[4];
  double ys[5];
#pragma unroll
  for (int v = 0; v < 5; ++v) ys[v] = y[v] + wsum<1, 5>(K, f, v) * h;   // (K unused for stage 1)
  double ysA = 0.0, ysB = 0.0, rA = 0.0, rB = 0.0, pA = 0.0, pB = 0.0;
#pragma unroll
  for (int s = 1; s <= 6; ++s) {
    double w = 0.0, cn = 0.0;
    switch (s) {
      case 1: quad_part<2, 1>(K, fA, fB, pA, pB); w = kW[2][1]; cn = kCs[2]; break;
      case 2: quad_part<3, 2>(K, fA, fB, pA, pB); w = kW[3][2]; cn = kCs[3]; break;
      case 3: quad_part<4, 3>(K, fA, fB, pA, pB); w = kW[4][3]; cn = kCs[4]; break;
      case 4: quad_part<5, 4>(K, fA, fB, pA, pB); w = kW[5][4]; cn = kCs[5]; break;
      case 5: quad_part<6, 5>(K, fA, fB, pA, pB); w = kW[6][5]; cn = kCs[6]; break;
      default: quad_epart(K, fA, fB, pA, pB); break;
    }
    (void)cn;   // (autonomous RHS: stage times unused)
    MARK("stage_part_done");
    quad_rhs(B, R, ys, rA, rB, aux);
    if (s < 6) {
      K.put(s, rA, rB);
      ysA = yA + (pA + rA * w) * h;
      ysB = yB + (pB + rB * w) * h;
      ys[0] = qbcast<0>(ysA);
      ys[1] = qbcast<1>(ysA);
      ys[2] = qbcast<2>(ysA);
      ys[3] = qbcast<3>(ysA);
      ys[4] = ysB;
    }
  }
  MARK("stages_done");
  // ys = y_new, (rA, rB) = K6; error estimate of the owned variables
#pragma unroll
  for (int v = 0; v < 5; ++v) ynew[v] = ys[v];
  k6[0] = qbcast<0>(rA);
  k6[1] = qbcast<1>(rA);
  k6[2] = qbcast<2>(rA);
  k6[3] = qbcast<3>(rA);
  k6[4] = rB;
  const double eA = h * (pA + rA * kE[6]), eB = h * (pB + rB * kE[6]);
  const double scA = atol + np_max(fabs(yA), fabs(ysA)) * rtol;
  const double scB = atol + np_max(fabs(yB), fabs(ysB)) * rtol;
  double xA, xB;
  div2(eA, scA, eB, scB, xA, xB);
  const double x0 = qbcast<0>(xA), x1 = qbcast<1>(xA), x2 = qbcast<2>(xA), x3 = qbcast<3>(xA);
  double ss = x0 * x0;
  ss = ss + x1 * x1;
  ss = ss + x2 * x2;
  ss = ss + x3 * x3;
  ss = ss + xB * xB;
  MARK("error_norm_done");
  return sqrt(ss) / RootN<5>::v;
}

// cal_dis_reaches for a quad (wr.py:844-850): the two half-difference sines
// on two lanes (role 0: latitude, role 1: longitude), then broadcast
__device__ __forceinline__ bool quad_dis_reaches(const QuadRole& R, double lon_c, double lat_c,
                                                 double lon_p, double lat_p, double cos_c,
                                                 double cos_p, double cut_off, double cut_a) {
  const double dlat2 = (lat_c - lat_p) / 2.0, dlon2 = (lon_c - lon_p) / 2.0;
  {   // (cal_dis_reaches' polynomial verdict, the same operations: selftest kinds 36/37)
    const double s1 = sin_small(dlat2), s2 = sin_small(dlon2);
    const double ap = s1 * s1 + (cos_p * cos_c) * (s2 * s2);
    if (fabs(dlat2) <= 0.0625 && fabs(dlon2) <= 0.0625 && ap < cut_a * (1.0 - 1e-12)) return false;
  }
  const double sv = k_sin(R.odd ? dlon2 : dlat2);
  const double sd = qbcast<0>(sv), sl = qbcast<1>(sv);
  const double a = sd * sd + (cos_p * cos_c) * (sl * sl);
  bool r = false;
  if (!(a < cut_a)) {
    asm volatile("");   // rare: near or past the threshold, or NaN
    r = fabs(2.0 * atan2(sqrt(a), sqrt(1.0 - a))) >= cut_off;
  }
  return r;
}

// Rows [it_begin, it_end) of rays order[0, n_heavy), one per quad (64 per
// block, no queue): rk45_run_kernel's loop, step control and post-processing.
// Run by rk45_run_kernel's first a.heavy_blocks blocks (one grid: those
// blocks are placed with the persistent ones, one per CU, whatever the
// dispatch order of concurrent kernels), in the run kernel's LDS: the cell
// cache where the run kernel keeps it, the owned stage values (20 KB) where
// the run kernel keeps its stages.
// quad_rays' interval loop from a ray's running state (also the drain-time
// hand-off of rk45_run_kernel's waves, run_rays): rows [it, it_end) of `ray`,
// its mid-step state included (in_step, rejected, hs), exactly where a run
// kernel lane left it between two attempts
template <bool kTrace>
__device__ __forceinline__ void quad_run(const RunArgs<StaticBG>& a, const CachedStaticBG& B, const QuadRole& R,
                                         KQuad& K, int64_t ray, double* rows, double (&y)[5], double (&f)[5],
                                         double (&aux)[3], double t, double habs, double hs, int64_t nacc,
                                         int64_t nrej, int64_t att0, int32_t nanrow, int32_t it, double prev_lon,
                                         double prev_lat, double cos_prev, bool in_step, bool rejected,
                                         int64_t w) {
  const bool writer = R.role == 0;
  for (;;) {
    const double tb = a.tbound[it];
    // ---- Lane::iterate (rkf45.py:222-253, 375-514)
    int st = 0;   // 0 step, 1 reached, 2 frozen
    if (!in_step) {
      const double sum = (((y[0] + y[1]) + y[2]) + y[3]) + y[4];
      if (isnan(sum)) {   // (== isnan(sum / 5.0): Lane::iterate)
        t = tb;
        st = 2;
      } else if (t == tb) {
        st = 1;
      } else {
        hs = np_max(habs, a.min_step);
        rejected = false;
        in_step = true;
      }
    }
    if (st == 0) {
      double tn = t + hs;
      if (tn - tb > 0.0) tn = tb;
      const double h = tn - t;
      const double ha = fabs(h);
      double yn[5], k6[5];
      double en = quad_attempt(B, R, K, y, f, h, a.rtol, a.atol, yn, k6, aux);
      MARK("attempt_done");
      if (en != en) en = 0.0;
      const double sp = kSafety * k_pow(en, kErrExp);
      MARK("pow_done");
      const bool acc = en < 1.0;
      double fac = np_min(kMaxFactor, sp);
      if (en == 0.0) fac = kMaxFactor;
      if (rejected) fac = np_min(1.0, fac);
      const double tnew = (tn != tn) ? tb : tn;
      habs = acc ? ha * fac : habs;
      hs = acc ? hs : ha * np_max(kMinFactor, sp);
      t = acc ? tnew : t;
#pragma unroll
      for (int v = 0; v < 5; ++v) {
        y[v] = acc ? yn[v] : y[v];
        f[v] = acc ? k6[v] : f[v];
      }
      in_step = !acc;
      rejected = rejected || !acc;
      nacc += acc ? 1 : 0;
      nrej += acc ? 0 : 1;
      MARK("control_done");
      if (!(acc && t - tb >= 0.0)) continue;
      st = 1;
    }
    // ---- interval it reached: rk45_run_kernel's post-processing (wr.py:835-885)
    MARK("row_end");
    const bool have = !isnan(aux[2]);
    double ug, vg, cos_c = kNaN;
    bool masked = fabs(y[1]) >= kHalfPi;
    if (!masked) {
      cos_c = aux[2];
      if (RARE(!have)) cos_c = cos_small(y[1]);   // (a branch: rare)
      masked = quad_dis_reaches(R, y[0], y[1], prev_lon, prev_lat, cos_c, cos_prev, a.cut_off, a.cut_a);
    }
    if (masked) {
#pragma unroll
      for (int v = 0; v < 5; ++v) y[v] = kNaN;
      ug = vg = kNaN;
      cos_c = kNaN;
      aux[2] = kNaN;
    } else if (have) {
      ug = aux[0];
      vg = aux[1];
    } else {
      ugvg_at(a.B, tb, y[0], y[1], y[2], y[3], ug, vg);
    }
    const int last = (st == 2) ? a.it_end : it + 1;
    if (writer && rows) {
      const double2 r0 = make_double2(y[0], y[1]), r1 = make_double2(y[2], y[3]);
      const double2 r2 = make_double2(y[4], ug), r3 = make_double2(vg, (double)nacc);
      for (int kr = it; kr < last; ++kr) {
        double2* o = reinterpret_cast<double2*>(rows + (size_t)(kr - a.it_begin) * RWRT_NOUT);
        store_row16<RWRT_ROW_NT>(o + 0, r0);
        store_row16<RWRT_ROW_NT>(o + 1, r1);
        store_row16<RWRT_ROW_NT>(o + 2, r2);
        store_row16<RWRT_ROW_NT>(o + 3, r3);
      }
    }
    if (nanrow == a.nt && isnan(y[0])) nanrow = it;   // wr.py:853-855 (host reduces)
    prev_lon = y[0];
    prev_lat = y[1];
    cos_prev = cos_c;
    it = last;
    if (st == 2) t = a.tbound[a.it_end - 1];
    if (it == a.it_end) break;
  }
  if (writer) {
#pragma unroll
    for (int v = 0; v < 5; ++v) {
      a.state[v * a.nray + ray] = y[v];
      a.state[(5 + v) * a.nray + ray] = f[v];
    }
    a.state[10 * a.nray + ray] = t;
    a.state[11 * a.nray + ray] = habs;
    a.count[2 * ray] = nacc;
    a.count[2 * ray + 1] = nrej;
    a.nanrow[ray] = nanrow;
    if (kTrace && w < a.trace_cap) trace_ray(a.trace, w, ray, nacc + nrej - att0, true);
  }
}

template <bool kTrace>
__device__ __forceinline__ void quad_rays(const RunArgs<StaticBG>& a, char* cache, double* Kq, int lb) {
  const CachedStaticBG B = LaneBG<StaticBG>::make(a.B, cache);
  QuadRole R;
  R.role = threadIdx.x & 3;
  R.odd = (R.role & 1) != 0;
  R.high = (R.role & 2) != 0;
  KQuad K{Kq + threadIdx.x};
  // order position of this quad's ray, a.quad_per_wave quads per wave
  const int qi = (threadIdx.x & 63) >> 2;
  // consecutive positions share a wave (p -> wave p / quad_per_wave): rays of
  // like weight, which on C3 are often near-copies whose row ends and cell
  // crossings stay aligned.  Dealing the heaviest one per wave instead (p ->
  // wave p % waves) mixed rays that diverge: the 256 heaviest C3 rays at 4 per
  // wave took 14.5 us per attempt of the heaviest, 9.6 us contiguous
  // (profiles/r4/sched/latency_xcd.txt)
  const int64_t w = (lb * 4 + (int64_t)(threadIdx.x >> 6)) * a.quad_per_wave + qi;
  const int64_t ray = (qi < a.quad_per_wave && w < a.n_heavy) ? a.order[w] : -1;
  if (ray < 0) return;   // (whole quads: the four lanes share w)
  // a ray frozen at the launch start is frozen_fill_kernel's (the C ABI asks
  // for live rays in order[0, n_heavy); a C caller's frozen one is skipped
  // here, not written twice)
  if (a.frozen && a.frozen[ray]) return;
  double y[5], f[5], aux[3];
#pragma unroll
  for (int v = 0; v < 5; ++v) {
    y[v] = a.state[v * a.nray + ray];
    f[v] = a.state[(5 + v) * a.nray + ray];
  }
  double t = a.state[10 * a.nray + ray], habs = a.state[11 * a.nray + ray], hs = 0.0;
  int64_t nacc = a.count[2 * ray], nrej = a.count[2 * ray + 1];
  const int64_t att0 = nacc + nrej;
  double* const rows = row_block(a, ray);
  if (kTrace && w < a.trace_cap && R.role == 0) trace_start(a.trace, w);
  int32_t nanrow = a.nanrow[ray];
  int32_t it = a.it_begin;
  double prev_lon = y[0], prev_lat = y[1], cos_prev = k_cos(prev_lat);
  aux[2] = kNaN;
  bool in_step = false, rejected = false;
  quad_run<kTrace>(a, B, R, K, ray, rows, y, f, aux, t, habs, hs, nacc, nrej, att0, nanrow, it, prev_lon,
                   prev_lat, cos_prev, in_step, rejected, w);
}

// WR.core_ray_run_rk45 (wr.py:767-887) for rows [it_begin, it_end): persistent
// lanes, one ray each, refilled from the work queue.
//
// Load balance: the work per ray per chunk spans 15x the mean (C3); the
// slowest rays set the makespan.  The host orders rays by the work they did in
// the previous chunk (longest first) and may hand the heaviest ones to the
// latency mode (quad_rays in the grid's first blocks, order[0, n_heavy)); the
// queue is the rest.
using KStore = KShared<5>;
// kTrace: the diagnostic instantiation (rwrt_ctx_set_trace) -- the product
// kernel carries none of the trace hooks
#ifndef RWRT_RUN_ALIGN
#define RWRT_RUN_ALIGN 256
#endif
// the latency mode's background of a time-varying run kernel (none: void)
template <class BG>
struct TvBlock {
  using type = void;
};
template <class T>
struct TvBlock<VaryingBG<T>> {
  using type = BlockVaryingBG<T>;
};

// The ray loop of rk45_run_kernel's blocks: each lane pulls rays from the
// work queue (hw = -1), or -- kReplica, the time-varying latency mode -- every
// lane of the wave runs the ray at order position hw, replicated, through a
// BlockVaryingBG, and lane 0 stores its rows and state.
template <class BG, class LBG, bool kTrace, bool kReplica, bool kPair = false>
__device__ __forceinline__ void run_rays(const RunArgs<BG>& a, const LBG& lbg, char* smem, int64_t hw) {
  using RayProblem = RayProblemT<LBG>;
  const RayProblem P{lbg};
  // (a latency wave's lane 0 stores; lane pairs: the lower lane)
  const bool writer = kReplica ? (threadIdx.x & 63u) == 0 : kPair ? (threadIdx.x & 63u) < 32u : true;
  Lane<RayProblem, KStore> L;
  L.K.p = reinterpret_cast<double*>(smem) + threadIdx.x;
  L.K.stride = 256;
  int64_t ray = -1, nacc = 0, nrej = 0;
  double* rows = nullptr;   // the ray's row block (row_block)
  int32_t it = 0, nanrow = 0, wpos = 0;   // (wpos: the ray's queue position, kTrace only)
  double prev_lon = 0.0, prev_lat = 0.0, cos_prev = 0.0;
  // drain-time hand-off (the static state's ray loop): see below the loop
  constexpr bool kHandoff = std::is_same<LBG, CachedStaticBG>::value && !kReplica && !kPair && !kTrace;
  bool handoff = false;
  // above frozen_fill_kernel's waves (priority 0) sharing the SIMD: the
  // fill takes the issue cycles the ray loop leaves idle
  __builtin_amdgcn_s_setprio(1);
  for (;;) {
    if (ray < 0) {
      int64_t w;
      if (kReplica) {   // a latency wave: its one ray, then done
        if (hw < 0) break;
        w = hw;
        hw = -1;
      } else if (kPair) {   // lane pairs: the lower lane pulls, the upper one takes the same ray
        int64_t w0 = 0;
        if ((threadIdx.x & 63u) < 32u) w0 = a.n_heavy + atomicAdd(&a.queue[1], 1);
        w = __shfl(w0, (int)(threadIdx.x & 31u));
      } else {
        w = a.n_heavy + atomicAdd(&a.queue[1], 1);
      }
      if (w >= a.nray) break;
      ray = a.order ? a.order[w] : w;
      if (kTrace) {
        wpos = (int32_t)w;
        if (w < a.trace_cap) trace_start(a.trace, w);
      }
      if (a.frozen && a.frozen[ray]) {   // its rows come from frozen_fill_kernel
        ray = -1;
        continue;
      }
#pragma unroll
      for (int v = 0; v < 5; ++v) {
        L.y[v] = a.state[v * a.nray + ray];
        L.f[v] = a.state[(5 + v) * a.nray + ray];
      }
      L.t = a.state[10 * a.nray + ray];
      L.habs = a.state[11 * a.nray + ray];
      rows = row_block(a, ray);
      L.in_step = false;
      L.rejected = false;
      L.hs = 0.0;
      nacc = a.count[2 * ray];
      nrej = a.count[2 * ray + 1];
      nanrow = a.nanrow[ray];
      it = a.it_begin;
      prev_lon = L.y[0];   // == rlon[it-1], rlat[it-1] (wr.py:844, 877-885)
      prev_lat = L.y[1];
      cos_prev = k_cos(prev_lat);
      L.aux[2] = kNaN;     // no evaluation at y yet
    }
    if constexpr (kHandoff) {
      // (wave-uniform) few rays left in this wave and none left in the queue:
      // hand them to the quad layout, between two attempts
      if (RARE(__builtin_popcountll(__builtin_amdgcn_ballot_w64(true)) <= (unsigned)a.handoff)) {
        const int32_t q = __atomic_load_n(&a.queue[1], __ATOMIC_RELAXED);
        if (a.n_heavy + (int64_t)q >= a.nray) {
          handoff = true;
          break;
        }
      }
    }
    const double tb = a.tbound[it];
    const int st = L.iterate(P, tb, a.min_step, a.rtol, a.atol, nacc, nrej);
    if (st == Lane<RayProblem, KStore>::kStep) continue;
    MARK("x_row_end");

    // ---- interval it reached: post-processing (wr.py:835-885) ----
    // The last accepted step's K6 evaluation was at this y: its cos(lat), ug
    // and vg are the values wr.py:844 and wr.py:856-865 recompute (same
    // inputs, same operations), so they are reused unless that evaluation was
    // masked (aux NaN) or y has changed since.
    double* y = L.y;
    // (a time-varying flow: K6 was evaluated at t + h, which can differ from
    // t_bound in the last bit -- its values are reused only when it does not:
    // t + (t_bound - t) == t_bound whenever t_bound / 2 <= t, i.e. at every
    // row end but the first few; otherwise ugvg_at recomputes at t_bound,
    // an HBM round trip per row end at 0.25 degrees)
#ifndef RWRT_TV_REUSE_K6
#define RWRT_TV_REUSE_K6 1
#endif
    const bool have = (!BG::kTimeVarying || (RWRT_TV_REUSE_K6 && L.tk6 == tb)) && !isnan(L.aux[2]);
    double ug, vg, cos_c = kNaN;
    bool masked = fabs(y[1]) >= kHalfPi;
    if (!masked) {
      cos_c = L.aux[2];
      if (RARE(!have)) cos_c = cos_small(y[1]);   // |y[1]| < pi/2 or NaN here (a branch: rare)
      masked = cal_dis_reaches(y[0], y[1], prev_lon, prev_lat, cos_c, cos_prev, a.cut_off, a.cut_a);
    }
    if (masked) {
#pragma unroll
      for (int v = 0; v < 5; ++v) y[v] = kNaN;
      ug = vg = kNaN;             // ugvg of a NaN position
      cos_c = kNaN;
      L.aux[2] = kNaN;
    } else if (have) {
      ug = L.aux[0];
      vg = L.aux[1];
    } else if (RARE(true)) {   // the last evaluation at y was masked (rare)
      ugvg_at(a.B, tb, y[0], y[1], y[2], y[3], ug, vg);
    }
    const double2 r0 = make_double2(y[0], y[1]), r1 = make_double2(y[2], y[3]);
    const double2 r2 = make_double2(y[4], ug), r3 = make_double2(vg, (double)nacc);
    // A frozen ray never changes again (its mean stays NaN; re-applying the
    // masks against itself is a no-op), so every remaining row of the chunk
    // equals this one: write them all and release the lane.
    const int last = (st == Lane<RayProblem, KStore>::kFrozen) ? a.it_end : it + 1;
    if (writer && rows) {
      double2* o = reinterpret_cast<double2*>(rows + (size_t)(it - a.it_begin) * RWRT_NOUT);
      store_row16<RWRT_ROW_NT>(o + 0, r0);
      store_row16<RWRT_ROW_NT>(o + 1, r1);
      store_row16<RWRT_ROW_NT>(o + 2, r2);
      store_row16<RWRT_ROW_NT>(o + 3, r3);
    }
    if (RARE(last > it + 1) && writer && rows) {
      asm volatile("");   // frozen: the remaining rows of the chunk (rare branch)
      for (int k = it + 1; k < last; ++k) {
        double2* o = reinterpret_cast<double2*>(rows + (size_t)(k - a.it_begin) * RWRT_NOUT);
        o[0] = r0;
        o[1] = r1;
        o[2] = r2;
        o[3] = r3;
      }
    }
    if (nanrow == a.nt && isnan(y[0])) nanrow = it;  // wr.py:853-855 (host reduces)
    prev_lon = y[0];
    prev_lat = y[1];
    cos_prev = cos_c;
    it = last;
    if (st == Lane<RayProblem, KStore>::kFrozen) L.t = a.tbound[a.it_end - 1];
    if (it == a.it_end && writer) {
#pragma unroll
      for (int v = 0; v < 5; ++v) {
        a.state[v * a.nray + ray] = y[v];
        a.state[(5 + v) * a.nray + ray] = L.f[v];
      }
      a.state[10 * a.nray + ray] = L.t;
      a.state[11 * a.nray + ray] = L.habs;
      if (kTrace && wpos < a.trace_cap)
        trace_ray(a.trace, wpos, ray, nacc + nrej - a.count[2 * ray] - a.count[2 * ray + 1], false);
      a.count[2 * ray] = nacc;
      a.count[2 * ray + 1] = nrej;
      a.nanrow[ray] = nanrow;
      ray = -1;
    }
    if ((kReplica || kPair) && it == a.it_end) ray = -1;   // (the other lanes of a latency wave or pair)
    MARK("x_row_end_done");
  }
  if constexpr (kHandoff) {
    // Drain-time hand-off.  The queue order is a prediction (the previous
    // launch's work): the rays that end a launch run nearly alone, one lane
    // of a wave each, for tens of ms (non-zonal C3: 3-14 rays for ~60 ms,
    // DESIGN.md §6).  Once the queue is drained, a wave with at most
    // a.handoff rays left moves them -- between two attempts, every register
    // of a ray's state by ds_bpermute -- to the quad layout of the latency
    // mode (quad_run: four lanes per ray, the divisions, stage sums and error
    // quotients dealt out over the quad; 1.26-1.37x per attempt, DESIGN.md
    // §4) and continues each from exactly where its lane stopped: the same
    // operations on the same values, so the rows and counters are the run
    // kernel's bit for bit.  The lanes that left the loop with no ray join in.
    const uint64_t hm = __builtin_amdgcn_ballot_w64(handoff);
    if (RARE(hm != 0)) {
      const int q = (int)((threadIdx.x & 63u) >> 2);
      const int nq = __builtin_popcountll(hm);
      uint64_t m = hm;
      for (int i = 0; i < q && m; ++i) m &= m - 1;   // the q-th ray's lane
      const int src = m ? __builtin_ctzll(m) : 0;
      auto sh = [&](double v) { return __shfl(v, src); };
      auto shl = [&](int64_t v) { return (int64_t)__shfl((long long)v, src); };
      auto shi = [&](int32_t v) { return (int32_t)__shfl((int)v, src); };
      double y[5], f[5], aux[3];
#pragma unroll
      for (int v = 0; v < 5; ++v) {
        y[v] = sh(L.y[v]);
        f[v] = sh(L.f[v]);
      }
#pragma unroll
      for (int v = 0; v < 3; ++v) aux[v] = sh(L.aux[v]);
      const int64_t qray = shl(ray), qnacc = shl(nacc), qnrej = shl(nrej);
      double* const qrows = reinterpret_cast<double*>(shl(reinterpret_cast<int64_t>(rows)));
      const double qt = sh(L.t), qhabs = sh(L.habs), qhs = sh(L.hs);
      const double qplon = sh(prev_lon), qplat = sh(prev_lat), qcos = sh(cos_prev);
      const int32_t qnanrow = shi(nanrow), qit = shi(it);
      const int32_t qflags = shi((L.in_step ? 1 : 0) | (L.rejected ? 2 : 0));
      if ((threadIdx.x & 63u) == 0) atomicAdd(&a.queue[0], nq);   // (rays handed off: d_work[0])
      if (q < nq) {   // (whole quads)
        CachedStaticBG QB = lbg;
        QB.key_x = QB.key_y = ~0u;   // the quad refill fills other slots of the slice
        QuadRole R;
        R.role = threadIdx.x & 3;
        R.odd = (R.role & 1) != 0;
        R.high = (R.role & 2) != 0;
        KQuad K{reinterpret_cast<double*>(smem) + threadIdx.x};
        quad_run<false>(a, QB, R, K, qray, qrows, y, f, aux, qt, qhabs, qhs, qnacc, qnrej, 0, qnanrow, qit,
                        qplon, qplat, qcos, (qflags & 1) != 0, (qflags & 2) != 0, 0);
      }
    }
  }
}

template <class BG, bool kTrace = false>
__global__ void __launch_bounds__(256, 1) __attribute__((aligned(RWRT_RUN_ALIGN)))
rk45_run_kernel(RunArgs<BG> a) {
  nm_stage<NM_ALL>();
  // all LDS in one array: the stages (5 x 5 doubles per lane) then the lookup cache
  constexpr int kKBytes = 5 * 5 * 256 * 8;
  __shared__ __attribute__((aligned(16))) char smem[kKBytes + LaneBG<BG>::kLdsBytes];
  if constexpr (std::is_same<BG, StaticBG>::value) {
    const int lb = (int)blockIdx.x;   // (latency block index)
#ifdef RWRT_ANALYZE_QUAD
    if (true) {   // (analysis build of the latency mode: its loop is the common path)
#else
    if (RARE(lb < a.heavy_blocks)) {   // (block-uniform) latency mode
#endif
      __builtin_amdgcn_s_setprio(1);
      quad_rays<kTrace>(a, smem + kKBytes, reinterpret_cast<double*>(smem), lb);
      return;
    }
  }
  if constexpr (!std::is_void<typename TvBlock<BG>::type>::value) {
    // latency mode of the time-varying loops: blocks [0, heavy_blocks) run
    // order[0, n_heavy), one ray per wave replicated on its 64 lanes
    // (BlockVaryingBG), consecutive positions on consecutive waves
    if (RARE((int)blockIdx.x < a.heavy_blocks)) {   // (block-uniform)
      const int64_t w = (int64_t)blockIdx.x * 4 + (int64_t)(threadIdx.x >> 6);
      if (w >= a.n_heavy) return;
      using BBG = typename TvBlock<BG>::type;
      run_rays<BG, BBG, false, true>(a, BBG::make(a.B, smem + kKBytes), smem, w);
      return;
    }
  }
  if constexpr (std::is_same<BG, VaryingBG<double>>::value) {
#ifdef RWRT_ANALYZE_PAIR
    if (true) {   // (analysis build: the lane-pair loop only)
#else
    if (a.B.half) {   // (kernel-uniform) 32 rays per wave: lane pairs
#endif
      run_rays<BG, PairVaryingBG64, false, false, true>(a, PairVaryingBG64::make(a.B, smem + kKBytes), smem, -1);
      return;
    }
  }
  run_rays<BG, typename LaneBG<BG>::type, kTrace, false>(a, LaneBG<BG>::make(a.B, smem + kKBytes), smem, -1);
}

// ---------------------------------------------------------------------------
// Rays frozen at the launch start (NaN mean: dead root slots, rays masked in
// an earlier chunk) never change again (rkf45.py:400-403); rk45_run_kernel's
// lanes would each spend one attempt-sized detour writing their constant
// rows (up to ~1000 x 64 B per ray, 70 % of C3's output bytes, with the other
// lanes of the wave idle).  launch_run instead flags them (frozen_flag_kernel),
// the run kernel skips them, and frozen_fill_kernel -- on a side stream,
// overlapping the run kernel in the registers and LDS it leaves free --
// computes each one's row exactly as the run kernel's frozen path does (the
// same masks and group velocity) and writes the chunk's rows with coalesced
// 16-B stores.
// ---------------------------------------------------------------------------
__global__ void frozen_flag_kernel(const double* __restrict__ state, int64_t nray,
                                   uint8_t* __restrict__ frozen, int32_t* __restrict__ tail_from = nullptr,
                                   int32_t it_begin = 0, int32_t it_end = 0) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nray;
       i += (int64_t)gridDim.x * blockDim.x) {
    double sum = state[i];
#pragma unroll
    for (int v = 1; v < 5; ++v) sum = sum + state[v * nray + i];
    const bool frz = isnan(sum / 5.0);   // Lane::iterate's NaN-mean test
    frozen[i] = frz ? 1 : 0;
    // tails: a frozen ray's tail starts at the launch (its row: frozen_tail_kernel);
    // the others have none (a ray that freezes inside the launch writes its
    // remaining rows as before: rare, and the ray loops stay as they are)
    if (tail_from) tail_from[i] = frz ? it_begin : it_end;
  }
}

// At most 128 VGPRs: a fill wave must fit beside the run kernel's wave in a
// SIMD's register file (256 VGPRs + its AGPRs of 512), and its LDS (the 3.5
// KB sin/cos table, one wave per block) beside the run kernel's 155 KB, or
// the fill would wait for the run to end.
constexpr int kFillThreads = 64;
// Every row of a launch for each frozen ray of a fill tile (one wave, ray
// base + lane): one ray's rows at a time, 16 B per thread, contiguous (a
// ray's rows are); thread t stores quarter t & 3 of the 64-B row, read from
// the ray's lane by cross-lane reads -- no LDS, so that a fill wave fits
// beside rk45_run_kernel's 155 KB block on every CU.
__device__ __forceinline__ void write_frozen_tile(double* out, int64_t base, int64_t nrows, bool mine,
                                                  double2 r0, double2 r1, double2 r2, double2 r3) {
  unsigned long long lanes = __ballot(mine);
  const int64_t nq = nrows * 4;
  const int qt = threadIdx.x & 3;
  while (lanes) {
    const int j = __builtin_ctzll(lanes);
    lanes &= lanes - 1;
    double2* o = reinterpret_cast<double2*>(out + (size_t)(base + j) * nrows * RWRT_NOUT);
    // (every lane reads lane j's quarters 0..3 in turn and keeps its own)
    const double2 q0 = make_double2(__shfl(r0.x, j), __shfl(r0.y, j));
    const double2 q1 = make_double2(__shfl(r1.x, j), __shfl(r1.y, j));
    const double2 q2 = make_double2(__shfl(r2.x, j), __shfl(r2.y, j));
    const double2 q3 = make_double2(__shfl(r3.x, j), __shfl(r3.y, j));
    const double2 v = qt == 0 ? q0 : qt == 1 ? q1 : qt == 2 ? q2 : q3;
    for (int64_t q = threadIdx.x; q < nq; q += kFillThreads) store_row16<1>(o + q, v);
    // pace the stores (~0.9 us per full 64 rows written; none for shorter
    // chunks): a full-rate fill floods the memory queues the run kernel's
    // lookups wait in
    for (int64_t z = 64; z <= nrows; z += 64) __builtin_amdgcn_s_sleep(32);
  }
}

// The row of a ray frozen at the launch start: rk45_run_kernel's fetch +
// kFrozen iteration + post-processing, verbatim (and its state update)
template <class BG>
__device__ __forceinline__ void frozen_row(const RunArgs<BG>& a, int64_t ray, double2& r0, double2& r1,
                                           double2& r2, double2& r3) {
  {
    double y[5];
#pragma unroll
    for (int v = 0; v < 5; ++v) y[v] = a.state[v * a.nray + ray];
    const int64_t nacc = a.count[2 * ray];
    int32_t nanrow = a.nanrow[ray];
    const int32_t it = a.it_begin;
    const double prev_lon = y[0], prev_lat = y[1];
    const double cos_prev = k_cos(prev_lat);
    const double tb = a.tbound[it];
    double ug, vg, cos_c = kNaN;
    bool masked = fabs(y[1]) >= kHalfPi;
    if (!masked) {
      cos_c = cos_small(y[1]);
      masked = cal_dis_reaches(y[0], y[1], prev_lon, prev_lat, cos_c, cos_prev, a.cut_off, a.cut_a);
    }
    if (masked) {
#pragma unroll
      for (int v = 0; v < 5; ++v) y[v] = kNaN;
      ug = vg = kNaN;
    } else {
      ugvg_at(a.B, tb, y[0], y[1], y[2], y[3], ug, vg);
    }
    r0 = make_double2(y[0], y[1]);
    r1 = make_double2(y[2], y[3]);
    r2 = make_double2(y[4], ug);
    r3 = make_double2(vg, (double)nacc);
    if (nanrow == a.nt && isnan(y[0])) nanrow = it;   // wr.py:853-855
#pragma unroll
    for (int v = 0; v < 5; ++v) a.state[v * a.nray + ray] = y[v];
    a.state[10 * a.nray + ray] = a.tbound[a.it_end - 1];
    a.nanrow[ray] = nanrow;
  }
}

template <class BG>
__global__ void __launch_bounds__(kFillThreads) __attribute__((amdgpu_num_vgpr(128)))
frozen_fill_kernel(RunArgs<BG> a) {
  nm_stage<NM_SINCOS>();
  const int64_t nrows = a.it_end - a.it_begin;
  const int64_t base = blockIdx.x * (int64_t)kFillThreads;
  const int64_t ray = base + threadIdx.x;
  const bool mine = ray < a.nray && a.frozen[ray];
  double2 r0 = make_double2(0.0, 0.0), r1 = r0, r2 = r0, r3 = r0;
  if (mine) frozen_row(a, ray, r0, r1, r2, r3);
  write_frozen_tile(a.out, base, nrows, mine, r0, r1, r2, r3);
}

// With tails (rwrt_rk45_run_tails) a frozen ray's rows are ONE row: this
// kernel stores each flagged ray's row as its constant tail from it_begin,
// on the side stream beside the run kernel like frozen_fill_kernel (the
// same register and LDS caps) -- 64 B per frozen ray instead of 64 B per
// frozen ray and row (C3: 116 GB of constant rows per 90-day step, which
// frozen_fill_kernel wrote beside the ray loop, competing for its memory
// queues).  rwrt_expand_tails materialises the rows for consumers that want
// them dense.
template <class BG>
__global__ void __launch_bounds__(kFillThreads) __attribute__((amdgpu_num_vgpr(128)))
frozen_tail_kernel(RunArgs<BG> a, double* __restrict__ tail_row) {
  nm_stage<NM_SINCOS>();
  const int64_t ray = blockIdx.x * (int64_t)kFillThreads + threadIdx.x;
  if (ray < a.nray && a.frozen[ray]) {
    double2 r0, r1, r2, r3;
    frozen_row(a, ray, r0, r1, r2, r3);
    store_tail(tail_row, ray, r0, r1, r2, r3);   // (tail_from: frozen_flag_kernel)
  }
}



__global__ void math_kernel(int kind, int64_t n, const double* __restrict__ x,
                            const double* __restrict__ y, double* __restrict__ out) {
  nm_stage<NM_ALL>();
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = x[i], b = y ? y[i] : 0.0;
  double r;
  switch (kind) {
    case 0: r = sin(a); break;
    case 1: r = cos(a); break;
    case 2: r = tan(a); break;
    case 3: r = pow(a, b); break;
    case 4: r = atan2(a, b); break;
    case 5: r = py_mod(a, b); break;
    case 6: r = sqrt(a); break;
    case 7: r = a / b; break;
    case 8: r = floor(a); break;
    case 9: { double sn, cs; sincos(a, &sn, &cs); r = sn; } break;
    case 10: { double sn, cs; sincos(a, &sn, &cs); r = cs; } break;
    case 11: r = div_rearth(a); break;
    case 12: r = fmod_pos(a, b); break;
    case 13: r = py_mod_2pi(a); break;
    case 14: r = py_mod_2pi_again(py_mod_2pi(a)); break;
    case 15: r = div_hw(a, b, recip_hw(b)); break;
    case 16: r = (double)floor_i32(a); break;
    case 23: { double q1, q2; div2(a, b, b, a, q1, q2); r = q1; } break;
    case 24: { double q1, q2; div2(b, a, a, b, q1, q2); r = q2; } break;
    case 25: r = np_math::nm_sin(a); break;
    case 26: r = np_math::nm_cos(a); break;
    case 27: r = np_math::nm_tan(a); break;
    case 28: r = np_math::nm_pow(a, b); break;
    case 29: r = np_math::nm_rcp14(a); break;
    case 30: { double sn, cs, tn; k_sincostan(a, sn, cs, tn); r = sn; } break;
    case 31: { double sn, cs, tn; k_sincostan(a, sn, cs, tn); r = cs; } break;
    case 32: { double sn, cs, tn; k_sincostan(a, sn, cs, tn); r = tn; } break;
    case 33: r = k_pow(a, b); break;
    case 34: r = qdiv(a, b, rcp2(b)); break;   // exact when kind 35 says so
    case 35: {   // 1 if qdiv(a, b, rcp2(b)) is in DivGuard's exact range, else 0
      DivGuard G;
      G.num(a);
      G.den(b);
      r = G.ok() ? 1.0 : 0.0;
    } break;
    default: r = kNaN; break;   // (unreachable: rwrt_selftest_math rejects other kinds)
  }
  out[i] = r;
}

// ---------------------------------------------------------------------------
// Fixed-step RK4: WR.core_ray_run_numpy (wr.py:702-765) + rk4_step_numpy
// (wr.py:583-622) + core_rk4_step (wr.py:89-95), the reference's default
// integrator (inte_method='').  Same RHS, same post-processing.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool rhs_bad(const double* y) {
  return fabs(y[1]) >= kHalfPi || fabs(y[3]) >= 100.0;   // diffun_numpy err_mask (wr.py:508-510)
}

struct Rk4Args {
  Field F;
  const char* img;    // cache image of F (the lookups' refills)
  int64_t nray;
  double dt, cut_off;
  int32_t nt, it_begin, it_end;
  const int64_t* order;
  double* state;      // rows 0..4 of the [12][nray] state: y
  int64_t* count;     // [nray][2]: steps taken, steps held (a masked stage)
  int32_t* nanrow;
  double* out;
  int32_t* queue;
  const uint8_t* frozen;   // rays whose rows rk4_fill_kernel writes (NULL: none)
};

__global__ void __launch_bounds__(256, 1) rk4_run_kernel(Rk4Args a) {
  nm_stage<NM_SINCOS | NM_TAN>();
  const int64_t nrows = a.it_end - a.it_begin;
  __shared__ __attribute__((aligned(16))) char smem[LaneBG<StaticBG>::kLdsBytes];
  const auto RB = LaneBG<StaticBG>::make(StaticBG{a.F, a.img}, smem);
  const double half = 0.5 * a.dt;        // 0.5 * dt      (wr.py:602-604)
  const double sixth = a.dt / 6.0;       // dt / 6.0      (wr.py:92)
  for (;;) {
    const int32_t w = atomicAdd(a.queue, 1);
    if (w >= a.nray) break;
    const int64_t ray = a.order ? a.order[w] : (int64_t)w;
    if (a.frozen && a.frozen[ray]) continue;   // its rows come from rk4_fill_kernel
    double y[5];
#pragma unroll
    for (int v = 0; v < 5; ++v) y[v] = a.state[v * a.nray + ray];
    int64_t nstep = a.count[2 * ray], nhold = a.count[2 * ray + 1];
    int32_t nanrow = a.nanrow[ray];
    double prev_lon = y[0], prev_lat = y[1];
    int it = a.it_begin;
    while (it < a.it_end) {
      // one RK4 step: k1 at y; k2, k3 at y + dt/2 k; k4 at y + dt k3 (one RHS copy)
      const bool bad1 = rhs_bad(y);
      // a state with a NaN in lon/lat/k/l is stepped (to all-NaN) but not
      // counted: the count is then the same however the run is chunked
      const bool nan_in = isnan(y[0]) || isnan(y[1]) || isnan(y[2]) || isnan(y[3]);
      bool held = bad1;
      double acc[5], k[5], ys[5];
#pragma nounroll
      for (int s = 0; s < 4; ++s) {
        const double c = (s == 3) ? a.dt : half;
#pragma unroll
        for (int v = 0; v < 5; ++v) ys[v] = (s == 0) ? y[v] : y[v] + c * k[v];
        if (s > 0 && rhs_bad(ys)) held = true;
        ray_rhs(RB, 0.0, ys, k);
        const double wgt = (s == 1 || s == 2) ? 2.0 : 1.0;
#pragma unroll
        for (int v = 0; v < 5; ++v) acc[v] = (s == 0) ? k[v] : acc[v] + wgt * k[v];
        if (bad1) break;   // wr.py:600: no later stage matters for this ray
      }
      if (!held) {
#pragma unroll
        for (int v = 0; v < 5; ++v) y[v] = y[v] + sixth * acc[v];
        nstep += nan_in ? 0 : 1;
      } else if (!nan_in) {
        // held by a masked stage; a masked FIRST stage holds the ray for every
        // remaining step (its rows repeat to the chunk's end, below), each counted
        nhold += bad1 ? (a.it_end - it) : 1;
      }
      // post-processing (wr.py:718-756)
      if (fabs(y[1]) >= kHalfPi) {
#pragma unroll
        for (int v = 0; v < 5; ++v) y[v] = kNaN;
      }
      if (cal_dis(y[0], y[1], prev_lon, prev_lat) >= a.cut_off) {
#pragma unroll
        for (int v = 0; v < 5; ++v) y[v] = kNaN;
      }
      double ug, vg;
      ugvg_at(StaticBG{a.F}, 0.0, y[0], y[1], y[2], y[3], ug, vg);
      const double2 r0 = make_double2(y[0], y[1]), r1 = make_double2(y[2], y[3]);
      const double2 r2 = make_double2(y[4], ug), r3 = make_double2(vg, (double)nstep);
      // A held ray (masked first stage) or an all-NaN state repeats this row
      // forever: write every remaining row of the chunk at once.
      const bool allnan = isnan(y[0]) && isnan(y[1]) && isnan(y[2]) && isnan(y[3]) && isnan(y[4]);
      const int last = (bad1 || allnan) ? a.it_end : it + 1;
      for (int q = it; q < last; ++q) {
        double2* o = reinterpret_cast<double2*>(a.out + ((size_t)ray * nrows + (q - a.it_begin)) * RWRT_NOUT);
        o[0] = r0;
        o[1] = r1;
        o[2] = r2;
        o[3] = r3;
      }
      if (nanrow == a.nt && isnan(y[0])) nanrow = it;
      prev_lon = y[0];
      prev_lat = y[1];
      it = last;
    }
#pragma unroll
    for (int v = 0; v < 5; ++v) a.state[v * a.nray + ray] = y[v];
    a.count[2 * ray] = nstep;
    a.count[2 * ray + 1] = nhold;
    a.nanrow[ray] = nanrow;
  }
}

// RK4 rays with a NaN in lon, lat, k or l at the launch start: their first
// step either holds them (a masked first stage, wr.py:600) or makes the whole
// state NaN (every derivative of such a state is NaN), and rk4_run_kernel
// then repeats that row to the end of the chunk -- so these rays' rows are
// known before the launch.  rk4_flag_kernel marks them, rk4_run_kernel skips
// them and rk4_fill_kernel (side stream, beside the run kernel) applies that
// step and the post-processing of wr.py:718-756 as the run kernel does and
// writes the rows like frozen_fill_kernel.
__global__ void rk4_flag_kernel(const double* __restrict__ state, int64_t nray,
                                uint8_t* __restrict__ frozen) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nray;
       i += (int64_t)gridDim.x * blockDim.x) {
    bool nan = false;
#pragma unroll
    for (int v = 0; v < 4; ++v) nan = nan || isnan(state[v * nray + i]);
    frozen[i] = nan ? 1 : 0;
  }
}

__global__ void __launch_bounds__(kFillThreads) __attribute__((amdgpu_num_vgpr(128)))
rk4_fill_kernel(Rk4Args a) {
  nm_stage<NM_SINCOS>();
  const int64_t nrows = a.it_end - a.it_begin;
  const int64_t base = blockIdx.x * (int64_t)kFillThreads;
  const int64_t ray = base + threadIdx.x;
  const bool mine = ray < a.nray && a.frozen[ray];
  double2 r0 = make_double2(0.0, 0.0), r1 = r0, r2 = r0, r3 = r0;
  if (mine) {
    double y[5];
#pragma unroll
    for (int v = 0; v < 5; ++v) y[v] = a.state[v * a.nray + ray];
    int64_t nstep = a.count[2 * ray];
    int32_t nanrow = a.nanrow[ray];
    const double prev_lon = y[0], prev_lat = y[1];
    const int it = a.it_begin;
    // rk4_run_kernel's step: held iff the first stage is masked; otherwise
    // every stage derivative is NaN and so is y + dt/6 * acc (not counted)
    if (!rhs_bad(y)) {
#pragma unroll
      for (int v = 0; v < 5; ++v) y[v] = kNaN;
    }
    if (fabs(y[1]) >= kHalfPi) {
#pragma unroll
      for (int v = 0; v < 5; ++v) y[v] = kNaN;
    }
    if (cal_dis(y[0], y[1], prev_lon, prev_lat) >= a.cut_off) {
#pragma unroll
      for (int v = 0; v < 5; ++v) y[v] = kNaN;
    }
    double ug, vg;
    ugvg_at(StaticBG{a.F}, 0.0, y[0], y[1], y[2], y[3], ug, vg);
    r0 = make_double2(y[0], y[1]);
    r1 = make_double2(y[2], y[3]);
    r2 = make_double2(y[4], ug);
    r3 = make_double2(vg, (double)nstep);
    if (nanrow == a.nt && isnan(y[0])) nanrow = it;
#pragma unroll
    for (int v = 0; v < 5; ++v) a.state[v * a.nray + ray] = y[v];
    a.count[2 * ray] = nstep;
    a.nanrow[ray] = nanrow;
  }
  write_frozen_tile(a.out, base, nrows, mine, r0, r1, r2, r3);
}

// rk45_simple_current (rkf45.py:672-724) over ncol columns, one lane each.
template <class P>
__global__ void kat_kernel(int64_t ncol, const double* __restrict__ y0, int32_t nt,
                           const double* __restrict__ teval, double rtol, double atol,
                           double min_step, double* __restrict__ out) {
  nm_stage<NM_ALL>();
  constexpr int NV = P::NV;
  const P fun{};
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= ncol) return;
  Lane<P, KRegs<P::NV>> L;
#pragma unroll
  for (int v = 0; v < NV; ++v) L.y[v] = y0[v * ncol + i];
  L.t = teval[0];
  fun(L.t, L.y, L.f);
  L.habs = initial_step(fun, L.t, L.y, L.f, rtol, atol);
  L.in_step = false;
  L.rejected = false;
  int64_t nacc = 0, nrej = 0;
  for (int v = 0; v < NV; ++v) out[(i * nt) * NV + v] = L.y[v];
  for (int it = 1; it < nt; ++it) {
    while (L.iterate(fun, teval[it], min_step, rtol, atol, nacc, nrej) == Lane<P, KRegs<P::NV>>::kStep) {
    }
    for (int v = 0; v < NV; ++v) out[(i * nt + it) * NV + v] = L.y[v];
  }
}

// ---------------------------------------------------------------------------
// Initial rays: WR.ray_initial_numpy (wr.py:344-395)
// ---------------------------------------------------------------------------
// change_roots_order (bs.py:942-982) on the nreal compacted real roots, then
// the |m| > 100 filter and the reversal of cal_ky (bs.py:1037-1040).
__device__ __forceinline__ void order_roots(double m[3], int nreal) {
  auto swap = [&](int a, int b) { const double t = m[a]; m[a] = m[b]; m[b] = t; };
  if (nreal == 3) {
    if (m[2] >= 0.0 && m[2] < m[1]) swap(1, 2);
    if (m[0] < 0.0) swap(0, 1);
    if ((m[1] < 0.0 && m[2] < 0.0 && m[1] < m[2]) || (m[1] > 0.0 && m[2] < 0.0)) swap(1, 2);
  } else if (nreal == 2) {
    if (!(m[0] > 0.0)) swap(0, 1);
  } else if (nreal == 1) {
    if (m[0] < 0.0) swap(0, 1);
  }
#pragma unroll
  for (int q = 0; q < 3; ++q)
    if (!isnan(m[q]) && fabs(m[q]) > 100.0) m[q] = kNaN;
  swap(0, 2);
}

// One thread per (source, zonal wavenumber).  zc = {k, k**2, k**3, freq/k*R}
// for every k (NumPy-evaluated on the host); rows[7][3][nsource][nzwn].
__global__ void ray_initial_kernel(Field F, int64_t nsource, const double* __restrict__ slon,
                                   const double* __restrict__ slat,
                                   const double* __restrict__ scos, int32_t nzwn,
                                   const double* __restrict__ zc, double* __restrict__ rows,
                                   int32_t* __restrict__ info) {
  const int64_t n = nsource * nzwn;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = i / nzwn;
    const int iz = (int)(i - s * nzwn);
    const double lon = slon[s], lat = slat[s];
    // BS.cal_bs_mercator_point at the source: fmu fmv fmqx fmqy (bs.py:856-883)
    double fu, fv, fqx, fqy;
    interp4(F, py_mod_2pi(lon), lat, fu, fv, fqx, fqy);
    const Merc M = merc_factors(lat, scos[s], 0.0);
    const double fmu = (fu / M.cp) * M.m;
    const double fmv = (fv / M.cp) * M.m;
    const double fmqx = fqx * M.m;
    const double fmqy = (fqy * M.cp) * M.m;
    const double k = zc[iz], k2 = zc[nzwn + iz], k3 = zc[2 * nzwn + iz], ps = zc[3 * nzwn + iz];
    double mr[3] = {kNaN, kNaN, kNaN};
    if (k != 0.0) {
      // cal_ky_numpy coefficients, lowest order first (bs.py:1005-1012)
      const double c[4] = {k3 * ((fmu - ps) - (fmqy / k2)), k2 * fmv + fmqx, k * (fmu - ps), fmv};
      int deg = 3;
      while (deg > 0 && fabs(c[deg]) == 0.0) --deg;    // exact-zero reduction
      if (deg >= 1) {
        double p[4];
        for (int q = 0; q <= deg; ++q) p[q] = c[deg - q];   // highest first
        nproots::cx r[3] = {{kNaN, kNaN}, {kNaN, kNaN}, {kNaN, kNaN}};
        bool finite = true;
        for (int q = 0; q <= deg; ++q) finite = finite && isfinite(p[q]);
        int st = finite ? nproots::np_roots(p, deg, r) : -1;
        if (st != 0) atomicAdd(info, 1);   // np.linalg.eigvals would raise
        // real roots (|Im| < delt), compacted in np.roots' order (bs.py:1030-1036)
        int nreal = 0;
        for (int q = 0; q < deg; ++q)
          if (st == 0 && fabs(r[q].im) < 1e-8) mr[nreal++] = r[q].re;
        order_roots(mr, nreal);
      }
    }
    // outputs: rows[v][slot][s][iz]
    const int64_t plane = 3 * n;
    for (int slot = 0; slot < 3; ++slot) {
      const double m = mr[slot];
      const int64_t o = (int64_t)slot * n + i;
      double ug, vg;
      if (k == 0.0) {
        ug = 0.0;
        vg = 0.0;
      } else {
        // cal_ugvg_numpy (wn.py:209-259)
        double nans = ((m * 0.0) * (((fmu * fmqx) * fmqy) * 0.0)) + 1.0;
        if (isnan(nans)) nans = 0.0;
        const double a = (k * k) - (m * m);
        const double b = (2.0 * k) * m;
        const double cc = (k * k) + (m * m);
        const double c2 = cc * cc;
        ug = (fmu + (((a * fmqy) - (b * fmqx)) / c2)) * nans;
        vg = (fmv + (((a * fmqx) + (b * fmqy)) / c2)) * nans;
      }
      rows[0 * plane + o] = lon;
      rows[1 * plane + o] = lat;
      rows[2 * plane + o] = k;
      rows[3 * plane + o] = m;
      rows[4 * plane + o] = isnan(m) ? kNaN : 1.0;
      rows[5 * plane + o] = ug;
      rows[6 * plane + o] = vg;
    }
  }
}

// ---------------------------------------------------------------------------
// Host side of the ABI
// ---------------------------------------------------------------------------
thread_local std::string g_err;

rwrt_status fail(rwrt_status s, const char* fmt, const char* detail = "") {
  char buf[512];
  snprintf(buf, sizeof buf, fmt, detail);
  g_err = buf;
  return s;
}

rwrt_status check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return RWRT_ERR_HIP;
  }
  return RWRT_OK;
}

rwrt_status make_field(const rwrt_grid* g, const double* packed, Field& F) {
  if (!g) return fail(RWRT_ERR_ARG, "grid is NULL%s");
  if (!packed) return fail(RWRT_ERR_ARG, "packed fields pointer is NULL%s");
  if (g->ncol < 2 || g->nrow < 2) return fail(RWRT_ERR_ARG, "grid must be at least 2x2%s");
  if (!(g->dlon != 0.0) || !(g->dlat != 0.0)) return fail(RWRT_ERR_ARG, "grid spacing is zero%s");
  if (reinterpret_cast<uintptr_t>(packed) % 16 != 0)
    return fail(RWRT_ERR_ARG, "packed fields must be 16-byte aligned%s");
  // the lookups address one level with 32-bit element offsets
  if (g->ncol > 65535 || g->nrow > 65535) return fail(RWRT_ERR_ARG, "grid dimension > 65535%s");
  if ((int64_t)g->ncol * g->nrow >= (1LL << 24))
    return fail(RWRT_ERR_ARG, "grid too large for one packed level (>= 2^24 records)%s");
  F.P = packed;
  F.W = g->ncol;
  F.H = g->nrow;
  F.lon0 = g->lon0;
  F.dlon = g->dlon;
  F.lat0 = g->lat0;
  F.dlat = g->dlat;
  return RWRT_OK;
}

unsigned grid_for(int64_t n, int block) {
  int64_t b = (n + block - 1) / block;
  if (b < 1) b = 1;
  if (b > 65535LL * 32) b = 65535LL * 32;
  return (unsigned)b;
}

// Occupancy-derived persistent grid of rk45_run_kernel<BG> on the current device.
template <class BG = StaticBG>
int persistent_blocks_on(int ncu) {
  int per = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per, reinterpret_cast<const void*>(rk45_run_kernel<BG>), 256, 0) != hipSuccess || per < 1)
    per = 1;
  return ncu * per;
}

// solver construction / ray loop launchers shared by the static and the
// time-varying entry points
template <class BG>
rwrt_status launch_init(const BG& B, int64_t nray, const double* d_y0, const rwrt_params* p,
                        double* d_state, int64_t* d_count, int32_t* d_nanrow, int32_t* d_live,
                        int64_t* d_summary, void* stream) {
  if (!p) return fail(RWRT_ERR_ARG, "params is NULL%s");
  if (nray < 0 || nray > 0x7fffffffLL) return fail(RWRT_ERR_ARG, "nray out of range%s");
  // per-ray buffers of an empty batch may be NULL (empty tensors)
  if (!d_summary || (nray > 0 && (!d_y0 || !d_state || !d_count || !d_nanrow || !d_live)))
    return fail(RWRT_ERR_ARG, "NULL buffer to rwrt_rk45_init%s");
  if (hipMemsetAsync(d_summary, 0, 2 * sizeof(int64_t), (hipStream_t)stream) != hipSuccess)
    return check_launch("hipMemsetAsync(summary)");
  if (nray == 0) return RWRT_OK;
  InitArgs<BG> a{B, nray, d_y0, p->rtol, p->atol, p->nt, d_state, d_count, d_nanrow, d_live, d_summary};
  hipLaunchKernelGGL(rk45_init_kernel<BG>, dim3(grid_for(nray, 256)), dim3(256), 0,
                     (hipStream_t)stream, a);
  return check_launch("rk45_init_kernel");
}

}  // namespace rwrt

// An execution context (include/rwrt.h rwrt_ctx): everything the ray-loop
// entry points need beyond the caller's buffers -- the frozen-ray flags (one
// byte per ray, grown on demand), the side stream the fill kernels run on and
// its events, and the device's launch geometry.  Distinct contexts share
// nothing, so calls through them are reentrant and may run concurrently on
// different streams; one context used from several threads is serialised by
// its mutex (host bookkeeping only -- the GPU work stays asynchronous), and a
// call on another stream than the context's previous call waits on the device
// for that call's end before it rewrites the flags.
struct rwrt_ctx {
  int device = 0;
  int ncu = 256;
  int blocks_static = 0, blocks_f32 = 0, blocks_f64 = 0, blocks_a32 = 0;   // persistent grids
  uint8_t* flags = nullptr;
  size_t cap = 0;
  char* img = nullptr;         // cache image of the static state (cache_image_kernel), rebuilt per call
  size_t img_cap = 0;
  hipStream_t side = nullptr;
  hipEvent_t flagged = nullptr, filled = nullptr;
  hipEvent_t done = nullptr;   // end of the last call on this context
  int quad_per_wave = 16;      // latency mode: rays per wave (rwrt_ctx_set_latency_density)
  int tv_lanes = 64;           // rays per wave of fp64 time-varying calls (rwrt_ctx_set_tv_lanes)
  int handoff = 16;            // drain-time hand-off threshold (rwrt_ctx_set_handoff)
  int64_t* trace = nullptr;    // rwrt_ctx_set_trace (diagnostic)
  int64_t trace_cap = 0;
  bool used = false;
  std::mutex mu;
};

namespace rwrt {

// Makes ctx->device current for the duration of a call (restored after).
struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// Flags for nray rays.  A buffer that earlier calls of this context may still
// read is freed only after the last of them (its `done` event) has finished.
rwrt_status ctx_flags(rwrt_ctx* c, int64_t nray) {
  if ((size_t)nray <= c->cap) return RWRT_OK;
  if (c->flags) {
    if ((c->used && hipEventSynchronize(c->done) != hipSuccess) || hipFree(c->flags) != hipSuccess)
      return check_launch("releasing the context's frozen-ray flags");
    c->flags = nullptr;
    c->cap = 0;
  }
  const size_t cap = ((size_t)nray + 4095) & ~(size_t)4095;
  if (hipMalloc(reinterpret_cast<void**>(&c->flags), cap) != hipSuccess)
    return fail(RWRT_ERR_HIP, "frozen-ray flag allocation failed%s");
  c->cap = cap;
  return RWRT_OK;
}

// The cache image of F for this call, built on `stream` (after ctx_begin:
// the previous call of the context, which may still read the old image, is
// finished on the device by then).  Rebuilt every call, so a caller may change
// the packed state between calls; ~1 MB at 2.5 degrees.
rwrt_status ctx_image(rwrt_ctx* c, const Field& F, hipStream_t stream, const char** out) {
  const size_t need = cache_image_bytes((int64_t)F.W * F.H);
  if (need > c->img_cap) {
    if (c->img) {
      if ((c->used && hipEventSynchronize(c->done) != hipSuccess) || hipFree(c->img) != hipSuccess)
        return check_launch("releasing the context's cache image");
      c->img = nullptr;
      c->img_cap = 0;
    }
    if (hipMalloc(reinterpret_cast<void**>(&c->img), need) != hipSuccess)
      return fail(RWRT_ERR_HIP, "cache image allocation failed%s");
    c->img_cap = need;
  }
  hipLaunchKernelGGL(cache_image_kernel, dim3(grid_for((int64_t)F.W * F.H * 6, 256)), dim3(256), 0, stream,
                     F, c->img);
  *out = c->img;
  return check_launch("cache_image_kernel");
}

template <class BG> int& ctx_blocks(rwrt_ctx* c);
template <> int& ctx_blocks<StaticBG>(rwrt_ctx* c) { return c->blocks_static; }
template <> int& ctx_blocks<VaryingBG<float>>(rwrt_ctx* c) { return c->blocks_f32; }
template <> int& ctx_blocks<VaryingBG<double>>(rwrt_ctx* c) { return c->blocks_f64; }
template <> int& ctx_blocks<VaryingBGA32>(rwrt_ctx* c) { return c->blocks_a32; }

template <class BG>
int ctx_persistent_blocks(rwrt_ctx* c) {
  int& b = ctx_blocks<BG>(c);
  if (!b) b = persistent_blocks_on<BG>(c->ncu);
  return b;
}

// flag kernel on `stream`, then the side stream waits for it
template <class Flag>
rwrt_status ctx_begin(rwrt_ctx* c, hipStream_t stream, Flag launch_flags) {
  // the flags belong to this context: a call on another stream must not
  // overwrite them while the previous call still reads them
  if (c->used && hipStreamWaitEvent(stream, c->done, 0) != hipSuccess)
    return check_launch("hipStreamWaitEvent(previous call of the context)");
  launch_flags();
  if (rwrt_status s = check_launch("flag kernel")) return s;
  if (hipEventRecord(c->flagged, stream) != hipSuccess || hipStreamWaitEvent(c->side, c->flagged, 0) != hipSuccess)
    return check_launch("hipEventRecord(frozen flags)");
  return RWRT_OK;
}
// `stream` waits for the fill on the side stream; the call ends there
rwrt_status ctx_end(rwrt_ctx* c, hipStream_t stream) {
  if (hipEventRecord(c->filled, c->side) != hipSuccess || hipStreamWaitEvent(stream, c->filled, 0) != hipSuccess ||
      hipEventRecord(c->done, stream) != hipSuccess)
    return check_launch("hipEventRecord(frozen fill)");
  c->used = true;
  return RWRT_OK;
}

rwrt_status ctx_check(rwrt_ctx* c) {
  if (!c) return fail(RWRT_ERR_ARG, "rwrt_ctx is NULL (create one with rwrt_ctx_create)%s");
  return RWRT_OK;
}

template <class BG>
rwrt_status launch_run(rwrt_ctx* ctx, const BG& B, int64_t nray, const rwrt_params* p,
                       const double* d_tbound, int32_t it_begin, int32_t it_end,
                       const int64_t* d_order, int64_t n_heavy, double* d_state, int64_t* d_count,
                       int32_t* d_nanrow, double* d_out, int32_t* d_tail_from, double* d_tail_row,
                       int32_t* d_work, void* stream, const int32_t* d_row_slot = nullptr) {
  if (rwrt_status s = ctx_check(ctx)) return s;
  if (!p) return fail(RWRT_ERR_ARG, "params is NULL%s");
  if (nray < 0 || nray > 0x7fffffffLL) return fail(RWRT_ERR_ARG, "nray out of range%s");
  if (it_begin < 1 || it_end > p->nt || it_begin >= it_end)
    return fail(RWRT_ERR_ARG, "need 1 <= it_begin < it_end <= nt%s");
  if (!d_tbound || !d_work || (nray > 0 && (!d_state || !d_count || !d_nanrow || !d_out)))
    return fail(RWRT_ERR_ARG, "NULL buffer to rwrt_rk45_run%s");
  if (reinterpret_cast<uintptr_t>(d_out) % 16 != 0)
    return fail(RWRT_ERR_ARG, "output rows must be 16-byte aligned%s");
  if (!d_tail_from != !d_tail_row) return fail(RWRT_ERR_ARG, "tails need both d_tail_from and d_tail_row%s");
  if (reinterpret_cast<uintptr_t>(d_tail_row) % 16 != 0)
    return fail(RWRT_ERR_ARG, "tail rows must be 16-byte aligned%s");
  if (d_row_slot && !d_tail_from)
    return fail(RWRT_ERR_ARG, "row slots need tails (the rays without a slot keep theirs there)%s");
  if (nray == 0) return RWRT_OK;
  if (n_heavy < 0 || n_heavy > nray) return fail(RWRT_ERR_ARG, "n_heavy out of range%s");
  if (n_heavy > 0 && !d_order) return fail(RWRT_ERR_ARG, "n_heavy > 0 needs d_order%s");
  // (latency mode: quad_rays on the static background, replicated waves with
  // a block cache on the time-varying ones -- rk45_run_kernel's first
  // heavy_blocks blocks either way; none for the fp32-arithmetic variant)
  if (n_heavy > 0 && std::is_void<typename TvBlock<BG>::type>::value && !std::is_same<BG, StaticBG>::value)
    return fail(RWRT_ERR_ARG, "latency mode (n_heavy > 0) is not built for fp32-arithmetic levels%s");
  // the context's settings are read once, under its lock: a concurrent
  // rwrt_ctx_set_latency_density cannot change the density between sizing the
  // latency-mode grid and launching it
  std::lock_guard<std::mutex> lock(ctx->mu);
  const int32_t quad_per_wave = ctx->quad_per_wave;
  const int32_t handoff = ctx->handoff;
  // rays per latency-mode block: quad_rays 4 x rays-per-wave, the
  // time-varying latency waves one ray per wave
  const int64_t per_block = BG::kTimeVarying ? 4 : 4 * (int64_t)quad_per_wave;
  const int64_t team_blocks = (n_heavy + per_block - 1) / per_block;
  if (team_blocks > ctx->ncu / 2)
    return fail(RWRT_ERR_ARG, "n_heavy exceeds the latency mode's capacity (per CU 4 x rays-per-wave, time-varying 4; half the CUs)%s");
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return check_launch("hipSetDevice(context device)");
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(d_work, 0, 2 * sizeof(int32_t), st) != hipSuccess)
    return check_launch("hipMemsetAsync(queue)");
  int64_t blocks = ctx_persistent_blocks<BG>(ctx);
  // latency-mode blocks take a CU each (their LDS does not fit beside a
  // persistent block): the persistent grid shrinks by as many CUs
  if (team_blocks) blocks = std::max<int64_t>(1, blocks - team_blocks * (blocks / ctx->ncu));
  int64_t block_rays = 256;   // rays a block runs at once
  if constexpr (BG::kTimeVarying) block_rays = B.half ? 128 : 256;
  const int64_t need = (nray - n_heavy + block_rays - 1) / block_rays;
  if (blocks > need) blocks = need;
  RunArgs<BG> a{B, nray, p->rtol, p->atol, p->min_step, p->cut_off, p->nt, it_begin, it_end,
                d_tbound, d_order, d_state, d_count, d_nanrow, d_out, d_work,
                n_heavy, 0, haversine_cut(p->cut_off), nullptr};
  a.row_slot = d_row_slot;
  a.handoff = handoff;
  // frozen rays: flagged on `stream`, filled on the context's side stream
  // while the run kernel (which skips them) integrates the rest; `stream` then
  // waits for the fill, so the call stays one stream-ordered operation.  With
  // tails, the side stream stores their constant tail rows instead of
  // filling (frozen_tail_kernel).
  if (rwrt_status s = ctx_flags(ctx, nray)) return s;
  a.frozen = ctx->flags;
  if (rwrt_status s = ctx_begin(ctx, st, [&] {
        hipLaunchKernelGGL(frozen_flag_kernel, dim3(grid_for(nray, 256)), dim3(256), 0, st, d_state, nray,
                           ctx->flags, d_tail_from, it_begin, it_end);
      }))
    return s;
  if constexpr (std::is_same<BG, StaticBG>::value) {
    if (rwrt_status s = ctx_image(ctx, B.F, st, &a.B.img)) return s;
  }
  // latency mode in the run kernel's first team_blocks blocks (quad_rays):
  // one grid, so they are placed beside the persistent blocks whatever the
  // hardware queues' dispatch order (a second kernel on another stream could
  // wait for a CU on its XCD until the persistent grid drains)
  a.heavy_blocks = (int32_t)team_blocks;
  a.quad_per_wave = quad_per_wave;
  if constexpr (std::is_same<BG, StaticBG>::value) {
    a.trace = ctx->trace;
    a.trace_cap = ctx->trace ? ctx->trace_cap : 0;
  }
  if (nray > n_heavy || team_blocks) {
    const int64_t grid = team_blocks + (nray > n_heavy ? blocks : 0);
    if (a.trace && std::is_same<BG, StaticBG>::value) {
      if constexpr (std::is_same<BG, StaticBG>::value)
        hipLaunchKernelGGL((rk45_run_kernel<BG, true>), dim3((unsigned)grid), dim3(256), 0, st, a);
    } else {
      hipLaunchKernelGGL(rk45_run_kernel<BG>, dim3((unsigned)grid), dim3(256), 0, st, a);
    }
    if (rwrt_status s = check_launch("rk45_run_kernel")) return s;
  }
  if (d_tail_from)
    hipLaunchKernelGGL(frozen_tail_kernel<BG>, dim3((unsigned)((nray + kFillThreads - 1) / kFillThreads)),
                       dim3(kFillThreads), 0, ctx->side, a, d_tail_row);
  else
    hipLaunchKernelGGL(frozen_fill_kernel<BG>, dim3((unsigned)((nray + kFillThreads - 1) / kFillThreads)),
                       dim3(kFillThreads), 0, ctx->side, a);
  if (rwrt_status s = check_launch(d_tail_from ? "frozen_tail_kernel" : "frozen_fill_kernel")) return s;
  return ctx_end(ctx, st);
}

// a time-varying background from the ABI description
template <class T>
rwrt_status make_varying(const rwrt_grid* g, const rwrt_background* b, VaryingBG<T>& B) {
  Field F;
  if (!b) return fail(RWRT_ERR_ARG, "background is NULL%s");
  if (rwrt_status s = make_field(g, reinterpret_cast<const double*>(b->d_levels), F)) return s;
  if (b->nlev < 1) return fail(RWRT_ERR_ARG, "background needs nlev >= 1%s");
  if (!(b->dt > 0.0)) return fail(RWRT_ERR_ARG, "background level spacing dt must be > 0%s");
  B.P = reinterpret_cast<const T*>(b->d_levels);
  B.W = F.W;
  B.H = F.H;
  B.nlev = b->nlev;
  B.lev_stride = (int64_t)F.W * F.H * kNF;
  B.lon0 = F.lon0;
  B.dlon = F.dlon;
  B.lat0 = F.lat0;
  B.dlat = F.dlat;
  B.t0 = b->t0;
  B.dt = b->dt;
  B.half = 0;
  return RWRT_OK;
}

// ---------------------------------------------------------------------------
// BS.ready on the device (bs.py:264-279, 291-305, 318-372 / our bs.py):
// three element passes over the (nlon, nlat) grid, every expression in the
// reference's NumPy evaluation order.
// ---------------------------------------------------------------------------
struct ReadyArgs {
  int nlon, nlat;
  const float* u;      // [nlat][nlon] as read (file layout; BS keeps u.T)
  const float* v;
  const double* trig;  // [3][nlat]: np.cos(lat) (ucos), and at 1..nlat-2 np.cos / np.sin of lat[1:-1]
  double dx2, dy2, dxx, dyy, dxy4, dx, dy;   // 2dx, 2dy, dx**2, dy**2, (4dx)dy, dx, dy
  double* q;           // scratch [nlon][nlat] x 4: q, qxx, qyy, qxy (unsmoothed)
  void* out;           // [nlon+1][nlat][12], double or float
};

__device__ __forceinline__ int wrapi(int i, int n) { return i < 0 ? i + n : (i >= n ? i - n : i); }
__device__ __forceinline__ double U(const ReadyArgs& a, int i, int j) { return (double)a.u[(size_t)j * a.nlon + i]; }
__device__ __forceinline__ double V(const ReadyArgs& a, int i, int j) { return (double)a.v[(size_t)j * a.nlon + i]; }

// pass 1: absolute vorticity q (calc_absolute_vorticity, bs.py:264-279)
__global__ void ready_q_kernel(ReadyArgs a) {
  const int64_t n = (int64_t)a.nlon * a.nlat;
  for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < n;
       id += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(id / a.nlat), j = (int)(id - (int64_t)i * a.nlat);
    const int jj = j < 1 ? 1 : (j > a.nlat - 2 ? a.nlat - 2 : j);   // q[:,0]=q[:,1], q[:,-1]=q[:,-2]
    const double vx = (V(a, wrapi(i + 1, a.nlon), jj) - V(a, wrapi(i - 1, a.nlon), jj)) / a.dx2;
    const double ucp = U(a, i, jj + 1) * a.trig[jj + 1];
    const double ucm = U(a, i, jj - 1) * a.trig[jj - 1];
    const double uy = (ucp - ucm) / a.dy2;
    a.q[(size_t)i * a.nlat + j] = (vx - uy) / a.trig[a.nlat + jj] +
                                  ((2.0 * kOmega) * a.trig[2 * a.nlat + jj]) * kREarth;
  }
}

// pass 2: unsmoothed qxx, qyy, qxy (gradient_xx / _yy / _xy)
__global__ void ready_q2_kernel(ReadyArgs a) {
  const int64_t n = (int64_t)a.nlon * a.nlat;
  const double* q = a.q;
  for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < n;
       id += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(id / a.nlat), j = (int)(id - (int64_t)i * a.nlat);
    const int H = a.nlat;
    const size_t ip = (size_t)wrapi(i + 1, a.nlon) * H, i0 = (size_t)i * H, im = (size_t)wrapi(i - 1, a.nlon) * H;
    const int jj = j < 1 ? 1 : (j > H - 2 ? H - 2 : j);
    const double qxx = ((q[ip + j] - 2.0 * q[i0 + j]) + q[im + j]) / a.dxx;
    const double qyy = ((q[i0 + jj + 1] - 2.0 * q[i0 + jj]) + q[i0 + jj - 1]) / a.dyy;
    const double qxy = (((q[ip + jj + 1] - q[ip + jj - 1]) - q[im + jj + 1]) + q[im + jj - 1]) / a.dxy4;
    a.q[n + id] = qxx;
    a.q[2 * n + id] = qyy;
    a.q[3 * n + id] = qxy;
  }
}

// smth9 (bs.py:291-305): f + convolve(f, w, 'constant') on [1:-2, 1:-2]
__device__ __forceinline__ double smth9_at(const double* f, int nlon, int H, int i, int j) {
  const double f0 = f[(size_t)i * H + j];
  if (i < 1 || i > nlon - 3 || j < 1 || j > H - 3) return f0;
  const double w[3][3] = {{0.0625, 0.125, 0.0625}, {0.125, -0.75, 0.125}, {0.0625, 0.125, 0.0625}};
  double acc = 0.0;
#pragma unroll
  for (int da = 0; da < 3; ++da)
#pragma unroll
    for (int db = 0; db < 3; ++db) acc = acc + f[(size_t)(i + da - 1) * H + (j + db - 1)] * w[da][db];
  return f0 + acc;
}

// gradient_y of column i of a field given by an accessor (bs.py gradient_y)
template <class G>
__device__ __forceinline__ double grad_y(const G& g, int j, int H, double dy2, double dy) {
  if (j == 0) return (g(1) - g(0)) / dy;
  if (j == H - 1) return (g(H - 1) - g(H - 2)) / dy;
  return (g(j + 1) - g(j - 1)) / dy2;
}

// pass 3: the packed record of every grid point (+ the cyclic column)
template <class T>
__global__ void ready_pack_kernel(ReadyArgs a) {
  const int H = a.nlat;
  const int64_t n = (int64_t)(a.nlon + 1) * H, nq = (int64_t)a.nlon * H;
  for (int64_t id = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; id < n;
       id += (int64_t)gridDim.x * blockDim.x) {
    const int ic = (int)(id / H), j = (int)(id - (int64_t)ic * H);
    const int i = ic == a.nlon ? 0 : ic;                     // bs.py:370-372 cyclic copy
    const int ip = wrapi(i + 1, a.nlon), im = wrapi(i - 1, a.nlon);
    const double* q = a.q;
    double r[12];
    r[F_U] = U(a, i, j);
    r[F_V] = V(a, i, j);
    r[F_UX] = (U(a, ip, j) - U(a, im, j)) / a.dx2;
    r[F_UY] = grad_y([&](int jj) { return U(a, i, jj); }, j, H, a.dy2, a.dy);
    r[F_VX] = (V(a, ip, j) - V(a, im, j)) / a.dx2;
    r[F_VY] = grad_y([&](int jj) { return V(a, i, jj); }, j, H, a.dy2, a.dy);
    r[F_QX] = (q[(size_t)ip * H + j] - q[(size_t)im * H + j]) / a.dx2;
    r[F_QY] = grad_y([&](int jj) { return q[(size_t)i * H + jj]; }, j, H, a.dy2, a.dy);
    r[F_QXX] = smth9_at(q + nq, a.nlon, H, i, j);
    r[F_QXY] = smth9_at(q + 3 * nq, a.nlon, H, i, j);
    r[F_QYY] = smth9_at(q + 2 * nq, a.nlon, H, i, j);
    r[F_PAD] = 0.0;
    T* o = reinterpret_cast<T*>(a.out) + id * kNF;
#pragma unroll
    for (int k = 0; k < 12; ++k) o[k] = (T)r[k];
  }
}

template <class BG>
__global__ void rhs_bg_kernel(BG B, int64_t n, const double* __restrict__ t,
                              const double* __restrict__ y, double* __restrict__ dydt) {
  nm_stage<NM_SINCOS | NM_TAN>();
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    double yy[5], d[5];
#pragma unroll
    for (int v = 0; v < 5; ++v) yy[v] = y[v * n + i];
    ray_rhs(B, t[i], yy, d);
#pragma unroll
    for (int v = 0; v < 5; ++v) dydt[v * n + i] = d[v];
  }
}

// rwrt_expand_tails: rows [tail_from[j], it_end) of every ray j := tail_row[j],
// one 16-B quarter of a row per thread (coalesced; rows without a tail untouched)
__global__ void expand_tails_kernel(double* __restrict__ out, int64_t nray, int32_t it_begin, int32_t nrows,
                                    const int32_t* __restrict__ tail_from, const double* __restrict__ tail_row) {
  const int64_t per = (int64_t)nrows * 4, n = nray * per;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = i / per;
    const int64_t q = i - j * per;
    if (it_begin + (int32_t)(q >> 2) >= tail_from[j])
      reinterpret_cast<double2*>(out)[i] = reinterpret_cast<const double2*>(tail_row)[j * 4 + (q & 3)];
  }
}

// rwrt_expand_slots: ray j's rows from its row block (compact rows of a
// rwrt_rk45_run_slots call) below tail_from[j], its tail row from there on
__global__ void expand_slots_kernel(double* __restrict__ out, int64_t nray, int32_t it_begin, int32_t nrows,
                                    const int32_t* __restrict__ row_slot, const int32_t* __restrict__ tail_from,
                                    const double* __restrict__ tail_row, const double* __restrict__ rows) {
  const int64_t per = (int64_t)nrows * 4, n = nray * per;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = i / per;
    const int64_t q = i - j * per;
    const int32_t sl = row_slot[j];
    if (it_begin + (int32_t)(q >> 2) >= tail_from[j])
      reinterpret_cast<double2*>(out)[i] = reinterpret_cast<const double2*>(tail_row)[j * 4 + (q & 3)];
    else if (sl >= 0)
      reinterpret_cast<double2*>(out)[i] = reinterpret_cast<const double2*>(rows)[(int64_t)sl * per + q];
  }
}

// rwrt_row_slots: the rays live at this point (finite state mean, the run
// kernels' frozen test) numbered in ray order -- an exclusive scan of the
// live flags over tiles of kSlotTile rays: per-tile counts (parked in each
// tile's first row_slot entry), one block scans them into offsets, then each
// tile numbers its rays (wave ballots).  No scratch beyond row_slot itself.
constexpr int kSlotTile = 4096;   // 256 threads x 16 rays
__device__ __forceinline__ bool slot_live(const double* __restrict__ state, int64_t nray, int64_t i) {
  double sum = state[i];
#pragma unroll
  for (int v = 1; v < 5; ++v) sum = sum + state[v * nray + i];
  return !isnan(sum / 5.0);   // frozen_flag_kernel's test
}
__global__ void __launch_bounds__(256) slot_count_kernel(const double* __restrict__ state, int64_t nray,
                                                         int32_t* __restrict__ row_slot) {
  const int64_t base = (int64_t)blockIdx.x * kSlotTile;
  int c = 0;
  for (int k = 0; k < kSlotTile / 256; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    c += (i < nray && slot_live(state, nray, i)) ? 1 : 0;
  }
  __shared__ int part[4];
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) row_slot[base] = part[0] + part[1] + part[2] + part[3];
}
__global__ void __launch_bounds__(1024) slot_offsets_kernel(int64_t nray, int32_t* __restrict__ row_slot,
                                                            int64_t* __restrict__ nslot) {
  const int64_t tiles = (nray + kSlotTile - 1) / kSlotTile;
  __shared__ int wsum[16];
  __shared__ int carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int64_t t0 = 0; t0 < tiles; t0 += 1024) {
    const int64_t t = t0 + threadIdx.x;
    const int v = t < tiles ? row_slot[t * kSlotTile] : 0;
    int x = v;   // inclusive scan within the wave
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int before = carry;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    if (t < tiles) row_slot[t * kSlotTile] = before + x - v;   // exclusive
    __syncthreads();
    if (threadIdx.x == 1023) carry = before + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) *nslot = carry;
}
__global__ void __launch_bounds__(256) slot_assign_kernel(const double* __restrict__ state, int64_t nray,
                                                          int32_t* __restrict__ row_slot) {
  const int64_t base = (int64_t)blockIdx.x * kSlotTile;
  __shared__ int off;
  __shared__ int wcnt[4];
  if (threadIdx.x == 0) off = row_slot[base];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int k = 0; k < kSlotTile / 256; ++k) {
    const int64_t i = base + k * 256 + threadIdx.x;
    const bool live = i < nray && slot_live(state, nray, i);
    const uint64_t m = __ballot(live);
    if (lane == 0) wcnt[wave] = __popcll(m);
    __syncthreads();
    int before = off;
    for (int w = 0; w < wave; ++w) before += wcnt[w];
    const int mine = before + __popcll(m & ((1ull << lane) - 1ull));
    if (i < nray) row_slot[i] = live ? mine : -1;
    __syncthreads();
    if (threadIdx.x == 0) off += wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
    __syncthreads();
  }
}

// rwrt_selftest_math kinds 36/37: the jump mask's verdict (1: jump) for a step
// of (dlat, dlon) = (x, y) from (lon, lat) = (1.0, 0.6), cut_off 0.05 rad:
// 36 with the ray loops' polynomial "no jump" shortcut, 37 without it.
// (Kernels added after round 4 are defined here, after the ray loops, so
// that the ray loops keep their place in the code object.)
__global__ void jump_verdict_kernel(int kind, int64_t n, const double* __restrict__ x,
                                    const double* __restrict__ y, double* __restrict__ out, double cut_a) {
  nm_stage<NM_SINCOS>();
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double lat_p = 0.6, lon_p = 1.0, cut = 0.05;
  const double lat_c = lat_p + x[i], lon_c = lon_p + y[i];
  const double cp = k_cos(lat_p), cc = k_cos(lat_c);
  const bool j = (kind == 36) ? cal_dis_reaches<true>(lon_c, lat_c, lon_p, lat_p, cc, cp, cut, cut_a)
                              : cal_dis_reaches<false>(lon_c, lat_c, lon_p, lat_p, cc, cp, cut, cut_a);
  out[i] = j ? 1.0 : 0.0;
}

}  // namespace rwrt

using namespace rwrt;

extern "C" {

const char* rwrt_version(void) { return "rwrt 0.4 (gfx950, abi 4)"; }

rwrt_status rwrt_ctx_create(int32_t device, rwrt_ctx** out) {
  if (!out) return fail(RWRT_ERR_ARG, "out is NULL%s");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(RWRT_ERR_ARG, "no such HIP device%s");
  DeviceGuard dg(device);
  if (!dg.ok) return check_launch("hipSetDevice");
  rwrt_ctx* c = new (std::nothrow) rwrt_ctx;
  if (!c) return fail(RWRT_ERR_HIP, "out of host memory%s");
  c->device = device;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0)
    c->ncu = ncu;
  if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->flagged, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->filled, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) {
    rwrt_status s = check_launch("creating the context's stream and events");
    rwrt_ctx_destroy(c);
    return s ? s : fail(RWRT_ERR_HIP, "creating the context's stream and events failed%s");
  }
  *out = c;
  return RWRT_OK;
}

rwrt_status rwrt_ctx_set_latency_density(rwrt_ctx* c, int32_t rays_per_wave) {
  if (!c) return fail(RWRT_ERR_ARG, "rwrt_ctx is NULL%s");
  if (rays_per_wave < 1 || rays_per_wave > 16) return fail(RWRT_ERR_ARG, "rays_per_wave must be 1..16%s");
  std::lock_guard<std::mutex> lock(c->mu);
  c->quad_per_wave = rays_per_wave;
  return RWRT_OK;
}

rwrt_status rwrt_ctx_set_tv_lanes(rwrt_ctx* c, int32_t lanes) {
  if (!c) return fail(RWRT_ERR_ARG, "rwrt_ctx is NULL%s");
  if (lanes != 32 && lanes != 64) return fail(RWRT_ERR_ARG, "time-varying lanes per wave must be 32 or 64%s");
  std::lock_guard<std::mutex> lock(c->mu);
  c->tv_lanes = lanes;
  return RWRT_OK;
}

rwrt_status rwrt_ctx_set_handoff(rwrt_ctx* ctx, int32_t max_rays) {
  if (rwrt_status s = ctx_check(ctx)) return s;
  if (max_rays < 0 || max_rays > 16) return fail(RWRT_ERR_ARG, "hand-off threshold must be 0..16 rays%s");
  std::lock_guard<std::mutex> lock(ctx->mu);
  ctx->handoff = max_rays;
  return RWRT_OK;
}

rwrt_status rwrt_ctx_set_trace(rwrt_ctx* c, int64_t* d_trace, int64_t capacity) {
  if (!c) return fail(RWRT_ERR_ARG, "rwrt_ctx is NULL%s");
  if (capacity < 0 || (capacity > 0 && !d_trace) || capacity > 0x7fffffffLL)
    return fail(RWRT_ERR_ARG, "trace capacity out of range or NULL trace buffer%s");
  std::lock_guard<std::mutex> lock(c->mu);
  c->trace = capacity ? d_trace : nullptr;
  c->trace_cap = capacity;
  return RWRT_OK;
}

rwrt_status rwrt_ctx_destroy(rwrt_ctx* c) {
  if (!c) return RWRT_OK;
  rwrt_status s = RWRT_OK;
  {
    std::lock_guard<std::mutex> lock(c->mu);
    DeviceGuard dg(c->device);
    // the last call's kernels may still read the flags / run on the side stream
    if (c->used && hipEventSynchronize(c->done) != hipSuccess) s = check_launch("rwrt_ctx_destroy");
    if (c->flags) (void)hipFree(c->flags);
    if (c->img) (void)hipFree(c->img);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->flagged) (void)hipEventDestroy(c->flagged);
    if (c->filled) (void)hipEventDestroy(c->filled);
    if (c->done) (void)hipEventDestroy(c->done);
  }
  delete c;
  return s;
}

const char* rwrt_last_error(void) { return g_err.c_str(); }

rwrt_status rwrt_pack_fields(const rwrt_grid* g, const double* d_fields, double* d_packed,
                             void* stream) {
  if (!g || !d_fields || !d_packed) return fail(RWRT_ERR_ARG, "NULL argument to rwrt_pack_fields%s");
  const int64_t npts = (int64_t)g->ncol * g->nrow;
  hipLaunchKernelGGL(pack_fields_kernel, dim3(grid_for(npts, 256)), dim3(256), 0,
                     (hipStream_t)stream, d_fields, d_packed, npts);
  return check_launch("pack_fields_kernel");
}

rwrt_status rwrt_mercator_point(const rwrt_grid* g, const double* d_packed, int64_t n,
                                const double* d_lon, const double* d_lat, double* d_out,
                                void* stream) {
  Field F;
  if (rwrt_status s = make_field(g, d_packed, F)) return s;
  if (n < 0 || (n > 0 && (!d_lon || !d_lat || !d_out))) return fail(RWRT_ERR_ARG, "bad point arrays%s");
  if (n == 0) return RWRT_OK;
  hipLaunchKernelGGL(mercator_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, F,
                     n, d_lon, d_lat, d_out);
  return check_launch("mercator_kernel");
}

rwrt_status rwrt_rhs(const rwrt_grid* g, const double* d_packed, int64_t n, const double* d_y,
                     double* d_dydt, void* stream) {
  Field F;
  if (rwrt_status s = make_field(g, d_packed, F)) return s;
  if (n < 0 || (n > 0 && (!d_y || !d_dydt))) return fail(RWRT_ERR_ARG, "bad state arrays%s");
  if (n == 0) return RWRT_OK;
  hipLaunchKernelGGL(rhs_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, F, n,
                     d_y, d_dydt);
  return check_launch("rhs_kernel");
}

rwrt_status rwrt_dp54_attempt(const rwrt_grid* g, const double* d_packed, int64_t n,
                              const double* d_y, const double* d_f, const double* d_h,
                              double rtol, double atol, double* d_K, double* d_ynew,
                              double* d_err, void* stream) {
  Field F;
  if (rwrt_status s = make_field(g, d_packed, F)) return s;
  if (n < 0 || (n > 0 && (!d_y || !d_f || !d_h || !d_K || !d_ynew || !d_err)))
    return fail(RWRT_ERR_ARG, "bad attempt arrays%s");
  if (n == 0) return RWRT_OK;
  hipLaunchKernelGGL(attempt_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, F,
                     n, d_y, d_f, d_h, rtol, atol, d_K, d_ynew, d_err);
  return check_launch("attempt_kernel");
}

rwrt_status rwrt_ray_initial(const rwrt_grid* g, const double* d_packed, int64_t nsource,
                             const double* d_src_lon, const double* d_src_lat,
                             const double* d_src_cos, int32_t nzwn, const double* d_zwn,
                             double* d_rows, int32_t* d_info, void* stream) {
  Field F;
  if (rwrt_status s = make_field(g, d_packed, F)) return s;
  if (nsource < 0 || nzwn < 0) return fail(RWRT_ERR_ARG, "negative size%s");
  if (!d_src_lon || !d_src_lat || !d_src_cos || !d_zwn || !d_rows || !d_info)
    return fail(RWRT_ERR_ARG, "NULL buffer%s");
  if (hipMemsetAsync(d_info, 0, sizeof(int32_t), (hipStream_t)stream) != hipSuccess)
    return check_launch("hipMemsetAsync(info)");
  const int64_t n = nsource * (int64_t)nzwn;
  if (n == 0) return RWRT_OK;
  hipLaunchKernelGGL(ray_initial_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream,
                     F, nsource, d_src_lon, d_src_lat, d_src_cos, nzwn, d_zwn, d_rows, d_info);
  return check_launch("ray_initial_kernel");
}

rwrt_status rwrt_rk45_init(const rwrt_grid* g, const double* d_packed, int64_t nray,
                           const double* d_y0, const rwrt_params* p, double* d_state,
                           int64_t* d_count, int32_t* d_nanrow, int32_t* d_live,
                           int64_t* d_summary, void* stream) {
  Field F;
  if (rwrt_status s = make_field(g, d_packed, F)) return s;
  return launch_init(StaticBG{F}, nray, d_y0, p, d_state, d_count, d_nanrow, d_live, d_summary,
                     stream);
}

rwrt_status rwrt_rk45_run(rwrt_ctx* ctx, const rwrt_grid* g, const double* d_packed,
                          int64_t nray, const rwrt_params* p, const double* d_tbound,
                          int32_t it_begin, int32_t it_end, const int64_t* d_order,
                          int64_t n_heavy, double* d_state, int64_t* d_count, int32_t* d_nanrow,
                          double* d_out, int32_t* d_work, void* stream) {
  return rwrt_rk45_run_tails(ctx, g, d_packed, nray, p, d_tbound, it_begin, it_end, d_order, n_heavy, d_state,
                             d_count, d_nanrow, d_out, nullptr, nullptr, d_work, stream);
}

rwrt_status rwrt_rk45_run_tails(rwrt_ctx* ctx, const rwrt_grid* g, const double* d_packed,
                                int64_t nray, const rwrt_params* p, const double* d_tbound,
                                int32_t it_begin, int32_t it_end, const int64_t* d_order,
                                int64_t n_heavy, double* d_state, int64_t* d_count, int32_t* d_nanrow,
                                double* d_out, int32_t* d_tail_from, double* d_tail_row, int32_t* d_work,
                                void* stream) {
  Field F;
  if (rwrt_status s = make_field(g, d_packed, F)) return s;
  return launch_run(ctx, StaticBG{F}, nray, p, d_tbound, it_begin, it_end, d_order, n_heavy, d_state,
                    d_count, d_nanrow, d_out, d_tail_from, d_tail_row, d_work, stream);
}

rwrt_status rwrt_rk45_run_slots(rwrt_ctx* ctx, const rwrt_grid* g, const double* d_packed,
                                int64_t nray, const rwrt_params* p, const double* d_tbound,
                                int32_t it_begin, int32_t it_end, const int64_t* d_order,
                                int64_t n_heavy, double* d_state, int64_t* d_count, int32_t* d_nanrow,
                                double* d_out, const int32_t* d_row_slot, int32_t* d_tail_from,
                                double* d_tail_row, int32_t* d_work, void* stream) {
  if (!d_row_slot) return fail(RWRT_ERR_ARG, "rwrt_rk45_run_slots needs d_row_slot%s");
  Field F;
  if (rwrt_status s = make_field(g, d_packed, F)) return s;
  return launch_run(ctx, StaticBG{F}, nray, p, d_tbound, it_begin, it_end, d_order, n_heavy, d_state,
                    d_count, d_nanrow, d_out, d_tail_from, d_tail_row, d_work, stream, d_row_slot);
}

rwrt_status rwrt_row_slots(int64_t nray, const double* d_state, int32_t* d_row_slot, int64_t* d_nslot,
                           void* stream) {
  if (nray < 0 || nray > 0x7fffffffLL) return fail(RWRT_ERR_ARG, "nray out of range%s");
  if (!d_nslot || (nray > 0 && (!d_state || !d_row_slot))) return fail(RWRT_ERR_ARG, "NULL buffer to rwrt_row_slots%s");
  hipStream_t st = (hipStream_t)stream;
  if (nray == 0) {
    if (hipMemsetAsync(d_nslot, 0, sizeof(int64_t), st) != hipSuccess) return check_launch("hipMemsetAsync(nslot)");
    return RWRT_OK;
  }
  const int64_t tiles = (nray + kSlotTile - 1) / kSlotTile;
  hipLaunchKernelGGL(slot_count_kernel, dim3((unsigned)tiles), dim3(256), 0, st, d_state, nray, d_row_slot);
  hipLaunchKernelGGL(slot_offsets_kernel, dim3(1), dim3(1024), 0, st, nray, d_row_slot, d_nslot);
  hipLaunchKernelGGL(slot_assign_kernel, dim3((unsigned)tiles), dim3(256), 0, st, d_state, nray, d_row_slot);
  return check_launch("row slot kernels");
}

rwrt_status rwrt_expand_slots(int64_t nray, int32_t it_begin, int32_t it_end, const int32_t* d_row_slot,
                              const int32_t* d_tail_from, const double* d_tail_row, const double* d_rows,
                              double* d_out, void* stream) {
  if (nray < 0 || it_begin >= it_end) return fail(RWRT_ERR_ARG, "bad rwrt_expand_slots shape%s");
  if (nray == 0) return RWRT_OK;
  if (!d_row_slot || !d_tail_from || !d_tail_row || !d_rows || !d_out)
    return fail(RWRT_ERR_ARG, "NULL buffer to rwrt_expand_slots%s");
  if (reinterpret_cast<uintptr_t>(d_out) % 16 != 0 || reinterpret_cast<uintptr_t>(d_tail_row) % 16 != 0 ||
      reinterpret_cast<uintptr_t>(d_rows) % 16 != 0)
    return fail(RWRT_ERR_ARG, "rows must be 16-byte aligned%s");
  const int64_t n = nray * (int64_t)(it_end - it_begin) * 4;
  hipLaunchKernelGGL(expand_slots_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, d_out,
                     nray, it_begin, it_end - it_begin, d_row_slot, d_tail_from, d_tail_row, d_rows);
  return check_launch("expand_slots_kernel");
}

rwrt_status rwrt_expand_tails(int64_t nray, int32_t it_begin, int32_t it_end, const int32_t* d_tail_from,
                              const double* d_tail_row, double* d_out, void* stream) {
  if (nray < 0 || it_begin >= it_end) return fail(RWRT_ERR_ARG, "bad rwrt_expand_tails shape%s");
  if (nray == 0) return RWRT_OK;
  if (!d_tail_from || !d_tail_row || !d_out) return fail(RWRT_ERR_ARG, "NULL buffer to rwrt_expand_tails%s");
  if (reinterpret_cast<uintptr_t>(d_out) % 16 != 0 || reinterpret_cast<uintptr_t>(d_tail_row) % 16 != 0)
    return fail(RWRT_ERR_ARG, "rows must be 16-byte aligned%s");
  const int64_t n = nray * (int64_t)(it_end - it_begin) * 4;
  hipLaunchKernelGGL(expand_tails_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, d_out,
                     nray, it_begin, it_end - it_begin, d_tail_from, d_tail_row);
  return check_launch("expand_tails_kernel");
}

rwrt_status rwrt_rk45_init_tv(const rwrt_grid* g, const rwrt_background* b, int64_t nray,
                              const double* d_y0, const rwrt_params* p, double* d_state,
                              int64_t* d_count, int32_t* d_nanrow, int32_t* d_live,
                              int64_t* d_summary, void* stream) {
  if (b && b->fp32 == 2) {
    VaryingBGA32 B;
    if (rwrt_status s = make_varying(g, b, static_cast<VaryingBG<float>&>(B))) return s;
    return launch_init(B, nray, d_y0, p, d_state, d_count, d_nanrow, d_live, d_summary, stream);
  }
  if (b && b->fp32) {
    VaryingBG<float> B;
    if (rwrt_status s = make_varying(g, b, B)) return s;
    return launch_init(B, nray, d_y0, p, d_state, d_count, d_nanrow, d_live, d_summary, stream);
  }
  VaryingBG<double> B;
  if (rwrt_status s = make_varying(g, b, B)) return s;
  return launch_init(B, nray, d_y0, p, d_state, d_count, d_nanrow, d_live, d_summary, stream);
}

rwrt_status rwrt_rk45_run_tv(rwrt_ctx* ctx, const rwrt_grid* g, const rwrt_background* b,
                             int64_t nray, const rwrt_params* p, const double* d_tbound, int32_t it_begin,
                             int32_t it_end, const int64_t* d_order, int64_t n_heavy,
                             double* d_state, int64_t* d_count, int32_t* d_nanrow, double* d_out,
                             int32_t* d_work, void* stream) {
  return rwrt_rk45_run_tv_tails(ctx, g, b, nray, p, d_tbound, it_begin, it_end, d_order, n_heavy, d_state,
                                d_count, d_nanrow, d_out, nullptr, nullptr, d_work, stream);
}

static rwrt_status run_tv(rwrt_ctx* ctx, const rwrt_grid* g, const rwrt_background* b,
                                   int64_t nray, const rwrt_params* p, const double* d_tbound,
                                   int32_t it_begin, int32_t it_end, const int64_t* d_order, int64_t n_heavy,
                                   double* d_state, int64_t* d_count, int32_t* d_nanrow, double* d_out,
                                   int32_t* d_tail_from, double* d_tail_row, int32_t* d_work, void* stream,
                          const int32_t* d_row_slot) {
  if (b && b->fp32 == 2) {
    VaryingBGA32 B;
    if (rwrt_status s = make_varying(g, b, static_cast<VaryingBG<float>&>(B))) return s;
    return launch_run(ctx, B, nray, p, d_tbound, it_begin, it_end, d_order, n_heavy, d_state, d_count,
                      d_nanrow, d_out, d_tail_from, d_tail_row, d_work, stream, d_row_slot);
  }
  if (b && b->fp32) {
    VaryingBG<float> B;
    if (rwrt_status s = make_varying(g, b, B)) return s;
    return launch_run(ctx, B, nray, p, d_tbound, it_begin, it_end, d_order, n_heavy, d_state, d_count,
                      d_nanrow, d_out, d_tail_from, d_tail_row, d_work, stream, d_row_slot);
  }
  int lanes = 64;
  if (ctx) {
    std::lock_guard<std::mutex> lock(ctx->mu);
    lanes = ctx->tv_lanes;
  }
  VaryingBG<double> B;
  if (rwrt_status s = make_varying(g, b, B)) return s;
  B.half = lanes == 32;
  return launch_run(ctx, B, nray, p, d_tbound, it_begin, it_end, d_order, n_heavy, d_state, d_count,
                    d_nanrow, d_out, d_tail_from, d_tail_row, d_work, stream, d_row_slot);
}

rwrt_status rwrt_rk45_run_tv_tails(rwrt_ctx* ctx, const rwrt_grid* g, const rwrt_background* b,
                                   int64_t nray, const rwrt_params* p, const double* d_tbound,
                                   int32_t it_begin, int32_t it_end, const int64_t* d_order, int64_t n_heavy,
                                   double* d_state, int64_t* d_count, int32_t* d_nanrow, double* d_out,
                                   int32_t* d_tail_from, double* d_tail_row, int32_t* d_work, void* stream) {
  return run_tv(ctx, g, b, nray, p, d_tbound, it_begin, it_end, d_order, n_heavy, d_state, d_count, d_nanrow,
                d_out, d_tail_from, d_tail_row, d_work, stream, nullptr);
}

rwrt_status rwrt_rk45_run_tv_slots(rwrt_ctx* ctx, const rwrt_grid* g, const rwrt_background* b,
                                   int64_t nray, const rwrt_params* p, const double* d_tbound,
                                   int32_t it_begin, int32_t it_end, const int64_t* d_order, int64_t n_heavy,
                                   double* d_state, int64_t* d_count, int32_t* d_nanrow, double* d_out,
                                   const int32_t* d_row_slot, int32_t* d_tail_from, double* d_tail_row,
                                   int32_t* d_work, void* stream) {
  if (!d_row_slot) return fail(RWRT_ERR_ARG, "rwrt_rk45_run_tv_slots needs d_row_slot%s");
  return run_tv(ctx, g, b, nray, p, d_tbound, it_begin, it_end, d_order, n_heavy, d_state, d_count, d_nanrow,
                d_out, d_tail_from, d_tail_row, d_work, stream, d_row_slot);
}

rwrt_status rwrt_rhs_tv(const rwrt_grid* g, const rwrt_background* b, int64_t n,
                        const double* d_t, const double* d_y, double* d_dydt, void* stream) {
  if (n < 0 || !d_t || !d_y || !d_dydt) return fail(RWRT_ERR_ARG, "bad rwrt_rhs_tv arguments%s");
  if (n == 0) return RWRT_OK;
  const dim3 grid(grid_for(n, 256)), block(256);
  if (b && b->fp32 == 2) {
    VaryingBGA32 B;
    if (rwrt_status s = make_varying(g, b, static_cast<VaryingBG<float>&>(B))) return s;
    hipLaunchKernelGGL(rhs_bg_kernel<VaryingBGA32>, grid, block, 0, (hipStream_t)stream, B, n,
                       d_t, d_y, d_dydt);
  } else if (b && b->fp32) {
    VaryingBG<float> B;
    if (rwrt_status s = make_varying(g, b, B)) return s;
    hipLaunchKernelGGL(rhs_bg_kernel<VaryingBG<float>>, grid, block, 0, (hipStream_t)stream, B, n,
                       d_t, d_y, d_dydt);
  } else {
    VaryingBG<double> B;
    if (rwrt_status s = make_varying(g, b, B)) return s;
    hipLaunchKernelGGL(rhs_bg_kernel<VaryingBG<double>>, grid, block, 0, (hipStream_t)stream, B, n,
                       d_t, d_y, d_dydt);
  }
  return check_launch("rhs_bg_kernel");
}

rwrt_status rwrt_bs_ready(int32_t nlon, int32_t nlat, const float* d_u, const float* d_v,
                          const double* d_trig, double dx, double dy, double* d_scratch,
                          void* d_packed, int32_t fp32, void* stream) {
  if (nlon < 3 || nlat < 4) return fail(RWRT_ERR_ARG, "bs_ready needs nlon >= 3 and nlat >= 4%s");
  if (!d_u || !d_v || !d_trig || !d_scratch || !d_packed) return fail(RWRT_ERR_ARG, "NULL buffer to rwrt_bs_ready%s");
  if (reinterpret_cast<uintptr_t>(d_packed) % 16 != 0)
    return fail(RWRT_ERR_ARG, "packed fields must be 16-byte aligned%s");
  ReadyArgs a{nlon, nlat, d_u, d_v, d_trig, 2.0 * dx, 2.0 * dy, dx * dx, dy * dy, (4.0 * dx) * dy,
              dx, dy, d_scratch, d_packed};
  const int64_t n = (int64_t)nlon * nlat, n1 = (int64_t)(nlon + 1) * nlat;
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(ready_q_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, a);
  hipLaunchKernelGGL(ready_q2_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st, a);
  if (fp32)
    hipLaunchKernelGGL(ready_pack_kernel<float>, dim3(grid_for(n1, 256)), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL(ready_pack_kernel<double>, dim3(grid_for(n1, 256)), dim3(256), 0, st, a);
  return check_launch("bs_ready kernels");
}

rwrt_status rwrt_rk4_run(rwrt_ctx* ctx, const rwrt_grid* g, const double* d_packed,
                         int64_t nray, const rwrt_params* p, int32_t it_begin, int32_t it_end,
                         const int64_t* d_order, double* d_state, int64_t* d_count,
                         int32_t* d_nanrow, double* d_out, int32_t* d_work, void* stream) {
  Field F;
  if (rwrt_status s = ctx_check(ctx)) return s;
  if (rwrt_status s = make_field(g, d_packed, F)) return s;
  if (!p) return fail(RWRT_ERR_ARG, "params is NULL%s");
  if (nray < 0 || nray > 0x7fffffffLL) return fail(RWRT_ERR_ARG, "nray out of range%s");
  if (it_begin < 1 || it_end > p->nt || it_begin >= it_end)
    return fail(RWRT_ERR_ARG, "need 1 <= it_begin < it_end <= nt%s");
  if (!(p->tstep > 0.0)) return fail(RWRT_ERR_ARG, "tstep must be positive%s");
  if (!d_work || (nray > 0 && (!d_state || !d_count || !d_nanrow || !d_out)))
    return fail(RWRT_ERR_ARG, "NULL buffer to rwrt_rk4_run%s");
  if (reinterpret_cast<uintptr_t>(d_out) % 16 != 0)
    return fail(RWRT_ERR_ARG, "output rows must be 16-byte aligned%s");
  if (nray == 0) return RWRT_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return check_launch("hipSetDevice(context device)");
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(d_work, 0, sizeof(int32_t), st) != hipSuccess)
    return check_launch("hipMemsetAsync(queue)");
  Rk4Args a{F, nullptr, nray, p->tstep, p->cut_off, p->nt, it_begin, it_end, d_order, d_state, d_count,
            d_nanrow, d_out, d_work, nullptr};
  int64_t blocks = ctx_persistent_blocks<StaticBG>(ctx);
  const int64_t need = (nray + 255) / 256;
  if (blocks > need) blocks = need;
  // rays whose rows are known at the start go to rk4_fill_kernel on the side
  // stream (as launch_run does for the RK45 loop)
  if (rwrt_status s = ctx_flags(ctx, nray)) return s;
  a.frozen = ctx->flags;
  if (rwrt_status s = ctx_begin(ctx, st, [&] {
        hipLaunchKernelGGL(rk4_flag_kernel, dim3(grid_for(nray, 256)), dim3(256), 0, st, d_state, nray,
                           ctx->flags);
      }))
    return s;
  if (rwrt_status s = ctx_image(ctx, F, st, &a.img)) return s;
  hipLaunchKernelGGL(rk4_run_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
  if (rwrt_status s = check_launch("rk4_run_kernel")) return s;
  hipLaunchKernelGGL(rk4_fill_kernel, dim3((unsigned)((nray + kFillThreads - 1) / kFillThreads)),
                     dim3(kFillThreads), 0, ctx->side, a);
  if (rwrt_status s = check_launch("rk4_fill_kernel")) return s;
  return ctx_end(ctx, st);
}

rwrt_status rwrt_kat_rk45(int32_t kind, int64_t ncol, const double* d_y0, int32_t nt,
                          const double* d_teval, double rtol, double atol, double min_step,
                          double* d_out, void* stream) {
  if (ncol <= 0 || nt < 1 || !d_y0 || !d_teval || !d_out) return fail(RWRT_ERR_ARG, "bad KAT arguments%s");
  const dim3 grid(grid_for(ncol, 64)), block(64);
  hipStream_t s = (hipStream_t)stream;
  switch (kind) {
    case 0: hipLaunchKernelGGL(kat_kernel<KatLinear>, grid, block, 0, s, ncol, d_y0, nt, d_teval, rtol, atol, min_step, d_out); break;
    case 1: hipLaunchKernelGGL(kat_kernel<KatExp>, grid, block, 0, s, ncol, d_y0, nt, d_teval, rtol, atol, min_step, d_out); break;
    case 2: hipLaunchKernelGGL(kat_kernel<KatLorenz>, grid, block, 0, s, ncol, d_y0, nt, d_teval, rtol, atol, min_step, d_out); break;
    default: return fail(RWRT_ERR_ARG, "unknown KAT kind%s");
  }
  return check_launch("kat_kernel");
}

rwrt_status rwrt_selftest_math(int32_t kind, int64_t n, const double* d_x, const double* d_y,
                               double* d_out, void* stream) {
  if (n < 0 || kind < 0 || kind > 37 || (n > 0 && (!d_x || !d_out)))
    return fail(RWRT_ERR_ARG, "bad selftest arguments%s");
  if (kind >= 17 && kind <= 22)   // retired device-libm restatements: never alias another kind
    return fail(RWRT_ERR_ARG, "selftest kinds 17-22 are retired%s");
  if (n == 0) return RWRT_OK;
  if (kind >= 36) {
    if (!d_y) return fail(RWRT_ERR_ARG, "selftest kinds 36/37 need d_y%s");
    hipLaunchKernelGGL(jump_verdict_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, kind,
                       n, d_x, d_y, d_out, haversine_cut(0.05));
    return check_launch("jump_verdict_kernel");
  }
  hipLaunchKernelGGL(math_kernel, dim3(grid_for(n, 256)), dim3(256), 0, (hipStream_t)stream, kind,
                     n, d_x, d_y, d_out);
  return check_launch("math_kernel");
}

// Host side of the drop-in delivery (hostio.HistorySink): the block starts as
// copies of the previous row, then the shipped columns are scattered in.
rwrt_status rwrt_host_fill_rows(double* dst, int64_t nrows, int64_t ncol, int64_t ld,
                                const double* prev, const double* src, int64_t nsrc,
                                int64_t ld_src, const int64_t* cols) {
  if (nrows < 0 || ncol < 0 || nsrc < 0 || nsrc > ncol || ld < ncol || ld_src < nsrc)
    return fail(RWRT_ERR_ARG, "bad rwrt_host_fill_rows shape%s");
  if (nrows == 0 || ncol == 0) return RWRT_OK;
  if (!dst || (nsrc < ncol && !prev) || (nsrc > 0 && (!src || !cols)))
    return fail(RWRT_ERR_ARG, "NULL buffer to rwrt_host_fill_rows%s");
  for (int64_t j = 0; j < nsrc; ++j)
    if (cols[j] < 0 || cols[j] >= ncol || (j > 0 && cols[j] <= cols[j - 1]))
      return fail(RWRT_ERR_ARG, "cols must be strictly ascending in [0, ncol)%s");
  typedef double v2d __attribute__((ext_vector_type(2)));
  for (int64_t i = 0; i < nrows; ++i) {
    double* d = dst + i * ld;
    const double* s = src + i * ld_src;
    if (nsrc == ncol) {
      std::memcpy(d, s, sizeof(double) * ncol);
      continue;
    }
    // Each 64-B line of the row is assembled from the previous row and the
    // shipped columns that fall in it, then written with non-temporal stores
    // (the block is far larger than the caches: no read-for-ownership).
    int64_t j = 0, c = 0;
    for (; c < ncol && (reinterpret_cast<uintptr_t>(d + c) & 63); ++c)
      d[c] = (j < nsrc && cols[j] == c) ? s[j++] : prev[c];
    for (; c + 8 <= ncol; c += 8) {
      double line[8];
      std::memcpy(line, prev + c, sizeof(line));
      for (; j < nsrc && cols[j] < c + 8; ++j) line[cols[j] - c] = s[j];
      for (int q = 0; q < 8; q += 2) {
        const v2d v = {line[q], line[q + 1]};
        __builtin_nontemporal_store(v, reinterpret_cast<v2d*>(d + c + q));
      }
    }
    for (; c < ncol; ++c) d[c] = (j < nsrc && cols[j] == c) ? s[j++] : prev[c];
  }
  __builtin_ia32_sfence();   // the streaming stores are visible before the caller's release
  return RWRT_OK;
}

}  // extern "C"
