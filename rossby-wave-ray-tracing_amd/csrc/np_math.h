// np_math.h -- sin, cos, tan and pow exactly as the reference's NumPy computes
// them on an AVX-512 x86-64 host, restated operation by operation so that the
// GPU reproduces the reference's ray histories bit for bit.
//
// The reference evaluates its transcendentals through NumPy 2.2.6 ufuncs
// (SURVEY.md §8(c)): np.sin / np.cos call glibc 2.35's libm, whose x86-64
// ifunc selects the FMA build of the IBM Accurate Mathematical Library's
// s_sin.c (__sin_fma / __cos_fma); np.tan and np.power run NumPy's SVML
// kernels __svml_tan8_ha and __svml_pow8_ha (AVX512_SKX dispatch).  Each
// function below follows the instruction sequence of that machine code --
// the FMA contractions the compiler made, the table lookups, the embedded
// rounding modes -- with the constants and tables read from the two shared
// objects by tools/gen_np_math.py (np_math_tables.h).  tests/test_np_math.py
// proves each one bitwise equal to NumPy on >= 16 M arguments; the GPU box's
// host computes the same bits (tools/host_libm_probe.py fingerprints).
//
// Domain: every argument the ray loop produces.  sin and cos follow glibc for
// |x| < 105414350 (the table path and reduce_sincos; beyond, glibc's
// Payne-Hanek __branred is not restated and the includer's library routine
// answers); tan follows SVML for |x| <= 65536 (beyond: the includer's
// routine); pow follows SVML's main path for finite x > 0 with |y log2 x| <=
// 1021.5 and the C99 special values elsewhere (SVML's rare-path routine is not
// restated: exact for the ray loop's pow(err, -0.2) and pow(0.01/d, 0.2)).
//
// The includer supplies:
//   NM_FN            function qualifiers
//   NM_CONST         qualifier of scalar constants (e.g. constexpr)
//   NM_TABLE         qualifier of the tables (device: __constant__ const)
//   NM_FMA_RZ(a,b,c) fused multiply-add rounded toward zero
//   NM_ADD_RZ(a,b)   addition rounded toward zero
//   NM_MUL_RZ(a,b)   multiplication rounded toward zero
//   NM_RCP14_TAB     the expanded VRCP14PD table (nm_rcp14_table(): 65536 x
//                    uint16 result fraction bits), declared after this header
//   NM_ADD_RD(a,b)   addition rounded toward -infinity
//   NM_FALLBACK_SIN/COS/TAN/POW  library routines outside the domain above
// Compile with -ffp-contract=off: every fused operation here is explicit.
#pragma once

#include "np_math_tables.h"

namespace np_math {

struct NmRcp14;

NM_FN double nm_d(unsigned long long u) { return __builtin_bit_cast(double, u); }
NM_FN unsigned long long nm_u(double x) { return __builtin_bit_cast(unsigned long long, x); }
NM_FN double nm_fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
NM_FN double nm_abs(double x) { return nm_d(nm_u(x) & 0x7FFFFFFFFFFFFFFFull); }
NM_FN double nm_sign(double x) { return nm_d(nm_u(x) & 0x8000000000000000ull); }
NM_FN double nm_copysign(double m, double s) {
  return nm_d((nm_u(m) & 0x7FFFFFFFFFFFFFFFull) | (nm_u(s) & 0x8000000000000000ull));
}
NM_FN double tabd(const unsigned long long* t, int i) { return nm_d(t[i]); }

// ---------------------------------------------------------------------------
// VRCP14PD: the result depends on the sign, the exponent and the top 16
// fraction bits of the input (an exact power of two has its exact
// reciprocal); the 16-bit result fraction comes from the table.  Normal
// inputs whose reciprocal is normal.
// ---------------------------------------------------------------------------
// The expanded table: entry i = the 16 result fraction bits for inputs with
// top fraction bits i; built at compile time from the 2-bit deltas of
// np_math_tables.h (the includer stores one: a __device__ const on the GPU).
struct NmRcp14 {
  unsigned short v[65536];
};
constexpr NmRcp14 nm_rcp14_table() {
  NmRcp14 t{};
  unsigned f = kRCP14_F0;
  t.v[0] = (unsigned short)f;
  for (int i = 1; i < 65536; ++i) {
    const int k = i - 1;
    f -= (kRCP14_DELTA[k >> 4] >> (2 * (k & 15))) & 3u;
    t.v[i] = (unsigned short)f;
  }
  return t;
}
NM_FN double nm_rcp14(double x) {
  const unsigned long long u = nm_u(x);
  const unsigned long long e = (u >> 52) & 0x7FF;
  const unsigned i = (unsigned)(u >> 36) & 0xFFFF;
  const unsigned long long s = u & 0x8000000000000000ull;
  if ((u & 0x000FFFFFFFFFFFFFull) == 0) return nm_d(s | ((2046ull - e) << 52));   // 2^-(e-1023)
  return nm_d(s | ((2045ull - e) << 52) | ((unsigned long long)NM_RCP14_TAB[i] << 36));
}

// ---------------------------------------------------------------------------
// glibc 2.35 s_sin.c, FMA build (__sin_fma / __cos_fma)
// ---------------------------------------------------------------------------
// TAYLOR_SIN(xx, a, da): ((POLY(xx) * a - 0.5 * da) * xx + da), then a + that
NM_FN double g_taylor_sin(double a, double da) {
  const double xx = a * a;
  double p = nm_fma(nm_d(kG_S5), xx, nm_d(kG_S4));
  p = nm_fma(p, xx, nm_d(kG_S3));
  p = nm_fma(p, xx, nm_d(kG_S2));
  p = nm_fma(p, xx, nm_d(kG_S1));
  const double t1 = nm_fma(p, a, -(da * nm_d(kG_CS2)));     // vfmsub: P a - 0.5 da
  return a + nm_fma(xx, t1, da);
}
// do_sin(x, dx): |x| >= 0.126 here unless the Taylor branch is taken
NM_FN double g_do_sin(double x, double dx) {
  if (nm_abs(x) < nm_d(kG_T126)) return g_taylor_sin(x, dx);
  if (!(0.0 < x)) dx = -dx;                                   // x <= 0 (or NaN)
  const double ax = nm_abs(x);
  const double u = nm_d(kG_BIG) + ax;
  const int k = (int)((unsigned)nm_u(u) << 2);
  const double xr = ax - (u - nm_d(kG_BIG));
  const double xx = xr * xr;
  const double t = nm_fma(nm_d(kG_SN5), xx, nm_d(kG_SN3));
  const double s = xr + nm_fma(xr * xx, t, dx);
  double c0 = nm_fma(nm_d(kG_CS6), xx, nm_d(kG_CS4));
  c0 = nm_fma(c0, xx, nm_d(kG_CS2));
  const double c = nm_fma(xr, dx, xx * c0);
  const double sn = tabd(kG_SINCOSTAB, k), ssn = tabd(kG_SINCOSTAB, k + 1);
  const double cs = tabd(kG_SINCOSTAB, k + 2), ccs = tabd(kG_SINCOSTAB, k + 3);
  const double cor = nm_fma(s, cs, nm_fma(-c, sn, nm_fma(ccs, s, ssn)));
  return nm_copysign(sn + cor, x);
}
// do_cos(x, dx)
NM_FN double g_do_cos(double x, double dx) {
  if (x < 0.0) dx = -dx;
  const double ax = nm_abs(x);
  const double u = nm_d(kG_BIG) + ax;
  const int k = (int)((unsigned)nm_u(u) << 2);
  const double xr = (ax - (u - nm_d(kG_BIG))) + dx;
  const double xx = xr * xr;
  const double t = nm_fma(nm_d(kG_SN5), xx, nm_d(kG_SN3));
  const double s = nm_fma(xr * xx, t, xr);
  double c0 = nm_fma(nm_d(kG_CS6), xx, nm_d(kG_CS4));
  c0 = nm_fma(c0, xx, nm_d(kG_CS2));
  const double c = xx * c0;
  const double sn = tabd(kG_SINCOSTAB, k), ssn = tabd(kG_SINCOSTAB, k + 1);
  const double cs = tabd(kG_SINCOSTAB, k + 2), ccs = tabd(kG_SINCOSTAB, k + 3);
  const double cor = nm_fma(-s, sn, nm_fma(-c, cs, nm_fma(-s, ssn, ccs)));
  return cs + cor;
}
// reduce_sincos: x = n pi/2 + (a + da), n mod 4
NM_FN int g_reduce(double x, double& a, double& da) {
  const double t = nm_fma(x, nm_d(kG_HPINV), nm_d(kG_TOINT));
  const double xn = t - nm_d(kG_TOINT);
  const int n = (int)(unsigned)nm_u(t) & 3;
  const double y = nm_fma(-xn, nm_d(kG_MP2), nm_fma(-xn, nm_d(kG_MP1), x));
  const double t2 = nm_fma(-xn, nm_d(kG_PP3), y);
  const double db = nm_fma(-xn, nm_d(kG_PP3), y - t2);
  const double b = nm_fma(-xn, nm_d(kG_PP4), t2);
  a = b;
  da = db + nm_fma(-xn, nm_d(kG_PP4), t2 - b);
  return n;
}
NM_FN double g_do_sincos(double a, double da, int n) {
  const double r = (n & 1) ? g_do_cos(a, da) : g_do_sin(a, da);
  return (n & 2) ? -r : r;
}
NM_FN unsigned g_hi(double x) { return (unsigned)(nm_u(x) >> 32) & 0x7FFFFFFFu; }

NM_FN double nm_sin(double x) {
  const unsigned k = g_hi(x);
  if (k < 0x3E500000u) return x;                              // |x| < 2^-26
  if (k < 0x3FEB6000u) return g_do_sin(x, 0.0);               // |x| < 0.855469
  if (k < 0x400368FDu) {                                      // |x| < 2.426265
    const double t = nm_d(kG_HP0) - nm_abs(x);
    return nm_copysign(g_do_cos(t, nm_d(kG_HP1)), x);
  }
  if (k < 0x419921FBu) {                                      // |x| < 105414350
    double a, da;
    const int n = g_reduce(x, a, da);
    return g_do_sincos(a, da, n);
  }
  return NM_FALLBACK_SIN(x);
}

NM_FN double nm_cos(double x) {
  const unsigned k = g_hi(x);
  if (k < 0x3E400000u) return 1.0;                            // |x| < 2^-27
  if (k < 0x3FEB6000u) return g_do_cos(x, 0.0);
  if (k < 0x400368FDu) {
    const double y = nm_d(kG_HP0) - nm_abs(x);
    const double a = y + nm_d(kG_HP1);
    const double da = (y - a) + nm_d(kG_HP1);
    return g_do_sin(a, da);
  }
  if (k < 0x419921FBu) {
    double a, da;
    const int n = g_reduce(x, a, da);
    return g_do_sincos(a, da, n + 1);
  }
  return NM_FALLBACK_COS(x);
}

// ---------------------------------------------------------------------------
// SVML __svml_tan8_ha (main path, |x| <= 65536): x = n pi/16 + r,
// tan x = (T + tan r) / (1 - T tan r), T = tan(n pi/16) in head + tail
// ---------------------------------------------------------------------------
NM_FN double nm_tan(double x) {
  if (!(nm_abs(x) <= nm_d(kT_BIGARG))) {
    if (x != x || nm_abs(x) == __builtin_inf()) return x - x;   // NaN
    return NM_FALLBACK_TAN(x);
  }
  const double y = nm_fma(nm_d(kT_INVPI16), x, nm_d(kT_SHIFT));
  const double n = y - nm_d(kT_SHIFT);
  const int j = (int)(nm_u(y) & 15);
  const double r1 = nm_fma(-n, nm_d(kT_PI16A), x);
  const double r2 = nm_fma(-n, nm_d(kT_PI16B), r1);
  const double r = nm_fma(-n, nm_d(kT_PI16C), r2);
  const double e2 = nm_fma(-nm_d(kT_PI16B), n, r1 - r2);
  const double e3 = nm_fma(nm_d(kT_PI16C), n, r - r2);
  const double rl = e2 - e3;
  const double r2q = r * r;
  double p = nm_fma(nm_d(kT_C5), r2q, nm_d(kT_C4));
  p = nm_fma(r2q, p, nm_d(kT_C3));
  p = nm_fma(r2q, p, nm_d(kT_C2));
  p = nm_fma(r2q, p, nm_d(kT_C1));
  const double pr = p * r;
  const double z9 = nm_fma(-r2q, pr, -rl);                    // vfnmsub: -(r^2 p r) - rl
  const double th = r - z9;                                   // tan r, head
  const double tl = (r - th) - z9;                            // and tail
  const double T = tabd(kT_TAN_HI, j), Tl = tabd(kT_TAN_LO, j);
  const double N = th + T;
  const double nl = (th - (N - T)) + Tl;
  const double D = nm_fma(-th, T, nm_d(kT_ONE));
  const double Nl = nl + tl;
  double dl = nm_fma(th, T, D - nm_d(kT_ONE));
  dl = nm_fma(tl, T, dl);
  dl = nm_fma(th, Tl, dl);
  double rc = nm_rcp14(D);
  double e = nm_fma(-D, rc, nm_d(kT_ONE));
  e = nm_fma(dl, rc, e);
  rc = nm_fma(e, rc, rc);
  const double q = rc * N;
  double res = nm_fma(q, D, -N);
  res = nm_fma(-q, dl, res);
  return nm_fma(-rc, res - Nl, q);
}

// ---------------------------------------------------------------------------
// SVML __svml_pow8_ha (main path): log2 x = k + log2 of the table point + a
// degree-10 polynomial in r = (m R - 1) / 2 (R = VRCP14 of the mantissa,
// rounded to 1/32), T = y log2 x by round-toward-zero double-double steps,
// 2^T from a 16-entry table and a degree-7 polynomial
// ---------------------------------------------------------------------------
NM_FN double nm_pow(double x, double y) {
  const double inf = __builtin_inf();
  const bool xs = !(x > 0.0) || x == inf || x != x;           // vfpclass 0xdf: NaN, 0, inf, < 0
  const bool ys = y != y || nm_abs(y) == inf;                  // vfpclass 0x99
  if (xs || ys) {
    // C99 / IEEE pow special values (what SVML's rare path returns)
    if (y == 0.0) return 1.0;
    if (x == 1.0) return 1.0;
    if (x != x || y != y) return x + y;
    const double ax = nm_abs(x);
    const bool yint = __builtin_trunc(y) == y && nm_abs(y) != inf;
    const bool yodd = yint && nm_abs(y) < 9007199254740992.0 && __builtin_fmod(y, 2.0) != 0.0;
    if (nm_abs(y) == inf) {
      if (ax == 1.0) return 1.0;
      return ((ax < 1.0) == (y < 0.0)) ? inf : 0.0;
    }
    if (x == 0.0) {
      const double v = (y < 0.0) ? inf : 0.0;
      return yodd ? nm_copysign(v, x) : v;
    }
    if (ax == inf) {
      const double v = (y < 0.0) ? 0.0 : inf;
      return (x < 0.0 && yodd) ? -v : v;
    }
    // finite x < 0
    if (!yint) return __builtin_nan("");
    const double m = NM_FALLBACK_POW(ax, y);
    return yodd ? -m : m;
  }
  // vgetmant (interval [0.5, 1)) and vgetexp of x > 0, normal or subnormal
  unsigned long long ux = nm_u(x);
  int ex = (int)((ux >> 52) & 0x7FF) - 1023;
  if ((ux >> 52) == 0) {                                       // subnormal: normalise
    const int lz = __builtin_clzll(ux) - 11;
    ux <<= lz;
    ex = -1022 - lz;
  }
  const double M = nm_d((ux & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);   // [1, 2)
  const double m = M * 0.5;                                                          // [0.5, 1)
  // VRCP14PD(m), rounded to 5 fraction bits (vrndscalepd 0x58, to nearest even)
  const double rc = nm_rcp14(m);
  const double R = __builtin_rint(rc * 32.0) * 0.03125;
  const int f = (int)((nm_u(R) >> 47) & 31);
  double e = (double)ex;
  if (R < 1.5) e = e + 1.0;
  const double Lh = tabd(kP_LOG_HI, f), Ll = tabd(kP_LOG_LO, f);
  const double r = nm_fma(m * nm_d(kP_HALF), R, -nm_d(kP_HALF));
  const double r2 = r * r;
  const double a9 = nm_fma(nm_d(kP_C10), r, nm_d(kP_C9));
  const double a7 = nm_fma(nm_d(kP_C8), r, nm_d(kP_C7));
  const double lo = nm_fma(nm_d(kP_LN), r, nm_d(kP_LP));
  const double a5 = nm_fma(nm_d(kP_C6), r, nm_d(kP_C5));
  const double a3 = nm_fma(nm_d(kP_C4), r, nm_d(kP_C3));
  const double r4 = r2 * r2;
  double q = nm_fma(r2, a9, a7);
  const double b5 = nm_fma(r2, a5, a3);
  q = nm_fma(r4, q, b5);
  q = nm_fma(r2, q, lo);
  q = nm_fma(r, q, Ll);
  const double LE = Lh + e;
  const double H = nm_fma(nm_d(kP_C1), r, LE);
  const double cr = H - LE;
  const double z4 = nm_fma(-r, cr, H);
  double z14 = nm_fma(r, nm_d(kP_C1), -cr);
  const double z5 = H - z4;
  z14 = nm_fma(-z14, r, z14);
  const double z12 = nm_fma(cr, r, -z5);
  const double z7 = z14 - z12;
  const double z8 = q + z7;
  const double L = z4 + z8;                                   // log2 x, head
  const double P = NM_MUL_RZ(L, y);
  const double Ld = L - z4;
  const double pe = NM_FMA_RZ(y, L, -P);
  const double Lt = z8 - Ld;                                  // log2 x, tail
  const double Pl = NM_FMA_RZ(y, Lt, pe);
  const double T = NM_ADD_RZ(P, Pl);                          // y log2 x
  const double Tl = Pl - (T - P);
  if (!(nm_abs(T) <= nm_d(kP_TOVF))) return NM_FALLBACK_POW(x, y);   // over/underflow (rare path)
  // 2^T: T = (k16 + fr) / 16 with fr in [0, 1) (vaddpd {rd-sae} on a shifter
  // and vreducepd 0x41: both the floor at 1/16)
  const double fl = __builtin_floor(T * 16.0);
  const double frac = NM_ADD_RD(T, -(fl * 0.0625));   // vreducepd subtracts under its own RD
  const long long k16 = (long long)fl;
  const int jj = (int)(k16 & 15);
  const long long kk = k16 >> 4;
  const double fz = nm_d(nm_u(frac + Tl) & 0xBFFFFFFFFFFFFFFFull);
  const double f2 = fz * fz;
  double p1 = nm_fma(nm_d(kP_E7), fz, nm_d(kP_E6));
  const double p3 = nm_fma(nm_d(kP_E4), fz, nm_d(kP_E3));
  const double p5 = nm_fma(nm_d(kP_E2), fz, nm_d(kP_E1));
  p1 = nm_fma(f2, p1, p3);
  p1 = nm_fma(f2, p1, p5);
  const double El = tabd(kP_EXP_LO, jj), Eh = tabd(kP_EXP_HI, jj);
  p1 = nm_fma(fz, p1, El);
  p1 = nm_fma(Eh, p1, Eh);
  const double scale = nm_d((unsigned long long)(kk + 1023) << 52);
  return p1 * scale;
}

}  // namespace np_math
