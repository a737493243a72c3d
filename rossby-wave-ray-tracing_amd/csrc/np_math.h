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
//   NM_ADD_RD(a,b)   addition rounded toward -infinity
//   NM_FALLBACK_SIN/COS/TAN/POW  library routines outside the domain above
// Compile with -ffp-contract=off: every fused operation here is explicit.
//
// Provenance and licences of what is restated: the algorithms and constants
// of glibc's IBM Accurate Mathematical Library (sysdeps/ieee754/dbl-64/
// s_sin.c, sincostab; GNU LGPL-2.1-or-later) and of Intel's SVML kernels
// shipped inside NumPy (numpy/_core/src/umath/svml; BSD-3-Clause).  No source
// file of either is copied: the operation sequences were read from the
// machine code of the two shared objects of the reference's host and the
// constants extracted from them (tools/gen_np_math.py); the reference
// repository itself contains none of this code.
#pragma once

#include "np_math_tables.h"

namespace np_math {

// NM_KVAL(u): an includer may serve the scalar constants from a faster copy
// (e.g. LDS) when u is a compile-time constant; default: the bit pattern.
#ifndef NM_KVAL
#define NM_KVAL(u) __builtin_bit_cast(double, (unsigned long long)(u))
#endif
NM_FN double nm_d(unsigned long long u) { return NM_KVAL(u); }
NM_FN unsigned long long nm_u(double x) { return __builtin_bit_cast(unsigned long long, x); }
#ifndef NM_FMA
#define NM_FMA(a, b, c) __builtin_fma((a), (b), (c))
#endif
NM_FN double nm_fma(double a, double b, double c) { return NM_FMA(a, b, c); }
NM_FN double nm_abs(double x) { return nm_d(nm_u(x) & 0x7FFFFFFFFFFFFFFFull); }
NM_FN double nm_sign(double x) { return nm_d(nm_u(x) & 0x8000000000000000ull); }
NM_FN double nm_copysign(double m, double s) {
  return nm_d((nm_u(m) & 0x7FFFFFFFFFFFFFFFull) | (nm_u(s) & 0x8000000000000000ull));
}
// Table reads go through NM_LD(table, i) (default: the array element); an
// includer can serve them from a faster copy (e.g. LDS).
//
// The common path of each function is straight-line code (the arms of the
// reference's data-dependent branches computed both and selected, table
// indices clamped into range), with the rare arguments fixed up at the end:
// on the GPU a wave then never splits on the argument ranges of its lanes
// and the table reads can be issued early.  The selected values are the
// reference's; what differs is only which dead values get computed.
#ifndef NM_LD
#define NM_LD(t, i) (t)[i]
#endif
#define tabd(t, i) nm_d(NM_LD(t, i))
// The reads that always come in pairs or quadruples can be served together
// (an includer storing the tables interleaved: one wide read each):
//   NM_SINCOS4(k, sn, ssn, cs, ccs)  kG_SINCOSTAB[k .. k+3] (k a multiple of 4)
//   NM_TAN2(j, hi, lo)               kT_TAN_HI[j], kT_TAN_LO[j]
//   NM_KNOT2(k, a, n)                kRCP14_KNOT[k], kRCP14_KNOT[k+1] (k even)
//   NM_LOG2(f, hi, lo), NM_EXP2(j, hi, lo)  kP_LOG_HI/LO[f], kP_EXP_HI/LO[j]
#ifndef NM_SINCOS4
#define NM_SINCOS4(k, a, b, c, d) \
  (a = tabd(kG_SINCOSTAB, k), b = tabd(kG_SINCOSTAB, (k) + 1), c = tabd(kG_SINCOSTAB, (k) + 2), \
   d = tabd(kG_SINCOSTAB, (k) + 3))
#endif
#ifndef NM_TAN2
#define NM_TAN2(j, hi, lo) (hi = tabd(kT_TAN_HI, j), lo = tabd(kT_TAN_LO, j))
#endif
#ifndef NM_KNOT2
#define NM_KNOT2(k, a, n) (a = NM_LD(kRCP14_KNOT, k), n = NM_LD(kRCP14_KNOT, (k) + 1))
#endif
#ifndef NM_LOG2
#define NM_LOG2(f, hi, lo) (hi = tabd(kP_LOG_HI, f), lo = tabd(kP_LOG_LO, f))
#endif
#ifndef NM_EXP2
#define NM_EXP2(j, hi, lo) (hi = tabd(kP_EXP_HI, j), lo = tabd(kP_EXP_LO, j))
#endif
// NM_ISSUE_FENCE(): the table reads above it are issued before the work below
// (e.g. a scheduling barrier); nothing on the host
#ifndef NM_ISSUE_FENCE
#define NM_ISSUE_FENCE()
#endif
// NM_RARE(c): the condition of a rarely taken branch (an includer's static
// analysis build may compile those branches away; default: the condition)
#ifndef NM_RARE
#define NM_RARE(c) (c)
#endif
// NM_RARE_ANY(c): the same for a branch the caller may take for every lane
// (a device build makes it wave-uniform)
#ifndef NM_RARE_ANY
#define NM_RARE_ANY(c) NM_RARE(c)
#endif

// ---------------------------------------------------------------------------
// VRCP14PD: the result depends on the sign, the exponent and the top 16
// fraction bits i of the input; its 16 fraction bits are the fixed-point
// interpolation (A[k] - N[k] o) >> 10, k = i >> 10, o = i & 1023 (knots
// recovered from the instruction itself for every i, tools/gen_np_math.py).
// An exact power of two has its exact reciprocal.  Normal inputs whose
// reciprocal is normal.
// ---------------------------------------------------------------------------
// (rcp14_knot: the knot index of x; nm_rcp14_k: the reciprocal given its knots)
NM_FN unsigned rcp14_knot(double x) { return 2u * ((unsigned)(nm_u(x) >> 46) & 63u); }
NM_FN double nm_rcp14_k(double x, unsigned A, unsigned N) {
  const unsigned long long u = nm_u(x);
  const unsigned long long e = (u >> 52) & 0x7FF;
  const unsigned long long s = u & 0x8000000000000000ull;
  const unsigned o = (unsigned)(u >> 36) & 1023u;
  const unsigned f = (A - N * o) >> 10;
  const double p2 = nm_d(s | ((2046ull - e) << 52));          // 2^-(e-1023)
  const double r = nm_d(s | ((2045ull - e) << 52) | ((unsigned long long)f << 36));
  return (u & 0x000FFFFFFFFFFFFFull) == 0 ? p2 : r;
}
NM_FN double nm_rcp14(double x) {
  const unsigned k = rcp14_knot(x);
  unsigned A, N;
  NM_KNOT2(k, A, N);
  return nm_rcp14_k(x, A, N);
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
// sincostab index of the table point nearest |x| (x + BIG rounds |x| to
// 1/128); clamped for arguments off the table (their value is not selected)
NM_FN unsigned g_index(double x) {
  const unsigned k = (unsigned)nm_u(nm_d(kG_BIG) + nm_abs(x)) << 2;
  return k < 436u ? k : 436u;
}
// sin and cos of the table point k as double-doubles
struct GTab {
  double sn, ssn, cs, ccs;
};
NM_FN GTab g_tab(unsigned k) {
  GTab T;
  NM_SINCOS4(k, T.sn, T.ssn, T.cs, T.ccs);
  return T;
}
// do_sin(x, dx) with the table entry of x fetched by the caller (below 0.126
// the Taylor branch's value is returned)
NM_FN double g_do_sin_t(double x, double dx, const GTab& T) {
  const double ts = g_taylor_sin(x, dx);                      // |x| < 0.126
  dx = (0.0 < x) ? dx : -dx;                                  // x <= 0 (or NaN): -dx
  const double ax = nm_abs(x);
  const double u = nm_d(kG_BIG) + ax;
  const double xr = ax - (u - nm_d(kG_BIG));
  const double xx = xr * xr;
  const double t = nm_fma(nm_d(kG_SN5), xx, nm_d(kG_SN3));
  const double s = xr + nm_fma(xr * xx, t, dx);
  double c0 = nm_fma(nm_d(kG_CS6), xx, nm_d(kG_CS4));
  c0 = nm_fma(c0, xx, nm_d(kG_CS2));
  const double c = nm_fma(xr, dx, xx * c0);
  const double cor = nm_fma(s, T.cs, nm_fma(-c, T.sn, nm_fma(T.ccs, s, T.ssn)));
  return nm_abs(x) < nm_d(kG_T126) ? ts : nm_copysign(T.sn + cor, x);
}
// do_cos(x, dx), the same
NM_FN double g_do_cos_t(double x, double dx, const GTab& T) {
  dx = (x < 0.0) ? -dx : dx;
  const double ax = nm_abs(x);
  const double u = nm_d(kG_BIG) + ax;
  const double xr = (ax - (u - nm_d(kG_BIG))) + dx;
  const double xx = xr * xr;
  const double t = nm_fma(nm_d(kG_SN5), xx, nm_d(kG_SN3));
  const double s = nm_fma(xr * xx, t, xr);
  double c0 = nm_fma(nm_d(kG_CS6), xx, nm_d(kG_CS4));
  c0 = nm_fma(c0, xx, nm_d(kG_CS2));
  const double c = xx * c0;
  const double cor = nm_fma(-s, T.sn, nm_fma(-c, T.cs, nm_fma(-s, T.ssn, T.ccs)));
  return T.cs + cor;
}
NM_FN double g_do_sin(double x, double dx) { return g_do_sin_t(x, dx, g_tab(g_index(x))); }
NM_FN double g_do_cos(double x, double dx) { return g_do_cos_t(x, dx, g_tab(g_index(x))); }
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
  if (NM_RARE(true)) {                                        // |x| >= 2.426265 (rare)
    if (k < 0x419921FBu) {                                    // |x| < 105414350
      double a, da;
      const int n = g_reduce(x, a, da);
      return g_do_sincos(a, da, n);
    }
    return NM_FALLBACK_SIN(x);
  }
  return x;   // (not reached)
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
  if (NM_RARE(true)) {                                        // |x| >= 2.426265 (rare)
    if (k < 0x419921FBu) {
      double a, da;
      const int n = g_reduce(x, a, da);
      return g_do_sincos(a, da, n + 1);
    }
    return NM_FALLBACK_COS(x);
  }
  return x;   // (not reached)
}

// sin and cos of one argument, bit for bit nm_sin(x) and nm_cos(x), with the
// work shared: below |x| = 2.426265 (every latitude) each of the two is one
// of glibc's do_sin / do_cos evaluations, and the pair is always one of each
// -- (do_sin(x, 0), do_cos(x, 0)) below 0.855469, (do_cos(pi/2 - |x|, pi/2
// tail), do_sin of the same point as a double-double) above -- so a lane
// evaluates exactly one do_sin and one do_cos whichever range it is in.
// (without the arguments |x| >= 2.426265, inf and NaN: nm_sincos below)
// split so that a caller can place work between the table reads and their
// use: nm_sincos_tab issues the two lookups, nm_sincos_fin evaluates
struct SinCosPre {
  GTab Ts, Tc;
};
// The two evaluations read the table points of x and x (below 0.855469) or
// of a = t + pi/2 tail and t (above), and a is within an ulp of t: the two
// points are one unless t lies within an ulp of a 1/128 rounding midpoint.
// (Reading one entry, and the second only where the two differ, halves the
// lane-random table reads -- the kernels' LDS bank conflicts, 0.187 -> 0.148
// of LDS-active cycles -- but measured 0.955x on C3: the wave-uniform branch's
// SGPRs add spill moves to the run kernel, profiles/r5/sched/sincos_entry.txt.)
NM_FN SinCosPre nm_sincos_tab(double x) {
  const bool far = g_hi(x) >= 0x3FEB6000u;
  const double t = nm_d(kG_HP0) - nm_abs(x);
  const double a = t + nm_d(kG_HP1);
  return SinCosPre{g_tab(g_index(far ? a : x)), g_tab(g_index(far ? t : x))};
}
NM_FN void nm_sincos_fin(double x, const SinCosPre& P, double& sn, double& cs) {
  const unsigned k = g_hi(x);
  const bool far = k >= 0x3FEB6000u;
  const double t = nm_d(kG_HP0) - nm_abs(x);
  const double a = t + nm_d(kG_HP1);
  const double da = (t - a) + nm_d(kG_HP1);
  const double S = g_do_sin_t(far ? a : x, far ? da : 0.0, P.Ts);
  const double C = g_do_cos_t(far ? t : x, far ? nm_d(kG_HP1) : 0.0, P.Tc);
  sn = far ? nm_copysign(C, x) : S;
  cs = far ? S : C;
  sn = (k < 0x3E500000u) ? x : sn;
  cs = (k < 0x3E400000u) ? 1.0 : cs;
}
NM_FN void nm_sincos_main(double x, double& sn, double& cs) {
  const SinCosPre P = nm_sincos_tab(x);
  NM_ISSUE_FENCE();
  nm_sincos_fin(x, P, sn, cs);
}
NM_FN bool nm_sincos_rare(double x) { return !(g_hi(x) < 0x400368FDu); }
NM_FN void nm_sincos(double x, double& sn, double& cs) {
  nm_sincos_main(x, sn, cs);
  if (NM_RARE(nm_sincos_rare(x))) {                                    // |x| >= 2.426265, inf, NaN (rare)
    sn = nm_sin(x);
    cs = nm_cos(x);
  }
}

// ---------------------------------------------------------------------------
// SVML __svml_tan8_ha (main path, |x| <= 65536): x = n pi/16 + r,
// tan x = (T + tan r) / (1 - T tan r), T = tan(n pi/16) in head + tail
// ---------------------------------------------------------------------------
// (without |x| > 65536, inf and NaN: nm_tan below).  t_index: the table
// point j of x; nm_tan_t: tan x given T = tan(j pi/16) as head + tail.
NM_FN int t_index(double x) { return (int)(nm_u(nm_fma(nm_d(kT_INVPI16), x, nm_d(kT_SHIFT))) & 15); }
// in two stages around the reciprocal's knot read: nm_tan_pre up to D = 1 -
// T tan r, nm_tan_fin from rcp14(D) on
struct TanPre {
  double N, Nl, D, dl;
};
NM_FN TanPre nm_tan_pre(double x, double T, double Tl) {
  const double y = nm_fma(nm_d(kT_INVPI16), x, nm_d(kT_SHIFT));
  const double n = y - nm_d(kT_SHIFT);
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
  const double N = th + T;
  const double nl = (th - (N - T)) + Tl;
  const double D = nm_fma(-th, T, nm_d(kT_ONE));
  const double Nl = nl + tl;
  double dl = nm_fma(th, T, D - nm_d(kT_ONE));
  dl = nm_fma(tl, T, dl);
  dl = nm_fma(th, Tl, dl);
  return TanPre{N, Nl, D, dl};
}
NM_FN double nm_tan_fin(const TanPre& t, unsigned A, unsigned Nk) {
  double rc = nm_rcp14_k(t.D, A, Nk);
  double e = nm_fma(-t.D, rc, nm_d(kT_ONE));
  e = nm_fma(t.dl, rc, e);
  rc = nm_fma(e, rc, rc);
  const double q = rc * t.N;
  double res = nm_fma(q, t.D, -t.N);
  res = nm_fma(-q, t.dl, res);
  return nm_fma(-rc, res - t.Nl, q);
}
NM_FN double nm_tan_t(double x, double T, double Tl) {
  const TanPre t = nm_tan_pre(x, T, Tl);
  const unsigned k = rcp14_knot(t.D);
  unsigned A, N;
  NM_KNOT2(k, A, N);
  return nm_tan_fin(t, A, N);
}
NM_FN double nm_tan_main(double x) {
  const int j = t_index(x);
  double T, Tl;
  NM_TAN2(j, T, Tl);
  return nm_tan_t(x, T, Tl);
}
NM_FN double nm_tan(double x) {
  const double v = nm_tan_main(x);
  if (!(nm_abs(x) <= nm_d(kT_BIGARG)))                        // |x| > 65536, inf, NaN (rare)
    return (x != x || nm_abs(x) == __builtin_inf()) ? x - x : NM_FALLBACK_TAN(x);
  return v;
}

// sin, cos and tan of one argument (the RHS's latitude): one straight-line
// block for the three, one rare-argument branch
//   reads: tan's table point, sin/cos's two | tan up to 1 - T tan r, the
//   reciprocal's knots | sin and cos | tan
NM_FN void nm_sincostan(double x, double& sn, double& cs, double& tn) {
  const int j = t_index(x);
  double T, Tl;
  NM_TAN2(j, T, Tl);
  const SinCosPre P = nm_sincos_tab(x);
  NM_ISSUE_FENCE();
  const TanPre tp = nm_tan_pre(x, T, Tl);
  const unsigned k = rcp14_knot(tp.D);
  unsigned A, Nk;
  NM_KNOT2(k, A, Nk);
  NM_ISSUE_FENCE();
  nm_sincos_fin(x, P, sn, cs);
  tn = nm_tan_fin(tp, A, Nk);
  if (NM_RARE(nm_sincos_rare(x))) {                                    // |x| >= 2.426265, inf, NaN (rare)
    sn = nm_sin(x);
    cs = nm_cos(x);
    tn = nm_tan(x);
  }
}
// The same in two halves, so that a caller can place independent work
// (the RHS: the lookup's cell arithmetic) beside the first half's table reads
// and tan polynomial: nm_sincostan_begin .. nm_sincostan_end(x, ...) gives
// nm_sincostan's values bit for bit (the same operations on the same operands).
struct SinCosTanPre {
  SinCosPre P;
  TanPre tp;
  unsigned A, Nk;
};
NM_FN SinCosTanPre nm_sincostan_begin(double x) {
  SinCosTanPre r;
  const int j = t_index(x);
  double T, Tl;
  NM_TAN2(j, T, Tl);
  r.P = nm_sincos_tab(x);
  NM_ISSUE_FENCE();
  r.tp = nm_tan_pre(x, T, Tl);
  const unsigned k = rcp14_knot(r.tp.D);
  NM_KNOT2(k, r.A, r.Nk);
  return r;
}
NM_FN void nm_sincostan_end(double x, const SinCosTanPre& r, double& sn, double& cs, double& tn) {
  nm_sincos_fin(x, r.P, sn, cs);
  tn = nm_tan_fin(r.tp, r.A, r.Nk);
  if (NM_RARE(nm_sincos_rare(x))) {                                    // |x| >= 2.426265, inf, NaN (rare)
    sn = nm_sin(x);
    cs = nm_cos(x);
    tn = nm_tan(x);
  }
}

// sin OR cos of one argument per lane, one instruction stream for both (the
// lanes of a ray team, csrc/rwrt.hip: lane pairs of the fp64 time-varying loop,
// quads of the latency mode): nm_sincos_fin evaluates one do_sin and one
// do_cos per lane; a lane that wants only sin(x) or only cos(x) needs one of
// them -- do_sin(x, 0) / do_cos(x, 0) below 0.855469, do_cos(t, pi/2 tail) /
// do_sin(a, da) above -- and do_sin_t and do_cos_t are the same operations on
// permuted operands: the table pair (sn, ssn, cs, ccs) read as (cs, ccs, sn,
// ssn), s negated, the tail added to xr or folded into s, the correction
// term's product dropped.  So a sin lane and a cos lane run one stream,
// selecting operands, and read ONE table point each.  Bit for bit nm_sin(x)
// / nm_cos(x) for |x| < 2.426265 (tests/test_np_math.py; the rest: the
// caller's rare branch, nm_sinorcostan_end).
NM_FN unsigned nm_sinorcos_index(double x, bool want_cos) {
  const bool far = g_hi(x) >= 0x3FEB6000u;
  const double t = nm_d(kG_HP0) - nm_abs(x);
  const double a = t + nm_d(kG_HP1);
  return g_index(far ? ((want_cos != far) ? t : a) : x);
}
NM_FN double nm_sinorcos_fin(double x, bool want_cos, const GTab& T) {
  const unsigned k = g_hi(x);
  const bool far = k >= 0x3FEB6000u;
  const double t = nm_d(kG_HP0) - nm_abs(x);
  const double a = t + nm_d(kG_HP1);
  const double da = (t - a) + nm_d(kG_HP1);
  const bool ev_cos = want_cos != far;                         // this lane's evaluation is do_cos
  const double u = far ? (ev_cos ? t : a) : x;
  const double du = far ? (ev_cos ? nm_d(kG_HP1) : da) : 0.0;
  const double ts = g_taylor_sin(u, du);                       // (do_sin, |u| < 0.126)
  const double dxs = ev_cos ? ((u < 0.0) ? -du : du) : ((0.0 < u) ? du : -du);
  const double au = nm_abs(u);
  const double uu = nm_d(kG_BIG) + au;
  const double r0 = au - (uu - nm_d(kG_BIG));
  const double xr = ev_cos ? r0 + dxs : r0;
  const double xx = xr * xr;
  const double tt = nm_fma(nm_d(kG_SN5), xx, nm_d(kG_SN3));
  const double q = nm_fma(xr * xx, tt, ev_cos ? xr : dxs);
  const double s = ev_cos ? q : xr + q;
  double c0 = nm_fma(nm_d(kG_CS6), xx, nm_d(kG_CS4));
  c0 = nm_fma(c0, xx, nm_d(kG_CS2));
  const double m = xx * c0;
  const double c = ev_cos ? m : nm_fma(xr, dxs, m);
  const double P = ev_cos ? T.cs : T.sn, p = ev_cos ? T.ccs : T.ssn;
  const double Q = ev_cos ? T.sn : T.cs, qq = ev_cos ? T.ssn : T.ccs;
  const double s2 = ev_cos ? -s : s;
  const double cor = nm_fma(s2, Q, nm_fma(-c, P, nm_fma(qq, s2, p)));
  const double r = P + cor;
  double v = ev_cos ? r : (nm_abs(u) < nm_d(kG_T126) ? ts : nm_copysign(r, u));
  v = (!want_cos && far) ? nm_copysign(v, x) : v;
  return want_cos ? ((k < 0x3E400000u) ? 1.0 : v) : ((k < 0x3E500000u) ? x : v);
}
// (sin or cos) and tan of one argument in two halves, as nm_sincostan_begin /
// _end: one table point for the trigonometric pair instead of two
struct SinOrCosTanPre {
  GTab T;
  TanPre tp;
  unsigned A, Nk;
};
NM_FN SinOrCosTanPre nm_sinorcostan_begin(double x, bool want_cos) {
  SinOrCosTanPre r;
  const int j = t_index(x);
  double T, Tl;
  NM_TAN2(j, T, Tl);
  r.T = g_tab(nm_sinorcos_index(x, want_cos));
  NM_ISSUE_FENCE();
  r.tp = nm_tan_pre(x, T, Tl);
  const unsigned k = rcp14_knot(r.tp.D);
  NM_KNOT2(k, r.A, r.Nk);
  return r;
}
NM_FN void nm_sinorcostan_end(double x, bool want_cos, const SinOrCosTanPre& r, double& sc, double& tn) {
  sc = nm_sinorcos_fin(x, want_cos, r.T);
  tn = nm_tan_fin(r.tp, r.A, r.Nk);
  if (NM_RARE(nm_sincos_rare(x))) {                                    // |x| >= 2.426265, inf, NaN (rare)
    sc = want_cos ? nm_cos(x) : nm_sin(x);
    tn = nm_tan(x);
  }
}

// ---------------------------------------------------------------------------
// SVML __svml_pow8_ha (main path): log2 x = k + log2 of the table point + a
// degree-10 polynomial in r = (m R - 1) / 2 (R = VRCP14 of the mantissa,
// rounded to 1/32), T = y log2 x by round-toward-zero double-double steps,
// 2^T from a 16-entry table and a degree-7 polynomial
// ---------------------------------------------------------------------------
// pow's special values: x NaN, 0, inf or < 0, y NaN or inf (C99 / IEEE pow,
// what SVML's rare path returns)
NM_FN double nm_pow_special(double x, double y) {
  const double inf = __builtin_inf();
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

NM_FN double nm_pow(double x, double y) {
  const double inf = __builtin_inf();
  const bool xs = !(x > 0.0) || x == inf || x != x;           // vfpclass 0xdf: NaN, 0, inf, < 0
  const bool ys = y != y || nm_abs(y) == inf;                  // vfpclass 0x99
  // vgetmant (interval [0.5, 1)) and vgetexp of x > 0, normal or subnormal
  unsigned long long ux = nm_u(x);
  int ex = (int)((ux >> 52) & 0x7FF) - 1023;
  {                                                            // subnormal: normalise
    const int lz = __builtin_clzll(ux | 1) - 11;
    const bool sub = (ux >> 52) == 0;
    ux = sub ? ux << lz : ux;
    ex = sub ? -1022 - lz : ex;
  }
  const double M = nm_d((ux & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);   // [1, 2)
  const double m = M * 0.5;                                                          // [0.5, 1)
  // VRCP14PD(m), rounded to 5 fraction bits (vrndscalepd 0x58, to nearest even)
  const double rc = nm_rcp14(m);
  const double R = __builtin_rint(rc * 32.0) * 0.03125;
  const int f = (int)((nm_u(R) >> 47) & 31);
  double e = (double)ex;
  if (R < 1.5) e = e + 1.0;
  double Lh, Ll;
  NM_LOG2(f, Lh, Ll);
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
  const bool ovf = !(nm_abs(T) <= nm_d(kP_TOVF));            // over/underflow (rare path)
  // 2^T: T = (k16 + fr) / 16 with fr in [0, 1) (vaddpd {rd-sae} on a shifter
  // and vreducepd 0x41: both the floor at 1/16)
  const double Tm = ovf ? 0.0 : T;                            // (a finite stand-in there)
  const double fl = __builtin_floor(Tm * 16.0);
  const double frac = NM_ADD_RD(Tm, -(fl * 0.0625));   // vreducepd subtracts under its own RD
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
  double Eh, El;
  NM_EXP2(jj, Eh, El);
  p1 = nm_fma(fz, p1, El);
  p1 = nm_fma(Eh, p1, Eh);
  const double scale = nm_d((unsigned long long)(kk + 1023) << 52);
  const double v = p1 * scale;
  if (NM_RARE(xs || ys)) return nm_pow_special(x, y);
  if (NM_RARE(ovf)) return NM_FALLBACK_POW(x, y);
  return v;
}

}  // namespace np_math
