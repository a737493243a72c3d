// nproots.h -- np.roots for polynomials of degree <= 3, operation for operation.
//
// The reference solves the t = 0 dispersion relation with np.roots
// (bs.py:1017-1040 cal_ky_numpy -> numpy/lib/polynomial.py roots), i.e. the
// eigenvalues of the companion matrix from LAPACK zgeev (numpy 2.2.6 linked
// against scipy_openblas 0.3.29, LAPACK 3.12.0).  The ORDER of those
// eigenvalues is what change_roots_order (bs.py:942-982) then permutes, so a
// closed-form cubic cannot reproduce the reference: this header restates the
// exact path for N <= 3
//
//   companion matrix  numpy complex division (npymath cdiv: reciprocal-scaled Smith)
//   zgeev('N','N')    ZLANGE range check, ZGEBAL('B'), ZGEHRD (identity here),
//                     ZHSEQR -> ZLAHQR (wantt = wantz = .false.)
//   ZLAHQR            Ahues-Tisseur deflation, Wilkinson / exceptional shifts,
//                     single-shift QR sweeps with ZLARFG reflectors
//   libm              glibc 2.35 hypot (cabs) and csqrt, restated below
//   BLAS              OpenBLAS dznrm2 (x87 extended sum of squares) and zscal
//
// with IEEE double arithmetic in the same order (compile with
// -ffp-contract=off).  Verified bit-for-bit against numpy's eigvals on the
// reference host (tests/test_nproots.py).  Compiled for the device (init
// kernel) and, for that test only, for the host.
//
// Provenance and licences of the restated algorithms: LAPACK 3.12 (ZGEBAL,
// ZLAHQR, ZLARFG, DLADIV, DLAPY3; modified BSD), OpenBLAS 0.3.29 (dznrm2,
// zscal kernels; BSD-3-Clause), NumPy's npymath complex division
// (BSD-3-Clause), glibc 2.35 hypot / csqrt (LGPL-2.1-or-later).  Written from
// the published algorithms and checked against their results; no source
// file of those projects is copied.
#pragma once
#include <cstdint>
#include <cstring>
#include <cmath>

#ifndef RWRT_HD
#define RWRT_HD __host__ __device__
#endif

namespace nproots {

struct cx {
  double re, im;
};

RWRT_HD inline cx mk(double r, double i) { return cx{r, i}; }
RWRT_HD inline cx add(cx a, cx b) { return cx{a.re + b.re, a.im + b.im}; }
RWRT_HD inline cx sub(cx a, cx b) { return cx{a.re - b.re, a.im - b.im}; }
// gfortran complex multiply (-fcx-fortran-rules: no NaN recovery)
RWRT_HD inline cx mul(cx a, cx b) { return cx{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
// Mixed real/complex operands: Fortran converts the real to (s, 0) and,
// because signed zeros are honoured, GCC lowers the FULL complex operation
// (no component-wise shortcut) -- the sign of a zero imaginary part, which
// decides csqrt's branch in the Wilkinson shift, depends on it.
RWRT_HD inline cx rmul_f(double s, cx a) { return mul(cx{s, 0.0}, a); }
// GCC complex division with Fortran rules (expand_complex_div_wide: Smith)
RWRT_HD inline cx div_f(cx a, cx b) {
  if (fabs(b.re) < fabs(b.im)) {
    const double ratio = b.re / b.im;
    const double div = (b.re * ratio) + b.im;
    const double tr = (a.re * ratio) + a.im;
    const double ti = (a.im * ratio) - a.re;
    return cx{tr / div, ti / div};
  }
  const double ratio = b.im / b.re;
  const double div = (b.im * ratio) + b.re;
  const double tr = (a.im * ratio) + a.re;
  const double ti = a.im - (a.re * ratio);
  return cx{tr / div, ti / div};
}
RWRT_HD inline cx rdiv_f(cx a, double s) { return div_f(a, cx{s, 0.0}); }
// ZDSCAL (OpenBLAS): component-wise, verified on signed zeros
RWRT_HD inline cx zdscal1(double s, cx a) { return cx{s * a.re, s * a.im}; }
// ZSCAL (OpenBLAS x86_64 zscal kernel): a purely real or purely imaginary
// alpha takes a component-wise branch (verified on signed zeros)
RWRT_HD inline cx zscal1(cx a, cx x) {
  if (a.im == 0.0) return cx{a.re * x.re, a.re * x.im};
  if (a.re == 0.0) return cx{-a.im * x.im, a.im * x.re};
  return mul(a, x);
}
RWRT_HD inline cx conj(cx a) { return cx{a.re, -a.im}; }
RWRT_HD inline double cabs1(cx a) { return fabs(a.re) + fabs(a.im); }

// glibc 2.35 __hypot (sysdeps/ieee754/dbl-64/e_hypot.c), non-FMA kernel
// (Borges' correction); finite inputs.
RWRT_HD inline double hypot_kernel(double ax, double ay) {
  double h = sqrt(ax * ax + ay * ay);
  double t1, t2;
  if (h <= 2.0 * ay) {
    const double delta = h - ay;
    t1 = ax * (2.0 * delta - ax);
    t2 = (delta - 2.0 * (ax - ay)) * delta;
  } else {
    const double delta = h - ax;
    t1 = 2.0 * delta * (ax - 2.0 * ay);
    t2 = (4.0 * delta - ay) * ay + delta * delta;
  }
  h -= (t1 + t2) / (2.0 * h);
  return h;
}

RWRT_HD inline double glibc_hypot(double x, double y) {
  if (!isfinite(x) || !isfinite(y)) {
    if ((isinf(x) || isinf(y))) return INFINITY;
    return x + y;
  }
  x = fabs(x);
  y = fabs(y);
  double ax = x < y ? y : x;
  double ay = x < y ? x : y;
  const double kScale = 0x1p-600, kLarge = 0x1p+511, kTiny = 0x1p-511, kEps = 0x1p-54;
  if (ax > kLarge) {
    if (ay <= ax * kEps) return ax + ay;
    return hypot_kernel(ax * kScale, ay * kScale) / kScale;
  }
  if (ay < kTiny) {
    if (ax >= ay / kEps) return ax + ay;
    return hypot_kernel(ax / kScale, ay / kScale) * kScale;
  }
  if (ay <= ax * kEps) return ax + ay;
  return hypot_kernel(ax, ay);
}

RWRT_HD inline double cabs(cx a) { return glibc_hypot(a.re, a.im); }

// glibc 2.35 csqrt (math/s_csqrt_template.c) for finite arguments of normal range.
RWRT_HD inline cx csqrt(cx x) {
  const double re = x.re, im = x.im;
  if (im == 0.0) {
    if (re < 0.0) return cx{0.0, copysign(sqrt(-re), im)};
    return cx{fabs(sqrt(re)), copysign(0.0, im)};
  }
  if (re == 0.0) {
    double r;
    if (fabs(im) >= 2.0 * 2.2250738585072014e-308)
      r = sqrt(0.5 * fabs(im));
    else
      r = 0.5 * sqrt(2.0 * fabs(im));
    return cx{r, copysign(r, im)};
  }
  const double d = glibc_hypot(re, im);
  double r, s;
  if (re > 0.0) {
    r = sqrt(0.5 * (d + re));
    s = 0.5 * (im / r);
  } else {
    s = sqrt(0.5 * (d - re));
    r = fabs(0.5 * (im / s));
  }
  return cx{r, copysign(s, im)};
}

// LAPACK 3.12 DLADIV (Baudin & Smith robust complex division)
RWRT_HD inline double dladiv2(double a, double b, double c, double d, double r, double t) {
  if (r != 0.0) {
    const double br = b * r;
    if (br != 0.0) return (a + br) * t;
    return a * t + (b * t) * r;
  }
  return (a + d * (b / c)) * t;
}

RWRT_HD inline void dladiv1(double a, double b, double c, double d, double& p, double& q) {
  const double r = d / c;
  const double t = 1.0 / (c + d * r);
  p = dladiv2(a, b, c, d, r, t);
  a = -a;
  q = dladiv2(b, a, c, d, r, t);
}

RWRT_HD inline cx zladiv(cx x, cx y) {
  double aa = x.re, bb = x.im, cc = y.re, dd = y.im;
  double ab = fmax(fabs(x.re), fabs(x.im));
  double cd = fmax(fabs(y.re), fabs(y.im));
  double s = 1.0;
  const double ov = 1.7976931348623157e308, un = 2.2250738585072014e-308, eps = 0x1p-53;
  const double be = 2.0 / (eps * eps);
  if (ab >= 0.5 * ov) { aa = 0.5 * aa; bb = 0.5 * bb; s = 2.0 * s; }
  if (cd >= 0.5 * ov) { cc = 0.5 * cc; dd = 0.5 * dd; s = 0.5 * s; }
  if (ab <= un * 2.0 / eps) { aa = aa * be; bb = bb * be; s = s / be; }
  if (cd <= un * 2.0 / eps) { cc = cc * be; dd = dd * be; s = s * be; }
  double p, q;
  if (fabs(y.im) <= fabs(y.re)) {
    dladiv1(aa, bb, cc, dd, p, q);
  } else {
    dladiv1(bb, aa, dd, cc, p, q);
    q = -q;
  }
  return cx{p * s, q * s};
}

// LAPACK 3.12 DLAPY3
RWRT_HD inline double dlapy3(double x, double y, double z) {
  const double hugeval = 1.7976931348623157e308;
  const double xa = fabs(x), ya = fabs(y), za = fabs(z);
  const double w = fmax(xa, fmax(ya, za));
  if (w == 0.0 || w > hugeval) return xa + ya + za;
  const double a = xa / w, b = ya / w, c = za / w;
  return w * sqrt(a * a + b * b + c * c);
}

// --- OpenBLAS dznrm2 (znrm2_k, kernel/x86_64/znrm2.S) ----------------------
// x87 code: squares and sums in 64-bit-mantissa extended precision, the real
// parts' squares in one accumulator and the imaginary parts' in another,
// total = (0 + A_re) + A_im, fsqrt, then one rounding to double (fstpl).
// Restated with a small soft float: value = m * 2^e, m a normalised 64-bit
// mantissa, round-to-nearest-even at every step (non-negative operands only).
struct Ext {
  uint64_t m;
  int e;
};
typedef unsigned __int128 u128;

RWRT_HD inline int clz128(u128 v) {
  const uint64_t hi = (uint64_t)(v >> 64), lo = (uint64_t)v;
  return hi ? __builtin_clzll(hi) : (lo ? 64 + __builtin_clzll(lo) : 128);
}

// round a 128-bit mantissa P (value P * 2^e0, P != 0) with extra sticky bits to 64 bits
RWRT_HD inline Ext ext_round(u128 P, int e0, bool sticky) {
  const int lz = clz128(P);
  P <<= lz;
  uint64_t m = (uint64_t)(P >> 64);
  const uint64_t low = (uint64_t)P;
  int e = e0 - lz + 64;
  const uint64_t half = 1ull << 63;
  if (low > half || (low == half && (sticky || (m & 1)))) {
    m += 1;
    if (m == 0) { m = 1ull << 63; e += 1; }
  }
  return Ext{m, e};
}

RWRT_HD inline Ext ext_sq(double x) {
  x = fabs(x);
  if (x == 0.0) return Ext{0, 0};
  uint64_t bits;
  memcpy(&bits, &x, 8);
  const int E = (int)(bits >> 52);
  uint64_t mx = bits & ((1ull << 52) - 1);
  int ex;
  if (E == 0) {
    ex = -1074;
  } else {
    mx |= 1ull << 52;
    ex = E - 1075;
  }
  return ext_round((u128)mx * mx, 2 * ex, false);
}

RWRT_HD inline Ext ext_add(Ext a, Ext b) {
  if (b.m == 0) return a;
  if (a.m == 0) return b;
  if (a.e < b.e) { const Ext t = a; a = b; b = t; }
  const int d = a.e - b.e;
  const u128 A = (u128)a.m << 64;
  u128 B = (u128)b.m << 64;
  bool sticky = false;
  if (d >= 128) {
    sticky = true;
    B = 0;
  } else if (d > 0) {
    sticky = (B << (128 - d)) != 0;
    B >>= d;
  }
  u128 S = A + B;
  int e0 = a.e - 64;
  if (S < A) {   // carry out of 128 bits
    sticky = sticky || (S & 1);
    S = (S >> 1) | ((u128)1 << 127);
    e0 += 1;
  }
  return ext_round(S, e0, sticky);
}

RWRT_HD inline Ext ext_sqrt(Ext a) {
  if (a.m == 0) return a;
  u128 N;
  int eh;
  if (a.e & 1) { N = (u128)a.m << 63; eh = (a.e - 63) / 2; }
  else { N = (u128)a.m << 64; eh = (a.e - 64) / 2; }
  // floor(sqrt(N)), N in [2^126, 2^128): double estimate, one corrective
  // step, then exact integer fix-up
  uint64_t r = (uint64_t)fmin(sqrt((double)N), 18446744073709549568.0);
  for (int it = 0; it < 2; ++it) {
    const u128 rr = (u128)r * r;
    const double diff = (rr > N) ? -(double)(rr - N) : (double)(N - rr);
    const double corr = diff / (2.0 * (double)r);
    const double rn = (double)r + corr;
    r = (uint64_t)fmin(fmax(rn, 9223372036854775808.0), 18446744073709549568.0);
  }
  while ((u128)r * r > N) --r;
  while (r != ~0ull && (u128)(r + 1) * (r + 1) <= N) ++r;
  const u128 rem = N - (u128)r * r;
  if (rem > (u128)r) {   // (r + 1/2)^2 = r^2 + r + 1/4 < N
    r += 1;
    if (r == 0) return Ext{1ull << 63, eh + 64 + 1 - 64};
  }
  return Ext{r, eh};
}

RWRT_HD inline double ext_to_double(Ext a) {
  if (a.m == 0) return 0.0;
  uint64_t mm = a.m >> 11;
  const uint64_t low = a.m & 0x7FF;
  int e = a.e + 11;
  if (low > 0x400 || (low == 0x400 && (mm & 1))) {
    mm += 1;
    if (mm == (1ull << 53)) { mm >>= 1; e += 1; }
  }
  return ldexp((double)mm, e);
}

template <int N>
RWRT_HD inline double dznrm2(const cx* x, int n, int inc) {
  Ext a0{0, 0}, a1{0, 0};
  for (int i = 0; i < n; ++i) {
    a0 = ext_add(a0, ext_sq(x[i * inc].re));
    a1 = ext_add(a1, ext_sq(x[i * inc].im));
  }
  return ext_to_double(ext_sqrt(ext_add(a0, a1)));
}

// LAPACK 3.12 ZLARFG for n = 2: alpha, x (one element); returns tau.
RWRT_HD inline cx zlarfg2(cx& alpha, cx& x) {
  const double xnorm = dznrm2<1>(&x, 1, 1);
  double alphr = alpha.re, alphi = alpha.im;
  if (xnorm == 0.0 && alphi == 0.0) return cx{0.0, 0.0};
  double beta = -copysign(dlapy3(alphr, alphi, xnorm), alphr);
  const double safmin = 2.2250738585072014e-308 / 0x1p-53;
  const double rsafmn = 1.0 / safmin;
  int knt = 0;
  if (fabs(beta) < safmin) {
    do {
      ++knt;
      x = zdscal1(rsafmn, x);
      beta = beta * rsafmn;
      alphi = alphi * rsafmn;
      alphr = alphr * rsafmn;
    } while (fabs(beta) < safmin && knt < 20);
    const double xn = dznrm2<1>(&x, 1, 1);
    alpha = cx{alphr, alphi};
    beta = -copysign(dlapy3(alphr, alphi, xn), alphr);
  }
  const cx tau{(beta - alphr) / beta, -alphi / beta};
  const cx a = zladiv(cx{1.0, 0.0}, cx{alpha.re - beta, alpha.im - 0.0});   // ALPHA - (BETA, 0)
  x = zscal1(a, x);   // ZSCAL(1, alpha, x)
  for (int j = 0; j < knt; ++j) beta = beta * safmin;
  alpha = cx{beta, 0.0};
  return tau;
}

// Column-major N x N complex matrix, H(i, j) with 1-based indices as in LAPACK.
template <int N>
struct Mat {
  cx a[N * N];
  RWRT_HD cx& operator()(int i, int j) { return a[(j - 1) * N + (i - 1)]; }
};


// LAPACK 3.12 ZGEBAL('B') restricted to what companion matrices can reach;
// returns ilo, ihi (scale factors are not needed for eigenvalues).
template <int N>
RWRT_HD inline void zgebal(Mat<N>& A, int& ilo, int& ihi) {
  int k = 1, l = N;
  // permutations: search rows isolating an eigenvalue, push them down
  bool noconv = true;
  while (noconv) {
    noconv = false;
    for (int i = l; i >= 1; --i) {
      bool canswap = true;
      for (int j = 1; j <= l; ++j)
        if (i != j && (A(i, j).re != 0.0 || A(i, j).im != 0.0)) { canswap = false; break; }
      if (canswap) {
        if (i != l) {
          for (int r = 1; r <= l; ++r) { cx t = A(r, i); A(r, i) = A(r, l); A(r, l) = t; }
          for (int c = k; c <= N; ++c) { cx t = A(i, c); A(i, c) = A(l, c); A(l, c) = t; }
        }
        noconv = true;
        if (l == 1) { ilo = 1; ihi = 1; return; }
        l = l - 1;
      }
    }
  }
  noconv = true;
  while (noconv) {
    noconv = false;
    for (int j = k; j <= l; ++j) {
      bool canswap = true;
      for (int i = k; i <= l; ++i)
        if (i != j && (A(i, j).re != 0.0 || A(i, j).im != 0.0)) { canswap = false; break; }
      if (canswap) {
        if (j != k) {
          for (int r = 1; r <= l; ++r) { cx t = A(r, j); A(r, j) = A(r, k); A(r, k) = t; }
          for (int c = k; c <= N; ++c) { cx t = A(j, c); A(j, c) = A(k, c); A(k, c) = t; }
        }
        noconv = true;
        k = k + 1;
      }
    }
  }
  double scale[N];
  for (int i = k; i <= l; ++i) scale[i - 1] = 1.0;
  const double sclfac = 2.0, factor = 0.95;
  const double sfmin1 = 2.2250738585072014e-308 / 0x1p-52;
  const double sfmax1 = 1.0 / sfmin1;
  const double sfmin2 = sfmin1 * sclfac;
  const double sfmax2 = 1.0 / sfmin2;
  noconv = true;
  while (noconv) {
    noconv = false;
    for (int i = k; i <= l; ++i) {
      cx col[N], row[N];
      for (int r = k; r <= l; ++r) { col[r - k] = A(r, i); row[r - k] = A(i, r); }
      double c = dznrm2<N>(col, l - k + 1, 1);
      double r = dznrm2<N>(row, l - k + 1, 1);
      int ica = 1;
      double best = -1.0;
      for (int q = 1; q <= l; ++q) {
        const double v = cabs1(A(q, i));
        if (v > best) { best = v; ica = q; }
      }
      double ca = cabs(A(ica, i));
      int ira = 1;
      best = -1.0;
      for (int q = 1; q <= N - k + 1; ++q) {
        const double v = cabs1(A(i, q + k - 1));
        if (v > best) { best = v; ira = q; }
      }
      double ra = cabs(A(i, ira + k - 1));
      if (c == 0.0 || r == 0.0) continue;
      if (isnan(c + ca + r + ra)) { ilo = k; ihi = l; return; }
      double g = r / sclfac;
      double f = 1.0;
      const double s = c + r;
      while (c < g && fmax(f, fmax(c, ca)) < sfmax2 && fmin(r, fmin(g, ra)) > sfmin2) {
        f = f * sclfac;
        c = c * sclfac;
        ca = ca * sclfac;
        r = r / sclfac;
        g = g / sclfac;
        ra = ra / sclfac;
      }
      g = c / sclfac;
      while (g >= r && fmax(r, ra) < sfmax2 && fmin(fmin(f, c), fmin(g, ca)) > sfmin2) {
        f = f / sclfac;
        c = c / sclfac;
        g = g / sclfac;
        ca = ca / sclfac;
        r = r * sclfac;
        ra = ra * sclfac;
      }
      if ((c + r) >= factor * s) continue;
      if (f < 1.0 && scale[i - 1] < 1.0) {
        if (f * scale[i - 1] <= sfmin1) continue;
      }
      if (f > 1.0 && scale[i - 1] > 1.0) {
        if (scale[i - 1] >= sfmax1 / f) continue;
      }
      g = 1.0 / f;
      scale[i - 1] = scale[i - 1] * f;
      noconv = true;
      for (int q = k; q <= N; ++q) A(i, q) = zdscal1(g, A(i, q));   // ZDSCAL row
      for (int q = 1; q <= l; ++q) A(q, i) = zdscal1(f, A(q, i));   // ZDSCAL column
    }
  }
  ilo = k;
  ihi = l;
}

// LAPACK 3.12 ZLAHQR with WANTT = WANTZ = .FALSE.; eigenvalues into w[0..N).
// Returns INFO (0 = converged).
template <int N>
RWRT_HD inline int zlahqr(Mat<N>& H, int ilo, int ihi, cx* w) {
  if (ilo == ihi) {
    w[ilo - 1] = H(ilo, ilo);
    return 0;
  }
  for (int j = ilo; j <= ihi - 3; ++j) {
    H(j + 2, j) = cx{0.0, 0.0};
    H(j + 3, j) = cx{0.0, 0.0};
  }
  if (ilo <= ihi - 2) H(ihi, ihi - 2) = cx{0.0, 0.0};
  const int jlo = ilo, jhi = ihi;
  for (int i = ilo + 1; i <= ihi; ++i) {
    if (H(i, i - 1).im != 0.0) {
      cx sc = rdiv_f(H(i, i - 1), cabs1(H(i, i - 1)));
      sc = rdiv_f(conj(sc), cabs(sc));
      H(i, i - 1) = cx{cabs(H(i, i - 1)), 0.0};
      for (int q = i; q <= jhi; ++q) H(i, q) = zscal1(sc, H(i, q));
      const int hi = (jhi < i + 1) ? jhi : i + 1;
      for (int q = jlo; q <= hi; ++q) H(q, i) = zscal1(conj(sc), H(q, i));
    }
  }
  const int nh = ihi - ilo + 1;
  const double safmin = 2.2250738585072014e-308;
  const double ulp = 0x1p-52;
  const double smlnum = safmin * ((double)nh / ulp);
  const int itmax = 30 * (nh > 10 ? nh : 10);
  const double dat1 = 3.0 / 4.0;
  const int kexsh = 10;
  int kdefl = 0;
  int i = ihi;
  while (i >= ilo) {
    int l = ilo;
    bool converged = false;
    for (int its = 0; its <= itmax; ++its) {
      int k;
      for (k = i; k >= l + 1; --k) {
        if (cabs1(H(k, k - 1)) <= smlnum) break;
        double tst = cabs1(H(k - 1, k - 1)) + cabs1(H(k, k));
        if (tst == 0.0) {
          if (k - 2 >= ilo) tst = tst + fabs(H(k - 1, k - 2).re);
          if (k + 1 <= ihi) tst = tst + fabs(H(k + 1, k).re);
        }
        if (fabs(H(k, k - 1).re) <= ulp * tst) {
          const double ab = fmax(cabs1(H(k, k - 1)), cabs1(H(k - 1, k)));
          const double ba = fmin(cabs1(H(k, k - 1)), cabs1(H(k - 1, k)));
          const double aa = fmax(cabs1(H(k, k)), cabs1(sub(H(k - 1, k - 1), H(k, k))));
          const double bb = fmin(cabs1(H(k, k)), cabs1(sub(H(k - 1, k - 1), H(k, k))));
          const double s = aa + ab;
          if (ba * (ab / s) <= fmax(smlnum, ulp * (bb * (aa / s)))) break;
        }
      }
      l = k;
      if (l > ilo) H(l, l - 1) = cx{0.0, 0.0};
      if (l >= i) { converged = true; break; }
      kdefl = kdefl + 1;
      const int i1 = l, i2 = i;
      cx t;
      if (kdefl % (2 * kexsh) == 0) {
        const double s = dat1 * fabs(H(i, i - 1).re);
        t = cx{s + H(i, i).re, 0.0 + H(i, i).im};   // (S, 0) + H(I, I)
      } else if (kdefl % kexsh == 0) {
        const double s = dat1 * fabs(H(l + 1, l).re);
        t = cx{s + H(l, l).re, 0.0 + H(l, l).im};
      } else {
        t = H(i, i);
        const cx u = mul(csqrt(H(i - 1, i)), csqrt(H(i, i - 1)));
        double s = cabs1(u);
        if (s != 0.0) {
          const cx x = rmul_f(0.5, sub(H(i - 1, i - 1), t));
          const double sx = cabs1(x);
          s = fmax(s, cabs1(x));
          const cx xs = rdiv_f(x, s), us = rdiv_f(u, s);
          cx y = rmul_f(s, csqrt(add(mul(xs, xs), mul(us, us))));
          if (sx > 0.0) {
            const cx xx = rdiv_f(x, sx);
            if (xx.re * y.re + xx.im * y.im < 0.0) y = cx{-y.re, -y.im};
          }
          t = sub(t, mul(u, zladiv(u, add(x, y))));
        }
      }
      int m;
      cx v[2];
      for (m = i - 1; m >= l + 1; --m) {
        const cx h11 = H(m, m), h22 = H(m + 1, m + 1);
        cx h11s = sub(h11, t);
        double h21 = H(m + 1, m).re;
        const double s = cabs1(h11s) + fabs(h21);
        h11s = rdiv_f(h11s, s);
        h21 = h21 / s;
        v[0] = h11s;
        v[1] = cx{h21, 0.0};
        const double h10 = H(m, m - 1).re;
        if (fabs(h10) * fabs(h21) <= ulp * (cabs1(h11s) * (cabs1(h11) + cabs1(h22)))) break;
      }
      if (m == l) {
        const cx h11 = H(l, l);
        cx h11s = sub(h11, t);
        double h21 = H(l + 1, l).re;
        const double s = cabs1(h11s) + fabs(h21);
        h11s = rdiv_f(h11s, s);
        h21 = h21 / s;
        v[0] = h11s;
        v[1] = cx{h21, 0.0};
      }
      for (int kk = m; kk <= i - 1; ++kk) {
        if (kk > m) {
          v[0] = H(kk, kk - 1);
          v[1] = H(kk + 1, kk - 1);
        }
        const cx t1 = zlarfg2(v[0], v[1]);
        if (kk > m) {
          H(kk, kk - 1) = v[0];
          H(kk + 1, kk - 1) = cx{0.0, 0.0};
        }
        const cx v2 = v[1];
        const double t2 = mul(t1, v2).re;
        for (int j = kk; j <= i2; ++j) {
          const cx sum = add(mul(conj(t1), H(kk, j)), rmul_f(t2, H(kk + 1, j)));
          H(kk, j) = sub(H(kk, j), sum);
          H(kk + 1, j) = sub(H(kk + 1, j), mul(sum, v2));
        }
        const int jend = (kk + 2 < i) ? kk + 2 : i;
        for (int j = i1; j <= jend; ++j) {
          const cx sum = add(mul(t1, H(j, kk)), rmul_f(t2, H(j, kk + 1)));
          H(j, kk) = sub(H(j, kk), sum);
          H(j, kk + 1) = sub(H(j, kk + 1), mul(sum, conj(v2)));
        }
        if (kk == m && m > l) {
          cx temp = sub(cx{1.0, 0.0}, t1);   // ONE - T1
          temp = rdiv_f(temp, cabs(temp));
          H(m + 1, m) = mul(H(m + 1, m), conj(temp));
          if (m + 2 <= i) H(m + 2, m + 1) = mul(H(m + 2, m + 1), temp);
          for (int j = m; j <= i; ++j) {
            if (j != m + 1) {
              if (i2 > j)
                for (int q = j + 1; q <= i2; ++q) H(j, q) = zscal1(temp, H(j, q));
              for (int q = i1; q <= j - 1; ++q) H(q, j) = zscal1(conj(temp), H(q, j));
            }
          }
        }
      }
      cx temp = H(i, i - 1);
      if (temp.im != 0.0) {
        const double rtemp = cabs(temp);
        H(i, i - 1) = cx{rtemp, 0.0};
        temp = rdiv_f(temp, rtemp);
        if (i2 > i)
          for (int q = i + 1; q <= i2; ++q) H(i, q) = zscal1(conj(temp), H(i, q));
        for (int q = i1; q <= i - 1; ++q) H(q, i) = zscal1(temp, H(q, i));
      }
    }
    if (!converged) return i;
    w[i - 1] = H(i, i);
    kdefl = 0;
    i = l - 1;
  }
  return 0;
}

// numpy complex division a / b (npymath: reciprocal-scaled Smith)
RWRT_HD inline cx np_cdiv(cx a, cx b) {
  const double ar = fabs(b.re), ai = fabs(b.im);
  if (ar >= ai) {
    if (ar == 0.0 && ai == 0.0) return cx{a.re / ar, a.im / ai};
    const double rat = b.im / b.re;
    const double scl = 1.0 / (b.re + b.im * rat);
    return cx{(a.re + a.im * rat) * scl, (a.im - a.re * rat) * scl};
  }
  const double rat = b.re / b.im;
  const double scl = 1.0 / (b.im + b.re * rat);
  return cx{(a.re * rat + a.im) * scl, (a.im * rat - a.re) * scl};
}

// zgeev('N', 'N') eigenvalues of the n x n (n <= 3) matrix in A (column-major
// in the leading n*n entries is NOT assumed: A is Mat<NM> with n == NM).
// Returns INFO.
template <int N>
RWRT_HD inline int zgeev_eigvals(Mat<N>& A, cx* w) {
  // ZLANGE('M') range check: data outside [SMLNUM, BIGNUM] would be rescaled
  // by ZLASCL (never for the dispersion relation); report it instead.
  double anrm = 0.0;
  for (int q = 0; q < N * N; ++q) {
    const double v = cabs(A.a[q]);
    if (anrm < v || isnan(v)) anrm = v;
  }
  const double smlnum = sqrt(2.2250738585072014e-308) / 0x1p-52;
  const double bignum = 1.0 / smlnum;
  if (isnan(anrm)) return -1;
  if ((anrm > 0.0 && anrm < smlnum) || anrm > bignum) return -2;
  int ilo, ihi;
  zgebal<N>(A, ilo, ihi);
  // ZGEHRD: the companion matrix is already Hessenberg with real
  // subdiagonal; its ZLARFG reflectors are identities (x = 0, alpha real).
  for (int q = 1; q < ilo; ++q) w[q - 1] = A(q, q);
  for (int q = ihi + 1; q <= N; ++q) w[q - 1] = A(q, q);
  return zlahqr<N>(A, ilo, ihi, w);
}

// np.roots(p) for p = highest-first real coefficients p[0..deg] with
// p[0] != 0 (cal_ky's degree reduction already stripped leading zeros).
// Fills roots[0..deg) in np.roots' order; returns INFO of zgeev.
RWRT_HD inline int np_roots(const double* p, int deg, cx* roots) {
  int last = deg;                    // index of the last non-zero coefficient
  while (last > 0 && p[last] == 0.0) --last;
  const int trailing = deg - last;
  int info = 0;
  const int n = last;                // companion size
  // complex128 coefficients p + 0j; companion first row = -p[1:] / p[0]
  const cx p0{p[0], 0.0};
  if (n == 1) {
    roots[0] = np_cdiv(cx{-p[1], -0.0}, p0);
  } else if (n == 2) {
    Mat<2> A;
    for (int q = 0; q < 4; ++q) A.a[q] = cx{0.0, 0.0};
    A(2, 1) = cx{1.0, 0.0};
    for (int j = 1; j <= 2; ++j) A(1, j) = np_cdiv(cx{-p[j], -0.0}, p0);
    info = zgeev_eigvals<2>(A, roots);
  } else if (n == 3) {
    Mat<3> A;
    for (int q = 0; q < 9; ++q) A.a[q] = cx{0.0, 0.0};
    A(2, 1) = cx{1.0, 0.0};
    A(3, 2) = cx{1.0, 0.0};
    for (int j = 1; j <= 3; ++j) A(1, j) = np_cdiv(cx{-p[j], -0.0}, p0);
    info = zgeev_eigvals<3>(A, roots);
  }
  for (int q = n; q < n + trailing; ++q) roots[q] = cx{0.0, 0.0};
  return info;
}

}  // namespace nproots
