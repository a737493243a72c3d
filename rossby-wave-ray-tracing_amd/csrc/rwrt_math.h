// rwrt_math.h -- the transcendental functions of the ray loop, written out
// operation by operation: sin/cos/tan of one argument with one reduction and
// pow, restating the ROCm device library's (ocml) f64 algorithms.
//
// The kernel (rwrt.hip) uses rm_sincostan_small for the Mercator factors
// (bs.py:856-883) and rm_pow for the step control (rkf45.py:34-99, 453-475);
// on the device both are bit-identical to ocml's sin/cos/tan/pow
// (tests/test_gpu_devmath.py).
//
// The same source also compiles for the HOST (oracle/devmath.cpp): the NumPy
// oracle can then run with the device's transcendentals instead of
// glibc/SVML, which isolates the only difference between the GPU path and
// the reference -- the last bit of libm -- and makes whole 90-day trajectories
// comparable bit for bit (tests/test_gpu_devmath.py).
//
// Everything here is IEEE-754 binary64 arithmetic (+ - * fma, rint, trunc,
// frexp, ldexp, bit casts).  The includer supplies the qualifiers and the two
// primitives whose instruction differs between the targets:
//   RM_FN           function qualifiers
//   RM_FMA3(a,b,c)  fused multiply-add (device: three-operand v_fma_f64)
//   RM_RECIP2(b)    ocml's refined reciprocal, v_rcp_f64 + two Newton steps;
//                   the host uses the IEEE quotient 1/b, which the device
//                   sequence equals (checked on the GPU for both call sites'
//                   argument ranges, tests/test_gpu_devmath.py)
// Compile with -ffp-contract=off.
#pragma once

namespace rwrt_math {

RM_FN double rm_bits(unsigned long long u) { return __builtin_bit_cast(double, u); }
RM_FN unsigned long long rm_ubits(double x) { return __builtin_bit_cast(unsigned long long, x); }

// ---------------------------------------------------------------------------
// sin, cos, tan of |x| < 2^30 (the caller routes larger, infinite and NaN
// arguments to the library): __ocmlpriv_trigredsmall_f64 (Cody-Waite, 3-part
// pi/2), __ocmlpriv_sincosred2_f64, __ocmlpriv_tanred2_f64 and the
// quadrant/sign logic of __ocml_sincos_f64 / __ocml_tan_f64.
// ---------------------------------------------------------------------------
RM_FN void rm_sincostan_small(double x, double& sn, double& cs, double& tn) {
  const double ax = fabs(x);
  // __ocmlpriv_trigredsmall_f64
  const double n = rint(ax * rm_bits(0x3FE45F306DC9C883ull));
  const double a = fma(n, rm_bits(0xBFF921FB54442D18ull), ax);
  const double b = fma(n, rm_bits(0xBC91A62633145C00ull), a);
  const double p = n * rm_bits(0x3C91A62633145C00ull);
  const double pl = fma(n, rm_bits(0x3C91A62633145C00ull), -p);
  const double s1 = a - p;
  const double s2 = (a - s1) - p;
  const double e = (((s1 - b) + s2) - pl);
  const double e2 = fma(n, rm_bits(0xB97B839A252049C0ull), e);
  const double rh = b + e2;                 // reduced argument, head
  const double rl = e2 - (rh - b);          // and tail
  const int q = (int)n & 3;
  // __ocmlpriv_sincosred2_f64(rh, rl)
  const double x2 = rh * rh;
  const double r = x2 * 0.5;
  const double t = 1.0 - r;
  const double u = (1.0 - t) - r;
  const double x4 = x2 * x2;
  double c = RM_FMA3(x2, rm_bits(0xBDA907DB46CC5E42ull), rm_bits(0x3E21EEB69037AB78ull));
  c = RM_FMA3(x2, c, rm_bits(0xBE927E4FA17F65F6ull));
  c = RM_FMA3(x2, c, rm_bits(0x3EFA01A019F4EC90ull));
  c = RM_FMA3(x2, c, rm_bits(0xBF56C16C16C16967ull));
  c = RM_FMA3(x2, c, rm_bits(0x3FA5555555555555ull));
  const double cosr = t + fma(x4, c, fma(rh, -rl, u));
  double sp = RM_FMA3(x2, rm_bits(0x3DE5E0B2F9A43BB8ull), rm_bits(0xBE5AE600B42FDFA7ull));
  sp = RM_FMA3(x2, sp, rm_bits(0x3EC71DE3796CDE01ull));
  sp = RM_FMA3(x2, sp, rm_bits(0xBF2A01A019E83E5Cull));
  sp = RM_FMA3(x2, sp, rm_bits(0x3F81111111110BB3ull));
  const double m = rh * (-x2);
  const double sq = fma(x2, fma(m, sp, rl * 0.5), -rl);
  const double sinr = rh - fma(m, rm_bits(0xBFC5555555555555ull), sq);
  // __ocml_sincos_f64 quadrant and sign
  const unsigned long long sgn_hi = (q > 1) ? 0x8000000000000000ull : 0ull;
  const unsigned long long xsgn = rm_ubits(x) & 0x8000000000000000ull;
  const bool even = (q & 1) == 0;
  sn = rm_bits(rm_ubits(even ? sinr : cosr) ^ xsgn ^ sgn_hi);
  cs = rm_bits(rm_ubits(even ? cosr : -sinr) ^ sgn_hi);
  // __ocmlpriv_tanred2_f64(rh, rl, q & 1)
  const double h2 = rh * rh;
  const double h2l = fma(rh, rh, -h2);
  const double s = h2 + fma(rh, rl * 2.0, h2l);
  double z = RM_FMA3(s, rm_bits(0x3EF5E089C751C08Cull), rm_bits(0xBF078809A9A29F71ull));
  z = RM_FMA3(s, z, rm_bits(0x3F17746F90A8AAE0ull));
  z = RM_FMA3(s, z, rm_bits(0xBEFBB44DA6FBF144ull));
  z = RM_FMA3(s, z, rm_bits(0x3F21E634A7943ACFull));
  z = RM_FMA3(s, z, rm_bits(0x3F2D250FDEB68FEBull));
  z = RM_FMA3(s, z, rm_bits(0x3F437FD9B58C4D95ull));
  z = RM_FMA3(s, z, rm_bits(0x3F57D5AF15120E2Cull));
  z = RM_FMA3(s, z, rm_bits(0x3F6D6D93E09491DFull));
  z = RM_FMA3(s, z, rm_bits(0x3F8226E12033784Dull));
  z = RM_FMA3(s, z, rm_bits(0x3F9664F49AC36AE2ull));
  z = RM_FMA3(s, z, rm_bits(0x3FABA1BA1B451C21ull));
  z = RM_FMA3(s, z, rm_bits(0x3FC11111111185B7ull));
  z = RM_FMA3(s, z, rm_bits(0x3FD55555555554EEull));
  const double w = s * z;
  const double v = rh * w;
  const double vl = fma(rh, w, -v);
  const double th0 = rh + v;
  const double vt = v - (th0 - rh);
  const double tl0 = (rl + vl) + vt;
  const double th = th0 + tl0;                // tan(reduced), head
  const double tl = tl0 - (th - th0);         // and tail
  const double rc = RM_RECIP2(th);
  const double pr = th * rc;
  const double pe = fma(rc, tl, fma(rc, th, -pr));
  const double ps = pr + pe;
  const double pt = pe - (ps - pr);
  const double o1 = 1.0 - ps;
  const double o2 = ((1.0 - o1) - ps) - pt;
  const double ncot = rc + rc * (o1 + o2);    // 1 / tan(reduced)
  const double tr = ((q & 1) == 0) ? th : -ncot;
  tn = rm_bits(rm_ubits(tr) ^ xsgn);
}

// ---------------------------------------------------------------------------
// pow(x, y): __ocml_pow_f64 = exp(y * log|x|) with log|x| in double-double
// (__ocmlpriv_epln_f64) and the product's tail folded in by
// __ocmlpriv_expep_f64, then the C99 special cases.
// ---------------------------------------------------------------------------
// __ocml_exp_f64 (finite_only off)
RM_FN double rm_exp(double x) {
  const double n = rint(x * rm_bits(0x3FF71547652B82FEull));
  double r = fma(-n, rm_bits(0x3FE62E42FEFA39EFull), x);
  r = fma(-n, rm_bits(0x3C7ABC9E3B39803Full), r);
  double p = RM_FMA3(r, rm_bits(0x3E5ADE156A5DCB37ull), rm_bits(0x3E928AF3FCA7AB0Cull));
  p = RM_FMA3(r, p, rm_bits(0x3EC71DEE623FDE64ull));
  p = RM_FMA3(r, p, rm_bits(0x3EFA01997C89E6B0ull));
  p = RM_FMA3(r, p, rm_bits(0x3F2A01A014761F6Eull));
  p = RM_FMA3(r, p, rm_bits(0x3F56C16C1852B7B0ull));
  p = RM_FMA3(r, p, rm_bits(0x3F81111111122322ull));
  p = RM_FMA3(r, p, rm_bits(0x3FA55555555502A1ull));
  p = RM_FMA3(r, p, rm_bits(0x3FC5555555555511ull));
  p = RM_FMA3(r, p, rm_bits(0x3FE000000000000Bull));
  p = RM_FMA3(r, p, 1.0);
  p = RM_FMA3(r, p, 1.0);
  double e = (x == x) ? ldexp(p, (int)fmax(fmin(n, 2100.0), -2100.0)) : p;   // NaN: p is NaN
  e = (x > 1024.0) ? rm_bits(0x7FF0000000000000ull) : e;
  return (x < -1075.0) ? 0.0 : e;
}

// __ocmlpriv_epln_f64: log(x) = hi + lo for finite x > 0
RM_FN void rm_epln(double x, double& hi, double& lo) {
  int ex0;
  const double m0 = frexp(x, &ex0);
  const bool lt = m0 < rm_bits(0x3FE5555555555555ull);
  const double m = m0 * (lt ? 2.0 : 1.0);
  const int ex = ex0 - (lt ? 1 : 0);
  const double a = m + -1.0;
  const double b = m + 1.0;
  const double bh = b + -1.0;
  const double bl = m - bh;
  const double r = RM_RECIP2(b);
  // u = a / b in double-double
  const double q = a * r;
  const double p = b * q;
  double pe = fma(q, b, -p);
  pe = fma(q, bl, pe);
  const double s = p + pe;
  const double se = pe - (s - p);
  const double d = a - s;
  const double dd = d + (((a - d) - s) - se);
  const double corr = r * dd;
  const double uh = q + corr;
  const double ul = corr - (uh - q);
  // v = u^2
  const double u2 = uh * uh;
  double u2e = fma(uh, uh, -u2);
  u2e = fma(uh, ul * 2.0, u2e);
  const double vh = u2 + u2e;
  const double vl = u2e - (vh - u2);
  double P = RM_FMA3(vh, rm_bits(0x3FBDEE674222DE17ull), rm_bits(0x3FBA6564968915A9ull));
  P = RM_FMA3(vh, P, rm_bits(0x3FBE25E43ABE935Aull));
  P = RM_FMA3(vh, P, rm_bits(0x3FC110EF47E6C9C2ull));
  P = RM_FMA3(vh, P, rm_bits(0x3FC3B13BCFA74449ull));
  P = RM_FMA3(vh, P, rm_bits(0x3FC745D171BF3C30ull));
  P = RM_FMA3(vh, P, rm_bits(0x3FCC71C71C7792CEull));
  P = RM_FMA3(vh, P, rm_bits(0x3FD24924924920DAull));
  P = RM_FMA3(vh, P, rm_bits(0x3FD999999999999Cull));
  // ex * ln2 in double-double
  const double fe = (double)ex;
  const double l2h = fe * rm_bits(0x3FE62E42FEFA39EFull);
  double l2e = fma(fe, rm_bits(0x3FE62E42FEFA39EFull), -l2h);
  l2e = fma(fe, rm_bits(0x3C7ABC9E3B39803Full), l2e);
  const double lh = l2h + l2e;
  const double ll = l2e - (lh - l2h);
  // 2u
  const double u2h = ldexp(uh, 1);
  const double u2l = ldexp(ul, 1);
  // u^3 = u * v
  const double c = uh * vh;
  double ce = fma(vh, uh, -c);
  ce = fma(vh, ul, ce);
  ce = fma(vl, uh, ce);
  const double ch = c + ce;
  const double cl = ce - (ch - c);
  // v * P
  const double w = vh * P;
  double we = fma(vh, P, -w);
  we = fma(vl, P, we);
  const double wh = w + we;
  const double wl = we - (wh - w);
  // + 2/3 (double-double)
  const double z = wh + rm_bits(0x3FE5555555555555ull);
  const double zd = wh - (z + rm_bits(0xBFE5555555555555ull));
  const double zl = (wl + rm_bits(0x3C8543B0D5DF274Dull)) + zd;
  const double zh2 = z + zl;
  const double zl2 = zl - (zh2 - z);
  // u^3 * (v P + 2/3)
  const double m86 = ch * zh2;
  double me = fma(ch, zh2, -m86);
  me = fma(ch, zl2, me);
  me = fma(cl, zh2, me);
  const double mh = m86 + me;
  const double ml = me - (mh - m86);
  // 2u + that
  const double s94 = u2h + mh;
  const double s96 = mh - (s94 - u2h);
  const double s98 = (u2l + ml) + s96;
  const double s99 = s94 + s98;
  const double s101 = s98 - (s99 - s94);
  // ex ln2 + that
  const double a102 = lh + s99;
  const double a103 = a102 - lh;
  const double a107 = (s99 - a103) + (lh - (a102 - a103));
  const double b108 = ll + s101;
  const double b109 = b108 - ll;
  const double b113 = (s101 - b109) + (ll - (b108 - b109));
  const double c114 = b108 + a107;
  const double c115 = a102 + c114;
  const double c117 = c114 - (c115 - a102);
  const double c118 = b113 + c117;
  hi = c115 + c118;
  lo = c118 - (hi - c115);
}

RM_FN double rm_pow(double x, double y) {
  const double inf = rm_bits(0x7FF0000000000000ull), nan = rm_bits(0x7FF8000000000000ull);
  const double yy = (x == 1.0) ? 1.0 : y;
  const double xx = (yy == 0.0) ? 1.0 : x;
  const double ax = fabs(xx);
  double lh = 0.0, ll = 0.0;
  if (ax > 0.0 && ax < inf) rm_epln(ax, lh, ll);   // else: a special case below
  const double pr = yy * lh;
  double pe = fma(yy, lh, -pr);
  pe = fma(yy, ll, pe);
  const double s = pr + pe;
  const double sl = pe - (s - pr);
  const double eh = (fabs(pr) == inf) ? pr : s;
  const double el = (fabs(eh) == inf) ? 0.0 : sl;
  // __ocmlpriv_expep_f64
  const double ex = rm_exp(eh);
  const double e = (fabs(ex) == inf) ? ex : fma(ex, el, ex);
  const bool yint = trunc(yy) == yy;
  const double yh = yy * 0.5;
  const bool yodd = yint && (trunc(yh) != yh);
  double ret = copysign(e, yodd ? xx : 1.0);
  if (xx < 0.0) ret = yint ? ret : nan;
  if (fabs(yy) == inf) {
    const bool big = (yy != fabs(yy)) != (ax < 1.0);
    ret = (ax == 1.0) ? 1.0 : (big ? 0.0 : inf);
  }
  if (xx == 0.0 || ax == inf) {
    const double v = ((yy < 0.0) != (xx == 0.0)) ? 0.0 : inf;
    ret = copysign(v, yodd ? xx : 0.0);
  }
  if (xx != xx || yy != yy) ret = nan;
  return ret;
}

}  // namespace rwrt_math
