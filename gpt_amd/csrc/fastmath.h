// Register-light fp64 log and sincos(2πu) for the Box–Muller transform of the Philox streams.
//
// The library versions carry Payne–Hanek reduction tables and long polynomial ladders whose
// constants the compiler hoists into registers next to the kernels' resident U / gradU tiles.
// Box–Muller only needs log on (0, 1] and sin/cos of 2πu with u in (0, 1), so:
//   log: fdlibm's e_log.c scheme (s = f/(2+f), degree-14 minimax in s; on the device the
//        quotient is f times a Newton-refined reciprocal) — error < 2 ulp;
//   sincos(2πu): exact quadrant reduction on 4u (no π rounding in the reduction), then
//        fdlibm's __kernel_sin / __kernel_cos on |φ| <= π/4 — error < 1 ulp.
// Results can differ from glibc (the oracle's numpy) in the last bit; parity tolerances cover it.
//
// The coefficients come from a table the caller passes (kernels pass an opaque pointer to a
// __constant__ copy, so they are fetched by scalar loads at their use instead of being hoisted
// into vector registers for the whole kernel).
#pragma once
#include <stdint.h>
#include <string.h>

#ifndef GPT_HD
#define GPT_HD __host__ __device__ __forceinline__
#endif

namespace gpt {

// [0..6] Lg1..Lg7  [7] ln2_hi  [8] ln2_lo  [9..14] S1..S6  [15..20] C1..C6  [21] π/2 hi  [22] π/2 lo
// [23] 2π·2⁻³²  [24..26] Taylor sin φ³, φ⁵, φ⁷  [27..30] Taylor cos φ², φ⁴, φ⁶, φ⁸ (fm_sincos_tab)
#define GPT_FM_COEF                                                                              \
  {6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01,                 \
   2.222219843214978396e-01, 1.818357216161805012e-01, 1.531383769920937332e-01,                 \
   1.479819860511658591e-01, 6.93147180369123816490e-01, 1.90821492927058770002e-10,             \
   -1.66666666666666324348e-01, 8.33333333332248946124e-03, -1.98412698298579493134e-04,         \
   2.75573137070700676789e-06, -2.50507602534068634195e-08, 1.58969099521155010221e-10,          \
   4.16666666666666019037e-02, -1.38888888888741095749e-03, 2.48015872894767294178e-05,          \
   -2.75573143513906633035e-07, 2.08757232129817482790e-09, -1.13596475577881948265e-11,         \
   1.57079632679489655800e+00, 6.12323399573676603587e-17,                                     \
   1.4629180792671596e-09, -1.66666666666666666667e-01, 8.33333333333333333333e-03,          \
   -1.98412698412698412698e-04, -5.0e-01, 4.16666666666666666667e-02,                           \
   -1.38888888888888888889e-03, 2.48015873015873015873e-05}

// 1/x: on the device the hardware reciprocal plus two Newton steps (within 1 ulp)
GPT_HD double fm_rcp(double x) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(GPT_FM_OLD)
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
#else
  return 1.0 / x;
#endif
}

template <class CP>
GPT_HD double fm_log_c(double x, CP c) {   // x in (0, +inf), finite
  uint64_t bits;
  memcpy(&bits, &x, 8);
  int e = (int)((bits >> 52) & 0x7ff) - 1023;
  uint64_t mb = (bits & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL;   // mantissa in [1, 2)
  double mnt;
  memcpy(&mnt, &mb, 8);
  if (mnt > 1.4142135623730951) { mnt *= 0.5; e += 1; }                  // [√½, √2)
  const double f = mnt - 1.0;
  const double s = f * fm_rcp(2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * (c[1] + w * (c[3] + w * c[5]));
  const double t2 = z * (c[0] + w * (c[2] + w * (c[4] + w * c[6])));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  const double dk = (double)e;
  return dk * c[7] - ((hfsq - (s * (hfsq + R) + dk * c[8])) - f);
}

// sin(2πu), cos(2πu) for u in [0, 1].
template <class CP>
GPT_HD void fm_sincos_2pi_c(double u, double& sn, double& cs, CP c) {
  const double x = 4.0 * u;                 // exact
  const double qd = rint(x);
  const double f = x - qd;                  // exact, |f| <= 1/2
  const int q = ((int)qd) & 3;
  const double ph = fma(f, c[21], f * c[22]);   // |φ| <= π/4
  const double z = ph * ph;
  const double v = z * ph;
  const double rs = c[10] + z * (c[11] + z * (c[12] + z * (c[13] + z * c[14])));
  const double s = ph + v * (c[9] + z * rs);
  const double rc = z * (c[15] + z * (c[16] + z * (c[17] + z * (c[18] + z * (c[19] + z * c[20])))));
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  const double cc = w + (((1.0 - w) - hz) + z * rc);
  // quadrant q: (sin, cos) = (s, cc), (cc, −s), (−s, −cc), (−cc, s) — selects and sign-bit flips
  // (no divergent branches, so the independent Box–Muller chains of a caller interleave)
  const bool odd = (q & 1) != 0;
  uint64_t bs, bc;
  const double s0 = odd ? cc : s, c0 = odd ? s : cc;
  memcpy(&bs, &s0, 8);
  memcpy(&bc, &c0, 8);
  bs ^= (uint64_t)((q >> 1) & 1) << 63;
  bc ^= (uint64_t)(((q + 1) >> 1) & 1) << 63;
  memcpy(&sn, &bs, 8);
  memcpy(&cs, &bc, 8);
}

// sin(2πu), cos(2πu) for u = (x + ½)·2⁻³² (the Box–Muller angle of a 32-bit Philox word) from
// a table of (sin, cos)(2πi/256), i < 256 (tab: 512 doubles, e.g. in LDS; fm_sincos_tab_fill):
// u = i/256 + δ with i = x >> 24 and δ = ((x mod 2²⁴) + ½)·2⁻³² exact, |2πδ| < 2π/256, where
// Taylor polynomials of degrees 7 / 8 are exact to < 1e-20; then the angle-sum formulas.  About
// half the instructions of fm_sincos_2pi_c, within 2 ulp of it.
template <class CP, class TP>
GPT_HD void fm_sincos_tab(uint32_t x, const TP* tab, double& sn, double& cs, CP c) {
  const unsigned i = x >> 24;
  const double ph = ((double)(x & 0xFFFFFFu) + 0.5) * c[23];
  const double z = ph * ph;
  double ts = fma(z, c[26], c[25]);
  ts = fma(z, ts, c[24]);
  const double sp = fma(ph * z, ts, ph);
  double tc = fma(z, c[30], c[29]);
  tc = fma(z, tc, c[28]);
  tc = fma(z, tc, c[27]);
  const double cp = fma(z, tc, 1.0);
  const double st = tab[2 * i], ct = tab[2 * i + 1];
  sn = fma(st, cp, ct * sp);
  cs = fma(ct, cp, -(st * sp));
}

// fm_sincos_tab with the 256-entry table factored into two 16-entry ones: tab[2j], tab[2j + 1] =
// (sin, cos)(2πj/16) and tab[32 + 2j], tab[33 + 2j] = (sin, cos)(2πj/256), j < 16, so i = 16·ih + il
// takes the angle sum of entries ih and il first.  Each 16-entry table is 256 contiguous bytes —
// every LDS bank once — so the per-lane 16-B reads of a wave never conflict (lanes with the same
// entry share it; the 256-entry table's random rows cost ~3 passes per read).  Within 3 ulp of
// fm_sincos_2pi_c.
template <class CP, class TP>
GPT_HD void fm_sincos_tab2(uint32_t x, const TP* tab, double& sn, double& cs, CP c) {
  const unsigned ih = x >> 28, il = (x >> 24) & 15u;
  const double ph = ((double)(x & 0xFFFFFFu) + 0.5) * c[23];
  const double z = ph * ph;
  double ts = fma(z, c[26], c[25]);
  ts = fma(z, ts, c[24]);
  const double sp = fma(ph * z, ts, ph);
  double tc = fma(z, c[30], c[29]);
  tc = fma(z, tc, c[28]);
  tc = fma(z, tc, c[27]);
  const double cp = fma(z, tc, 1.0);
  const double s1 = tab[2 * ih], c1 = tab[2 * ih + 1];
  const double s2 = tab[32 + 2 * il], c2 = tab[33 + 2 * il];
  const double st = fma(s1, c2, c1 * s2), ct = fma(c1, c2, -(s1 * s2));
  sn = fma(st, cp, ct * sp);
  cs = fma(ct, cp, -(st * sp));
}

// √x for finite normal x > 0 (the Box–Muller radius: x = −2 ln u in [2e-10, 46]): on the device
// the hardware rsq refined by two Newton steps (the refinement of the library expansion without
// its denormal scaling and class checks).
GPT_HD double fm_sqrt_pos(double x) {
#if defined(__HIP_DEVICE_COMPILE__) && !defined(GPT_FM_OLD)
  double y = __builtin_amdgcn_rsq(x);
  double g = x * y, h = 0.5 * y;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  h = fma(h, r, h);
  double d = fma(-g, g, x);
  g = fma(d, h, g);
  d = fma(-g, g, x);
  return fma(d, h, g);
#else
  return sqrt(x);
#endif
}

struct FmHostCoef {
  double v[31];
  GPT_HD double operator[](int i) const { return v[i]; }
};
GPT_HD double fm_log(double x) {
  const FmHostCoef c{GPT_FM_COEF};
  return fm_log_c(x, c);
}
GPT_HD void fm_sincos_2pi(double u, double& sn, double& cs) {
  const FmHostCoef c{GPT_FM_COEF};
  fm_sincos_2pi_c(u, sn, cs, c);
}

}  // namespace gpt
