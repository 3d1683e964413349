/*
 * pt_fmath.h -- the path tracer's float32 transcendentals, correctly rounded in
 * all but vanishingly rare cases, bit-reproducible across the CPU and the GPU.
 *
 * GLSL leaves sin/cos/atan/asin/log/pow precision to the driver (the
 * reference's pass1.fsh uses them at IS:148-149,176,489-490,502-505,525,
 * 582,639,660), so no reference output pins them to the ulp. This header fixes
 * them to the one implementation-independent choice: the exact function value
 * rounded to float. Each function evaluates its float argument in double
 * precision -- exact argument reductions (pi/2 and ln 2 split in parts,
 * tan(k pi/16) breakpoints), Taylor series truncated far below double
 * rounding, Horner steps as explicit fused multiply-adds, IEEE double division
 * -- to ~1e-16 relative and rounds once to float, so the result is the
 * correctly rounded one unless the exact value lies within ~1e-16 of a
 * rounding midpoint (probability ~1e-8 per call). Written with only correctly
 * rounded IEEE operations (+, -, *, /, float sqrtf, double fma), so the HIP
 * kernels (v_fma_f64, v_div_*_f64) and the CPU checker produce identical bits.
 *
 * Why: the oracle's shader-text build (oracle/ref_glsl.cpp) binds the GLSL
 * built-ins to the host C library's double functions rounded to float -- an
 * implementation this repository did not write -- and the GPU's images equal
 * that build's (tests/test_gpu_libm_pin.py). tests/test_fmath.py checks every
 * function against float64 numpy rounded to float, and records its distance
 * from glibc's own float functions (sinf ... powf), which are not correctly
 * rounded in 0.07-16 % of inputs.
 *
 * Valid ranges: sin/cos |x| < 2^19 (the reduction's parts; the kernels use
 * |x| <= 2 pi), everything else the whole float range.
 *
 * Usable from C (oracle), C++ and HIP device code.
 */
#ifndef PT_FMATH_H
#define PT_FMATH_H

#if defined(__HIPCC__) || defined(__HIP__)
#define PTM_FN static inline __host__ __device__ __attribute__((always_inline))
#else
#define PTM_FN static inline
#endif
#define PTM_CORE PTM_FN

#ifdef __cplusplus
#include <cmath>
#define PTM_FMAD(a, b, c) ::fma((double)(a), (double)(b), (double)(c))
#define PTM_FLOORD(a) ::floor((double)(a))
#define PTM_SQRTF(a) ::sqrtf(a)
#else
#include <math.h>
#define PTM_FMAD(a, b, c) fma((double)(a), (double)(b), (double)(c))
#define PTM_FLOORD(a) floor((double)(a))
#define PTM_SQRTF(a) sqrtf(a)
#endif
#include <stdint.h>

PTM_FN uint32_t ptm_f2u(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
PTM_FN float ptm_u2f(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }
PTM_FN uint64_t ptm_d2u(double f) { uint64_t u; __builtin_memcpy(&u, &f, 8); return u; }
PTM_FN double ptm_u2d(uint64_t u) { double f; __builtin_memcpy(&f, &u, 8); return f; }
/* Every double constant of the cores below passes through PTM_K: its bits XOR a zero the
   compiler cannot see (device code: an SGPR pair set by s_mov_b64 in front of each use), so its
   materialization stays where it is used. Plain literals were hoisted out of the kernels' loops
   into ~120 SGPRs, which spilled into VGPR lanes and then to scratch (the Lambert regen kernel
   127 VGPRs with none spilled -> 125 spilled); calls instead of inlining wait for every
   outstanding memory operation at the callee's entry (c4 0.23 -> 0.30 ms per frame). */
#if defined(__HIP_DEVICE_COMPILE__)
PTM_FN uint64_t ptm_zero(void) {
  uint64_t z;
  __asm__ volatile("s_mov_b64 %0, 0" : "=s"(z));
  return z;
}
#else
PTM_FN uint64_t ptm_zero(void) { return 0; }
#endif
#define PTM_K(c) ptm_u2d(ptm_d2u(c) ^ z_)

/* pi/2 = P1 + P2 + P3 (33 + 33 + 53 significant bits: k * P1 and k * P2 are exact for |k| < 2^20) */
#define PTM_PIO2_1 1.5707963267341256
#define PTM_PIO2_2 6.077100506303966e-11
#define PTM_PIO2_3 2.0222662487959506e-21
#define PTM_2OPI 0.6366197723675814
#define PTM_PI_D 3.141592653589793
#define PTM_PIO2_D 1.5707963267948966
/* ln 2 = LN2_HI (40 bits: e * LN2_HI exact for |e| < 2^13) + LN2_LO */
#define PTM_LN2_HI 0.6931471805601177
#define PTM_LN2_LO -1.7239444525614835e-13
#define PTM_INV_LN2 1.4426950408889634

/* sin(r), cos(r) for |r| <= pi/4: Taylor to r^17 / r^18 (the next terms < 1e-19 relative) */
PTM_CORE double ptm_sin_d(double r) {
  const uint64_t z_ = ptm_zero();
  double z = r * r;
  double p = PTM_FMAD(z, PTM_K(2.8114572543455206e-15), PTM_K(-7.647163731819816e-13));
  p = PTM_FMAD(p, z, PTM_K(1.6059043836821613e-10));
  p = PTM_FMAD(p, z, PTM_K(-2.505210838544172e-08));
  p = PTM_FMAD(p, z, PTM_K(2.7557319223985893e-06));
  p = PTM_FMAD(p, z, PTM_K(-0.0001984126984126984));
  p = PTM_FMAD(p, z, PTM_K(0.008333333333333333));
  p = PTM_FMAD(p, z, PTM_K(-0.16666666666666666));
  return PTM_FMAD(r * z, p, r);
}
PTM_CORE double ptm_cos_d(double r) {
  const uint64_t z_ = ptm_zero();
  double z = r * r;
  double p = PTM_FMAD(z, PTM_K(-1.5619206968586225e-16), PTM_K(4.779477332387385e-14));
  p = PTM_FMAD(p, z, PTM_K(-1.1470745597729725e-11));
  p = PTM_FMAD(p, z, PTM_K(2.08767569878681e-09));
  p = PTM_FMAD(p, z, PTM_K(-2.755731922398589e-07));
  p = PTM_FMAD(p, z, PTM_K(2.48015873015873e-05));
  p = PTM_FMAD(p, z, PTM_K(-0.001388888888888889));
  p = PTM_FMAD(p, z, PTM_K(0.041666666666666664));
  return PTM_FMAD(z * z, p, 1.0 - 0.5 * z);
}
/* x = k pi/2 + r, |r| <= pi/4 (+ rounding), q = k */
PTM_FN double ptm_reduce_d(float x, int* q) {
  double xd = (double)x;
  double k = PTM_FLOORD(PTM_FMAD(xd, PTM_2OPI, 0.5));
  double r = PTM_FMAD(-k, PTM_PIO2_1, xd);
  r = PTM_FMAD(-k, PTM_PIO2_2, r);
  r = PTM_FMAD(-k, PTM_PIO2_3, r);
  *q = (int)k;
  return r;
}
PTM_FN float ptm_sinf(float x) {
  int q;
  double r = ptm_reduce_d(x, &q);
  double s = (q & 1) ? ptm_cos_d(r) : ptm_sin_d(r);
  return (float)((q & 2) ? -s : s);
}
PTM_FN float ptm_cosf(float x) {
  int q;
  double r = ptm_reduce_d(x, &q);
  double c = (q & 1) ? ptm_sin_d(r) : ptm_cos_d(r);
  return (float)(((q + 1) & 2) ? -c : c);
}
/* the same bits as ptm_sinf and ptm_cosf, one reduction */
PTM_FN void ptm_sincosf(float x, float* s, float* c) {
  int q;
  double r = ptm_reduce_d(x, &q);
  double sk = ptm_sin_d(r), ck = ptm_cos_d(r);
  double ss = (q & 1) ? ck : sk;
  double cc = (q & 1) ? sk : ck;
  *s = (float)((q & 2) ? -ss : ss);
  *c = (float)(((q + 1) & 2) ? -cc : cc);
}

/* atan(num / den) for 0 <= num <= den, den > 0: breakpoint c = tan(k pi/16) nearest the
   ratio, u = (num - c den) / (den + c num) (one division; the fmas keep u's error relative),
   |u| <= tan(pi/32), atan = atan(c) + u (1 - u^2/3 + ... - u^18/19) */
PTM_CORE double ptm_atan_ratio(double num, double den) {
  const uint64_t z_ = ptm_zero();
  double c, a;
  if (num < PTM_K(0.09849140335716425) * den) { c = 0.0; a = 0.0; }
  else if (num < PTM_K(0.3033466836073424) * den) { c = PTM_K(0.198912367379658); a = PTM_K(0.19634954084936207); }
  else if (num < PTM_K(0.5345111359507916) * den) { c = PTM_K(0.41421356237309503); a = PTM_K(0.39269908169872414); }
  else if (num < PTM_K(0.8206787908286602) * den) { c = PTM_K(0.6681786379192989); a = PTM_K(0.5890486225480862); }
  else { c = 1.0; a = PTM_K(0.7853981633974483); }
  double u = PTM_FMAD(-c, den, num) / PTM_FMAD(c, num, den);
  double z = u * u;
  double p = PTM_FMAD(z, PTM_K(-0.05263157894736842), PTM_K(0.058823529411764705));
  p = PTM_FMAD(p, z, PTM_K(-0.06666666666666667));
  p = PTM_FMAD(p, z, PTM_K(0.07692307692307693));
  p = PTM_FMAD(p, z, PTM_K(-0.09090909090909091));
  p = PTM_FMAD(p, z, PTM_K(0.1111111111111111));
  p = PTM_FMAD(p, z, PTM_K(-0.14285714285714285));
  p = PTM_FMAD(p, z, PTM_K(0.2));
  p = PTM_FMAD(p, z, PTM_K(-0.3333333333333333));
  return a + PTM_FMAD(u * z, p, u);
}
/* atan2 of doubles (finite or infinite magnitudes from float inputs), libm's quadrant and
   signed-zero rules */
PTM_FN double ptm_atan2_d(double y, double x) {
  double ax = x < 0.0 ? -x : x, ay = y < 0.0 ? -y : y;
  double a;
  if (ax == 0.0 && ay == 0.0) a = 0.0;
  else if (ay <= ax) a = ax == 1.0 / 0.0 ? (ay == ax ? 0.7853981633974483 : 0.0) : ptm_atan_ratio(ay, ax);
  else a = ay == 1.0 / 0.0 ? PTM_PIO2_D : PTM_PIO2_D - ptm_atan_ratio(ax, ay);
  if (ptm_d2u(x) >> 63) a = PTM_PI_D - a; /* x < 0 or x == -0 */
  return (ptm_d2u(y) >> 63) ? -a : a;
}
PTM_FN float ptm_atan2f(float y, float x) {
  if (y != y || x != x) return y + x;
  return (float)ptm_atan2_d((double)y, (double)x);
}

/* sqrt(a) in double for a >= 0: the float square root, then two Newton steps as fmas */
PTM_FN double ptm_sqrt_d(double a) {
  if (a == 0.0) return 0.0;
  double y = (double)PTM_SQRTF((float)a);
  double h = 0.5 / y;
  y = PTM_FMAD(PTM_FMAD(-y, y, a), h, y);
  return PTM_FMAD(PTM_FMAD(-y, y, a), h, y);
}
/* asin(x) = atan2(x, sqrt(1 - x^2)); 1 - x^2 is exact in double for a float x */
PTM_FN float ptm_asinf(float x) {
  if (x != x) return x;
  double xd = (double)x;
  double ax = xd < 0.0 ? -xd : xd;
  if (ax > 1.0) return (x - x) / (x - x); /* NaN */
  double s = ptm_sqrt_d(PTM_FMAD(-xd, xd, 1.0));
  double a = ax <= s ? ptm_atan_ratio(ax, s) : PTM_PIO2_D - ptm_atan_ratio(s, ax);
  return (float)(xd < 0.0 ? -a : a);
}

/* natural log of a positive finite double (every float, subnormals included, is a normal
   double): x = m 2^e, m in [sqrt(1/2), sqrt(2)), log m = 2 atanh(s), s = (m - 1) / (m + 1) */
PTM_CORE double ptm_log_d(double x) {
  const uint64_t z_ = ptm_zero();
  uint64_t u = ptm_d2u(x);
  int e = (int)((u >> 52) & 0x7ff) - 1023;
  double m = ptm_u2d((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull); /* [1, 2) */
  if (m > PTM_K(1.4142135623730951)) {
    m = m * 0.5;
    e += 1;
  }
  double s = (m - 1.0) / (m + 1.0);
  double z = s * s;
  double p = PTM_FMAD(z, PTM_K(0.043478260869565216), PTM_K(0.047619047619047616));
  p = PTM_FMAD(p, z, PTM_K(0.05263157894736842));
  p = PTM_FMAD(p, z, PTM_K(0.058823529411764705));
  p = PTM_FMAD(p, z, PTM_K(0.06666666666666667));
  p = PTM_FMAD(p, z, PTM_K(0.07692307692307693));
  p = PTM_FMAD(p, z, PTM_K(0.09090909090909091));
  p = PTM_FMAD(p, z, PTM_K(0.1111111111111111));
  p = PTM_FMAD(p, z, PTM_K(0.14285714285714285));
  p = PTM_FMAD(p, z, PTM_K(0.2));
  p = PTM_FMAD(p, z, PTM_K(0.3333333333333333));
  double s2 = s + s;
  double lm = PTM_FMAD(s2 * z, p, s2);
  double fe = (double)e;
  return PTM_FMAD(fe, PTM_LN2_HI, PTM_FMAD(fe, PTM_LN2_LO, lm));
}
PTM_FN float ptm_logf(float x) {
  if (x != x || x < 0.0f) return (x - x) / (x - x);
  if (x == 0.0f) return -1.0f / 0.0f;
  if (x > 3.40282346e38f) return x;
  return (float)ptm_log_d((double)x);
}

/* exp(w) for w in [-746, 710]: w = k ln 2 + r, |r| <= ln 2 / 2, Taylor to r^15 */
PTM_CORE double ptm_exp_d(double w) {
  const uint64_t z_ = ptm_zero();
  double k = PTM_FLOORD(PTM_FMAD(w, PTM_INV_LN2, 0.5));
  double r = PTM_FMAD(-k, PTM_LN2_HI, w);
  r = PTM_FMAD(-k, PTM_LN2_LO, r);
  double p = PTM_FMAD(r, PTM_K(7.647163731819816e-13), PTM_K(1.1470745597729725e-11));
  p = PTM_FMAD(p, r, PTM_K(1.6059043836821613e-10));
  p = PTM_FMAD(p, r, PTM_K(2.08767569878681e-09));
  p = PTM_FMAD(p, r, PTM_K(2.505210838544172e-08));
  p = PTM_FMAD(p, r, PTM_K(2.755731922398589e-07));
  p = PTM_FMAD(p, r, PTM_K(2.7557319223985893e-06));
  p = PTM_FMAD(p, r, PTM_K(2.48015873015873e-05));
  p = PTM_FMAD(p, r, PTM_K(0.0001984126984126984));
  p = PTM_FMAD(p, r, PTM_K(0.001388888888888889));
  p = PTM_FMAD(p, r, PTM_K(0.008333333333333333));
  p = PTM_FMAD(p, r, PTM_K(0.041666666666666664));
  p = PTM_FMAD(p, r, PTM_K(0.16666666666666666));
  p = PTM_FMAD(p, r, 0.5);
  double y = PTM_FMAD(r * r, p, r) + 1.0;
  /* y * 2^k in two exact steps (k in [-1100, 1030]: each half a normal power of two) */
  int ki = (int)k;
  int k1 = ki / 2, k2 = ki - k1;
  y = y * ptm_u2d((uint64_t)(k1 + 1023) << 52);
  return y * ptm_u2d((uint64_t)(k2 + 1023) << 52);
}
PTM_FN float ptm_expf(float x) {
  if (x != x) return x;
  if (x > 88.8f) return 1.0f / 0.0f;
  if (x < -104.0f) return 0.0f;
  return (float)ptm_exp_d((double)x);
}

/* pow for x > 0 (the only uses: SampleGTR1 IS:525 and the tonemap gamma): exp(y log x) in
   double, rounded once */
PTM_FN float ptm_powf(float x, float y) {
  if (y == 0.0f) return 1.0f;
  if (x == 1.0f) return 1.0f;
  if (x == 0.0f) return y > 0.0f ? 0.0f : 1.0f / 0.0f;
  if (x < 0.0f || x != x || y != y) return (x - x) / (x - x);
  if (x > 3.40282346e38f) return y > 0.0f ? x : 0.0f;
  double w = (double)y * ptm_log_d((double)x);
  if (w > 88.8) return 1.0f / 0.0f;
  if (w < -104.0) return 0.0f;
  return (float)ptm_exp_d(w);
}


/* ---- float approximations for decisions only (ptm_sph_texel in the kernels' pt_device.h):
   S. L. Moshier's single-precision Cephes atan / asin with explicit fmaf -- at most 4 / 3 ulp
   from the exact value (tests/test_fmath.py), the same bits on the CPU and the GPU. Their
   results never reach an image: they only decide a texel when no rounding of the correctly
   rounded functions could decide it otherwise. */
#ifdef __cplusplus
#define PTM_FMAF(a, b, c) ::fmaf((a), (b), (c))
#else
#define PTM_FMAF(a, b, c) fmaf((a), (b), (c))
#endif
PTM_FN float ptm_atan_pos_fast(float t) {
  float base = 0.0f, x = t;
  if (t > 2.414213562373095f) {
    base = 1.57079632679489661923f;
    x = -1.0f / t;
  } else if (t > 0.4142135623730950f) {
    base = 0.785398163397448309616f;
    x = (t - 1.0f) / (t + 1.0f);
  }
  float z = x * x;
  float p = PTM_FMAF(8.05374449538e-2f, z, -1.38776856032e-1f);
  p = PTM_FMAF(p, z, 1.99777106478e-1f);
  p = PTM_FMAF(p, z, -3.33329491539e-1f);
  return base + PTM_FMAF(p * z, x, x);
}
PTM_FN float ptm_atan2f_fast(float y, float x) {
  if (y != y || x != x) return y + x;
  float ax = x < 0.0f ? -x : x, ay = y < 0.0f ? -y : y;
  float a;
  if (ax == 0.0f && ay == 0.0f) a = 0.0f;
  else if (ay <= ax) a = ptm_atan_pos_fast(ay / ax);
  else a = 1.57079632679489661923f - ptm_atan_pos_fast(ax / ay);
  if (ptm_f2u(x) >> 31) a = 3.14159265358979323846f - a;
  return (ptm_f2u(y) >> 31) ? -a : a;
}
PTM_FN float ptm_asinf_fast(float x) {
  float ax = x < 0.0f ? -x : x;
  if (ax > 1.0f) return (x - x) / (x - x);
  float z, sq, r;
  int big = ax > 0.5f;
  if (big) {
    z = 0.5f * (1.0f - ax);
    sq = PTM_SQRTF(z);
  } else {
    z = ax * ax;
    sq = ax;
  }
  float p = PTM_FMAF(4.2163199048e-2f, z, 2.4181311049e-2f);
  p = PTM_FMAF(p, z, 4.5470025998e-2f);
  p = PTM_FMAF(p, z, 7.4953002686e-2f);
  p = PTM_FMAF(p, z, 1.6666752422e-1f);
  r = PTM_FMAF(p * z, sq, sq);
  if (big) r = 1.57079632679489661923f - (r + r);
  return x < 0.0f ? -r : r;
}

#endif /* PT_FMATH_H */
