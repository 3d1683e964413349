/*
 * pt_fmath.h -- the path tracer's float32 transcendentals, bit-reproducible
 * across the CPU and the GPU.
 *
 * GLSL leaves sin/cos/atan/asin/log/pow precision to the driver (the
 * reference's pass1.fsh uses them at IS:148-149,176,489-490,502-505,525,
 * 582,639,660), so no reference output pins them to the ulp. This header fixes
 * them as part of the numerics contract: Cephes-style argument reduction +
 * minimax polynomials (S. L. Moshier's single-precision coefficients), written
 * with only correctly-rounded IEEE operations (+, -, *, /, sqrtf) and explicit
 * fused multiply-adds (fmaf), so the HIP kernels (v_fma_f32) and the CPU
 * checker (x86 FMA / glibc fmaf) produce identical bits. Accuracy against a
 * float64 libm is tested in tests/test_fmath.py: sin 2, cos 5 (abs 2e-8 near
 * its zeros), atan2 4, asin 3, log 1, exp 1, pow 16 ulp on the ranges used;
 * GLSL only requires sin/cos to 2^-11 absolute.
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

#ifdef __cplusplus
#include <cmath>
#define PTM_FMA(a, b, c) ::fmaf((a), (b), (c))
#define PTM_SQRT(a) ::sqrtf(a)
#define PTM_FLOOR(a) ::floorf(a)
#else
#include <math.h>
#define PTM_FMA(a, b, c) fmaf((a), (b), (c))
#define PTM_SQRT(a) sqrtf(a)
#define PTM_FLOOR(a) floorf(a)
#endif
#include <stdint.h>

PTM_FN uint32_t ptm_f2u(float f) { uint32_t u; __builtin_memcpy(&u, &f, 4); return u; }
PTM_FN float ptm_u2f(uint32_t u) { float f; __builtin_memcpy(&f, &u, 4); return f; }

#define PTM_PIO2_1 1.5703125f               /* pi/2 in three parts (Cody-Waite) */
#define PTM_PIO2_2 4.837512969970703125e-4f
#define PTM_PIO2_3 7.54978995489188216e-8f
#define PTM_2OPI 0.636619772367581343f
#define PTM_PIO2 1.57079632679489661923f
#define PTM_PIO4 0.785398163397448309616f

/* sin and cos of r in [-pi/4, pi/4] */
PTM_FN float ptm_sin_kernel(float r) {
  float z = r * r;
  float p = PTM_FMA(-1.9515295891e-4f, z, 8.3321608736e-3f);
  p = PTM_FMA(p, z, -1.6666654611e-1f);
  return PTM_FMA(p * z, r, r);
}
PTM_FN float ptm_cos_kernel(float r) {
  float z = r * r;
  float p = PTM_FMA(2.443315711809948e-5f, z, -1.388731625493765e-3f);
  p = PTM_FMA(p, z, 4.166664568298827e-2f);
  return PTM_FMA(p * z, z, PTM_FMA(-0.5f, z, 1.0f));
}
/* range reduction x = k*pi/2 + r, |x| up to ~1e5 */
PTM_FN float ptm_reduce(float x, int* q) {
  float k = PTM_FLOOR(PTM_FMA(x, PTM_2OPI, 0.5f));
  float r = PTM_FMA(-k, PTM_PIO2_1, x);
  r = PTM_FMA(-k, PTM_PIO2_2, r);
  r = PTM_FMA(-k, PTM_PIO2_3, r);
  *q = (int)k;
  return r;
}
PTM_FN float ptm_sinf(float x) {
  int q;
  float r = ptm_reduce(x, &q);
  float s = (q & 1) ? ptm_cos_kernel(r) : ptm_sin_kernel(r);
  return (q & 2) ? -s : s;
}
PTM_FN float ptm_cosf(float x) {
  int q;
  float r = ptm_reduce(x, &q);
  float c = (q & 1) ? ptm_sin_kernel(r) : ptm_cos_kernel(r);
  return ((q + 1) & 2) ? -c : c;
}
PTM_FN void ptm_sincosf(float x, float* s, float* c) {
  int q;
  float r = ptm_reduce(x, &q);
  float sk = ptm_sin_kernel(r), ck = ptm_cos_kernel(r);
  float ss = (q & 1) ? ck : sk;
  float cc = (q & 1) ? sk : ck;
  *s = (q & 2) ? -ss : ss;
  *c = ((q + 1) & 2) ? -cc : cc;
}

/* atan(t) for t >= 0 */
PTM_FN float ptm_atan_pos(float t) {
  float base = 0.0f, x = t;
  if (t > 2.414213562373095f) {
    base = PTM_PIO2;
    x = -1.0f / t;
  } else if (t > 0.4142135623730950f) {
    base = PTM_PIO4;
    x = (t - 1.0f) / (t + 1.0f);
  }
  float z = x * x;
  float p = PTM_FMA(8.05374449538e-2f, z, -1.38776856032e-1f);
  p = PTM_FMA(p, z, 1.99777106478e-1f);
  p = PTM_FMA(p, z, -3.33329491539e-1f);
  return base + PTM_FMA(p * z, x, x);
}
PTM_FN float ptm_atan2f(float y, float x) {
  if (y != y || x != x) return y + x;
  float ax = x < 0.0f ? -x : x, ay = y < 0.0f ? -y : y;
  float a;
  if (ax == 0.0f && ay == 0.0f) {
    a = 0.0f;
  } else if (ay <= ax) {
    a = ptm_atan_pos(ay / ax);
  } else {
    a = PTM_PIO2 - ptm_atan_pos(ax / ay);
  }
  if (ptm_f2u(x) >> 31) a = 3.14159265358979323846f - a; /* x < 0 or x == -0: libm's signed-zero rules */
  return (ptm_f2u(y) >> 31) ? -a : a;
}

PTM_FN float ptm_asinf(float x) {
  float ax = x < 0.0f ? -x : x;
  if (ax > 1.0f) return (x - x) / (x - x); /* NaN */
  float z, s, r;
  int big = ax > 0.5f;
  if (big) {
    z = 0.5f * (1.0f - ax);
    s = PTM_SQRT(z);
  } else {
    z = ax * ax;
    s = ax;
  }
  float p = PTM_FMA(4.2163199048e-2f, z, 2.4181311049e-2f);
  p = PTM_FMA(p, z, 4.5470025998e-2f);
  p = PTM_FMA(p, z, 7.4953002686e-2f);
  p = PTM_FMA(p, z, 1.6666752422e-1f);
  r = PTM_FMA(p * z, s, s);
  if (big) r = PTM_PIO2 - (r + r);
  return x < 0.0f ? -r : r;
}

/* natural log, x > 0 normal or subnormal */
PTM_FN float ptm_logf(float x) {
  if (x != x || x < 0.0f) return (x - x) / (x - x);
  if (x == 0.0f) return -1.0f / 0.0f;
  if (x > 3.40282346e38f) return x;
  int e = 0;
  if (x < 1.17549435e-38f) { x *= 16777216.0f; e = -24; } /* subnormal */
  uint32_t u = ptm_f2u(x);
  e += (int)((u >> 23) & 0xff) - 126;
  float m = ptm_u2f((u & 0x007fffffu) | 0x3f000000u); /* [0.5, 1) */
  if (m < 0.70710678118654752f) {
    e -= 1;
    m = m + m - 1.0f;
  } else {
    m = m - 1.0f;
  }
  float z = m * m;
  float p = PTM_FMA(7.0376836292e-2f, m, -1.1514610310e-1f);
  p = PTM_FMA(p, m, 1.1676998740e-1f);
  p = PTM_FMA(p, m, -1.2420140846e-1f);
  p = PTM_FMA(p, m, 1.4249322787e-1f);
  p = PTM_FMA(p, m, -1.6668057665e-1f);
  p = PTM_FMA(p, m, 2.0000714765e-1f);
  p = PTM_FMA(p, m, -2.4999993993e-1f);
  p = PTM_FMA(p, m, 3.3333331174e-1f);
  float y = p * m * z;
  float fe = (float)e;
  y = PTM_FMA(fe, -2.12194440e-4f, y);
  y = PTM_FMA(-0.5f, z, y);
  float r = m + y;
  return PTM_FMA(fe, 0.693359375f, r);
}

PTM_FN float ptm_expf(float x) {
  if (x != x) return x;
  if (x > 88.72283905206835f) return 1.0f / 0.0f;
  if (x < -103.97208f) return 0.0f;
  float n = PTM_FLOOR(PTM_FMA(x, 1.44269504088896341f, 0.5f));
  float r = PTM_FMA(-n, 0.693359375f, x);
  r = PTM_FMA(-n, -2.12194440e-4f, r);
  float z = r * r;
  float p = PTM_FMA(1.9875691500e-4f, r, 1.3981999507e-3f);
  p = PTM_FMA(p, r, 8.3334519073e-3f);
  p = PTM_FMA(p, r, 4.1665795894e-2f);
  p = PTM_FMA(p, r, 1.6666665459e-1f);
  p = PTM_FMA(p, r, 5.0000001201e-1f);
  float y = PTM_FMA(p, z, r) + 1.0f;
  int k = (int)n;
  /* y * 2^k in two steps so 2^k never under/overflows on its own */
  int k1 = k / 2, k2 = k - k1;
  y = y * ptm_u2f((uint32_t)(k1 + 127) << 23);
  return y * ptm_u2f((uint32_t)(k2 + 127) << 23);
}

/* pow for x > 0 (the only use: SampleGTR1 IS:525 and the tonemap gamma) */
PTM_FN float ptm_powf(float x, float y) {
  if (y == 0.0f) return 1.0f;
  if (x == 1.0f) return 1.0f;
  if (x == 0.0f) return y > 0.0f ? 0.0f : 1.0f / 0.0f;
  if (x < 0.0f) return (x - x) / (x - x);
  return ptm_expf(y * ptm_logf(x));
}

#endif /* PT_FMATH_H */
