// fastmath.hpp — short-latency f64 math shared by the HIP kernels; also compiles as plain
// C++ (g++) for the host accuracy test.
#pragma once
#include <cmath>
#ifndef __HIP__
#define __host__
#define __device__
#define __forceinline__ inline
#endif

// Horner step c + z * acc as one v_fma_f64 with a separate destination. Written plainly, the
// compiler keeps the (hoisted) polynomial constant in a VGPR and emits v_mov_b64 + v_fmac_f64
// (the accumulate form ties the addend to the destination): two issue slots per term on the
// latency-bound LM chains of k_sba_lm.
__host__ __device__ __forceinline__ double hfma(double z, double acc, double c) {
#ifdef __HIP_DEVICE_COMPILE__
  double d;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(z), "v"(acc), "v"(c));
  return d;
#else
  return std::fma(z, acc, c);
#endif
}

// ------------------------------------------------------------------------------------
// Short-latency f64 math for the per-iteration dependency chains (measured on gfx950,
// tools/probe/valu_lat_probe.hip: IEEE 1/x 72 cycles, sqrt 109, log1p 569; v_rcp_f64 +
// two Newton steps 39, v_rsq_f64 + two Newton steps 49). Each result is within ~1 ulp of
// the correctly rounded value (tests/test_fastmath.py builds this header with g++ and checks
// it against libm). On the host the hardware estimates are replaced by the exact operation.
// ------------------------------------------------------------------------------------
__host__ __device__ __forceinline__ double rcp_nr(double p) {
#ifdef __HIP_DEVICE_COMPILE__
  double r = __builtin_amdgcn_rcp(p);
  r = fma(r, fma(-p, r, 1.0), r);
  return fma(r, fma(-p, r, 1.0), r);
#else
  return 1.0 / p;
#endif
}
// 1/sqrt(x), x > 0
__host__ __device__ __forceinline__ double rsq_nr(double x) {
#ifdef __HIP_DEVICE_COMPILE__
  const double h = 0.5 * x;
  double r = __builtin_amdgcn_rsq(x);
  r = r * fma(-h * r, r, 1.5);
  return r * fma(-h * r, r, 1.5);
#else
  return 1.0 / std::sqrt(x);
#endif
}
// log1p(t) for t >= 0 (finite): u = 1 + t with its exact rounding error c, u = 2^k m with
// m in [1/sqrt2, sqrt2), log m = f - f^2/2 + s (f^2/2 + R(s^2)), s = f / (2 + f), f = m - 1
// (the classic fdlibm reduction and minimax coefficients), one reciprocal, no table.
// log1p_pos with u = 1 + t and ru ~ 1 / u already formed by the caller (k_sba_lm shares that
// reciprocal with the Cauchy weights)
__host__ __device__ __forceinline__ double log1p_pos_ur(double t, double u, double ru) {
  const double c = (t >= 1.0 ? 1.0 - (u - t) : t - (u - 1.0)) * ru;
  int k;
  double m = std::frexp(u, &k);  // [0.5, 1)
  if (m < 0.70710678118654752440) {
    m *= 2.0;
    --k;
  }
  const double f = m - 1.0;
  const double s = f * rcp_nr(2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * hfma(w, hfma(w, 1.531383769920937332e-01, 2.222219843214978396e-01), 3.999999999940941908e-01);
  const double t2 =
      z * hfma(w, hfma(w, hfma(w, 1.479819860511658591e-01, 1.818357216161805012e-01), 2.857142874366239149e-01),
               6.666666666666735130e-01);
  const double R = t2 + t1, hfsq = 0.5 * f * f, dk = (double)k;
  return dk * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + (dk * 1.90821492927058770002e-10 + c))) - f);
}
__host__ __device__ __forceinline__ double log1p_pos(double t) {
  const double u = 1.0 + t;
  return log1p_pos_ur(t, u, rcp_nr(u));
}

// atan(x) for x >= 0 with one reciprocal: |v| <= tan(pi/8) after
//   x <= tan(pi/8):            v = x,                 atan x = atan v
//   tan(pi/8) < x <= tan(3pi/8): v = (x - 1)/(x + 1),   atan x = pi/4 + atan v
//   x > tan(3pi/8):            v = -1/x,               atan x = pi/2 + atan v
// and atan v = v - v (z S1(z^2) + z^2 S2(z^2)), z = v^2, with the fdlibm minimax
// coefficients for |v| < 7/16 (odd and even halves evaluated as two independent chains).
__host__ __device__ __forceinline__ double atan_pos(double x) {
  const bool a = x <= 0.41421356237309504880, c = x > 2.41421356237309504880;
  const double num = a ? x : (c ? -1.0 : x - 1.0);
  const double den = a ? 1.0 : (c ? x : x + 1.0);
  const double v = a ? x : num * rcp_nr(den);
  const double hi = a ? 0.0 : (c ? 1.57079632679489655800e+00 : 7.85398163397448278999e-01);
  const double lo = a ? 0.0 : (c ? 6.12323399573676603587e-17 : 3.06161699786838301793e-17);
  const double z = v * v, w = z * z;
  const double s1 =
      z * hfma(w,
               hfma(w,
                    hfma(w, hfma(w, hfma(w, 1.62858201153657823623e-02, 4.97687799461593236017e-02),
                                 6.66107313738753120669e-02),
                         9.09088713343650656196e-02),
                    1.42857142725034663711e-01),
               3.33333333333329318027e-01);
  const double s2 =
      w * hfma(w,
               hfma(w, hfma(w, hfma(w, -3.65315727442169155270e-02, -5.83357013379057348645e-02),
                            -7.69187620504482999495e-02),
                    -1.11111104054623557880e-01),
               -1.99999999998764832476e-01);
  return hi + ((v - v * (s1 + s2)) + lo);
}
