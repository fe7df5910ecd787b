// fastmath.hpp — short-latency f64 math shared by the HIP kernels; also compiles as plain
// C++ (g++) for the host accuracy test.
#pragma once
#include <cmath>
#ifndef __HIP__
#define __host__
#define __device__
#define __forceinline__ inline
#endif

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
__host__ __device__ __forceinline__ double log1p_pos(double t) {
  const double u = 1.0 + t;
  const double c = (t >= 1.0 ? 1.0 - (u - t) : t - (u - 1.0)) * rcp_nr(u);
  int k;
  double m = std::frexp(u, &k);  // [0.5, 1)
  if (m < 0.70710678118654752440) {
    m *= 2.0;
    --k;
  }
  const double f = m - 1.0;
  const double s = f * rcp_nr(2.0 + f);
  const double z = s * s, w = z * z;
  const double t1 = w * (3.999999999940941908e-01 + w * (2.222219843214978396e-01 + w * 1.531383769920937332e-01));
  const double t2 = z * (6.666666666666735130e-01 +
                         w * (2.857142874366239149e-01 + w * (1.818357216161805012e-01 + w * 1.479819860511658591e-01)));
  const double R = t2 + t1, hfsq = 0.5 * f * f, dk = (double)k;
  return dk * 6.93147180369123816490e-01 - ((hfsq - (s * (hfsq + R) + (dk * 1.90821492927058770002e-10 + c))) - f);
}
