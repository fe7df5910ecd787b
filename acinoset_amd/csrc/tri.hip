// tri.hip — fisheye triangulation on gfx950 (the SBA / FTE initialisation).
//
// triangulate_points_fisheye (src/lib/calib.py:120-129): cv::fisheye::undistortPoints
// (Newton on theta, default criteria: 10 iterations, eps 1e-8, non-converged or
// theta-flipped points -> -1e6) of both views, then cv::triangulatePoints' homogeneous
// DLT: the right singular vector of the smallest singular value of the 4x4 system,
// here by one-sided (Hestenes) Jacobi in registers, one thread per pair.
// get_pairwise_3d_points_from_df (src/lib/utils.py:319-349): adjacent camera pairs
// (c, c+1 mod C) of every (frame, marker) seen by both, mean over the pairs in pair order.
#include "common.hpp"

__device__ void fisheye_undistort(const double* __restrict__ c, double u, double v, double& xn, double& yn) {
  const double pwx = (u - c[2]) / c[0], pwy = (v - c[3]) / c[1];
  double theta_d = sqrt(pwx * pwx + pwy * pwy);
  theta_d = fmin(fmax(-M_PI / 2.0, theta_d), M_PI / 2.0);
  bool converged = false;
  double theta = theta_d, scale = 0.0;
  if (fabs(theta_d) > 1e-8) {
    for (int j = 0; j < 10; ++j) {
      const double t2 = theta * theta, t4 = t2 * t2, t6 = t4 * t2, t8 = t6 * t2;
      const double k0t2 = c[4] * t2, k1t4 = c[5] * t4, k2t6 = c[6] * t6, k3t8 = c[7] * t8;
      const double fix = (theta * (1 + k0t2 + k1t4 + k2t6 + k3t8) - theta_d) /
                         (1 + 3 * k0t2 + 5 * k1t4 + 7 * k2t6 + 9 * k3t8);
      theta = theta - fix;
      if (fabs(fix) < 1e-8) {
        converged = true;
        break;
      }
    }
    scale = tan(theta) / theta_d;
  } else {
    converged = true;
  }
  const bool flipped = (theta_d < 0 && theta > 0) || (theta_d > 0 && theta < 0);
  if (converged && !flipped) {
    xn = pwx * scale;
    yn = pwy * scale;
  } else {
    xn = yn = -1e6;
  }
}

// Null vector of a 4x4 (row-major) by one-sided Jacobi on its columns.
__device__ void dlt_null4(double A[16], double out[4]) {
  double V[16];
  for (int i = 0; i < 16; ++i) V[i] = (i % 5 == 0) ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 30; ++sweep) {
    // a pair is rotated while |gamma| / sqrt(alpha beta) >= 1e-15, tested squared (no square
    // root or division); the sweeps stop when no pair was. Rotation by the short-latency
    // reciprocal / reciprocal square root (fastmath.hpp, ~1 ulp)
    bool any = false;
#pragma unroll
    for (int p = 0; p < 3; ++p)
#pragma unroll
      for (int q = p + 1; q < 4; ++q) {
        double alpha = 0.0, beta = 0.0, gamma = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          alpha += A[i * 4 + p] * A[i * 4 + p];
          beta += A[i * 4 + q] * A[i * 4 + q];
          gamma += A[i * 4 + p] * A[i * 4 + q];
        }
        if (gamma == 0.0) continue;
        if (gamma * gamma < 1e-30 * (alpha * beta)) continue;
        any = true;
        const double zeta = (beta - alpha) * rcp_nr(2.0 * gamma);
        const double z2 = 1.0 + zeta * zeta;
        const double t = (zeta >= 0 ? 1.0 : -1.0) * rcp_nr(fabs(zeta) + z2 * rsq_nr(z2));
        const double cs = rsq_nr(1.0 + t * t), sn = cs * t;
        for (int i = 0; i < 4; ++i) {
          const double ap = A[i * 4 + p], aq = A[i * 4 + q];
          A[i * 4 + p] = cs * ap - sn * aq;
          A[i * 4 + q] = sn * ap + cs * aq;
          const double vp = V[i * 4 + p], vq = V[i * 4 + q];
          V[i * 4 + p] = cs * vp - sn * vq;
          V[i * 4 + q] = sn * vp + cs * vq;
        }
      }
    if (!any) break;
  }
  int best = 0;
  double bn = 1e300;
  for (int j = 0; j < 4; ++j) {
    double n2 = 0.0;
    for (int i = 0; i < 4; ++i) n2 += A[i * 4 + j] * A[i * 4 + j];
    if (n2 < bn) {
      bn = n2;
      best = j;
    }
  }
  for (int i = 0; i < 4; ++i) out[i] = V[i * 4 + best];
}

// the DLT of one pair from both views' undistorted points
__device__ void triangulate_und(const double* ca, const double* cb, double xa, double ya, double xb, double yb,
                                double X[3]) {
  // P = [R | t]; rows: x*P2 - P0, y*P2 - P1
  const double* Ra = ca + 8;
  const double* ta = ca + 17;
  const double* Rb = cb + 8;
  const double* tb = cb + 17;
  double A[16];
  for (int j = 0; j < 4; ++j) {
    const double pa0 = j < 3 ? Ra[j] : ta[0], pa1 = j < 3 ? Ra[3 + j] : ta[1], pa2 = j < 3 ? Ra[6 + j] : ta[2];
    const double pb0 = j < 3 ? Rb[j] : tb[0], pb1 = j < 3 ? Rb[3 + j] : tb[1], pb2 = j < 3 ? Rb[6 + j] : tb[2];
    A[0 * 4 + j] = xa * pa2 - pa0;
    A[1 * 4 + j] = ya * pa2 - pa1;
    A[2 * 4 + j] = xb * pb2 - pb0;
    A[3 * 4 + j] = yb * pb2 - pb1;
  }
  double h[4];
  dlt_null4(A, h);
  X[0] = h[0] / h[3];
  X[1] = h[1] / h[3];
  X[2] = h[2] / h[3];
}

__device__ void triangulate_one(const double* ca, const double* cb, double ua, double va, double ub, double vb,
                                double X[3]) {
  double xa, ya, xb, yb;
  fisheye_undistort(ca, ua, va, xa, ya);
  fisheye_undistort(cb, ub, vb, xb, yb);
  triangulate_und(ca, cb, xa, ya, xb, yb, X);
}

__global__ __launch_bounds__(256) void k_tri_pairs(const double* __restrict__ cams, int n_cams,
                                                   const double* __restrict__ uva, const double* __restrict__ uvb,
                                                   const int32_t* __restrict__ ca, const int32_t* __restrict__ cb,
                                                   int64_t n, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int a = ca[i], b = cb[i];
  if (a < 0 || a >= n_cams || b < 0 || b >= n_cams) {
    out[3 * i] = out[3 * i + 1] = out[3 * i + 2] = __builtin_nan("");
    return;
  }
  double X[3];
  triangulate_one(cams + a * ACS_CAM_STRIDE, cams + b * ACS_CAM_STRIDE, uva[2 * i], uva[2 * i + 1], uvb[2 * i],
                  uvb[2 * i + 1], X);
  out[3 * i] = X[0];
  out[3 * i + 1] = X[1];
  out[3 * i + 2] = X[2];
}

__global__ __launch_bounds__(256) void k_tri_dense(const double* __restrict__ cams, int C,
                                                   const double* __restrict__ uv, const uint8_t* __restrict__ mask,
                                                   int64_t n_pts, double* __restrict__ out, int32_t* __restrict__ cnt) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pts) return;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  int n = 0;
  // every observed view undistorted once: camera c's point serves the pairs (c - 1, c) and
  // (c, c + 1) (triangulate_one undistorted it for both); camera 0's is kept for the last pair
  const bool m0 = mask[p * C] != 0;
  double x0 = 0.0, y0 = 0.0;
  if (m0) fisheye_undistort(cams, uv[p * C * 2], uv[p * C * 2 + 1], x0, y0);
  double xa = x0, ya = y0;
  bool ma = m0;
  for (int c = 0; c < C; ++c) {
    const int c2 = (c + 1) % C;
    const bool mb = mask[p * C + c2] != 0;
    double xb = x0, yb = y0;
    if (c2 != 0 && mb)
      fisheye_undistort(cams + c2 * ACS_CAM_STRIDE, uv[(p * C + c2) * 2], uv[(p * C + c2) * 2 + 1], xb, yb);
    if (ma && mb) {
      double X[3];
      triangulate_und(cams + c * ACS_CAM_STRIDE, cams + c2 * ACS_CAM_STRIDE, xa, ya, xb, yb, X);
      s0 += X[0];
      s1 += X[1];
      s2 += X[2];
      ++n;
    }
    xa = xb;
    ya = yb;
    ma = mb;
  }
  const double nan = __builtin_nan("");
  out[3 * p] = n ? s0 / n : nan;
  out[3 * p + 1] = n ? s1 / n : nan;
  out[3 * p + 2] = n ? s2 / n : nan;
  if (cnt) cnt[p] = n;
}

int acs_tri_dense_enqueue(acs_ctx* ctx, const double* dcams, int C, const double* duv, const uint8_t* dmask,
                          int64_t n_pts, double* dout, int32_t* dcnt) {
  if (n_pts == 0) return ACS_OK;
  hipLaunchKernelGGL(k_tri_dense, dim3(acs_grid(n_pts, 256)), dim3(256), 0, ctx->stream, dcams, C, duv, dmask, n_pts,
                     dout, dcnt);
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

extern "C" {

int acs_triangulate_pairs(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv_a, const double* uv_b,
                          const int32_t* cam_a, const int32_t* cam_b, int64_t n, double* xyz_out, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, n >= 0 && n_cams >= 1, "acs_triangulate_pairs: bad sizes");
  if (n == 0) return ACS_OK;
  void *dc, *da, *db, *dca, *dcb;
  int rc;
  if ((rc = acs_stage_in(ctx, WS_CAMS, cams, sizeof(double) * ACS_CAM_STRIDE * n_cams, flags, &dc))) return rc;
  if ((rc = acs_stage_in(ctx, WS_TMP0, uv_a, sizeof(double) * 2 * n, flags, &da))) return rc;
  if ((rc = acs_stage_in(ctx, WS_TMP1, uv_b, sizeof(double) * 2 * n, flags, &db))) return rc;
  if ((rc = acs_stage_in(ctx, WS_TMP2, cam_a, sizeof(int32_t) * n, flags, &dca))) return rc;
  if ((rc = acs_stage_in(ctx, WS_TMP3, cam_b, sizeof(int32_t) * n, flags, &dcb))) return rc;
  double* dout = (double*)acs_out_buf(ctx, WS_OUT0, xyz_out, sizeof(double) * 3 * n, flags);
  if (!dout) return ACS_E_NOMEM;
  hipLaunchKernelGGL(k_tri_pairs, dim3(acs_grid(n, 256)), dim3(256), 0, ctx->stream, (const double*)dc, n_cams,
                     (const double*)da, (const double*)db, (const int32_t*)dca, (const int32_t*)dcb, n, dout);
  ACS_HIP(ctx, hipGetLastError());
  if ((rc = acs_stage_out(ctx, xyz_out, dout, sizeof(double) * 3 * n, flags))) return rc;
  if (!(flags & ACS_DEVICE_PTRS)) ACS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ACS_OK;
}

int acs_triangulate_dense(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv, const uint8_t* mask,
                          int64_t n_pts, double* xyz_out, int32_t* n_pairs_out, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, n_pts >= 0 && n_cams >= 2, "acs_triangulate_dense: bad sizes");
  if (n_pts == 0) return ACS_OK;
  void *dc, *duv, *dm;
  int rc;
  if ((rc = acs_stage_in(ctx, WS_CAMS, cams, sizeof(double) * ACS_CAM_STRIDE * n_cams, flags, &dc))) return rc;
  if ((rc = acs_stage_in(ctx, WS_UV, uv, sizeof(double) * 2 * n_pts * n_cams, flags, &duv))) return rc;
  if ((rc = acs_stage_in(ctx, WS_MASK, mask, (size_t)n_pts * n_cams, flags, &dm))) return rc;
  double* dout = (double*)acs_out_buf(ctx, WS_OUT0, xyz_out, sizeof(double) * 3 * n_pts, flags);
  int32_t* dcnt = n_pairs_out ? (int32_t*)acs_out_buf(ctx, WS_OUT1, n_pairs_out, sizeof(int32_t) * n_pts, flags)
                              : nullptr;
  if (!dout || (n_pairs_out && !dcnt)) return ACS_E_NOMEM;
  if ((rc = acs_tri_dense_enqueue(ctx, (const double*)dc, n_cams, (const double*)duv, (const uint8_t*)dm, n_pts, dout,
                                   dcnt)))
    return rc;
  if ((rc = acs_stage_out(ctx, xyz_out, dout, sizeof(double) * 3 * n_pts, flags))) return rc;
  if (n_pairs_out && (rc = acs_stage_out(ctx, n_pairs_out, dcnt, sizeof(int32_t) * n_pts, flags))) return rc;
  if (!(flags & ACS_DEVICE_PTRS)) ACS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ACS_OK;
}

}  // extern "C"
