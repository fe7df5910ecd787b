// pipeline.hip — configs[4]: SBA + EKF fused on one HBM-resident observation tensor.
//
// The reference runs the two reconstructions as separate drivers over one DLC DataFrame:
// core.sba (src/core/sba.py:27-70: pairwise triangulation, then points-only SBA) and
// core.ekf (src/core/ekf.py:26-298: the nose / lure line fit as the initial state, then the
// EKF + RTS smoother). Here they are one enqueue on the context stream, every stage reading
// the previous stage's device buffers:
//   k_pipe_gather     (S, N, C, L, 2) pixels + likelihoods -> dense SBA slots (S N L, C)
//                     with the core.sba likelihood filter (likelihood > thresh, :41)
//   k_tri_dense       pairwise fisheye triangulation of every (sequence, frame, marker)
//   k_pipe_prune      points no adjacent pair saw leave the SBA (the reference's inner merge
//                     on (frame, marker), src/lib/sba.py:299)
//   k_sba_lm          the fused per-point robust LM (sba.hip)
//   k_pipe_ekf_init   per sequence, the line fits of src/core/ekf.py:121-157 on the SBA points
//                     (fused) or on the triangulated points (core.ekf's own initial state)
//   k_pipe_ekf_gather the EKF model's markers out of the observation tensor (when the model
//                     uses a subset, e.g. the head model on the 20-keypoint DLC output)
//   k_ekf_filter, k_ekf_gain, k_ekf_smooth_x   (ekf.hip)
// No stage copies anything back to the host; a report (SBA convergence, outliers) is the
// only synchronisation, and only when asked for.
#include "common.hpp"
#include "fk.hpp"

// slot (p = (s N + n) L + l, camera c) <- meas[s, n, c, l]; the SBA mask keeps finite pixels
// with likelihood > thresh
__global__ __launch_bounds__(256) void k_pipe_gather(const double* __restrict__ meas, const double* __restrict__ lik,
                                                     int64_t SN, int C, int L, double thresh, double2* __restrict__ uv,
                                                     uint8_t* __restrict__ mask) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (s n, c, l), l fastest
  if (e >= SN * C * L) return;
  const int l = (int)(e % L);
  const int64_t r = e / L;
  const int c = (int)(r % C);
  const int64_t sn = r / C;
  const double2 m = reinterpret_cast<const double2*>(meas)[e];
  const bool ok = lik[e] > thresh && isfinite(m.x) && isfinite(m.y);
  const int64_t slot = (sn * L + l) * C + c;
  uv[slot] = ok ? m : make_double2(0.0, 0.0);
  mask[slot] = ok ? 1 : 0;
}

// a point no adjacent camera pair triangulated is not an SBA point (its start is NaN)
__global__ __launch_bounds__(256) void k_pipe_prune(const int32_t* __restrict__ cnt, int64_t n_pts, int C,
                                                    uint8_t* __restrict__ mask) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_pts * C) return;
  if (cnt[e / C] == 0) mask[e] = 0;
}

// fixed-order workgroup sum (blockDim 256): halving tree through LDS, result to every thread
__device__ double pipe_block_sum(double v, double* s) {
  const int t = threadIdx.x;
  s[t] = v;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (t < h) s[t] += s[t + h];
    __syncthreads();
  }
  const double r = s[0];
  __syncthreads();
  return r;
}

// Least-squares line through (frame, coordinate) of marker `m`'s finite points of sequence
// `seq` (scipy.stats.linregress: slope = S_fx / S_ff about the means, intercept = mean_x -
// slope mean_f), two passes with fixed-order sums. Returns the number of points used.
__device__ int pipe_line_fit(const double* __restrict__ pts, int seq, int N, int L, int m, double* s_red,
                             double slope[2], double icpt[2]) {
  double n = 0.0, sf = 0.0, sx = 0.0, sy = 0.0;
  for (int f = threadIdx.x; f < N; f += blockDim.x) {
    const double* p = pts + 3 * (((size_t)seq * N + f) * L + m);
    if (isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2])) {
      n += 1.0;
      sf += (double)f;
      sx += p[0];
      sy += p[1];
    }
  }
  n = pipe_block_sum(n, s_red);
  sf = pipe_block_sum(sf, s_red);
  sx = pipe_block_sum(sx, s_red);
  sy = pipe_block_sum(sy, s_red);
  if (n < 2.0) return (int)n;
  const double mf = sf / n, mx = sx / n, my = sy / n;
  double sff = 0.0, sfx = 0.0, sfy = 0.0;
  for (int f = threadIdx.x; f < N; f += blockDim.x) {
    const double* p = pts + 3 * (((size_t)seq * N + f) * L + m);
    if (isfinite(p[0]) && isfinite(p[1]) && isfinite(p[2])) {
      const double df = (double)f - mf;
      sff += df * df;
      sfx += df * (p[0] - mx);
      sfy += df * (p[1] - my);
    }
  }
  sff = pipe_block_sum(sff, s_red);
  sfx = pipe_block_sum(sfx, s_red);
  sfy = pipe_block_sum(sfy, s_red);
  slope[0] = sfx / sff;
  slope[1] = sfy / sff;
  icpt[0] = mx - slope[0] * mf;
  icpt[1] = my - slope[1] * mf;
  return (int)n;
}

// src/core/ekf.py:121-157 per sequence (start frame 0 of the sequence): lure x, y and their
// velocities from the lure line (when the model has a lure and it was seen twice), nose x, y,
// velocities and psi_0 = atan2(slope_y, slope_x) from the nose line; every other state 0.
// A sequence whose nose was seen in fewer than two frames gets NaN states and counts in *bad.
__global__ __launch_bounds__(256) void k_pipe_ekf_init(const double* __restrict__ pts, int N, int L, int P,
                                                       acs_ekf_init_spec sp, double sT, double* __restrict__ s0,
                                                       int* __restrict__ bad) {
  __shared__ double s_red[256];
  const int seq = blockIdx.x, n = 3 * P;
  double* s = s0 + (size_t)seq * n;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s[i] = 0.0;
  __syncthreads();
  double sl[2], ic[2];
  if (sp.lure >= 0 && sp.xl >= 0 && sp.yl >= 0) {
    if (pipe_line_fit(pts, seq, N, L, sp.lure, s_red, sl, ic) >= 2 && threadIdx.x == 0) {
      s[sp.xl] = ic[0];
      s[sp.yl] = ic[1];
      s[P + sp.xl] = sl[0] / sT;
      s[P + sp.yl] = sl[1] / sT;
    }
  }
  const int cnt = pipe_line_fit(pts, seq, N, L, sp.nose, s_red, sl, ic);
  if (threadIdx.x == 0) {
    if (cnt >= 2) {
      s[sp.x0] = ic[0];
      s[sp.y0] = ic[1];
      s[sp.psi0] = atan2(sl[1], sl[0]);
      s[P + sp.x0] = sl[0] / sT;
      s[P + sp.y0] = sl[1] / sT;
    } else {
      for (int i = 0; i < n; ++i) s[i] = __builtin_nan("");
      atomicAdd(bad, 1);
    }
  }
}

// EKF model markers out of the observation tensor: out[s n, c, k] = in[s n, c, map[k]]
__global__ __launch_bounds__(256) void k_pipe_ekf_gather(const double* __restrict__ meas, const double* __restrict__ lik,
                                                         int64_t SN, int C, int L, int Le, const int* __restrict__ map,
                                                         double* __restrict__ meas_e, double* __restrict__ lik_e) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= SN * C * Le) return;
  const int k = (int)(e % Le);
  const int64_t r = e / Le;  // (s n) C + c
  const int64_t src = r * L + map[k];
  reinterpret_cast<double2*>(meas_e)[e] = reinterpret_cast<const double2*>(meas)[src];
  lik_e[e] = lik[src];
}

extern "C" {

int acs_sba_ekf_pipeline(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                         int64_t n_reals, const double* cams, int32_t n_cams, const double* meas,
                         const double* likelihood, int32_t n_seq, int32_t n_frames, int32_t n_markers,
                         const int32_t* ekf_markers, double fps, double thresh, double max_pixel_err,
                         const double* r_std_base, const double* Q, const double* P0, const acs_sba_opts* sba_opts,
                         const acs_ekf_init_spec* init, int32_t ref_numerics, double eps, double* pts_out,
                         double* x_est, double* x_smooth, int64_t* outliers, acs_report* sba_report,
                         uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, skel_ints && skel_reals && ekf_markers && init, "pipeline: null descriptor");
  ACS_CHECK(ctx, n_ints >= FK_HDR, "pipeline: skeleton table");
  const int* hdr = skel_ints;  // host descriptor
  const int P = hdr[2], Le = hdr[3], n = 3 * P;
  ACS_CHECK(ctx, n_seq >= 1 && n_frames >= 1 && n_cams >= 2 && n_cams <= 64 && n_markers >= 1 && fps > 0,
            "pipeline: n_seq=%d n_frames=%d n_cams=%d n_markers=%d", n_seq, n_frames, n_cams, n_markers);
  ACS_CHECK(ctx, P >= 3 && P <= FK_MAXP && Le >= 1 && Le <= n_markers, "pipeline: EKF model P=%d L=%d", P, Le);
  bool ident = Le == n_markers;
  for (int k = 0; k < Le; ++k) {
    ACS_CHECK(ctx, ekf_markers[k] >= 0 && ekf_markers[k] < n_markers, "pipeline: ekf_markers[%d]=%d", k,
              ekf_markers[k]);
    ident = ident && ekf_markers[k] == k;
  }
  const acs_ekf_init_spec sp = *init;
  ACS_CHECK(ctx, sp.nose >= 0 && sp.nose < n_markers && sp.lure < n_markers && sp.x0 >= 0 && sp.x0 < P &&
                     sp.y0 >= 0 && sp.y0 < P && sp.psi0 >= 0 && sp.psi0 < P && sp.xl < P && sp.yl < P,
            "pipeline: bad acs_ekf_init_spec");
  const int64_t SN = (int64_t)n_seq * n_frames, n_pts = SN * n_markers;
  hipStream_t s = ctx->stream;
  int rc;
  // inputs (skeleton tables are host descriptors; arrays follow `flags`)
  void *dI, *dR, *dC, *dM, *dL, *dRb, *dQ, *dP0;
  if ((rc = acs_stage_in(ctx, WS_FTE0, skel_ints, sizeof(int32_t) * n_ints, 0, &dI))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE1, skel_reals, sizeof(double) * n_reals, 0, &dR))) return rc;
  if ((rc = acs_stage_in(ctx, WS_CAMS, cams, sizeof(double) * ACS_CAM_STRIDE * n_cams, flags, &dC))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE2, meas, sizeof(double) * n_pts * n_cams * 2, flags, &dM))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE3, likelihood, sizeof(double) * n_pts * n_cams, flags, &dL))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE4, r_std_base, sizeof(double) * n_cams, flags, &dRb))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE7, Q, sizeof(double) * n * n, flags, &dQ))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE8, P0, sizeof(double) * n * n, flags, &dP0))) return rc;
  // stage buffers
  double2* uvp = (double2*)acs_ws(ctx, WS_PIPE0, sizeof(double2) * n_pts * n_cams);
  uint8_t* mk = (uint8_t*)acs_ws(ctx, WS_PIPE1, (size_t)n_pts * n_cams);
  double* pts0 = (double*)acs_ws(ctx, WS_PIPE2, sizeof(double) * 3 * n_pts);
  int32_t* cnt = (int32_t*)acs_ws(ctx, WS_PIPE3, sizeof(int32_t) * n_pts + 256);
  double* s0 = (double*)acs_ws(ctx, WS_PIPE4, sizeof(double) * n_seq * n);
  int* dbad = (int*)(cnt + n_pts);
  double* dpts = (double*)acs_out_buf(ctx, WS_PIPE5, pts_out, sizeof(double) * 3 * n_pts, flags);
  if (!uvp || !mk || !pts0 || !cnt || !s0 || !dpts) return ACS_E_NOMEM;
  // 1. observations -> SBA slots; 2. triangulation; 3. prune; 4. SBA
  hipLaunchKernelGGL(k_pipe_gather, dim3(acs_grid(n_pts * n_cams, 256)), dim3(256), 0, s, (const double*)dM,
                     (const double*)dL, SN, n_cams, n_markers, thresh, uvp, mk);
  ACS_HIP(ctx, hipGetLastError());
  if ((rc = acs_tri_dense_enqueue(ctx, (const double*)dC, n_cams, (const double*)uvp, mk, n_pts, pts0, cnt)))
    return rc;
  hipLaunchKernelGGL(k_pipe_prune, dim3(acs_grid(n_pts * n_cams, 256)), dim3(256), 0, s, (const int32_t*)cnt, n_pts,
                     n_cams, mk);
  ACS_HIP(ctx, hipGetLastError());
  if ((rc = acs_sba_dense_enqueue(ctx, (const double*)dC, n_cams, uvp, mk, n_pts, pts0, dpts, sba_opts, sba_report)))
    return rc;
  // 5. EKF initial states
  ACS_HIP(ctx, hipMemsetAsync(dbad, 0, sizeof(int), s));
  hipLaunchKernelGGL(k_pipe_ekf_init, dim3(n_seq), dim3(256), 0, s, sp.from_sba ? (const double*)dpts : pts0,
                     n_frames, n_markers, P, sp, 1.0 / fps, s0, dbad);
  ACS_HIP(ctx, hipGetLastError());
  // 6. the EKF model's observations
  const double *dMe = (const double*)dM, *dLe = (const double*)dL;
  if (!ident) {
    int* dmap = (int*)acs_ws(ctx, WS_PIPE6, sizeof(int) * ((Le + 3) & ~3) + sizeof(double) * SN * n_cams * Le * 3);
    if (!dmap) return ACS_E_NOMEM;
    double* me = (double*)(dmap + ((Le + 3) & ~3));  // 16-byte aligned: stored through double2
    double* le = me + SN * n_cams * Le * 2;
    ACS_HIP(ctx, hipMemcpyAsync(dmap, ekf_markers, sizeof(int) * Le, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_pipe_ekf_gather, dim3(acs_grid(SN * n_cams * Le, 256)), dim3(256), 0, s, (const double*)dM,
                       (const double*)dL, SN, n_cams, n_markers, Le, (const int*)dmap, me, le);
    ACS_HIP(ctx, hipGetLastError());
    dMe = me;
    dLe = le;
  }
  // 7. EKF + RTS smoother
  EkfIo io;
  io.I = (const int*)dI;
  io.R = (const double*)dR;
  io.cams = (const double*)dC;
  io.meas = dMe;
  io.lik = dLe;
  io.rstd = (const double*)dRb;
  io.Q = (const double*)dQ;
  io.P0 = (const double*)dP0;
  io.s0 = s0;
  io.x_est = (double*)acs_out_buf(ctx, WS_FTE11, x_est, sizeof(double) * SN * n, flags);
  io.x_smooth = (double*)acs_out_buf(ctx, WS_FTE12, x_smooth, sizeof(double) * SN * n, flags);
  if (!io.x_est || !io.x_smooth) return ACS_E_NOMEM;
  if ((rc = acs_ekf_enqueue(ctx, (int)n_ints, (int)n_reals, hdr, n_cams, n_seq, n_frames, fps, thresh, max_pixel_err,
                            eps, ref_numerics, io)))
    return rc;
  if ((rc = acs_stage_out(ctx, pts_out, dpts, sizeof(double) * 3 * n_pts, flags))) return rc;
  if ((rc = acs_stage_out(ctx, x_est, io.x_est, sizeof(double) * SN * n, flags))) return rc;
  if ((rc = acs_stage_out(ctx, x_smooth, io.x_smooth, sizeof(double) * SN * n, flags))) return rc;
  if (outliers || !(flags & ACS_DEVICE_PTRS)) {
    std::vector<long long> ho(n_seq);
    int hbad = 0, hsing = 0;
    ACS_HIP(ctx, hipMemcpyAsync(ho.data(), io.outliers, sizeof(long long) * n_seq, hipMemcpyDeviceToHost, s));
    ACS_HIP(ctx, hipMemcpyAsync(&hbad, dbad, sizeof(int), hipMemcpyDeviceToHost, s));
    ACS_HIP(ctx, hipMemcpyAsync(&hsing, io.bad, sizeof(int), hipMemcpyDeviceToHost, s));
    ACS_HIP(ctx, hipStreamSynchronize(s));
    if (outliers)
      for (int q = 0; q < n_seq; ++q) outliers[q] = ho[q];
    ACS_CHECK(ctx, hbad == 0, "pipeline: %d sequence(s) with the nose in fewer than two frames (no initial state, "
                              "src/core/ekf.py:144-152)", hbad);
    ACS_CHECK(ctx, hsing == 0, "pipeline: %d singular EKF solve(s) (I + A P_xx or P_pred)", hsing);
  }
  return ACS_OK;
}

}  // extern "C"
