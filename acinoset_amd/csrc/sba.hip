// sba.hip — points-only sparse bundle adjustment on gfx950.
//
// Replaces the numeric body of bundle_adjust_points_only (src/lib/sba.py:181-195):
// scipy least_squares(trf, loss='cauchy', f_scale=50) over cost_func_points_only
// (src/lib/sba.py:149-153). With the cameras fixed the Jacobian sparsity
// (src/lib/sba.py:11-22) is block-diagonal per 3-D point, so the solve is a batch of
// independent 3-parameter robust least-squares problems.
//
// Mapping: one point = one aligned group of G lanes (G = next pow2 of the observation
// slots, <= 64) — lane l owns slot l (+ j*G). Observations are an (n_pts, K) slot tensor
// (slot = camera for the dense core.sba layout) read once, coalesced, into registers;
// the camera records are staged in LDS (the HOIST instance loads each lane's record into its
// registers instead). Each LM iteration: every lane projects its
// observation(s) and forms its contribution to the gradient g = sum rho'(z) r J (3), the
// Gauss-Newton matrix H = sum max(rho' + 2 z rho'', 0.1 rho') J^T J (6; Triggs-corrected,
// which converges quadratically where IRLS weights only converge linearly) and the Cauchy
// cost (1); a butterfly __shfl_xor reduction inside the group gives every lane
// bit-identical sums, so all lanes take the same accept/reject decision with no LDS
// round trip and no atomics. The whole LM loop runs inside one launch: HBM traffic is
// the observation tensor once plus the points in and out.
//
// LM spec (shared with oracle/sba.py): lam0 = 1e-3, Marquardt damping H + lam*diag(H),
// xtol default 1e-9 (scipy's default, used by the reference, is 1e-8),
// accept on strict decrease (lam /= 10, floor 1e-15), reject (lam *= 10); stop on
// gtol / ftol / xtol / lam > 1e16 / max_iters.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

struct SbaParams {
  int max_iters;
  double f_scale, ftol, xtol, gtol;
};

// HOIST: each lane keeps its camera record in registers for the whole LM loop instead of
// re-reading it from LDS in every projection (198 VGPRs: 2 waves per SIMD), chosen for
// grids of at most 2 waves per SIMD, where nothing else would fill the SIMD anyway.
// The other instances are not occupancy-bound either: <4, 3> (the configs[4] shape) holds 186
// VGPRs, 2 waves per SIMD, and register budgets for 2 / 3 / 4 waves per SIMD
// (amdgpu_waves_per_eu) ran it in 0.270 / 0.273 / 0.454 ms against 0.268-0.272 unconstrained
// (profiles/r06/bench_sba_w*_r06h.log): three independent slot chains per lane already keep the
// VALU issuing, and the 4-wave budget spills.
template <int G, int S, bool CAMID, bool HOIST>
__global__ __launch_bounds__(256) void k_sba_lm(const double* __restrict__ cams, int C, int K,
                                                const double2* __restrict__ uv,
                                                const uint8_t* __restrict__ mask,
                                                const uint8_t* __restrict__ camid, int64_t n_pts,
                                                const double* pts_in, double* pts,  // may alias
                                                SbaParams prm,
                                                double* __restrict__ cost0, double* __restrict__ cost1,
                                                int* __restrict__ stat) {
  extern __shared__ double s_cam[];
  const int lane = threadIdx.x & (G - 1);
  const int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const bool live = p < n_pts;
  // every global load is issued before the first wait: the slot's observation, its mask and
  // camera id, and the point (none depends on another), then the camera records for LDS.
  // One memory round trip instead of three before the LM loop starts.
  double2 q[S];
  uint8_t mk[S], cid[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int slot = lane + s * G;
    q[s] = double2{0.0, 0.0};
    mk[s] = 0;
    cid[s] = (uint8_t)slot;
    if (live && slot < K) {
      const int64_t o = p * K + slot;
      mk[s] = mask[o];
      q[s] = uv[o];
      if (CAMID) cid[s] = camid[o];
    }
  }
  double x0 = 0.0, x1 = 0.0, x2 = 0.0;
  if (live) {
    x0 = pts_in[3 * p];
    x1 = pts_in[3 * p + 1];
    x2 = pts_in[3 * p + 2];
  }
  // the null camera (record C): R = 0, t = (0, 0, 1), K = 0. Slots without an observation
  // project through it to u = v = 0 with a zero Jacobian, so with a zero observation they add
  // exact zeros to every sum: linearize() needs no branch around its projection
  double cr[HOIST ? S : 1][ACS_CAM_STRIDE];
  if constexpr (HOIST) {
    // S = 1 and slot = camera: the lane's record is loaded from global memory (L2-resident,
    // C x 160 B) in the same round trip as the observation, straight into its registers; no
    // LDS copy and no barrier ahead of the LM loop
    const double* cg = cams + (size_t)(lane < C ? lane : C - 1) * ACS_CAM_STRIDE;
#pragma unroll
    for (int i = 0; i < ACS_CAM_STRIDE; ++i) cr[0][i] = cg[i];
    if (!live) return;  // whole group leaves together
  } else {
    for (int i = threadIdx.x; i < C * ACS_CAM_STRIDE; i += blockDim.x) s_cam[i] = cams[i];
    if (threadIdx.x < ACS_CAM_STRIDE) s_cam[C * ACS_CAM_STRIDE + threadIdx.x] = threadIdx.x == 19 ? 1.0 : 0.0;
    __syncthreads();
    if (!live) return;  // whole group leaves together
  }

  double ou[S], ov[S];
  const double* oc[S];
  bool ok[S];
  int mine = 0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int slot = lane + s * G;
    const int cam = cid[s];
    ok[s] = slot < K && mk[s] && cam < C;
    ou[s] = ok[s] ? q[s].x : 0.0;
    ov[s] = ok[s] ? q[s].y : 0.0;
    oc[s] = s_cam + (ok[s] ? cam : C) * ACS_CAM_STRIDE;
    if constexpr (HOIST) {
#pragma unroll
      for (int i = 0; i < ACS_CAM_STRIDE; ++i) cr[s][i] = ok[s] ? cr[s][i] : (i == 19 ? 1.0 : 0.0);
    }
    mine += ok[s] ? 1 : 0;
  }
  const double nobs = group_sum<G>((double)mine);
  if (nobs == 0.0) {
    if (lane == 0) {
      pts[3 * p] = x0;
      pts[3 * p + 1] = x1;
      pts[3 * p + 2] = x2;
      if (stat) {
        cost0[p] = 0.0;
        cost1[p] = 0.0;
        stat[3 * p] = ACS_STATUS_NOOBS;
        stat[3 * p + 1] = 0;
        stat[3 * p + 2] = 0;
      }
    }
    return;
  }
  const double f2 = prm.f_scale * prm.f_scale;
  const double if2 = 1.0 / f2;

  // One pass over the observations at X: robust cost, Triggs-weighted GN matrix (packed
  // upper 3x3) and IRLS gradient, group-reduced. The trial point of every LM iteration is
  // linearised speculatively, so an accepted step (the common case) costs one projection.
  auto linearize = [&](double X0, double X1, double X2, double* Ho, double* go, double& Fo) {
#pragma unroll
    for (int i = 0; i < 6; ++i) Ho[i] = 0.0;
    go[0] = go[1] = go[2] = 0.0;
    double Fl = 0.0;
    // S > 1: the lane's slots share one logarithm too. With T = prod_s (1 + t_s) - 1 formed as
    // T + t + T t (exact algebra, relative rounding only), sum_s log1p(t_s) = log1p(T), and
    // prod_s 1 / (1 + t_s) is the reciprocal it needs. An empty slot (t = 0, 1 / (1 + t) = 1)
    // leaves both unchanged exactly.
    double Tl = 0.0, rTl = 1.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      // slots without an observation: the null camera, exact zero contributions
      double pu, pv, J[6];
      if constexpr (HOIST)
        fisheye_uvj(cr[s], X0, X1, X2, pu, pv, J);
      else
        fisheye_uvj(oc[s], X0, X1, X2, pu, pv, J);
      const double r[2] = {pu - ou[s], pv - ov[s]};
      const double zu = r[0] * r[0] * if2, zv = r[1] * r[1] * if2;
      // log1p(zu) + log1p(zv) with one logarithm, and the two Cauchy weights 1 / (1 + z) from
      // the logarithm's own reciprocal of (1 + zu)(1 + zv)
      const double t = zu + zv + zu * zv, u1 = 1.0 + t, ru = rcp_nr(u1);
      if constexpr (S == 1) {
        Fl += log1p_pos_ur(t, u1, ru);
      } else {
        Tl = s == 0 ? t : fma(Tl, t, Tl + t);
        rTl = s == 0 ? ru : rTl * ru;
      }
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const double z = d ? zv : zu;
        const double w = (d ? 1.0 + zu : 1.0 + zv) * ru;    // rho'(z): gradient weight
        const double wh = fmax((1.0 - z) * w * w, 0.1 * w);  // rho' + 2 z rho'' (Triggs), floored
        const double j0 = J[3 * d], j1 = J[3 * d + 1], j2 = J[3 * d + 2];
        const double hj0 = wh * j0, hj1 = wh * j1, hj2 = wh * j2;
        Ho[0] += hj0 * j0;
        Ho[1] += hj0 * j1;
        Ho[2] += hj0 * j2;
        Ho[3] += hj1 * j1;
        Ho[4] += hj1 * j2;
        Ho[5] += hj2 * j2;
        const double wr = w * r[d];
        go[0] += wr * j0;
        go[1] += wr * j1;
        go[2] += wr * j2;
      }
    }
    if constexpr (S > 1) Fl = log1p_pos_ur(Tl, 1.0 + Tl, rTl);
#pragma unroll
    for (int i = 0; i < 6; ++i) Ho[i] = group_sum<G>(Ho[i]);
#pragma unroll
    for (int i = 0; i < 3; ++i) go[i] = group_sum<G>(go[i]);
    Fo = 0.5 * f2 * group_sum<G>(Fl);
  };

  double H[6], g[3], F;
  linearize(x0, x1, x2, H, g, F);
  const double F_before = F;
  double lam = 1e-3;
  int status = ACS_STATUS_RUNNING, iters = 0, nfev = 1;
  while (status == ACS_STATUS_RUNNING) {
    if (iters >= prm.max_iters) {
      status = ACS_STATUS_MAXITER;
      break;
    }
    const double gmax = fmax(fabs(g[0]), fmax(fabs(g[1]), fabs(g[2])));
    if (gmax <= prm.gtol) {
      status = ACS_STATUS_GTOL;
      break;
    }
    // Cholesky of H + lam*diag(H)
    const double dl = 1.0 + lam;
    const double a00 = H[0] * dl, a11 = H[3] * dl, a22 = H[5] * dl;
    bool pd = a00 > 0.0;
    // reciprocal Cholesky diagonal; the argument, not the result, is selected (rsq_nr(1) = 1):
    // no branch around the reciprocal square roots
    const double i00 = rsq_nr(pd ? a00 : 1.0);
    const double L10 = H[1] * i00, L20 = H[2] * i00;
    const double d11 = a11 - L10 * L10;
    pd = pd && d11 > 0.0;
    const double i11 = rsq_nr(pd ? d11 : 1.0);
    const double L21 = (H[4] - L20 * L10) * i11;
    const double d22 = a22 - L20 * L20 - L21 * L21;
    pd = pd && d22 > 0.0;
    const double i22 = rsq_nr(pd ? d22 : 1.0);
    double dx0 = 0.0, dx1 = 0.0, dx2 = 0.0;
    if (pd) {
      const double y0 = -g[0] * i00;
      const double y1 = (-g[1] - L10 * y0) * i11;
      const double y2 = (-g[2] - L20 * y0 - L21 * y1) * i22;
      dx2 = y2 * i22;
      dx1 = (y1 - L21 * dx2) * i11;
      dx0 = (y0 - L10 * dx1 - L20 * dx2) * i00;
      // model decrease of the step, -g.dx - dx.H.dx/2: below the resolution of the
      // float64 cost the step can only be accepted or rejected by rounding -> converged
      const double Hd0 = H[0] * dx0 + H[1] * dx1 + H[2] * dx2;
      const double Hd1 = H[1] * dx0 + H[3] * dx1 + H[4] * dx2;
      const double Hd2 = H[2] * dx0 + H[4] * dx1 + H[5] * dx2;
      const double pred = -(g[0] * dx0 + g[1] * dx1 + g[2] * dx2) - 0.5 * (dx0 * Hd0 + dx1 * Hd1 + dx2 * Hd2);
      if (pred <= ACS_COST_RES * F) {
        status = ACS_STATUS_FTOL;
        break;
      }
    }
    ++iters;
    if (!pd) {
      // not positive definite (lam near its floor on a degenerate point): no step, so no
      // trial and no xtol test; raise lam as a rejection would (uniform over the group:
      // pd comes from the group-summed H)
      lam *= 10.0;
      if (lam > 1e16) status = ACS_STATUS_STALLED;
      continue;
    }
    const double n0 = x0 + dx0, n1 = x1 + dx1, n2 = x2 + dx2;
    double Hn[6], gn[3], Fn;
    linearize(n0, n1, n2, Hn, gn, Fn);
    ++nfev;
    // |dx| <= xtol (xtol + |x|), compared squared
    const double xx = x0 * x0 + x1 * x1 + x2 * x2;
    const double xn = xx > 0.0 ? xx * rsq_nr(xx > 0.0 ? xx : 1.0) : 0.0;
    const double xb = prm.xtol * (prm.xtol + xn);
    const bool small = dx0 * dx0 + dx1 * dx1 + dx2 * dx2 <= xb * xb;
    if (Fn < F) {
      const bool fconv = (F - Fn) <= prm.ftol * F;
      x0 = n0;
      x1 = n1;
      x2 = n2;
      lam = fmax(lam * 0.1, 1e-15);
      F = Fn;
#pragma unroll
      for (int i = 0; i < 6; ++i) H[i] = Hn[i];
      g[0] = gn[0];
      g[1] = gn[1];
      g[2] = gn[2];
      if (fconv)
        status = ACS_STATUS_FTOL;
      else if (small)
        status = ACS_STATUS_XTOL;
    } else {
      lam *= 10.0;
      if (small)
        status = ACS_STATUS_XTOL;
      else if (lam > 1e16)
        status = ACS_STATUS_STALLED;
    }
  }
  if (lane == 0) {
    pts[3 * p] = x0;
    pts[3 * p + 1] = x1;
    pts[3 * p + 2] = x2;
    // the per-point costs and status feed k_sba_report only: not written (28 B per point)
    // when no report is asked for
    if (stat) {
      cost0[p] = F_before;
      cost1[p] = F;
      stat[3 * p] = status;
      stat[3 * p + 1] = iters;
      stat[3 * p + 2] = nfev;
    }
  }
}

// Deterministic single-block reduction of the per-point outputs into an acs_report.
__global__ __launch_bounds__(256) void k_sba_report(const double* __restrict__ cost0,
                                                    const double* __restrict__ cost1,
                                                    const int* __restrict__ stat, int64_t n,
                                                    acs_report* __restrict__ rep) {
  __shared__ double s_c0[256], s_c1[256];
  __shared__ long long s_i[256][ACS_N_STATUS + 3];
  const int t = threadIdx.x;
  double c0 = 0.0, c1 = 0.0;
  long long cnt[ACS_N_STATUS] = {0}, isum = 0, imax = 0, nf = 0;
  for (int64_t i = t; i < n; i += 256) {
    c0 += cost0[i];
    c1 += cost1[i];
    int s = stat[3 * i];
    if (s >= 0 && s < ACS_N_STATUS) cnt[s]++;
    isum += stat[3 * i + 1];
    imax = max(imax, (long long)stat[3 * i + 1]);
    nf += stat[3 * i + 2];
  }
  s_c0[t] = c0;
  s_c1[t] = c1;
  for (int k = 0; k < ACS_N_STATUS; ++k) s_i[t][k] = cnt[k];
  s_i[t][ACS_N_STATUS] = isum;
  s_i[t][ACS_N_STATUS + 1] = imax;
  s_i[t][ACS_N_STATUS + 2] = nf;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (t < h) {
      s_c0[t] += s_c0[t + h];
      s_c1[t] += s_c1[t + h];
      for (int k = 0; k < ACS_N_STATUS + 3; ++k) {
        if (k == ACS_N_STATUS + 1)
          s_i[t][k] = max(s_i[t][k], s_i[t + h][k]);
        else
          s_i[t][k] += s_i[t + h][k];
      }
    }
    __syncthreads();
  }
  if (t == 0) {
    rep->n_problems = n;
    for (int k = 0; k < ACS_N_STATUS; ++k) rep->status_counts[k] = s_i[0][k];
    rep->iters_sum = s_i[0][ACS_N_STATUS];
    rep->iters_max = s_i[0][ACS_N_STATUS + 1];
    rep->nfev_sum = s_i[0][ACS_N_STATUS + 2];
    rep->cost_before = s_c0[0];
    rep->cost_after = s_c1[0];
  }
}

// ------------------------------------------------------------------------------------
// obs list -> (n_pts, K) slot tensor, deterministic (stable radix sort by point index)
// ------------------------------------------------------------------------------------
__global__ void k_iota(int32_t* v, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) v[i] = (int32_t)i;
}
__global__ void k_count(const int32_t* __restrict__ key, int64_t n, int32_t* __restrict__ cnt, int64_t n_pts,
                        int32_t* __restrict__ bad) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int32_t k = key[i];
  if (k < 0 || k >= n_pts) {
    atomicAdd(bad, 1);
    return;
  }
  atomicAdd(&cnt[k], 1);
}
__global__ void k_scatter_slots(const int32_t* __restrict__ skey, const int32_t* __restrict__ sval, int64_t n,
                                const int32_t* __restrict__ start, const double2* __restrict__ uv,
                                const int32_t* __restrict__ cam_idx, int K, int n_cams,
                                double2* __restrict__ uv_pad, uint8_t* __restrict__ mask,
                                uint8_t* __restrict__ camid) {
  int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const int32_t p = skey[j];
  const int32_t o = sval[j];
  const int64_t slot = j - start[p];
  const int64_t d = (int64_t)p * K + slot;
  const int c = cam_idx[o];
  uv_pad[d] = uv[o];
  camid[d] = (uint8_t)(c >= 0 && c < n_cams ? c : 255);
  mask[d] = (c >= 0 && c < n_cams) ? 1 : 0;
}


// residual vector in the caller's observation order (cost_func_points_only, src/lib/sba.py:149-153)
__global__ __launch_bounds__(256) void k_residuals_ext(const double* __restrict__ cams, int n_cams,
                                                       const double* __restrict__ uvobs,
                                                       const int32_t* __restrict__ pt_idx,
                                                       const int32_t* __restrict__ cam_idx, int64_t n_obs,
                                                       const double* __restrict__ pts, int64_t n_pts,
                                                       double* __restrict__ res) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_obs) return;
  const int c = cam_idx[i];
  const int64_t p = pt_idx[i];
  if (c < 0 || c >= n_cams || p < 0 || p >= n_pts) {
    res[2 * i] = res[2 * i + 1] = __builtin_nan("");
    return;
  }
  ProjOut o;
  fisheye_project<false>(cams + c * ACS_CAM_STRIDE, pts[3 * p], pts[3 * p + 1], pts[3 * p + 2], o);
  res[2 * i] = o.u - uvobs[2 * i];
  res[2 * i + 1] = o.v - uvobs[2 * i + 1];
}

static int next_pow2(int v) {
  int g = 1;
  while (g < v) g <<= 1;
  return g;
}

template <int G, int S, bool CAMID>
static void launch_lm_t(acs_ctx* ctx, int blocks, int block, const double* cams, int C, int K, const double2* uv,
                        const uint8_t* mask, const uint8_t* camid, int64_t n_pts, const double* pts_in, double* pts,
                        SbaParams prm, double* c0, double* c1, int* st) {
  // register-resident camera records when the grid holds at most 2 waves per SIMD
  const int64_t waves = (n_pts * G + 63) / 64;
  const bool hoist = S == 1 && !CAMID && G <= 16 && waves <= 8 * (int64_t)ctx->n_cu;
  if constexpr (S == 1 && !CAMID && G <= 16) {
    if (hoist) {
      hipLaunchKernelGGL((k_sba_lm<G, S, CAMID, true>), dim3(blocks), dim3(block),
                         sizeof(double) * ACS_CAM_STRIDE * (C + 1), ctx->stream, cams, C, K, uv, mask, camid, n_pts, pts_in,
                         pts, prm, c0, c1, st);
      return;
    }
  }
  hipLaunchKernelGGL((k_sba_lm<G, S, CAMID, false>), dim3(blocks), dim3(block), sizeof(double) * ACS_CAM_STRIDE * (C + 1),
                     ctx->stream, cams, C, K, uv, mask, camid, n_pts, pts_in, pts, prm, c0, c1, st);
}

template <int S, bool CAMID>
static int launch_lm_g(acs_ctx* ctx, int G, int blocks, int block, const double* cams, int C, int K,
                       const double2* uv, const uint8_t* mask, const uint8_t* camid, int64_t n_pts,
                       const double* pts_in, double* pts, SbaParams prm, double* c0, double* c1, int* st) {
  switch (G) {
#define ACS_G(g)                                                                                      \
  case g:                                                                                             \
    launch_lm_t<g, S, CAMID>(ctx, blocks, block, cams, C, K, uv, mask, camid, n_pts, pts_in, pts, prm, c0, c1, st); \
    break;
    ACS_G(2) ACS_G(4) ACS_G(8) ACS_G(16) ACS_G(32) ACS_G(64)
#undef ACS_G
    default:
      return acs_fail(ctx, ACS_E_INVALID, "unsupported group size %d", G);
  }
  return ACS_OK;
}

// Launch the LM kernel over an (n_pts, K) slot tensor already on the device; initial points
// from dpts_in, solution to dpts (may alias).
static int run_lm(acs_ctx* ctx, const double* dcams, int C, int K, const double2* duv, const uint8_t* dmask,
                  const uint8_t* dcamid, int64_t n_pts, const double* dpts_in, double* dpts,
                  const acs_sba_opts* opts, bool report, double** c0_out,
                  double** c1_out, int** st_out) {
  acs_sba_opts o;
  acs_sba_default_opts(&o);
  if (opts) o = *opts;
  ACS_CHECK(ctx, o.f_scale > 0 && o.max_iters >= 0, "bad acs_sba_opts");
  ACS_CHECK(ctx, K >= 1 && K <= 256, "observations per point (%d) must be in [1, 256]", K);
  ACS_CHECK(ctx, C >= 1 && C <= 255, "n_cams (%d) must be in [1, 255]", C);
  SbaParams prm{o.max_iters, o.f_scale, o.ftol, o.xtol, o.gtol};
  double *c0 = nullptr, *c1 = nullptr;
  int* st = nullptr;
  if (report) {
    c0 = (double*)acs_ws(ctx, WS_PERPT_F0, sizeof(double) * n_pts);
    c1 = (double*)acs_ws(ctx, WS_PERPT_F1, sizeof(double) * n_pts);
    st = (int*)acs_ws(ctx, WS_PERPT_I, sizeof(int) * 3 * n_pts);
    if (!c0 || !c1 || !st) return ACS_E_NOMEM;
  }
  int G = next_pow2(K < 2 ? 2 : K);
  int S = 1;
  if (G > 64) {
    G = 64;
    S = 4;
  } else if (G > K && (int64_t)((n_pts * G + 63) / 64) > 16 * (int64_t)ctx->n_cu) {
    // a throughput-bound grid (more than 4 waves per SIMD) whose slot count is not a power of
    // two: three slots per lane in groups of G / 4 lanes wherever that wastes fewer lanes
    // (K = 12: 4 lanes x 3 slots, where 16-lane groups ran 4 lanes per point through the null
    // camera record; the per-point LM arithmetic is also repeated by 4 lanes instead of 16)
    const int g3 = next_pow2((K + 2) / 3);
    if (3 * g3 < G) {
      G = g3 < 2 ? 2 : g3;
      S = 3;
    }
  }
  const int64_t threads = n_pts * G;
  int block = 256;
  if (threads < (int64_t)256 * 2 * ctx->n_cu) block = 64;  // small problem: spread over more CUs
  const int blocks = acs_grid(threads, block);
  int rc;
  if (dcamid) {
    rc = (S == 1) ? launch_lm_g<1, true>(ctx, G, blocks, block, dcams, C, K, duv, dmask, dcamid, n_pts, dpts_in, dpts, prm,
                                         c0, c1, st)
         : (S == 3) ? launch_lm_g<3, true>(ctx, G, blocks, block, dcams, C, K, duv, dmask, dcamid, n_pts, dpts_in, dpts,
                                           prm, c0, c1, st)
                    : launch_lm_g<4, true>(ctx, G, blocks, block, dcams, C, K, duv, dmask, dcamid, n_pts, dpts_in, dpts,
                                           prm, c0, c1, st);
  } else {
    rc = (S == 1) ? launch_lm_g<1, false>(ctx, G, blocks, block, dcams, C, K, duv, dmask, dcamid, n_pts, dpts_in, dpts,
                                          prm, c0, c1, st)
         : (S == 3) ? launch_lm_g<3, false>(ctx, G, blocks, block, dcams, C, K, duv, dmask, dcamid, n_pts, dpts_in,
                                            dpts, prm, c0, c1, st)
                    : launch_lm_g<4, false>(ctx, G, blocks, block, dcams, C, K, duv, dmask, dcamid, n_pts, dpts_in,
                                            dpts, prm, c0, c1, st);
  }
  if (rc) return rc;
  ACS_HIP(ctx, hipGetLastError());
  *c0_out = c0;
  *c1_out = c1;
  *st_out = st;
  return ACS_OK;
}

static int run_report(acs_ctx* ctx, const double* c0, const double* c1, const int* st, int64_t n,
                      acs_report* report) {
  acs_report* drep = (acs_report*)acs_ws(ctx, WS_REPORT, sizeof(acs_report));
  if (!drep) return ACS_E_NOMEM;
  hipLaunchKernelGGL(k_sba_report, dim3(1), dim3(256), 0, ctx->stream, c0, c1, st, n, drep);
  ACS_HIP(ctx, hipGetLastError());
  ACS_HIP(ctx, hipMemcpyAsync(report, drep, sizeof(acs_report), hipMemcpyDeviceToHost, ctx->stream));
  ACS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return ACS_OK;
}

int acs_sba_dense_enqueue(acs_ctx* ctx, const double* dcams, int C, const double2* duv, const uint8_t* dmask,
                          int64_t n_pts, const double* dpts_in, double* dpts_out, const acs_sba_opts* opts,
                          acs_report* report) {
  if (n_pts == 0) {
    if (report) std::memset(report, 0, sizeof(*report));
    return ACS_OK;
  }
  double *c0, *c1;
  int* st;
  int rc;
  if ((rc = run_lm(ctx, dcams, C, C, duv, dmask, nullptr, n_pts, dpts_in, dpts_out, opts, report != nullptr, &c0, &c1,
                   &st)))
    return rc;
  if (report) return run_report(ctx, c0, c1, st, n_pts, report);
  return ACS_OK;
}

int acs_obs_to_slots(acs_ctx* ctx, const double* duv, const int32_t* dpi, const int32_t* dci, int64_t n_obs,
                     int64_t n_pts, int n_cams, double2** uv_pad, uint8_t** mask, uint8_t** camid, int* K_out) {
  hipStream_t s = ctx->stream;
  // stable sort of observation ids by point id
  int32_t* skey = (int32_t*)acs_ws(ctx, WS_SORT0, sizeof(int32_t) * n_obs);
  int32_t* vin = (int32_t*)acs_ws(ctx, WS_SORT1, sizeof(int32_t) * n_obs);
  int32_t* sval = (int32_t*)acs_ws(ctx, WS_SORT2, sizeof(int32_t) * n_obs);
  int32_t* cnt = (int32_t*)acs_ws(ctx, WS_TMP0, sizeof(int32_t) * (n_pts + 2));
  int32_t* start = (int32_t*)acs_ws(ctx, WS_TMP1, sizeof(int32_t) * (n_pts + 1));
  if (!skey || !vin || !sval || !cnt || !start) return ACS_E_NOMEM;
  hipLaunchKernelGGL(k_iota, dim3(acs_grid(n_obs, 256)), dim3(256), 0, s, vin, n_obs);
  size_t tb0 = 0, tb1 = 0, tb2 = 0;
  ACS_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, tb0, dpi, skey, (const int32_t*)vin, sval,
                                                   (int)n_obs, 0, 32, s));
  ACS_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(nullptr, tb1, cnt, start, (int)n_pts, s));
  ACS_HIP(ctx, hipcub::DeviceReduce::Max(nullptr, tb2, cnt, cnt + n_pts, (int)n_pts, s));
  size_t tb = std::max(tb0, std::max(tb1, tb2));
  void* tmp = acs_ws(ctx, WS_SORT3, tb);
  if (!tmp) return ACS_E_NOMEM;
  ACS_HIP(ctx, hipcub::DeviceRadixSort::SortPairs(tmp, tb, dpi, skey, (const int32_t*)vin, sval,
                                                   (int)n_obs, 0, 32, s));
  ACS_HIP(ctx, hipMemsetAsync(cnt, 0, sizeof(int32_t) * (n_pts + 2), s));
  hipLaunchKernelGGL(k_count, dim3(acs_grid(n_obs, 256)), dim3(256), 0, s, dpi, n_obs, cnt, n_pts,
                     cnt + n_pts + 1);
  ACS_HIP(ctx, hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, start, (int)n_pts, s));
  ACS_HIP(ctx, hipcub::DeviceReduce::Max(tmp, tb, cnt, cnt + n_pts, (int)n_pts, s));
  int32_t hk[2] = {0, 0};
  ACS_HIP(ctx, hipMemcpyAsync(hk, cnt + n_pts, sizeof(int32_t) * 2, hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipStreamSynchronize(s));
  ACS_CHECK(ctx, hk[1] == 0, "acs_sba_points: %d point indices out of [0, %lld)", hk[1], (long long)n_pts);
  const int K = hk[0] < 1 ? 1 : hk[0];
  ACS_CHECK(ctx, K <= 256, "acs_sba_points: a point has %d observations (max 256)", K);
  double2* uvp = (double2*)acs_ws(ctx, WS_TMP2, sizeof(double2) * n_pts * K);
  uint8_t* mk = (uint8_t*)acs_ws(ctx, WS_TMP3, (size_t)n_pts * K);
  uint8_t* cid = (uint8_t*)acs_ws(ctx, WS_TMP4, (size_t)n_pts * K);
  if (!uvp || !mk || !cid) return ACS_E_NOMEM;
  ACS_HIP(ctx, hipMemsetAsync(mk, 0, (size_t)n_pts * K, s));
  hipLaunchKernelGGL(k_scatter_slots, dim3(acs_grid(n_obs, 256)), dim3(256), 0, s, skey, sval, n_obs, start,
                     (const double2*)duv, dci, K, n_cams, uvp, mk, cid);
  ACS_HIP(ctx, hipGetLastError());

  *uv_pad = uvp;
  *mask = mk;
  *camid = cid;
  *K_out = K;
  return ACS_OK;
}

extern "C" {

int acs_sba_points_dense_io(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv,
                            const uint8_t* mask, int64_t n_pts, const double* pts_in, double* pts_out,
                            const acs_sba_opts* opts, acs_report* report, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, n_pts >= 0 && n_cams >= 1 && n_cams <= 64, "acs_sba_points_dense: n_pts=%lld n_cams=%d (1..64)",
            (long long)n_pts, n_cams);
  if (n_pts == 0) {
    if (report) std::memset(report, 0, sizeof(*report));
    return ACS_OK;
  }
  void *dc, *duv, *dm, *dpi;
  int rc;
  if ((rc = acs_stage_in(ctx, WS_CAMS, cams, sizeof(double) * ACS_CAM_STRIDE * n_cams, flags, &dc))) return rc;
  if ((rc = acs_stage_in(ctx, WS_UV, uv, sizeof(double) * 2 * n_pts * n_cams, flags, &duv))) return rc;
  if ((rc = acs_stage_in(ctx, WS_MASK, mask, (size_t)n_pts * n_cams, flags, &dm))) return rc;
  if ((rc = acs_stage_in(ctx, WS_PTS, pts_in, sizeof(double) * 3 * n_pts, flags, &dpi))) return rc;
  double* dpo = (double*)acs_out_buf(ctx, WS_OUT0, pts_out, sizeof(double) * 3 * n_pts, flags);
  if (!dpo) return ACS_E_NOMEM;
  double *c0, *c1;
  int* st;
  if ((rc = run_lm(ctx, (const double*)dc, n_cams, n_cams, (const double2*)duv, (const uint8_t*)dm, nullptr, n_pts,
                   (const double*)dpi, dpo, opts, report != nullptr, &c0, &c1, &st)))
    return rc;
  if ((rc = acs_stage_out(ctx, pts_out, dpo, sizeof(double) * 3 * n_pts, flags))) return rc;
  if (report) {
    if ((rc = run_report(ctx, c0, c1, st, n_pts, report))) return rc;
  } else if (!(flags & ACS_DEVICE_PTRS)) {
    ACS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  }
  return ACS_OK;
}

int acs_sba_points_dense(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv, const uint8_t* mask,
                         int64_t n_pts, double* pts, const acs_sba_opts* opts, acs_report* report, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  return acs_sba_points_dense_io(ctx, cams, n_cams, uv, mask, n_pts, pts, pts, opts, report, flags);
}

int acs_sba_points(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv, const int32_t* pt_idx,
                   const int32_t* cam_idx, int64_t n_obs, double* pts, int64_t n_pts, const acs_sba_opts* opts,
                   double* resid_before, double* resid_after, acs_report* report, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, n_obs >= 0 && n_pts >= 0 && n_cams >= 1 && n_cams <= 255, "acs_sba_points: bad sizes");
  ACS_CHECK(ctx, n_obs < (int64_t)INT32_MAX, "acs_sba_points: n_obs too large");
  if (n_pts == 0 || n_obs == 0) {
    if (report) std::memset(report, 0, sizeof(*report));
    return ACS_OK;
  }
  void *dc, *duv, *dpi, *dci, *dp;
  int rc;
  if ((rc = acs_stage_in(ctx, WS_CAMS, cams, sizeof(double) * ACS_CAM_STRIDE * n_cams, flags, &dc))) return rc;
  if ((rc = acs_stage_in(ctx, WS_UV, uv, sizeof(double) * 2 * n_obs, flags, &duv))) return rc;
  if ((rc = acs_stage_in(ctx, WS_PTIDX, pt_idx, sizeof(int32_t) * n_obs, flags, &dpi))) return rc;
  if ((rc = acs_stage_in(ctx, WS_CAMIDX, cam_idx, sizeof(int32_t) * n_obs, flags, &dci))) return rc;
  if ((rc = acs_stage_in(ctx, WS_PTS, pts, sizeof(double) * 3 * n_pts, flags, &dp))) return rc;
  hipStream_t s = ctx->stream;

  // residuals at the initial points (residuals['before'])
  double* drb = nullptr;
  if (resid_before) {
    drb = (double*)acs_out_buf(ctx, WS_OUT0, resid_before, sizeof(double) * 2 * n_obs, flags);
    if (!drb) return ACS_E_NOMEM;
    hipLaunchKernelGGL(k_residuals_ext, dim3(acs_grid(n_obs, 256)), dim3(256), 0, s, (const double*)dc, n_cams,
                       (const double*)duv, (const int32_t*)dpi, (const int32_t*)dci, n_obs, (const double*)dp, n_pts,
                       drb);
    ACS_HIP(ctx, hipGetLastError());
  }

  double2* uvp;
  uint8_t *mk, *cid;
  int K;
  if ((rc = acs_obs_to_slots(ctx, (const double*)duv, (const int32_t*)dpi, (const int32_t*)dci, n_obs, n_pts, n_cams,
                             &uvp, &mk, &cid, &K)))
    return rc;

  double *c0, *c1;
  int* st;
  if ((rc = run_lm(ctx, (const double*)dc, n_cams, K, uvp, mk, cid, n_pts, (const double*)dp, (double*)dp, opts,
                   report != nullptr, &c0, &c1, &st)))
    return rc;

  double* dra = nullptr;
  if (resid_after) {
    dra = (double*)acs_out_buf(ctx, WS_OUT1, resid_after, sizeof(double) * 2 * n_obs, flags);
    if (!dra) return ACS_E_NOMEM;
    hipLaunchKernelGGL(k_residuals_ext, dim3(acs_grid(n_obs, 256)), dim3(256), 0, s, (const double*)dc, n_cams,
                       (const double*)duv, (const int32_t*)dpi, (const int32_t*)dci, n_obs, (const double*)dp, n_pts,
                       dra);
    ACS_HIP(ctx, hipGetLastError());
  }
  if ((rc = acs_stage_out(ctx, pts, dp, sizeof(double) * 3 * n_pts, flags))) return rc;
  if (resid_before && (rc = acs_stage_out(ctx, resid_before, drb, sizeof(double) * 2 * n_obs, flags))) return rc;
  if (resid_after && (rc = acs_stage_out(ctx, resid_after, dra, sizeof(double) * 2 * n_obs, flags))) return rc;
  if (report) {
    if ((rc = run_report(ctx, c0, c1, st, n_pts, report))) return rc;
  } else if (!(flags & ACS_DEVICE_PTRS)) {
    ACS_HIP(ctx, hipStreamSynchronize(s));
  }
  return ACS_OK;
}

}  // extern "C"
