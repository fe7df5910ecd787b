// ekf.hip — extended Kalman filter + RTS smoother on gfx950.
//
// Replaces the frame loop of core.ekf (src/core/ekf.py:229-287); spec: oracle/ekf.py.
// One workgroup owns one sequence and walks its frames (the filter is sequential in
// time); independent sequences run on independent workgroups / GPUs ("replicas only").
//
// Per frame (k_ekf_filter, 512 threads = 8 waves):
//   1. constant-acceleration prediction; P <- F P F^T + Q column/row-wise in LDS (F is
//      identity plus two scaled block shifts, so no dense product is needed)
//   2. measurement model: the P+1 poses of the forward-difference Jacobian (:81-96) are
//      evaluated one per wave (table FK in LDS + fisheye projection of C x L markers)
//   3. Kalman update in information form on the pose block: with H = [H_x 0 0] and R
//      diagonal, K r = P[:,x] (I + A P_xx)^-1 b and (I - K H) P = P - P[:,x] (I + A P_xx)^-1
//      A P[x,:], A = H_x^T R^-1 H_x, b = H_x^T R^-1 r (Woodbury; one P x P solve by
//      Gauss-Jordan with partial pivoting instead of inverting the 2CL x 2CL S of :267)
//   4. the reference's 3-sigma outlier count from diag(S) = diag(H_x P_xx H_x^T) + diag R
// With F32 (the reference numerics) the predicted state is rounded to float32 (:79), the
// FK trig runs in float32, and the Jacobian perturbation is x + 1e-3 in float32.
//
// k_ekf_smooth (256 threads): RTS backward pass (:280-287) with the predicted covariance
// inverted by blocked Gauss-Jordan on f64 MFMA tiles and the gain / covariance products on
// wg_mgemm.
#include "fk.hpp"
#include "mfma64.hpp"

#define EKF_WAVES 8

struct EkfDims {
  int N, C, L, P, n, npad, Ppad, m, S;
  double sT, thresh, maxpix, eps;
};

__device__ __forceinline__ void ekf_pose(const double* s, int P, int q, bool f32, double eps, double* xq, int lane) {
  for (int p = lane; p < P; p += 64) {
    double v = s[p];
    if (q > 0 && p == q - 1) v = f32 ? (double)((float)v + (float)eps) : v + eps;
    xq[p] = v;
  }
}

template <bool F32>
__global__ __launch_bounds__(512) void k_ekf_filter(EkfDims d, const int* __restrict__ I,
                                                    const double* __restrict__ Rl, const double* __restrict__ cams,
                                                    const double* __restrict__ meas, const double* __restrict__ lik,
                                                    const double* __restrict__ rbase, const double* __restrict__ Q,
                                                    const double* __restrict__ P0, const double* __restrict__ s0,
                                                    double* __restrict__ xpred, double* __restrict__ xest,
                                                    double* __restrict__ Ppred, double* __restrict__ Pest,
                                                    double* __restrict__ scratch, long long* __restrict__ outliers) {
  const int seq = blockIdx.x;
  const int tid = threadIdx.x, nth = blockDim.x, lane = tid & 63, wave = tid >> 6;
  const int n = d.n, P = d.P, m = d.m, LDP = d.npad + 1, Pp = d.Ppad;
  const int AW = Pp + d.npad + 1;  // [M | G | b]
  extern __shared__ double lds[];
  double* sP = lds;                                   // npad x LDP: covariance
  double* U = sP + (size_t)d.npad * LDP;              // union: FK phase / algebra phase
  FkShared* fks = reinterpret_cast<FkShared*>(U);     // EKF_WAVES poses
  double* sPx = U;                                    // npad x Pp: P[:, x] before the update
  double* aug = sPx + (size_t)d.npad * Pp;            // Pp x AW
  double* sA = aug + (size_t)Pp * AW;                 // Pp x Pp
  double* ss = sA + (size_t)Pp * Pp;                  // n: state
  double* sx = ss + d.npad;                           // EKF_WAVES x FK_MAXP pose vectors
  __shared__ int s_piv;
  __shared__ unsigned long long s_out;
  const SkelView sk = skel_view(I, Rl);
  const double sT = d.sT, h2 = 0.5 * sT * sT;
  // per-sequence scratch: hpose (P+1) x m, H m x Pp, res m, w m
  double* hpose = scratch + (size_t)seq * ((size_t)(P + 1) * m + (size_t)m * Pp + 2 * m);
  double* H = hpose + (size_t)(P + 1) * m;
  double* res = H + (size_t)m * Pp;
  double* wr = res + m;
  const size_t fstride = (size_t)d.C * d.L;  // measurements per frame
  for (int e = tid; e < d.npad * LDP; e += nth) {
    const int r = e / LDP, c = e % LDP;
    sP[e] = (r < n && c < n) ? P0[r * n + c] : 0.0;
  }
  for (int r = tid; r < d.npad; r += nth) ss[r] = r < n ? s0[(size_t)seq * n + r] : 0.0;
  if (tid == 0) s_out = 0;
  __syncthreads();

  for (int i = 0; i < d.N; ++i) {
    const size_t fo = ((size_t)seq * d.N + i);
    // ---- 1. prediction --------------------------------------------------------------
    double sn = 0.0;
    if (tid < n) {
      if (tid >= 2 * P) {
        sn = ss[tid];
      } else if (tid >= P) {
        sn = ss[tid] + sT * ss[tid + P];
      } else {
        const double vel = ss[tid + P] + sT * ss[tid + 2 * P];
        sn = ss[tid] + sT * vel + h2 * ss[tid + 2 * P];
      }
      if (F32) sn = (double)(float)sn;
    }
    __syncthreads();
    if (tid < n) {
      ss[tid] = sn;
      xpred[fo * n + tid] = sn;
    }
    // F X (per column, rows in increasing order read only not-yet-updated rows)
    if (tid < n) {
      const int c = tid;
      for (int r = 0; r < n; ++r) {
        double v = sP[r * LDP + c];
        if (r < 2 * P) v += sT * sP[(r + P) * LDP + c];
        if (r < P) v += h2 * sP[(r + 2 * P) * LDP + c];
        sP[r * LDP + c] = v;
      }
    }
    __syncthreads();
    if (tid < n) {  // (F X) F^T + Q (per row)
      const int r = tid;
      for (int c = 0; c < n; ++c) {
        double v = sP[r * LDP + c];
        if (c < 2 * P) v += sT * sP[r * LDP + c + P];
        if (c < P) v += h2 * sP[r * LDP + c + 2 * P];
        sP[r * LDP + c] = v + Q[r * n + c];
      }
    }
    __syncthreads();
    for (int e = tid; e < n * n; e += nth) Ppred[fo * n * n + e] = sP[(e / n) * LDP + e % n];

    // ---- 2. poses of the forward-difference Jacobian --------------------------------
    for (int b0 = 0; b0 <= P; b0 += EKF_WAVES) {
      const int q = b0 + wave;
      double* xq = sx + wave * FK_MAXP;
      ekf_pose(ss, P, q <= P ? q : 0, F32, d.eps, xq, lane);
      __syncthreads();
      fk_frame<F32>(sk, xq, fks[wave], lane, 64);
      __syncthreads();
      if (q <= P) {
        for (int o = lane; o < d.C * d.L; o += 64) {
          const int c = o / d.L, l = o % d.L;
          const int node = sk.outn[l];
          ProjOut po;
          fisheye_project<false>(cams + c * ACS_CAM_STRIDE, fks[wave].pos[node][0], fks[wave].pos[node][1],
                                 fks[wave].pos[node][2], po);
          hpose[(size_t)q * m + 2 * o] = po.u;
          hpose[(size_t)q * m + 2 * o + 1] = po.v;
        }
      }
      __syncthreads();
    }
    // H, residual, R^-1 (row r = 2 (c L + l) + d, the reference's ordering)
    for (int r = tid; r < m; r += nth) {
      const double h0 = hpose[r];
      for (int q = 0; q < Pp; ++q) H[(size_t)r * Pp + q] = q < P ? (hpose[(size_t)(q + 1) * m + r] - h0) / d.eps : 0.0;
      const int o = r >> 1, c = o / d.L;
      const double z = meas[fo * fstride * 2 + r];
      double e = z - h0;
      if (!isfinite(e)) e = (e != e) ? 0.0 : (e > 0 ? 1.7976931348623157e308 : -1.7976931348623157e308);
      res[r] = e;
      const double lk = lik[fo * fstride + o];
      const double sd = (lk < d.thresh) ? d.maxpix : rbase[c];
      wr[r] = 1.0 / (sd * sd);
    }
    __syncthreads();
    // ---- 3. information-form update -------------------------------------------------
    for (int e = tid; e < Pp * Pp; e += nth) {  // A = H^T R^-1 H
      const int a = e / Pp, b = e % Pp;
      double v = 0.0;
      if (a < P && b < P)
        for (int r = 0; r < m; ++r) v += wr[r] * H[(size_t)r * Pp + a] * H[(size_t)r * Pp + b];
      sA[e] = v;
    }
    for (int e = tid; e < d.npad * Pp; e += nth) {  // P[:, x]
      const int r = e / Pp, c = e % Pp;
      sPx[e] = (r < n && c < P) ? sP[r * LDP + c] : 0.0;
    }
    for (int a = tid; a < Pp; a += nth) {  // b = H^T R^-1 r
      double v = 0.0;
      if (a < P)
        for (int r = 0; r < m; ++r) v += wr[r] * H[(size_t)r * Pp + a] * res[r];
      aug[a * AW + Pp + d.npad] = v;
    }
    // 3-sigma outlier count (:259-264): diag S = H_x P_xx H_x^T + R
    unsigned long long cnt = 0;
    for (int pt = tid; pt < m / 2; pt += nth) {
      bool outl = false;
      for (int dd = 0; dd < 2; ++dd) {
        const int r = 2 * pt + dd;
        const double* hr = H + (size_t)r * Pp;
        double q = 0.0;
        for (int a = 0; a < P; ++a) {
          double t = 0.0;
          for (int b = 0; b < P; ++b) t += sP[a * LDP + b] * hr[b];
          q += hr[a] * t;
        }
        const double Srr = q + 1.0 / wr[r];
        if (fabs(res[r]) > 3.0 * sqrt(Srr)) outl = true;
      }
      cnt += outl;
    }
    if (cnt) atomicAdd(&s_out, cnt);
    __syncthreads();
    // aug = [I + A P_xx | A P[x, :] | b]  (rows a < P; padding rows identity)
    for (int e = tid; e < Pp * (Pp + d.npad); e += nth) {
      const int a = e / (Pp + d.npad), c = e % (Pp + d.npad);
      double v = 0.0;
      if (a < P) {
        const int cc = c < Pp ? c : c - Pp;
        const bool live = c < Pp ? cc < P : cc < n;
        if (live)
          for (int k = 0; k < P; ++k) v += sA[a * Pp + k] * sP[k * LDP + cc];
        if (c < Pp && c == a) v += 1.0;
      } else if (c == a) {
        v = 1.0;
      }
      aug[a * AW + c] = v;
    }
    if (tid >= P && tid < Pp) aug[tid * AW + Pp + d.npad] = 0.0;
    __syncthreads();
    // Gauss-Jordan with partial pivoting on the P x P block
    for (int k = 0; k < P; ++k) {
      if (wave == 0) {
        double best = -1.0;
        int bi = k;
        for (int r = k + lane; r < P; r += 64) {
          const double v = fabs(aug[r * AW + k]);
          if (v > best) {
            best = v;
            bi = r;
          }
        }
        for (int off = 32; off > 0; off >>= 1) {
          const double ob = __shfl_xor(best, off);
          const int oi = __shfl_xor(bi, off);
          if (ob > best || (ob == best && oi < bi)) {
            best = ob;
            bi = oi;
          }
        }
        if (lane == 0) s_piv = bi;
      }
      __syncthreads();
      const int pv = s_piv;
      if (pv != k)
        for (int c = tid; c < AW; c += nth) {
          const double t = aug[k * AW + c];
          aug[k * AW + c] = aug[pv * AW + c];
          aug[pv * AW + c] = t;
        }
      __syncthreads();
      const double ip = 1.0 / aug[k * AW + k];
      __syncthreads();
      for (int c = tid; c < AW; c += nth) aug[k * AW + c] *= ip;
      __syncthreads();
      for (int e = tid; e < P * AW; e += nth) {
        const int r = e / AW, c = e % AW;
        if (r == k) continue;
        const double f = aug[r * AW + k];
        if (c != k) aug[e] -= f * aug[k * AW + c];
      }
      __syncthreads();
      for (int r = tid; r < P; r += nth)
        if (r != k) aug[r * AW + k] = 0.0;
      __syncthreads();
    }
    // s += P[:, x] Z_b ;  P -= P[:, x] Z_G
    if (tid < n) {
      double v = 0.0;
      for (int k = 0; k < P; ++k) v += sPx[tid * Pp + k] * aug[k * AW + Pp + d.npad];
      ss[tid] += v;
    }
    for (int e = tid; e < n * n; e += nth) {
      const int r = e / n, c = e % n;
      double v = 0.0;
      for (int k = 0; k < P; ++k) v += sPx[r * Pp + k] * aug[k * AW + Pp + c];
      sP[r * LDP + c] -= v;
    }
    __syncthreads();
    if (tid < n) xest[fo * n + tid] = ss[tid];
    for (int e = tid; e < n * n; e += nth) Pest[fo * n * n + e] = sP[(e / n) * LDP + e % n];
    __syncthreads();
  }
  if (tid == 0) outliers[seq] = (long long)s_out;
}

// RTS smoother (src/core/ekf.py:280-287), one workgroup per sequence.
__global__ __launch_bounds__(256) void k_ekf_smooth(EkfDims d, const double* __restrict__ xpred,
                                                    const double* __restrict__ xest, const double* __restrict__ Ppred,
                                                    const double* __restrict__ Pest, double* __restrict__ xs,
                                                    double* __restrict__ Ps, double* __restrict__ scratch,
                                                    int* __restrict__ bad, int keep_P) {
  const int seq = blockIdx.x, tid = threadIdx.x, nth = blockDim.x;
  const int n = d.n, P = d.P, np_ = d.npad, LD = np_ + 1;
  const double sT = d.sT, h2 = 0.5 * sT * sT;
  extern __shared__ double lds[];
  double* sInv = lds;                  // np x LD
  double* tmp = sInv + (size_t)np_ * LD;  // 512
  double* sv = tmp + 512;              // np
  const size_t nn = (size_t)np_ * np_;
  double* T = scratch + (size_t)seq * 5 * nn;  // P_est F^T
  double* A = T + nn;                           // gain
  double* D = A + nn;                           // Ps[i+1] - Ppred[i+1]
  double* E = D + nn;                           // A D
  double* Pn = E + nn;                          // Ps[i+1] (padded)
  const size_t nn0 = (size_t)n * n;
  const size_t base = (size_t)seq * d.N;
  for (int e = tid; e < (int)nn; e += nth) {
    const int r = e / np_, c = e % np_;
    Pn[e] = (r < n && c < n) ? Pest[(base + d.N - 1) * nn0 + r * n + c] : 0.0;
  }
  for (int r = tid; r < n; r += nth) xs[(base + d.N - 1) * n + r] = xest[(base + d.N - 1) * n + r];
  if (keep_P)
    for (int e = tid; e < (int)nn0; e += nth) Ps[(base + d.N - 1) * nn0 + e] = Pest[(base + d.N - 1) * nn0 + e];
  __syncthreads();
  for (int i = d.N - 2; i >= 0; --i) {
    const double* Pe = Pest + (base + i) * nn0;
    const double* Pp1 = Ppred + (base + i + 1) * nn0;
    for (int e = tid; e < np_ * LD; e += nth) {
      const int r = e / LD, c = e % LD;
      sInv[e] = (r < n && c < n) ? Pp1[r * n + c] : (r == c ? 1.0 : 0.0);
    }
    for (int e = tid; e < (int)nn; e += nth) {  // T = P_est F^T ; D = Ps[i+1] - Ppred[i+1]
      const int r = e / np_, c = e % np_;
      double t = 0.0, dd = 0.0;
      if (r < n && c < n) {
        t = Pe[r * n + c];
        if (c < 2 * P) t += sT * Pe[r * n + c + P];
        if (c < P) t += h2 * Pe[r * n + c + 2 * P];
        dd = Pn[e] - Pp1[r * n + c];
      }
      T[e] = t;
      D[e] = dd;
    }
    __syncthreads();
    wg_gj_inverse<false>(sInv, LD, np_ >> 4, tmp, bad);
    wg_mgemm<false, false>(A, np_, T, np_, sInv, LD, np_, np_, np_, 1.0, 0.0);  // A = T Pp^-1
    for (int r = tid; r < np_; r += nth)
      sv[r] = r < n ? xs[(base + i + 1) * n + r] - xpred[(base + i + 1) * n + r] : 0.0;
    __syncthreads();
    for (int r = tid; r < n; r += nth) {
      double v = xest[(base + i) * n + r];
      for (int c = 0; c < n; ++c) v += A[(size_t)r * np_ + c] * sv[c];
      xs[(base + i) * n + r] = v;
    }
    wg_mgemm<false, false>(E, np_, A, np_, D, np_, np_, np_, np_, 1.0, 0.0);  // E = A D
    for (int e = tid; e < (int)nn; e += nth) {
      const int r = e / np_, c = e % np_;
      Pn[e] = (r < n && c < n) ? Pe[r * n + c] : 0.0;
    }
    __syncthreads();
    wg_mgemm<false, true>(Pn, np_, E, np_, A, np_, np_, np_, np_, 1.0, 1.0);  // Ps[i] = P_est + E A^T
    if (keep_P)
      for (int e = tid; e < (int)nn0; e += nth) Ps[(base + i) * nn0 + e] = Pn[(size_t)(e / n) * np_ + e % n];
    __syncthreads();
  }
}

extern "C" {

int acs_ekf_run(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals, int64_t n_reals,
                const double* cams, int32_t n_cams, const double* meas, const double* likelihood, int32_t n_seq,
                int32_t n_frames, double fps, double thresh, double max_pixel_err, const double* r_std_base,
                const double* Q, const double* P0, const double* s0, int32_t ref_numerics, double eps,
                double* x_pred, double* x_est, double* x_smooth, double* P_est, double* P_smooth,
                int64_t* outliers, uint32_t flags) {
  int hdr[FK_HDR];
  if (flags & ACS_DEVICE_PTRS)
    ACS_HIP(ctx, hipMemcpy(hdr, skel_ints, sizeof(hdr), hipMemcpyDeviceToHost));
  else
    std::memcpy(hdr, skel_ints, sizeof(hdr));
  const int Jn = hdr[0], K = hdr[1], P = hdr[2], L = hdr[3];
  ACS_CHECK(ctx, Jn > 0 && Jn <= FK_MAXJ && K <= FK_MAXN && P >= 3 && P <= FK_MAXP && L >= 1 && L <= K,
            "ekf: skeleton table out of range");
  ACS_CHECK(ctx, n_ints == FK_HDR + 9 * Jn + 4 * K + L + 4 * P + K * P && n_reals == 3 * K, "ekf: blob sizes");
  ACS_CHECK(ctx, n_seq >= 1 && n_frames >= 1 && n_cams >= 1 && n_cams <= 64 && fps > 0 && eps > 0,
            "ekf: n_seq=%d n_frames=%d n_cams=%d", n_seq, n_frames, n_cams);
  ACS_CHECK(ctx, x_est && x_smooth, "ekf: x_est and x_smooth are required");
  EkfDims d;
  d.N = n_frames;
  d.C = n_cams;
  d.L = L;
  d.P = P;
  d.n = 3 * P;
  d.npad = ((d.n + 15) / 16) * 16;
  d.Ppad = ((P + 15) / 16) * 16;
  d.m = 2 * n_cams * L;
  d.S = n_seq;
  d.sT = 1.0 / fps;
  d.thresh = thresh;
  d.maxpix = max_pixel_err;
  d.eps = eps;
  const int n = d.n;
  const size_t NF = (size_t)n_seq * n_frames;
  hipStream_t s = ctx->stream;
  int rc;
  void *dI, *dR, *dC, *dM, *dL, *dRb, *dQ, *dP0, *dS0;
  if ((rc = acs_stage_in(ctx, WS_FTE0, skel_ints, sizeof(int32_t) * n_ints, flags, &dI))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE1, skel_reals, sizeof(double) * n_reals, flags, &dR))) return rc;
  if ((rc = acs_stage_in(ctx, WS_CAMS, cams, sizeof(double) * ACS_CAM_STRIDE * n_cams, flags, &dC))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE2, meas, sizeof(double) * NF * n_cams * L * 2, flags, &dM))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE3, likelihood, sizeof(double) * NF * n_cams * L, flags, &dL))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE4, r_std_base, sizeof(double) * n_cams, flags, &dRb))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE7, Q, sizeof(double) * n * n, flags, &dQ))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE8, P0, sizeof(double) * n * n, flags, &dP0))) return rc;
  if ((rc = acs_stage_in(ctx, WS_FTE9, s0, sizeof(double) * n_seq * n, flags, &dS0))) return rc;
  double* dxp = (double*)acs_out_buf(ctx, WS_FTE10, x_pred, sizeof(double) * NF * n, flags);
  double* dxe = (double*)acs_out_buf(ctx, WS_FTE11, x_est, sizeof(double) * NF * n, flags);
  double* dxs = (double*)acs_out_buf(ctx, WS_FTE12, x_smooth, sizeof(double) * NF * n, flags);
  if (!x_pred) dxp = (double*)acs_ws(ctx, WS_FTE10, sizeof(double) * NF * n);
  // covariance histories: always needed by the smoother; the caller's buffers when given
  double* dPe = (flags & ACS_DEVICE_PTRS) && P_est ? P_est : (double*)acs_ws(ctx, WS_FTE13, sizeof(double) * NF * n * n);
  double* dPp = (double*)acs_ws(ctx, WS_FTE14, sizeof(double) * NF * n * n);
  double* dPs = P_smooth ? ((flags & ACS_DEVICE_PTRS) ? P_smooth
                                                      : (double*)acs_ws(ctx, WS_FTE15, sizeof(double) * NF * n * n))
                         : nullptr;
  const size_t scr_f = (size_t)n_seq * ((size_t)(P + 1) * d.m + (size_t)d.m * d.Ppad + 2 * d.m);
  const size_t scr_s = (size_t)n_seq * 5 * d.npad * d.npad;
  double* scr = (double*)acs_ws(ctx, WS_FTE6, sizeof(double) * std::max(scr_f, scr_s) + 64 * (size_t)n_seq * 8);
  if (!dxp || !dxe || !dxs || !dPe || !dPp || !scr || (P_smooth && !dPs)) return ACS_E_NOMEM;
  long long* dout = (long long*)(scr + std::max(scr_f, scr_s));
  int* dbad = (int*)(dout + n_seq);
  ACS_HIP(ctx, hipMemsetAsync(dbad, 0, sizeof(int), s));
  const size_t U = std::max((size_t)EKF_WAVES * sizeof(FkShared) / sizeof(double),
                            (size_t)d.npad * d.Ppad + (size_t)d.Ppad * (d.Ppad + d.npad + 1) + (size_t)d.Ppad * d.Ppad);
  const size_t lds_f = sizeof(double) * ((size_t)d.npad * (d.npad + 1) + U + d.npad + EKF_WAVES * FK_MAXP);
  ACS_CHECK(ctx, lds_f <= 160 * 1024, "ekf: P = %d needs %zu bytes of LDS", P, lds_f);
  if (ref_numerics)
    hipLaunchKernelGGL(k_ekf_filter<true>, dim3(n_seq), dim3(512), lds_f, s, d, (const int*)dI, (const double*)dR,
                       (const double*)dC, (const double*)dM, (const double*)dL, (const double*)dRb, (const double*)dQ,
                       (const double*)dP0, (const double*)dS0, dxp, dxe, dPp, dPe, scr, dout);
  else
    hipLaunchKernelGGL(k_ekf_filter<false>, dim3(n_seq), dim3(512), lds_f, s, d, (const int*)dI, (const double*)dR,
                       (const double*)dC, (const double*)dM, (const double*)dL, (const double*)dRb, (const double*)dQ,
                       (const double*)dP0, (const double*)dS0, dxp, dxe, dPp, dPe, scr, dout);
  ACS_HIP(ctx, hipGetLastError());
  const size_t lds_s = sizeof(double) * ((size_t)d.npad * (d.npad + 1) + 512 + d.npad);
  hipLaunchKernelGGL(k_ekf_smooth, dim3(n_seq), dim3(256), lds_s, s, d, dxp, dxe, dPp, dPe, dxs, dPs, scr, dbad,
                     dPs ? 1 : 0);
  ACS_HIP(ctx, hipGetLastError());
  if (x_pred && (rc = acs_stage_out(ctx, x_pred, dxp, sizeof(double) * NF * n, flags))) return rc;
  if ((rc = acs_stage_out(ctx, x_est, dxe, sizeof(double) * NF * n, flags))) return rc;
  if ((rc = acs_stage_out(ctx, x_smooth, dxs, sizeof(double) * NF * n, flags))) return rc;
  if (P_est && !(flags & ACS_DEVICE_PTRS) && (rc = acs_stage_out(ctx, P_est, dPe, sizeof(double) * NF * n * n, flags)))
    return rc;
  if (P_smooth && !(flags & ACS_DEVICE_PTRS) &&
      (rc = acs_stage_out(ctx, P_smooth, dPs, sizeof(double) * NF * n * n, flags)))
    return rc;
  if (outliers) {
    std::vector<long long> ho(n_seq);
    ACS_HIP(ctx, hipMemcpyAsync(ho.data(), dout, sizeof(long long) * n_seq, hipMemcpyDeviceToHost, s));
    ACS_HIP(ctx, hipStreamSynchronize(s));
    for (int q = 0; q < n_seq; ++q) outliers[q] = ho[q];
  } else if (!(flags & ACS_DEVICE_PTRS)) {
    ACS_HIP(ctx, hipStreamSynchronize(s));
  }
  return ACS_OK;
}

}  // extern "C"
