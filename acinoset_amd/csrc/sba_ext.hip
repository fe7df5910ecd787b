// sba_ext.hip — bundle adjustment of points AND camera extrinsics on gfx950.
//
// Replaces bundle_adjust_points_and_extrinsics (src/lib/sba.py:158-178): scipy TRF with
// loss='cauchy' (f_scale 1) over cost_func_points_extrinsics (:142-146), where every
// camera's Rodrigues vector + translation is shared by all of its observations
// (create_bundle_adjustment_jacobian_sparsity_matrix :11-22 with 6 camera columns).
//
// LM with the points eliminated by Schur complement (spec: oracle/sba_ext.py):
//   k_ext_linearize [point groups] per observation: residual, J_pt = J_Y R, J_cam =
//                   J_Y [-[R X]x | I]; per point V (3x3), g_p; per slot the camera-side
//                   blocks U (6x6), g_c (6), W = J_cam^T J_pt (6x3). One point = one
//                   aligned lane group (as k_sba_lm), butterfly sums.
//   k_ext_schur     [point chunks] fixed-order partial reduced camera system
//                   S = U - sum W M W^T, b = -g_c + sum W M g_p, M = (V + lam D)^-1
//   k_ext_solve     [1 block] chunk sums in order, Marquardt damping, SPD inverse
//                   (blocked Gauss-Jordan on f64 MFMA tiles), camera step
//   k_ext_back      [points] point steps dX = -M (g_p + sum W^T dc), trial points
//   k_ext_cam       [1 block] trial cameras R <- exp([dw]x) R, t <- t + dt
//   k_ext_cost      [point groups] robust cost at the trial state
//   k_ext_lm        [1 block] accept / reject, lambda, stop tests
// In a multi-GPU run the per-rank partial (S, b) is what one all-reduce would sum.
#include <algorithm>

#include "mfma64.hpp"

#define EXT_MAXC 16
#define EXT_CHUNK 64
#define EXT_Q 45  // per slot: U (21 packed upper) + g_c (6) + W (18)
// damping floor: the 7-DoF similarity gauge is left free (as in the reference), so the
// reduced camera system is singular up to lambda; below ~1e-8 its gauge directions are
// resolved by rounding alone. Spec shared with oracle/sba_ext.py (LAM_MIN).
#define EXT_LAM_MIN 1e-7

struct ExtDims {
  int n, K, C, G, chunk;  // chunk: points per k_ext_schur block (LDS-sized)
  double f2;
};

struct ExtState {
  double F, F0, lam, gmax, dnorm, xnorm;
  int cur, status, iters, nacc, relin, pad;
  // rank round protocol (acs_sba_ext_dist_round): first round pending, a trial awaiting
  // its decision, the speculative swap of the state for the next system
  int first, pending, spec_on, save_cur;
  double save_lam;
};
#define EXT_STATUS_SKIP 100  // a rejected round: no step, the system is re-formed only

struct ExtOpts {
  int max_iters;
  double ftol, xtol, gtol;
};

__device__ __forceinline__ int upk(int i, int j) {  // packed upper-triangular index, 6x6
  if (i > j) {
    const int t = i;
    i = j;
    j = t;
  }
  return i * 6 - i * (i - 1) / 2 + (j - i);
}

template <int G>
__global__ __launch_bounds__(256) void k_ext_linearize(ExtDims d, const ExtState* __restrict__ st,
                                                       const double* __restrict__ camsbuf,
                                                       const double* __restrict__ ptsbuf,
                                                       const double2* __restrict__ uv,
                                                       const uint8_t* __restrict__ mask,
                                                       const uint8_t* __restrict__ camid, double* __restrict__ Q,
                                                       double* __restrict__ Vg, double* __restrict__ Fp) {
  if (st->status != 0 || !st->relin) return;
  const int cur = st->cur;
  const double* cams = camsbuf + cur * d.C * ACS_CAM_STRIDE;
  const double* pts = ptsbuf + (size_t)cur * d.n * 3;
  __shared__ double s_cam[EXT_MAXC * ACS_CAM_STRIDE];
  for (int i = threadIdx.x; i < d.C * ACS_CAM_STRIDE; i += blockDim.x) s_cam[i] = cams[i];
  __syncthreads();
  const int lane = threadIdx.x & (G - 1);
  const int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  if (p >= d.n) return;
  const double X0 = pts[3 * p], X1 = pts[3 * p + 1], X2 = pts[3 * p + 2];
  double V[6] = {0, 0, 0, 0, 0, 0}, gp[3] = {0, 0, 0}, F = 0.0;
  for (int slot = lane; slot < d.K; slot += G) {
    const int64_t o = p * d.K + slot;
    double* q = Q + (size_t)o * EXT_Q;
    if (!mask[o] || camid[o] >= d.C) {
      for (int e = 0; e < EXT_Q; ++e) q[e] = 0.0;
      continue;
    }
    const double* c = s_cam + camid[o] * ACS_CAM_STRIDE;
    ProjOut po;
    fisheye_project<true>(c, X0, X1, X2, po);
    const double2 m = uv[o];
    const double r[2] = {po.u - m.x, po.v - m.y};
    // R X = Y - t
    const double v0 = po.Y[0] - c[17], v1 = po.Y[1] - c[18], v2 = po.Y[2] - c[19];
    double U[21];
    for (int e = 0; e < 21; ++e) U[e] = 0.0;
    double gc[6] = {0, 0, 0, 0, 0, 0}, W[18];
    for (int e = 0; e < 18; ++e) W[e] = 0.0;
    for (int dd = 0; dd < 2; ++dd) {
      const double* jy = po.JY + 3 * dd;
      const double* jp = po.J + 3 * dd;
      // J_cam = [-(J_Y [v]x), J_Y]
      const double jc[6] = {-(jy[1] * v2 - jy[2] * v1), -(jy[2] * v0 - jy[0] * v2), -(jy[0] * v1 - jy[1] * v0),
                            jy[0], jy[1], jy[2]};
      const double z = r[dd] * r[dd] / d.f2;
      const double w = 1.0 / (1.0 + z);
      const double wh = fmax((1.0 - z) * w * w, 0.1 * w);
      F += 0.5 * d.f2 * log1p(z);
      for (int i = 0; i < 6; ++i) {
        gc[i] += w * r[dd] * jc[i];
        for (int j = i; j < 6; ++j) U[upk(i, j)] += wh * jc[i] * jc[j];
        for (int j = 0; j < 3; ++j) W[i * 3 + j] += wh * jc[i] * jp[j];
      }
      for (int i = 0; i < 3; ++i) {
        gp[i] += w * r[dd] * jp[i];
        for (int j = i; j < 3; ++j) V[i == 0 ? j : (i == 1 ? 2 + j : 5)] += wh * jp[i] * jp[j];
      }
    }
    for (int e = 0; e < 21; ++e) q[e] = U[e];
    for (int e = 0; e < 6; ++e) q[21 + e] = gc[e];
    for (int e = 0; e < 18; ++e) q[27 + e] = W[e];
  }
  for (int e = 0; e < 6; ++e) V[e] = group_sum<G>(V[e]);
  for (int e = 0; e < 3; ++e) gp[e] = group_sum<G>(gp[e]);
  F = group_sum<G>(F);
  if (lane == 0) {
    double* vg = Vg + (size_t)p * 10;
    for (int e = 0; e < 6; ++e) vg[e] = V[e];
    for (int e = 0; e < 3; ++e) vg[6 + e] = gp[e];
    vg[9] = F;
    Fp[p] = F;
  }
}

// damped point block inverse M = (V + lam diag V)^-1, V packed [00 01 02 11 12 22]
__device__ __forceinline__ void point_minv(const double* V, double lam, double M[9]) {
  const double a = V[0] * (1.0 + lam) + 1e-300, b = V[1], c = V[2];
  const double e = V[3] * (1.0 + lam) + 1e-300, f = V[4], i = V[5] * (1.0 + lam) + 1e-300;
  const double A = e * i - f * f, B = -(b * i - c * f), Cc = b * f - c * e;
  const double det = a * A + b * B + c * Cc;
  if (!(det > 1e-280)) {  // point without observations: no step
    for (int k = 0; k < 9; ++k) M[k] = 0.0;
    return;
  }
  const double id = 1.0 / det;
  M[0] = A * id;
  M[1] = B * id;
  M[2] = Cc * id;
  M[3] = B * id;
  M[4] = (a * i - c * c) * id;
  M[5] = -(a * f - b * c) * id;
  M[6] = Cc * id;
  M[7] = M[5];
  M[8] = (a * e - b * b) * id;
}

// entries of a chunk partial: S (6C x 6C), b (6C), U diagonal (6C), g_c (6C)
__global__ __launch_bounds__(256) void k_ext_schur(ExtDims d, const ExtState* __restrict__ st,
                                                   const double* __restrict__ Q, const double* __restrict__ Vg,
                                                   const uint8_t* __restrict__ mask,
                                                   const uint8_t* __restrict__ camid, double* __restrict__ part) {
  if (st->status != 0) return;
  const int ch = blockIdx.x;
  const int p0 = ch * d.chunk, p1 = min(d.n, p0 + d.chunk), np = p1 - p0;
  const int NC = 6 * d.C, nE = NC * NC + 3 * NC;
  const double lam = st->lam;
  extern __shared__ double lds[];
  double* sZ = lds;                              // np x K x 18  (W M)
  double* sg = sZ + (size_t)d.chunk * d.K * 18;  // np x 3 (g_p)
  int* scam = (int*)(sg + d.chunk * 3);          // np x K camera id (-1 = none)
  for (int t = threadIdx.x; t < np; t += blockDim.x) {
    const int p = p0 + t;
    double M[9];
    point_minv(Vg + (size_t)p * 10, lam, M);
    for (int j = 0; j < 3; ++j) sg[t * 3 + j] = Vg[(size_t)p * 10 + 6 + j];
    for (int s = 0; s < d.K; ++s) {
      const int64_t o = (int64_t)p * d.K + s;
      const bool ok = mask[o] && camid[o] < d.C;
      scam[t * d.K + s] = ok ? camid[o] : -1;
      const double* W = Q + (size_t)o * EXT_Q + 27;
      for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 3; ++j)
          sZ[((size_t)t * d.K + s) * 18 + i * 3 + j] =
              ok ? W[i * 3] * M[j] + W[i * 3 + 1] * M[3 + j] + W[i * 3 + 2] * M[6 + j] : 0.0;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < nE; e += blockDim.x) {
    double acc = 0.0;
    if (e < NC * NC) {
      const int a = e / NC, b = e % NC, c1 = a / 6, k1 = a % 6, c2 = b / 6, k2 = b % 6;
      for (int t = 0; t < np; ++t) {
        const int64_t base = (int64_t)(p0 + t) * d.K;
        for (int s1 = 0; s1 < d.K; ++s1) {
          if (scam[t * d.K + s1] != c1) continue;
          if (c1 == c2) acc += Q[(size_t)(base + s1) * EXT_Q + upk(k1, k2)];
          const double* z = sZ + ((size_t)t * d.K + s1) * 18 + k1 * 3;
          for (int s2 = 0; s2 < d.K; ++s2) {
            if (scam[t * d.K + s2] != c2) continue;
            const double* w = Q + (size_t)(base + s2) * EXT_Q + 27 + k2 * 3;
            acc -= z[0] * w[0] + z[1] * w[1] + z[2] * w[2];
          }
        }
      }
    } else {
      const int r = e - NC * NC, kind = r / NC, a = r % NC, c1 = a / 6, k1 = a % 6;
      for (int t = 0; t < np; ++t) {
        const int64_t base = (int64_t)(p0 + t) * d.K;
        for (int s1 = 0; s1 < d.K; ++s1) {
          if (scam[t * d.K + s1] != c1) continue;
          const double* q = Q + (size_t)(base + s1) * EXT_Q;
          if (kind == 0) {  // b = -g_c + Z g_p
            const double* z = sZ + ((size_t)t * d.K + s1) * 18 + k1 * 3;
            acc += -q[21 + k1] + z[0] * sg[t * 3] + z[1] * sg[t * 3 + 1] + z[2] * sg[t * 3 + 2];
          } else if (kind == 1) {  // U diagonal
            acc += q[upk(k1, k1)];
          } else {  // g_c
            acc += q[21 + k1];
          }
        }
      }
    }
    part[(size_t)ch * nE + e] = acc;
  }
}

__global__ __launch_bounds__(256) void k_ext_solve(ExtDims d, ExtState* __restrict__ st, int nchunk,
                                                   const double* __restrict__ part, const double* __restrict__ Vg,
                                                   int n_gp, const double* __restrict__ slots, int n_slots,
                                                   double* __restrict__ dc, double* __restrict__ Sg,
                                                   int* __restrict__ bad) {
  // part: nchunk partials of [S | b | diag U | g_c]; the point-gradient max comes from
  // Vg (n_gp points) and/or per-rank slots (distributed: points live on their ranks)
  if (st->status != 0) return;
  const int NC = 6 * d.C, NP = ((NC + 15) / 16) * 16, nE = NC * NC + 3 * NC, LD = NP + 1;
  const double lam = st->lam;
  extern __shared__ double lds[];
  double* sS = lds;               // NP x LD
  double* sb = sS + NP * LD;      // NP
  double* tmp = sb + NP;          // 512
  double* s_red = tmp + 512;      // 256
  for (int e = threadIdx.x; e < NP * NP; e += blockDim.x) {
    const int r = e / NP, c = e % NP;
    double v = 0.0;
    if (r < NC && c < NC) {
      for (int ch = 0; ch < nchunk; ++ch) v += part[(size_t)ch * nE + r * NC + c];
      if (r == c) {
        double u = 0.0;
        for (int ch = 0; ch < nchunk; ++ch) u += part[(size_t)ch * nE + NC * NC + NC + r];
        v += lam * fmax(u, 1e-12);
      }
    } else if (r == c) {
      v = 1.0;
    }
    sS[r * LD + c] = v;
    if (r < NC && c < NC) Sg[r * NC + c] = v;  // kept for the refinement step
  }
  double gm = 0.0;
  for (int r = threadIdx.x; r < NP; r += blockDim.x) {
    double v = 0.0, g = 0.0;
    if (r < NC)
      for (int ch = 0; ch < nchunk; ++ch) {
        v += part[(size_t)ch * nE + NC * NC + r];
        g += part[(size_t)ch * nE + NC * NC + 2 * NC + r];
      }
    sb[r] = v;
    gm = fmax(gm, fabs(g));
  }
  for (int p = threadIdx.x; p < n_gp; p += blockDim.x)
    for (int j = 0; j < 3; ++j) gm = fmax(gm, fabs(Vg[(size_t)p * 10 + 6 + j]));
  for (int t = threadIdx.x; t < n_slots; t += blockDim.x) gm = fmax(gm, slots[t]);
  __syncthreads();
  {  // block max
    s_red[threadIdx.x] = gm;
    __syncthreads();
    for (int h = (int)blockDim.x / 2; h > 0; h >>= 1) {
      if ((int)threadIdx.x < h) s_red[threadIdx.x] = fmax(s_red[threadIdx.x], s_red[threadIdx.x + h]);
      __syncthreads();
    }
    if (threadIdx.x == 0 && st->relin) st->gmax = s_red[0];
    __syncthreads();
  }
  wg_spd_inverse(sS, LD, NP >> 4, tmp, bad);
  // dc = S^-1 b, then one step of iterative refinement dc += S^-1 (b - S dc): with the
  // gauge left free (as in the reference) S is conditioned like 1/lambda at small damping
  double* sx = tmp;  // NC <= 96 < 512
  double* sr = tmp + 256;
  for (int r = threadIdx.x; r < NC; r += blockDim.x) {
    double v = 0.0;
    for (int c = 0; c < NC; ++c) v += sS[r * LD + c] * sb[c];
    sx[r] = v;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < NC; r += blockDim.x) {
    double v = sb[r];
    for (int c = 0; c < NC; ++c) v -= Sg[r * NC + c] * sx[c];
    sr[r] = v;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < NC; r += blockDim.x) {
    double v = sx[r];
    for (int c = 0; c < NC; ++c) v += sS[r * LD + c] * sr[c];
    dc[r] = v;
  }
}

__global__ __launch_bounds__(256) void k_ext_back(ExtDims d, const ExtState* __restrict__ st,
                                                  const double* __restrict__ Q, const double* __restrict__ Vg,
                                                  const uint8_t* __restrict__ mask,
                                                  const uint8_t* __restrict__ camid, const double* __restrict__ dc,
                                                  double* __restrict__ ptsbuf, double* __restrict__ normp) {
  if (st->status != 0) return;
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= d.n) return;
  const int cur = st->cur;
  const double* X = ptsbuf + (size_t)cur * d.n * 3;
  double* Xn = ptsbuf + (size_t)(cur ^ 1) * d.n * 3;
  double M[9];
  point_minv(Vg + (size_t)p * 10, st->lam, M);
  double acc[3] = {Vg[(size_t)p * 10 + 6], Vg[(size_t)p * 10 + 7], Vg[(size_t)p * 10 + 8]};
  for (int s = 0; s < d.K; ++s) {
    const int64_t o = p * d.K + s;
    if (!mask[o] || camid[o] >= d.C) continue;
    const double* W = Q + (size_t)o * EXT_Q + 27;
    const double* dcc = dc + 6 * camid[o];
    for (int j = 0; j < 3; ++j)
      for (int i = 0; i < 6; ++i) acc[j] += W[i * 3 + j] * dcc[i];
  }
  double dn = 0.0, xn = 0.0;
  for (int j = 0; j < 3; ++j) {
    const double dx = -(M[j * 3] * acc[0] + M[j * 3 + 1] * acc[1] + M[j * 3 + 2] * acc[2]);
    Xn[3 * p + j] = X[3 * p + j] + dx;
    dn += dx * dx;
    xn += X[3 * p + j] * X[3 * p + j];
  }
  normp[2 * p] = dn;
  normp[2 * p + 1] = xn;
}

__global__ void k_ext_cam(ExtDims d, const ExtState* __restrict__ st, const double* __restrict__ dc,
                          double* __restrict__ camsbuf, double* __restrict__ camnorm) {
  if (st->status != 0) return;
  const int c = threadIdx.x;
  if (c >= d.C) return;
  const int cur = st->cur;
  const double* cm = camsbuf + (cur * d.C + c) * ACS_CAM_STRIDE;
  double* cn = camsbuf + ((cur ^ 1) * d.C + c) * ACS_CAM_STRIDE;
  for (int i = 0; i < 8; ++i) cn[i] = cm[i];
  const double w0 = dc[6 * c], w1 = dc[6 * c + 1], w2 = dc[6 * c + 2];
  const double th = sqrt(w0 * w0 + w1 * w1 + w2 * w2);
  double E[9];
  if (th < 1e-300) {
    for (int i = 0; i < 9; ++i) E[i] = (i % 4 == 0) ? 1.0 : 0.0;
  } else {
    const double k0 = w0 / th, k1 = w1 / th, k2 = w2 / th, cs = cos(th), sn = sin(th), oc = 1.0 - cs;
    E[0] = cs + oc * k0 * k0;
    E[1] = oc * k0 * k1 - sn * k2;
    E[2] = oc * k0 * k2 + sn * k1;
    E[3] = oc * k1 * k0 + sn * k2;
    E[4] = cs + oc * k1 * k1;
    E[5] = oc * k1 * k2 - sn * k0;
    E[6] = oc * k2 * k0 - sn * k1;
    E[7] = oc * k2 * k1 + sn * k0;
    E[8] = cs + oc * k2 * k2;
  }
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      cn[8 + i * 3 + j] = E[i * 3] * cm[8 + j] + E[i * 3 + 1] * cm[8 + 3 + j] + E[i * 3 + 2] * cm[8 + 6 + j];
  double dn = 0.0, xn = 0.0;
  for (int i = 0; i < 3; ++i) {
    cn[17 + i] = cm[17 + i] + dc[6 * c + 3 + i];
    dn += dc[6 * c + i] * dc[6 * c + i] + dc[6 * c + 3 + i] * dc[6 * c + 3 + i];
    xn += cm[17 + i] * cm[17 + i];
  }
  camnorm[2 * c] = dn;
  camnorm[2 * c + 1] = xn;
}

template <int G>
__global__ __launch_bounds__(256) void k_ext_cost(ExtDims d, const ExtState* __restrict__ st, int which,
                                                  const double* __restrict__ camsbuf,
                                                  const double* __restrict__ ptsbuf, const double2* __restrict__ uv,
                                                  const uint8_t* __restrict__ mask,
                                                  const uint8_t* __restrict__ camid, double* __restrict__ Fp) {
  if (which == 1 && st->status != 0) return;
  const int buf = which == 1 ? (st->cur ^ 1) : st->cur;
  const double* cams = camsbuf + buf * d.C * ACS_CAM_STRIDE;
  const double* pts = ptsbuf + (size_t)buf * d.n * 3;
  __shared__ double s_cam[EXT_MAXC * ACS_CAM_STRIDE];
  for (int i = threadIdx.x; i < d.C * ACS_CAM_STRIDE; i += blockDim.x) s_cam[i] = cams[i];
  __syncthreads();
  const int lane = threadIdx.x & (G - 1);
  const int64_t p = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  if (p >= d.n) return;
  double F = 0.0;
  for (int slot = lane; slot < d.K; slot += G) {
    const int64_t o = p * d.K + slot;
    if (!mask[o] || camid[o] >= d.C) continue;
    ProjOut po;
    fisheye_project<false>(s_cam + camid[o] * ACS_CAM_STRIDE, pts[3 * p], pts[3 * p + 1], pts[3 * p + 2], po);
    const double2 m = uv[o];
    const double ru = po.u - m.x, rv = po.v - m.y;
    F += 0.5 * d.f2 * (log1p(ru * ru / d.f2) + log1p(rv * rv / d.f2));
  }
  F = group_sum<G>(F);
  if (lane == 0) Fp[p] = F;
}

__global__ __launch_bounds__(256) void k_ext_lm(ExtDims d, ExtState* __restrict__ st, ExtOpts o, int init,
                                                const double* __restrict__ Fp, const double* __restrict__ normp,
                                                const double* __restrict__ camnorm) {
  __shared__ double s_red[256];
  const int tid = threadIdx.x;
  auto bsum = [&](double v) {
    s_red[tid] = v;
    __syncthreads();
    for (int h = (int)blockDim.x / 2; h > 0; h >>= 1) {
      if (tid < h) s_red[tid] += s_red[tid + h];
      __syncthreads();
    }
    const double r = s_red[0];
    __syncthreads();
    return r;
  };
  double f = 0.0, dn = 0.0, xn = 0.0;
  for (int p = tid; p < d.n; p += blockDim.x) {
    f += Fp[p];
    if (!init) {
      dn += normp[2 * p];
      xn += normp[2 * p + 1];
    }
  }
  f = bsum(f);
  if (init) {
    if (tid == 0) st->F = st->F0 = f;
    return;
  }
  if (st->status != 0) return;
  dn = bsum(dn);
  xn = bsum(xn);
  if (tid != 0) return;
  for (int c = 0; c < d.C; ++c) {
    dn += camnorm[2 * c];
    xn += camnorm[2 * c + 1];
  }
  if (st->gmax <= o.gtol) {
    st->status = ACS_STATUS_GTOL;
    return;
  }
  st->iters += 1;
  st->dnorm = sqrt(dn);
  st->xnorm = sqrt(xn);
  const bool small = sqrt(dn) <= o.xtol * (o.xtol + sqrt(xn));
  if (f < st->F) {
    const bool fconv = (st->F - f) <= o.ftol * fabs(st->F);
    st->nacc += 1;
    st->F = f;
    st->cur ^= 1;
    st->lam = fmax(st->lam * 0.1, EXT_LAM_MIN);
    st->relin = 1;
    if (fconv)
      st->status = ACS_STATUS_FTOL;
    else if (small)
      st->status = ACS_STATUS_XTOL;
  } else {
    st->lam *= 10.0;
    st->relin = 0;
    if (st->lam > 1e16) st->status = ACS_STATUS_STALLED;
  }
  if (st->status == 0 && st->iters >= o.max_iters) st->status = ACS_STATUS_MAXITER;
}

// ---------------------------------------------------------------------------------------
static size_t ext_schur_lds(const ExtDims& d) {
  return sizeof(double) * ((size_t)d.chunk * d.K * 18 + d.chunk * 3) + sizeof(int) * d.chunk * d.K;
}

template <int G>
static void ext_enqueue(hipStream_t s, const ExtDims& d, ExtState* st, const ExtOpts& o, double* cams, double* pts,
                        const double2* uv, const uint8_t* mk, const uint8_t* cid, double* Q, double* Vg, double* Fp,
                        double* part, double* dc, double* Sg, double* normp, double* camnorm, int* bad,
                        int nchunk) {
  const int blocks = acs_grid((int64_t)d.n * G, 256);
  const size_t lds = ext_schur_lds(d);
  const int NP = ((6 * d.C + 15) / 16) * 16;
  const size_t lds_solve = sizeof(double) * ((size_t)NP * (NP + 1) + NP + 512 + 256);
  hipLaunchKernelGGL((k_ext_linearize<G>), dim3(blocks), dim3(256), 0, s, d, st, cams, pts, uv, mk, cid, Q, Vg, Fp);
  hipLaunchKernelGGL(k_ext_schur, dim3(nchunk), dim3(256), lds, s, d, st, Q, Vg, mk, cid, part);
  hipLaunchKernelGGL(k_ext_solve, dim3(1), dim3(256), lds_solve, s, d, st, nchunk, part, Vg, d.n, nullptr, 0, dc, Sg,
                     bad);
  hipLaunchKernelGGL(k_ext_back, dim3(acs_grid(d.n, 256)), dim3(256), 0, s, d, st, Q, Vg, mk, cid, dc, pts, normp);
  hipLaunchKernelGGL(k_ext_cam, dim3(1), dim3(64), 0, s, d, st, dc, cams, camnorm);
  hipLaunchKernelGGL((k_ext_cost<G>), dim3(blocks), dim3(256), 0, s, d, st, 1, cams, pts, uv, mk, cid, Fp);
  hipLaunchKernelGGL(k_ext_lm, dim3(1), dim3(256), 0, s, d, st, o, 0, Fp, normp, camnorm);
}

extern "C" {

void acs_sba_ext_default_opts(acs_sba_ext_opts* o) {
  o->max_iters = 500;
  o->reserved = 0;
  o->f_scale = 1.0;
  o->ftol = 1e-12;
  o->xtol = 1e-12;
  o->gtol = 1e-8;
  o->lambda0 = 1e-3;
}

int acs_sba_extrinsics(acs_ctx* ctx, double* cams, int32_t n_cams, const double* uv, const int32_t* pt_idx,
                       const int32_t* cam_idx, int64_t n_obs, double* pts, int64_t n_pts,
                       const acs_sba_ext_opts* opts, double* resid_before, double* resid_after,
                       acs_sba_ext_report* report, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  acs_sba_ext_opts op;
  acs_sba_ext_default_opts(&op);
  if (opts) op = *opts;
  ACS_CHECK(ctx, n_cams >= 1 && n_cams <= EXT_MAXC, "acs_sba_extrinsics: n_cams=%d (1..%d)", n_cams, EXT_MAXC);
  ACS_CHECK(ctx, n_obs >= 1 && n_pts >= 1 && n_obs < (int64_t)INT32_MAX, "acs_sba_extrinsics: bad sizes");
  ACS_CHECK(ctx, op.f_scale > 0 && op.max_iters >= 0, "acs_sba_extrinsics: bad options");
  hipStream_t s = ctx->stream;
  void *dcam0, *duv, *dpi, *dci, *dp0;
  int rc;
  if ((rc = acs_stage_in(ctx, WS_CAMS, cams, sizeof(double) * ACS_CAM_STRIDE * n_cams, flags, &dcam0))) return rc;
  if ((rc = acs_stage_in(ctx, WS_UV, uv, sizeof(double) * 2 * n_obs, flags, &duv))) return rc;
  if ((rc = acs_stage_in(ctx, WS_PTIDX, pt_idx, sizeof(int32_t) * n_obs, flags, &dpi))) return rc;
  if ((rc = acs_stage_in(ctx, WS_CAMIDX, cam_idx, sizeof(int32_t) * n_obs, flags, &dci))) return rc;
  if ((rc = acs_stage_in(ctx, WS_PTS, pts, sizeof(double) * 3 * n_pts, flags, &dp0))) return rc;
  double* drb = nullptr;
  if (resid_before) {
    drb = (double*)acs_out_buf(ctx, WS_OUT0, resid_before, sizeof(double) * 2 * n_obs, flags);
    if (!drb || (rc = acs_sba_residuals(ctx, (const double*)dcam0, n_cams, (const double*)duv, (const int32_t*)dpi,
                                        (const int32_t*)dci, n_obs, (const double*)dp0, n_pts, drb, ACS_DEVICE_PTRS)))
      return rc ? rc : ACS_E_NOMEM;
  }
  double2* uvp;
  uint8_t *mk, *cid;
  int K;
  if ((rc = acs_obs_to_slots(ctx, (const double*)duv, (const int32_t*)dpi, (const int32_t*)dci, n_obs, n_pts, n_cams,
                             &uvp, &mk, &cid, &K)))
    return rc;
  ACS_CHECK(ctx, K <= 64, "acs_sba_extrinsics: a point has %d observations (max 64)", K);
  ExtDims d{(int)n_pts, K, n_cams, 2, EXT_CHUNK, op.f_scale * op.f_scale};
  int G = 2;
  while (G < K) G <<= 1;
  d.G = G;
  // points per Schur block: W M tiles of a chunk must fit ~96 KB of LDS
  d.chunk = std::max(1, std::min(EXT_CHUNK, (int)(96 * 1024 / (148 * K + 24))));
  const int nchunk = (int)((n_pts + d.chunk - 1) / d.chunk);
  const int NC = 6 * n_cams, nE = NC * NC + 3 * NC;
  size_t off = 0;
  auto take = [&](size_t cnt) {
    size_t o = off;
    off += ((cnt * sizeof(double) + 255) / 256) * 256 / sizeof(double);
    return o;
  };
  const size_t oC = take(2 * (size_t)n_cams * ACS_CAM_STRIDE), oP = take(6 * (size_t)n_pts),
               oQ = take((size_t)n_pts * K * EXT_Q), oV = take((size_t)n_pts * 10), oF = take(n_pts),
               oPart = take((size_t)nchunk * nE), odc = take(96), oSg = take(96 * 96), onp = take(2 * (size_t)n_pts), ocn = take(64),
               ost = take(16), obad = take(2);
  double* arena = (double*)acs_ws(ctx, WS_FTE6, off * sizeof(double));
  if (!arena) return ACS_E_NOMEM;
  double *dcams = arena + oC, *dpts = arena + oP, *Q = arena + oQ, *Vg = arena + oV, *Fp = arena + oF,
         *part = arena + oPart, *dc = arena + odc, *Sg = arena + oSg, *normp = arena + onp, *camnorm = arena + ocn;
  ExtState* st = (ExtState*)(arena + ost);
  int* bad = (int*)(arena + obad);
  ACS_HIP(ctx, hipMemcpyAsync(dcams, dcam0, sizeof(double) * ACS_CAM_STRIDE * n_cams, hipMemcpyDeviceToDevice, s));
  ACS_HIP(ctx, hipMemcpyAsync(dcams + n_cams * ACS_CAM_STRIDE, dcam0, sizeof(double) * ACS_CAM_STRIDE * n_cams,
                              hipMemcpyDeviceToDevice, s));
  ACS_HIP(ctx, hipMemcpyAsync(dpts, dp0, sizeof(double) * 3 * n_pts, hipMemcpyDeviceToDevice, s));
  ACS_HIP(ctx, hipMemsetAsync(bad, 0, sizeof(int), s));
  ExtState st0;
  std::memset(&st0, 0, sizeof(st0));
  st0.lam = op.lambda0;
  st0.relin = 1;
  ACS_HIP(ctx, hipMemcpyAsync(st, &st0, sizeof(st0), hipMemcpyHostToDevice, s));
  ExtOpts o{op.max_iters, op.ftol, op.xtol, op.gtol};
  const int blocks = acs_grid((int64_t)n_pts * G, 256);
  auto launch_cost0 = [&]() {
    switch (G) {
#define EXT_C0(g) \
  case g: hipLaunchKernelGGL((k_ext_cost<g>), dim3(blocks), dim3(256), 0, s, d, st, 0, dcams, dpts, uvp, mk, cid, Fp); break;
      EXT_C0(2) EXT_C0(4) EXT_C0(8) EXT_C0(16) EXT_C0(32) EXT_C0(64)
#undef EXT_C0
    }
  };
  launch_cost0();
  hipLaunchKernelGGL(k_ext_lm, dim3(1), dim3(256), 0, s, d, st, o, 1, Fp, normp, camnorm);
  ACS_HIP(ctx, hipGetLastError());
  auto enqueue = [&]() {
    switch (G) {
#define EXT_IT(g) \
  case g: ext_enqueue<g>(s, d, st, o, dcams, dpts, uvp, mk, cid, Q, Vg, Fp, part, dc, Sg, normp, camnorm, bad, nchunk); \
    break;
      EXT_IT(2) EXT_IT(4) EXT_IT(8) EXT_IT(16) EXT_IT(32) EXT_IT(64)
#undef EXT_IT
    }
  };
  const int chunk = 4;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  bool use_graph = op.max_iters > 0 && hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed) == hipSuccess;
  if (use_graph) {
    for (int c = 0; c < chunk; ++c) enqueue();
    if (hipStreamEndCapture(s, &graph) != hipSuccess ||
        hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0) != hipSuccess) {
      if (graph) (void)hipGraphDestroy(graph);
      (void)hipGetLastError();
      graph = nullptr;
      exec = nullptr;
      use_graph = false;
    }
  }
  ExtState hs;
  std::memset(&hs, 0, sizeof(hs));
  for (int it = 0; it < op.max_iters + chunk; it += chunk) {
    if (use_graph) {
      ACS_HIP(ctx, hipGraphLaunch(exec, s));
    } else {
      for (int c = 0; c < chunk; ++c) enqueue();
    }
    ACS_HIP(ctx, hipGetLastError());
    ACS_HIP(ctx, hipMemcpyAsync(&hs, st, sizeof(hs), hipMemcpyDeviceToHost, s));
    ACS_HIP(ctx, hipStreamSynchronize(s));
    if (hs.status != 0) break;
  }
  if (exec) (void)hipGraphExecDestroy(exec);
  if (graph) (void)hipGraphDestroy(graph);
  if (op.max_iters == 0) {
    ACS_HIP(ctx, hipMemcpyAsync(&hs, st, sizeof(hs), hipMemcpyDeviceToHost, s));
    ACS_HIP(ctx, hipStreamSynchronize(s));
  }
  const double* fcams = dcams + hs.cur * n_cams * ACS_CAM_STRIDE;
  const double* fpts = dpts + (size_t)hs.cur * n_pts * 3;
  const hipMemcpyKind kout = (flags & ACS_DEVICE_PTRS) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  if (resid_after) {
    double* dra = (double*)acs_out_buf(ctx, WS_OUT1, resid_after, sizeof(double) * 2 * n_obs, flags);
    if (!dra || (rc = acs_sba_residuals(ctx, fcams, n_cams, (const double*)duv, (const int32_t*)dpi,
                                        (const int32_t*)dci, n_obs, fpts, n_pts, dra, ACS_DEVICE_PTRS)))
      return rc ? rc : ACS_E_NOMEM;
    if ((rc = acs_stage_out(ctx, resid_after, dra, sizeof(double) * 2 * n_obs, flags))) return rc;
  }
  if (resid_before && (rc = acs_stage_out(ctx, resid_before, drb, sizeof(double) * 2 * n_obs, flags))) return rc;
  ACS_HIP(ctx, hipMemcpyAsync(cams, fcams, sizeof(double) * ACS_CAM_STRIDE * n_cams, kout, s));
  ACS_HIP(ctx, hipMemcpyAsync(pts, fpts, sizeof(double) * 3 * n_pts, kout, s));
  int nbad = 0;
  ACS_HIP(ctx, hipMemcpyAsync(&nbad, bad, sizeof(int), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipStreamSynchronize(s));
  if (report) {
    report->status = hs.status == 0 ? ACS_STATUS_MAXITER : hs.status;
    report->iters = hs.iters;
    report->n_accepted = hs.nacc;
    report->n_bad_pivots = nbad;
    report->cost_before = hs.F0;
    report->cost_after = hs.F;
    report->grad_max = hs.gmax;
    report->lambda_final = hs.lam;
  }
  return ACS_OK;
}

}  // extern "C"

// =======================================================================================
// distributed points + extrinsics: points are split over the ranks,
// cameras replicated. Per LM step one all-reduce of the reduced camera system (p1 =
// [S | b | diag U | g_c | per-rank point |g| max]) and one of 3 doubles (cost, point
// step norms). Every rank solves the same camera system and takes the same decision.
// Spec: oracle/sba_ext_dist.py.
// =======================================================================================
__global__ __launch_bounds__(256) void k_ext_pack1(ExtDims d, const ExtState* __restrict__ st, int nchunk,
                                                   const double* __restrict__ part, const double* __restrict__ Vg,
                                                   int rank, double* __restrict__ p1) {
  if (st->status != 0) return;
  __shared__ double s_red[256];
  const int NC = 6 * d.C, nE = NC * NC + 3 * NC;
  for (int e = threadIdx.x; e < nE; e += blockDim.x) {
    double v = 0.0;
    for (int ch = 0; ch < nchunk; ++ch) v += part[(size_t)ch * nE + e];
    p1[e] = v;
  }
  double gm = 0.0;
  for (int p = threadIdx.x; p < d.n; p += blockDim.x)
    for (int j = 0; j < 3; ++j) gm = fmax(gm, fabs(Vg[(size_t)p * 10 + 6 + j]));
  s_red[threadIdx.x] = gm;
  __syncthreads();
  for (int h = (int)blockDim.x / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) s_red[threadIdx.x] = fmax(s_red[threadIdx.x], s_red[threadIdx.x + h]);
    __syncthreads();
  }
  if (threadIdx.x == 0) p1[nE + rank] = s_red[0];
}

__global__ __launch_bounds__(256) void k_ext_pack3(ExtDims d, const ExtState* __restrict__ st, int which,
                                                   const double* __restrict__ Fp, const double* __restrict__ normp,
                                                   double* __restrict__ p3) {
  if (which == 1 && st->status != 0) return;
  __shared__ double s_red[3][256];
  double a = 0.0, b = 0.0, c = 0.0;
  for (int p = threadIdx.x; p < d.n; p += blockDim.x) {
    a += Fp[p];
    if (which) {
      b += normp[2 * p];
      c += normp[2 * p + 1];
    }
  }
  s_red[0][threadIdx.x] = a;
  s_red[1][threadIdx.x] = b;
  s_red[2][threadIdx.x] = c;
  __syncthreads();
  for (int h = (int)blockDim.x / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h)
      for (int k = 0; k < 3; ++k) s_red[k][threadIdx.x] += s_red[k][threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0)
    for (int k = 0; k < 3; ++k) p3[k] = s_red[k][0];
}

// Rank round protocol: the decision on the pending trial from the all-reduced (cost,
// |dX|^2, |X|^2) of the previous round (k_ext_lm's rule); a rejection marks the round
// SKIP (no step: the system is re-formed at the current state with the raised damping).
__global__ void k_ext_decide(ExtDims d, ExtState* __restrict__ st, ExtOpts o, const double* __restrict__ p3,
                             const double* __restrict__ camnorm) {
  if (threadIdx.x != 0) return;
  if (st->first) {
    st->first = 0;
    st->F = st->F0 = p3[0];
    if (o.max_iters <= 0) st->status = ACS_STATUS_MAXITER;  // no step at all
    return;
  }
  if (st->status != 0 || !st->pending) return;
  st->pending = 0;
  double dn = p3[1], xn = p3[2];
  for (int c = 0; c < d.C; ++c) {
    dn += camnorm[2 * c];
    xn += camnorm[2 * c + 1];
  }
  if (st->gmax <= o.gtol) {
    st->status = ACS_STATUS_GTOL;
    return;
  }
  const double f = p3[0];
  st->iters += 1;
  st->dnorm = sqrt(dn);
  st->xnorm = sqrt(xn);
  const bool small = sqrt(dn) <= o.xtol * (o.xtol + sqrt(xn));
  if (f < st->F) {
    const bool fconv = (st->F - f) <= o.ftol * fabs(st->F);
    st->nacc += 1;
    st->F = f;
    st->cur ^= 1;
    st->lam = fmax(st->lam * 0.1, EXT_LAM_MIN);
    st->relin = 1;
    if (fconv)
      st->status = ACS_STATUS_FTOL;
    else if (small)
      st->status = ACS_STATUS_XTOL;
  } else {
    st->lam *= 10.0;
    st->relin = 0;
    if (st->lam > 1e16) st->status = ACS_STATUS_STALLED;
  }
  if (st->status == 0 && st->iters >= o.max_iters) st->status = ACS_STATUS_MAXITER;
  if (st->status == 0 && !st->relin) st->status = EXT_STATUS_SKIP;
}

// Around the system of a round: a round that took a step forms the next system at its trial
// state (points / cameras copy cur ^ 1) with the damping an acceptance sets (speculation:
// the next round's decision keeps it or discards it); the LM state is swapped for those
// kernels and restored after them. A rejected round re-linearises at the current state
// (the speculative system overwrote its linearisation).
__global__ void k_ext_spec(ExtState* __restrict__ st, int enter) {
  if (threadIdx.x != 0) return;
  if (enter) {
    if (st->status == EXT_STATUS_SKIP) {
      st->status = 0;
      st->relin = 1;
    } else if (st->status == 0) {
      st->pending = 1;
      st->spec_on = 1;
      st->save_cur = st->cur;
      st->save_lam = st->lam;
      st->cur ^= 1;
      st->lam = fmax(st->lam * 0.1, EXT_LAM_MIN);
      st->relin = 1;
    }
  } else if (st->spec_on) {
    st->spec_on = 0;
    st->cur = st->save_cur;
    st->lam = st->save_lam;
  }
}

#define EXT_DIST_RING 4

struct acs_sba_ext_dist {
  acs_ctx* ctx;
  void* own = nullptr;
  ExtDims d;
  ExtOpts o;
  int R, rank, nchunk;
  double *dcams, *dpts, *Q, *Vg, *Fp, *part, *dc, *Sg, *normp, *camnorm;
  double2* uvp;
  uint8_t *mk, *cid;
  ExtState* st;
  int* bad;
  // status after each round: pinned ring with completion events (acs_sba_ext_dist_poll)
  int32_t* snap = nullptr;
  hipEvent_t snap_ev[EXT_DIST_RING] = {};
  int64_t rounds = 0;
};

template <int G>
static void ext_dist_linearize(acs_sba_ext_dist* h, hipStream_t s) {
  const ExtDims& d = h->d;
  const int blocks = acs_grid((int64_t)d.n * G, 256);
  hipLaunchKernelGGL((k_ext_linearize<G>), dim3(blocks), dim3(256), 0, s, d, h->st, h->dcams, h->dpts, h->uvp, h->mk,
                     h->cid, h->Q, h->Vg, h->Fp);
}

template <int G>
static void ext_dist_cost(acs_sba_ext_dist* h, hipStream_t s, int which) {
  const ExtDims& d = h->d;
  const int blocks = acs_grid((int64_t)d.n * G, 256);
  hipLaunchKernelGGL((k_ext_cost<G>), dim3(blocks), dim3(256), 0, s, d, h->st, which, h->dcams, h->dpts, h->uvp,
                     h->mk, h->cid, h->Fp);
}

#define EXT_G_SWITCH(G, CALL)                  \
  switch (G) {                                 \
    case 2: CALL(2); break;                    \
    case 4: CALL(4); break;                    \
    case 8: CALL(8); break;                    \
    case 16: CALL(16); break;                  \
    case 32: CALL(32); break;                  \
    default: CALL(64); break;                  \
  }

extern "C" {

int acs_sba_ext_dist_create(acs_ctx* ctx, const double* cams, int32_t n_cams, const double* uv,
                            const int32_t* pt_idx, const int32_t* cam_idx, int64_t n_obs, const double* pts,
                            int64_t n_pts, const acs_sba_ext_opts* opts, int32_t rank, int32_t world,
                            acs_sba_ext_dist** out, int64_t* payload_sizes, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  acs_sba_ext_opts op;
  acs_sba_ext_default_opts(&op);
  if (opts) op = *opts;
  ACS_CHECK(ctx, n_cams >= 1 && n_cams <= EXT_MAXC, "sba_ext_dist: n_cams=%d (1..%d)", n_cams, EXT_MAXC);
  ACS_CHECK(ctx, n_obs >= 1 && n_pts >= 1 && n_obs < (int64_t)INT32_MAX, "sba_ext_dist: bad sizes");
  ACS_CHECK(ctx, op.f_scale > 0 && op.max_iters >= 0, "sba_ext_dist: bad options");
  ACS_CHECK(ctx, world >= 1 && rank >= 0 && rank < world, "sba_ext_dist: rank %d / world %d", rank, world);
  hipStream_t s = ctx->stream;
  void *dcam0, *duv, *dpi, *dci, *dp0;
  int rc;
  if ((rc = acs_stage_in(ctx, WS_CAMS, cams, sizeof(double) * ACS_CAM_STRIDE * n_cams, flags, &dcam0))) return rc;
  if ((rc = acs_stage_in(ctx, WS_UV, uv, sizeof(double) * 2 * n_obs, flags, &duv))) return rc;
  if ((rc = acs_stage_in(ctx, WS_PTIDX, pt_idx, sizeof(int32_t) * n_obs, flags, &dpi))) return rc;
  if ((rc = acs_stage_in(ctx, WS_CAMIDX, cam_idx, sizeof(int32_t) * n_obs, flags, &dci))) return rc;
  if ((rc = acs_stage_in(ctx, WS_PTS, pts, sizeof(double) * 3 * n_pts, flags, &dp0))) return rc;
  double2* uvp;
  uint8_t *mk, *cid;
  int K;
  if ((rc = acs_obs_to_slots(ctx, (const double*)duv, (const int32_t*)dpi, (const int32_t*)dci, n_obs, n_pts, n_cams,
                             &uvp, &mk, &cid, &K)))
    return rc;
  ACS_CHECK(ctx, K <= 64, "sba_ext_dist: a point has %d observations (max 64)", K);
  acs_sba_ext_dist* h = new acs_sba_ext_dist();
  h->ctx = ctx;
  ExtDims& d = h->d;
  d = ExtDims{(int)n_pts, K, n_cams, 2, EXT_CHUNK, op.f_scale * op.f_scale};
  while (d.G < K) d.G <<= 1;
  d.chunk = std::max(1, std::min(EXT_CHUNK, (int)(96 * 1024 / (148 * K + 24))));
  h->nchunk = (int)((n_pts + d.chunk - 1) / d.chunk);
  h->R = world;
  h->rank = rank;
  h->o = ExtOpts{op.max_iters, op.ftol, op.xtol, op.gtol};
  const int NC = 6 * n_cams, nE = NC * NC + 3 * NC;
  size_t off = 0;
  auto take = [&](size_t cnt) {
    size_t o = off;
    off += ((cnt * sizeof(double) + 255) / 256) * 256 / sizeof(double);
    return o;
  };
  const size_t oC = take(2 * (size_t)n_cams * ACS_CAM_STRIDE), oP = take(6 * (size_t)n_pts),
               oQ = take((size_t)n_pts * K * EXT_Q), oV = take((size_t)n_pts * 10), oF = take(n_pts),
               oPart = take((size_t)h->nchunk * nE), odc = take(96), oSg = take(96 * 96), onp = take(2 * (size_t)n_pts),
               ocn = take(64), ost = take(16), obad = take(2), ouv = take(2 * (size_t)n_pts * K),
               omk = take(((size_t)n_pts * K + 7) / 8), ocid = take(((size_t)n_pts * K + 7) / 8);
  if (acs_dev_malloc(&h->own, off * sizeof(double)) != hipSuccess) {
    delete h;
    return acs_fail(ctx, ACS_E_NOMEM, "sba_ext_dist: allocation failed");
  }
  double* a = (double*)h->own;
  h->dcams = a + oC;
  h->dpts = a + oP;
  h->Q = a + oQ;
  h->Vg = a + oV;
  h->Fp = a + oF;
  h->part = a + oPart;
  h->dc = a + odc;
  h->Sg = a + oSg;
  h->normp = a + onp;
  h->camnorm = a + ocn;
  h->st = (ExtState*)(a + ost);
  h->bad = (int*)(a + obad);
  h->uvp = (double2*)(a + ouv);
  h->mk = (uint8_t*)(a + omk);
  h->cid = (uint8_t*)(a + ocid);
  ACS_HIP(ctx, hipMemcpyAsync(h->uvp, uvp, sizeof(double2) * n_pts * K, hipMemcpyDeviceToDevice, s));
  ACS_HIP(ctx, hipMemcpyAsync(h->mk, mk, (size_t)n_pts * K, hipMemcpyDeviceToDevice, s));
  ACS_HIP(ctx, hipMemcpyAsync(h->cid, cid, (size_t)n_pts * K, hipMemcpyDeviceToDevice, s));
  for (int b = 0; b < 2; ++b)
    ACS_HIP(ctx, hipMemcpyAsync(h->dcams + b * n_cams * ACS_CAM_STRIDE, dcam0, sizeof(double) * ACS_CAM_STRIDE * n_cams,
                                hipMemcpyDeviceToDevice, s));
  ACS_HIP(ctx, hipMemcpyAsync(h->dpts, dp0, sizeof(double) * 3 * n_pts, hipMemcpyDeviceToDevice, s));
  ACS_HIP(ctx, hipMemsetAsync(h->bad, 0, sizeof(int), s));
  ExtState st0;
  std::memset(&st0, 0, sizeof(st0));
  st0.lam = op.lambda0;
  st0.relin = 1;
  st0.first = 1;
  ACS_HIP(ctx, hipMemcpyAsync(h->st, &st0, sizeof(st0), hipMemcpyHostToDevice, s));
  ACS_HIP(ctx, hipStreamSynchronize(s));
  bool snap_ok = acs_host_malloc((void**)&h->snap, sizeof(int32_t) * EXT_DIST_RING, hipHostMallocDefault) == hipSuccess;
  for (auto& e : h->snap_ev)
    if (snap_ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      e = nullptr;
      snap_ok = false;
    }
  if (!snap_ok) {
    acs_sba_ext_dist_destroy(h);
    return acs_fail(ctx, ACS_E_HIP, "sba_ext_dist: pinned status ring allocation failed");
  }
  if (payload_sizes) {
    payload_sizes[0] = nE + world + 3;  // [reduced camera system | (cost, |dX|^2, |X|^2)]
    payload_sizes[1] = 3;
  }
  *out = h;
  return ACS_OK;
}

int acs_sba_ext_dist_destroy(acs_sba_ext_dist* h) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  if (!h) return ACS_OK;
  (void)hipStreamSynchronize(h->ctx->stream);
  for (auto& e : h->snap_ev)
    if (e) (void)hipEventDestroy(e);
  if (h->snap) (void)acs_host_free(h->snap);
  if (h->own) (void)acs_dev_free(h->own);
  delete h;
  return ACS_OK;
}

}  // extern "C"

// the rank's reduced camera system at the current state (payload part 1, zeroed first)
static int ext_dist_system(acs_sba_ext_dist* h, double* p1) {
  acs_ctx* ctx = h->ctx;
  hipStream_t s = ctx->stream;
  const ExtDims& d = h->d;
  const int NC = 6 * d.C, nE = NC * NC + 3 * NC;
  ACS_HIP(ctx, hipMemsetAsync(p1, 0, sizeof(double) * (nE + h->R), s));
#define EXT_LIN(g) ext_dist_linearize<g>(h, s)
  EXT_G_SWITCH(d.G, EXT_LIN)
#undef EXT_LIN
  hipLaunchKernelGGL(k_ext_schur, dim3(h->nchunk), dim3(256), ext_schur_lds(d), s, d, h->st, h->Q, h->Vg, h->mk,
                     h->cid, h->part);
  hipLaunchKernelGGL(k_ext_pack1, dim3(1), dim3(256), 0, s, d, h->st, h->nchunk, h->part, h->Vg, h->rank, p1);
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

// solve the summed system p1, step cameras and this rank's points, (cost, |dX|^2, |X|^2) of
// the trial into p3
static int ext_dist_step(acs_sba_ext_dist* h, const double* p1, double* p3) {
  acs_ctx* ctx = h->ctx;
  hipStream_t s = ctx->stream;
  const ExtDims& d = h->d;
  const int NC = 6 * d.C, nE = NC * NC + 3 * NC;
  const int NP = ((NC + 15) / 16) * 16;
  const size_t lds_solve = sizeof(double) * ((size_t)NP * (NP + 1) + NP + 512 + 256);
  hipLaunchKernelGGL(k_ext_solve, dim3(1), dim3(256), lds_solve, s, d, h->st, 1, p1, h->Vg, 0, p1 + nE, h->R, h->dc,
                     h->Sg, h->bad);
  hipLaunchKernelGGL(k_ext_back, dim3(acs_grid(d.n, 256)), dim3(256), 0, s, d, h->st, h->Q, h->Vg, h->mk, h->cid,
                     h->dc, h->dpts, h->normp);
  hipLaunchKernelGGL(k_ext_cam, dim3(1), dim3(64), 0, s, d, h->st, h->dc, h->dcams, h->camnorm);
#define EXT_COST1(g) ext_dist_cost<g>(h, s, 1)
  EXT_G_SWITCH(d.G, EXT_COST1)
#undef EXT_COST1
  hipLaunchKernelGGL(k_ext_pack3, dim3(1), dim3(256), 0, s, d, h->st, 1, h->Fp, h->normp, p3);
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

extern "C" {

// payload [p1 | p3] of the starting state: its system and its cost
int acs_sba_ext_dist_init(acs_sba_ext_dist* h, double* payload) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  hipStream_t s = h->ctx->stream;
  const int NC = 6 * h->d.C, n1 = NC * NC + 3 * NC + h->R;
#define EXT_COST0(g) ext_dist_cost<g>(h, s, 0)
  EXT_G_SWITCH(h->d.G, EXT_COST0)
#undef EXT_COST0
  hipLaunchKernelGGL(k_ext_pack3, dim3(1), dim3(256), 0, s, h->d, h->st, 0, h->Fp, h->normp, payload + n1);
  ACS_HIP(h->ctx, hipGetLastError());
  return ext_dist_system(h, payload);
}

// One round: decide on the pending trial (in: all-reduced payload of the previous round),
// step from its system, and the next system (speculatively at the trial state) with the
// trial's cost into out - one all-reduce per LM step, the status polled a round late.
int acs_sba_ext_dist_round(acs_sba_ext_dist* h, const double* in, double* out) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  acs_ctx* ctx = h->ctx;
  ACS_CHECK(ctx, in && out && in != out, "sba_ext_dist_round: in and out must be distinct buffers");
  hipStream_t s = ctx->stream;
  const int NC = 6 * h->d.C, n1 = NC * NC + 3 * NC + h->R;
  int rc;
  hipLaunchKernelGGL(k_ext_decide, dim3(1), dim3(64), 0, s, h->d, h->st, h->o, in + n1, (const double*)h->camnorm);
  if ((rc = ext_dist_step(h, in, out + n1))) return rc;
  hipLaunchKernelGGL(k_ext_spec, dim3(1), dim3(64), 0, s, h->st, 1);
  if ((rc = ext_dist_system(h, out))) return rc;
  hipLaunchKernelGGL(k_ext_spec, dim3(1), dim3(64), 0, s, h->st, 0);
  ACS_HIP(ctx, hipGetLastError());
  const int slot = (int)(h->rounds % EXT_DIST_RING);
  ACS_HIP(ctx, hipMemcpyAsync(h->snap + slot, &h->st->status, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipEventRecord(h->snap_ev[slot], s));
  h->rounds++;
  return ACS_OK;
}

// LM status after round r (waits for that round only)
int acs_sba_ext_dist_poll(acs_sba_ext_dist* h, int64_t round, int32_t* status) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  ACS_CHECK(h ? h->ctx : nullptr, h && status && round >= 0 && round < h->rounds && round >= h->rounds - EXT_DIST_RING,
            "sba_ext_dist_poll: round %lld not among the last %d enqueued", (long long)round, EXT_DIST_RING);
  const int slot = (int)(round % EXT_DIST_RING);
  ACS_HIP(h->ctx, hipEventSynchronize(h->snap_ev[slot]));
  *status = h->snap[slot];
  return ACS_OK;
}

int acs_sba_ext_dist_result(acs_sba_ext_dist* h, double* cams, double* pts, acs_sba_ext_report* report,
                            uint32_t flags) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  acs_ctx* ctx = h->ctx;
  hipStream_t s = ctx->stream;
  const ExtDims& d = h->d;
  ExtState hs;
  ACS_HIP(ctx, hipMemcpyAsync(&hs, h->st, sizeof(hs), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipStreamSynchronize(s));
  const hipMemcpyKind kout = (flags & ACS_DEVICE_PTRS) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  if (cams)
    ACS_HIP(ctx, hipMemcpyAsync(cams, h->dcams + hs.cur * d.C * ACS_CAM_STRIDE, sizeof(double) * ACS_CAM_STRIDE * d.C,
                                kout, s));
  if (pts) ACS_HIP(ctx, hipMemcpyAsync(pts, h->dpts + (size_t)hs.cur * d.n * 3, sizeof(double) * 3 * d.n, kout, s));
  int nbad = 0;
  ACS_HIP(ctx, hipMemcpyAsync(&nbad, h->bad, sizeof(int), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipStreamSynchronize(s));
  if (report) {
    report->status = hs.status == 0 ? ACS_STATUS_MAXITER : hs.status;
    report->iters = hs.iters;
    report->n_accepted = hs.nacc;
    report->n_bad_pivots = nbad;
    report->cost_before = hs.F0;
    report->cost_after = hs.F;
    report->grad_max = hs.gmax;
    report->lambda_final = hs.lam;
  }
  return ACS_OK;
}

}  // extern "C"
