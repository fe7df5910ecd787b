// fte.hip — Full Trajectory Estimation solve on gfx950.
//
// Replaces the Pyomo model + IPOPT solve of src/core/fte.py:176-555. The NLP's
// equalities (FK :323-328, measurement :435-462, backward-Euler / constant-acceleration
// integration :467-487) are eliminated exactly: unknowns are the pose parameters of the
// N frames plus two virtual leading frames (which carry the reference's free dx[1],
// ddx[1]) and the C shutter delays (tau_0 = 0, |tau| <= Ts; :304-318). The objective
// (:492-510) is  sum rho(w * (proj(FK(x_n) + shift) - meas)) + sum (Delta^3 x / Ts^2)^2 / Q.
// It is minimised by Levenberg-Marquardt with the spec in oracle/fte.py.
//
// One LM iteration = 7 launches, all device-resident (state in FteState):
//   k_fte_linearize  [N blocks]  FK + analytic FK Jacobian (fk.hpp), fisheye projection
//                                and its Jacobian, loss derivatives, per-frame local
//                                Jacobian rows (2CL x NZ) in LDS and the per-frame normal
//                                block J^T W J via v_mfma_f64_16x16x4f64 (the dense small
//                                GEMM of the path), gradient, cost
//   k_fte_assemble   [M blocks]  block-banded (bandwidth 3) normal matrix + tau border
//                                + exact model term (third differences)
//   k_fte_window     [W blocks]  per-window band Cholesky of the interior, fill columns
//                                Y = L^-1 [A_IS | A_Itau | b_I], window Schur block Y^T Y
//   k_fte_reduced    [1 block ]  block-tridiagonal separator system + tau border, solved
//   k_fte_backsolve  [W blocks]  interior back substitution, trial state
//   k_fte_cost       [N blocks]  exact objective at the trial state (per-frame partials)
//   k_fte_lm         [1 block ]  fixed-order reduction, accept/reject, lambda, stop tests
// Windows are a partition of frames into interiors separated by 3-frame separators; with
// bandwidth 3 the interiors decouple exactly (a SPIKE/substructuring direct solve).
#include "fk.hpp"
#include "wgla.hpp"

#define FTE_NZP 64
#define FTE_MAXC 16
#define FTE_CH 32  // observations per LDS chunk (64 Jacobian rows)

typedef double dbl4 __attribute__((ext_vector_type(4)));

struct FteDims {
  int N, M, P, L, C, Cg, NZ, im, W, NCOL, B;
  double Ts, la, lb, lc;
};

struct FteState {
  double F, F0, lam, gmax, Fmeas, Fmodel, dnorm, xnorm;
  int cur, status, iters, nacc, relin, bad, pad0, pad1;
};

struct FteOptsDev {
  int max_iters;
  double ftol, xtol, gtol;
};

// ---------------------------------------------------------------------------------------
// shared helpers
// ---------------------------------------------------------------------------------------
struct ShiftCoef {
  double own, prev, prev2;
};
__device__ __forceinline__ ShiftCoef shift_coef(int im, double tc, double Ts) {
  ShiftCoef s{0.0, 0.0, 0.0};
  if (im >= 1) {
    s.own += tc / Ts;
    s.prev -= tc / Ts;
  }
  if (im == 2) {
    const double q = tc * tc / (Ts * Ts);
    s.own += q;
    s.prev -= 2.0 * q;
    s.prev2 += q;
  }
  return s;
}

__device__ __forceinline__ double loss_curv(double e, const LossOut& l) {
  double c = l.d2;
  if (e != 0.0) c = fmax(c, l.d1 / e);
  return fmax(c, 0.0);
}

// fixed-order block sum (blockDim.x must be a power of two <= 256)
__device__ double block_sum(double v, double* s_red) {
  const int t = threadIdx.x;
  s_red[t] = v;
  __syncthreads();
  for (int h = blockDim.x / 2; h > 0; h >>= 1) {
    if (t < h) s_red[t] += s_red[t + h];
    __syncthreads();
  }
  const double r = s_red[0];
  __syncthreads();
  return r;
}
__device__ double block_max(double v, double* s_red) {
  const int t = threadIdx.x;
  s_red[t] = v;
  __syncthreads();
  for (int h = blockDim.x / 2; h > 0; h >>= 1) {
    if (t < h) s_red[t] = fmax(s_red[t], s_red[t + h]);
    __syncthreads();
  }
  const double r = s_red[0];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------------------
// 1. per-frame linearisation
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fte_linearize(FteDims d, const int* __restrict__ I,
                                                       const double* __restrict__ Rl,
                                                       const double* __restrict__ cams,
                                                       const double* __restrict__ meas,
                                                       const double* __restrict__ wts,
                                                       const double* __restrict__ Xbuf,
                                                       const double* __restrict__ taubuf,
                                                       const FteState* __restrict__ st, int force,
                                                       double* __restrict__ Hloc, double* __restrict__ gloc,
                                                       double* __restrict__ Floc) {
  if (!force && (st->status != 0 || !st->relin)) return;
  const int k = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int P = d.P, C = d.C, L = d.L;
  const int cur = force ? 0 : st->cur;
  const double* X = Xbuf + (size_t)cur * d.M * P;
  const double* tau = taubuf + cur * C;
  __shared__ FkShared fk;
  __shared__ double s_cam[FTE_MAXC * ACS_CAM_STRIDE];
  __shared__ double s_J[2 * FTE_CH][FTE_NZP + 1];
  __shared__ double s_sq[2 * FTE_CH], s_gs[2 * FTE_CH];
  __shared__ double s_jp[FTE_CH][6];
  __shared__ int s_node[FTE_CH], s_cid[FTE_CH], s_ok[FTE_CH];
  __shared__ double s_dx[3], s_ddx[3], s_tau[FTE_MAXC];
  __shared__ double s_red[256];
  const SkelView s = skel_view(I, Rl);
  const int f = k + 2;
  for (int i = tid; i < C * ACS_CAM_STRIDE; i += blockDim.x) s_cam[i] = cams[i];
  if (tid < 3) {
    const double x0 = X[f * P + tid], x1 = X[(f - 1) * P + tid], x2 = X[(f - 2) * P + tid];
    s_dx[tid] = (x0 - x1) / d.Ts;
    s_ddx[tid] = (x0 - 2.0 * x1 + x2) / (d.Ts * d.Ts);
  }
  if (tid < C) s_tau[tid] = d.Cg ? tau[tid] : 0.0;
  fk_frame(s, X + f * P, fk, tid, blockDim.x);
  __syncthreads();

  // tiles of the symmetric 64x64 product: upper triangle, 10 tiles over 4 waves
  const int tI[10] = {0, 0, 0, 0, 1, 1, 1, 2, 2, 3};
  const int tJ[10] = {0, 1, 2, 3, 1, 2, 3, 2, 3, 3};
  dbl4 acc[3];
  for (int q = 0; q < 3; ++q) acc[q] = dbl4{0.0, 0.0, 0.0, 0.0};
  double gacc = 0.0, rho = 0.0;
  const int nobs = C * L;
  for (int ch = 0; ch < nobs; ch += FTE_CH) {
    if (tid < FTE_CH) {
      const int o = ch + tid;
      s_ok[tid] = 0;
      s_sq[2 * tid] = s_sq[2 * tid + 1] = 0.0;
      s_gs[2 * tid] = s_gs[2 * tid + 1] = 0.0;
      if (o < nobs) {
        const int c = o / L, l = o - (o / L) * L;
        const int node = s.outn[l];
        const double tc = s_tau[c];
        double sh[3];
        for (int i = 0; i < 3; ++i) {
          sh[i] = 0.0;
          if (d.im >= 1) sh[i] += s_dx[i] * tc;
          if (d.im == 2) sh[i] += s_ddx[i] * (tc * tc);
        }
        ProjOut po;
        fisheye_project<true, true>(s_cam + c * ACS_CAM_STRIDE, fk.pos[node][0] + sh[0], fk.pos[node][1] + sh[1],
                                    fk.pos[node][2] + sh[2], po);
        const size_t mi = ((size_t)k * C + c) * L + l;
        const double wt = wts[mi];
        const double mu = wt != 0.0 ? meas[2 * mi] : 0.0, mv = wt != 0.0 ? meas[2 * mi + 1] : 0.0;
        const double eu = wt * (po.u - mu), ev = wt * (po.v - mv);
        const LossOut lu = redescending(eu, d.la, d.lb, d.lc);
        const LossOut lv = redescending(ev, d.la, d.lb, d.lc);
        rho += lu.f + lv.f;
        s_sq[2 * tid] = sqrt(loss_curv(eu, lu));
        s_sq[2 * tid + 1] = sqrt(loss_curv(ev, lv));
        s_gs[2 * tid] = lu.d1;
        s_gs[2 * tid + 1] = lv.d1;
        for (int i = 0; i < 6; ++i) s_jp[tid][i] = wt * po.J[i];
        s_node[tid] = node;
        s_cid[tid] = c;
        s_ok[tid] = (wt != 0.0);
      }
    }
    __syncthreads();
    for (int idx = tid; idx < FTE_CH * FTE_NZP; idx += blockDim.x) {
      const int t = idx / FTE_NZP, q = idx - t * FTE_NZP;
      double v0 = 0.0, v1 = 0.0;
      if (s_ok[t] && q < d.NZ) {
        const int c = s_cid[t];
        const ShiftCoef sc = shift_coef(d.im, s_tau[c], d.Ts);
        double dp[3] = {0.0, 0.0, 0.0};
        if (q < P) {
          fk_dpos(s, fk, s_node[t], q, dp);
          if (q < 3) dp[q] += sc.own;
        } else if (q < P + 3) {
          dp[q - P] = sc.prev;
        } else if (q < P + 6) {
          dp[q - P - 3] = sc.prev2;
        } else {
          const int cc = q - P - 6;
          if (cc == c && c > 0) {
            for (int i = 0; i < 3; ++i) dp[i] = s_dx[i] + (d.im == 2 ? 2.0 * s_tau[c] * s_ddx[i] : 0.0);
          }
        }
        v0 = s_jp[t][0] * dp[0] + s_jp[t][1] * dp[1] + s_jp[t][2] * dp[2];
        v1 = s_jp[t][3] * dp[0] + s_jp[t][4] * dp[1] + s_jp[t][5] * dp[2];
      }
      s_J[2 * t][q] = v0;
      s_J[2 * t + 1][q] = v1;
    }
    __syncthreads();
    // gradient (one column per thread) and normal blocks (MFMA f64 16x16x4)
    if (tid < FTE_NZP) {
      for (int r = 0; r < 2 * FTE_CH; ++r) gacc = fma(s_gs[r], s_J[r][tid], gacc);
    }
    for (int q = 0; q < 3; ++q) {
      const int tile = wave + 4 * q;
      if (tile >= 10) break;
      const int ci = tI[tile] * 16 + (lane & 15), cj = tJ[tile] * 16 + (lane & 15);
      for (int r0 = 0; r0 < 2 * FTE_CH; r0 += 4) {
        const int r = r0 + (lane >> 4);
        const double sq = s_sq[r];
        const double a = s_J[r][ci] * sq, b = s_J[r][cj] * sq;
        acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[q], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  double* H = Hloc + (size_t)k * FTE_NZP * FTE_NZP;
  for (int q = 0; q < 3; ++q) {
    const int tile = wave + 4 * q;
    if (tile >= 10) break;
    for (int rg = 0; rg < 4; ++rg) {
      const int row = tI[tile] * 16 + (lane >> 4) + 4 * rg, col = tJ[tile] * 16 + (lane & 15);
      H[row * FTE_NZP + col] = acc[q][rg];
      H[col * FTE_NZP + row] = acc[q][rg];
    }
  }
  if (tid < FTE_NZP) gloc[(size_t)k * FTE_NZP + tid] = gacc;
  const double tot = block_sum(rho, s_red);
  if (tid == 0) Floc[k] = tot;
}

// ---------------------------------------------------------------------------------------
// 2. assembly of the banded normal matrix (row f: blocks (f, f-d), d = 0..3)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fte_assemble(FteDims d, const double* __restrict__ Xbuf,
                                                      const double* __restrict__ qinv,
                                                      const FteState* __restrict__ st, int force,
                                                      const double* __restrict__ Hloc,
                                                      const double* __restrict__ gloc, double* __restrict__ Ab,
                                                      double* __restrict__ gb, double* __restrict__ Bt,
                                                      double* __restrict__ gmaxp) {
  if (!force && (st->status != 0 || !st->relin)) return;
  const int f = blockIdx.x;
  const int tid = threadIdx.x, nth = blockDim.x;
  const int P = d.P, Cg = d.Cg, N = d.N;
  const int cur = force ? 0 : st->cur;
  const double* X = Xbuf + (size_t)cur * d.M * P;
  double* A = Ab + (size_t)f * 4 * P * P;
  double* g = gb + (size_t)f * P;
  double* B = Bt + (size_t)f * P * Cg;
  __shared__ double s_red[256];
  for (int i = tid; i < 4 * P * P; i += nth) A[i] = 0.0;
  for (int i = tid; i < P * Cg; i += nth) B[i] = 0.0;
  for (int i = tid; i < P; i += nth) g[i] = 0.0;
  __syncthreads();
  const int kown = f - 2, kprev = f - 1, kprev2 = f;
  if (kown >= 0 && kown < N) {
    const double* H = Hloc + (size_t)kown * FTE_NZP * FTE_NZP;
    for (int i = tid; i < P * P; i += nth) {
      const int r = i / P, c = i % P;
      A[r * P + c] += H[r * FTE_NZP + c];
    }
    for (int i = tid; i < P * 3; i += nth) {
      const int r = i / 3, c = i % 3;
      A[1 * P * P + r * P + c] += H[r * FTE_NZP + P + c];
      A[2 * P * P + r * P + c] += H[r * FTE_NZP + P + 3 + c];
    }
    for (int i = tid; i < P * Cg; i += nth) {
      const int r = i / Cg, c = i % Cg;
      B[r * Cg + c] += H[r * FTE_NZP + P + 6 + c];
    }
    for (int i = tid; i < P; i += nth) g[i] += gloc[(size_t)kown * FTE_NZP + i];
  }
  __syncthreads();
  if (kprev >= 0 && kprev < N) {
    const double* H = Hloc + (size_t)kprev * FTE_NZP * FTE_NZP;
    for (int i = tid; i < 9; i += nth) {
      const int r = i / 3, c = i % 3;
      A[r * P + c] += H[(P + r) * FTE_NZP + P + c];
      A[1 * P * P + r * P + c] += H[(P + r) * FTE_NZP + P + 3 + c];
    }
    for (int i = tid; i < 3 * Cg; i += nth) {
      const int r = i / Cg, c = i % Cg;
      B[r * Cg + c] += H[(P + r) * FTE_NZP + P + 6 + c];
    }
    for (int i = tid; i < 3; i += nth) g[i] += gloc[(size_t)kprev * FTE_NZP + P + i];
  }
  __syncthreads();
  if (kprev2 >= 0 && kprev2 < N) {
    const double* H = Hloc + (size_t)kprev2 * FTE_NZP * FTE_NZP;
    for (int i = tid; i < 9; i += nth) {
      const int r = i / 3, c = i % 3;
      A[r * P + c] += H[(P + 3 + r) * FTE_NZP + P + 3 + c];
    }
    for (int i = tid; i < 3 * Cg; i += nth) {
      const int r = i / Cg, c = i % Cg;
      B[r * Cg + c] += H[(P + 3 + r) * FTE_NZP + P + 6 + c];
    }
    for (int i = tid; i < 3; i += nth) g[i] += gloc[(size_t)kprev2 * FTE_NZP + P + 3 + i];
  }
  __syncthreads();
  // model term: stencils m in [3, M-1], s_m = (X_m - 3X_{m-1} + 3X_{m-2} - X_{m-3}) / Ts^2
  const double cf[4] = {1.0, -3.0, 3.0, -1.0};
  const double its2 = 1.0 / (d.Ts * d.Ts);
  for (int p = tid; p < P; p += nth) {
    double gm = 0.0;
    double hd[4] = {0.0, 0.0, 0.0, 0.0};
    for (int i = 0; i < 4; ++i) {
      const int m = f + i;
      if (m < 3 || m > d.M - 1) continue;
      const double sm = (X[m * P + p] - 3.0 * X[(m - 1) * P + p] + 3.0 * X[(m - 2) * P + p] - X[(m - 3) * P + p]) * its2;
      gm += 2.0 * qinv[p] * cf[i] * its2 * sm;
      for (int dd = 0; dd < 4 && i + dd < 4; ++dd) hd[dd] += 2.0 * qinv[p] * cf[i] * cf[i + dd] * its2 * its2;
    }
    g[p] += gm;
    for (int dd = 0; dd < 4; ++dd) A[dd * P * P + p * P + p] += hd[dd];
  }
  __syncthreads();
  double mx = 0.0;
  for (int i = tid; i < P; i += nth) mx = fmax(mx, fabs(g[i]));
  mx = block_max(mx, s_red);
  if (tid == 0) gmaxp[f] = mx;
}

// ---------------------------------------------------------------------------------------
// 3. window factorisation
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fte_window(FteDims d, const int* __restrict__ wstart,
                                                    const int* __restrict__ wlen, const FteState* __restrict__ st,
                                                    int force, double lam_force, const double* __restrict__ Ab,
                                                    const double* __restrict__ gb, const double* __restrict__ Bt,
                                                    double* __restrict__ Lb, double* __restrict__ Y,
                                                    double* __restrict__ Sw, int* __restrict__ bad) {
  if (!force && st->status != 0) return;
  const int w = blockIdx.x;
  const int tid = threadIdx.x, nth = blockDim.x;
  const int P = d.P, PP = P * P, NCOL = d.NCOL, Cg = d.Cg;
  const int s0 = wstart[w], n = wlen[w];
  const bool hasL = w > 0, hasR = w < d.W - 1;
  const int cL = 0, cR = 3 * P, cT = 6 * P, cb = 6 * P + Cg;
  const double lam = force ? lam_force : st->lam;
  for (int j = 0; j < n; ++j) {
    const int f = s0 + j;
    double* Lrow = Lb + (size_t)f * 4 * PP;
    const double* Arow = Ab + (size_t)f * 4 * PP;
    for (int i = tid; i < 4 * PP; i += nth) {
      const int blk = i / PP;
      double v = (blk == 0 || f - blk >= s0) ? Arow[i] : 0.0;
      if (blk == 0) {
        const int r = (i % PP) / P, c = i % P;
        if (r == c) v += lam * fmax(v, 1e-12);
      }
      Lrow[i] = v;
    }
    __syncthreads();
    for (int dd = 3; dd >= 1; --dd) {
      if (f - dd < s0) continue;
      for (int e = dd + 1; e <= 3; ++e) {
        if (f - e < s0) continue;
        wg_gemm<false, true>(Lrow + dd * PP, P, Lrow + e * PP, P, Lb + (size_t)(f - dd) * 4 * PP + (e - dd) * PP, P,
                             P, P, P, -1.0);
      }
      wg_trsm_rlt(Lrow + dd * PP, P, Lb + (size_t)(f - dd) * 4 * PP, P, P, P);
    }
    for (int dd = 1; dd <= 3; ++dd) {
      if (f - dd < s0) continue;
      wg_gemm<false, true>(Lrow, P, Lrow + dd * PP, P, Lrow + dd * PP, P, P, P, P, -1.0);
    }
    wg_chol(Lrow, P, P, bad);
    // E row
    double* Yrow = Y + (size_t)f * P * NCOL;
    for (int i = tid; i < P * NCOL; i += nth) {
      const int r = i / NCOL, c = i % NCOL;
      double v = 0.0;
      if (c < cR) {
        if (hasL) {
          const int sfi = c / P, sc = c % P;  // separator frame s0-3+sfi
          const int sf = s0 - 3 + sfi, dd = f - sf;
          if (dd >= 1 && dd <= 3) v = Arow[dd * PP + r * P + sc];
        }
      } else if (c < cT) {
        if (hasR) {
          const int sfi = (c - cR) / P, sc = (c - cR) % P;
          const int sf = s0 + n + sfi, dd = sf - f;
          if (dd >= 1 && dd <= 3) v = Ab[(size_t)sf * 4 * PP + dd * PP + sc * P + r];
        }
      } else if (c < cb) {
        v = Bt[(size_t)f * P * Cg + r * Cg + (c - cT)];
      } else {
        v = -gb[(size_t)f * P + r];
      }
      Yrow[i] = v;
    }
    __syncthreads();
    for (int dd = 1; dd <= 3; ++dd) {
      if (f - dd < s0) continue;
      wg_gemm<false, false>(Yrow, NCOL, Lrow + dd * PP, P, Y + (size_t)(f - dd) * P * NCOL, NCOL, P, NCOL, P, -1.0);
    }
    wg_trsm_lln(Yrow, NCOL, Lrow, P, P, NCOL);
  }
  // Schur block of this window: Sw = Y^T Y over its interior rows
  double* S = Sw + (size_t)w * NCOL * NCOL;
  const double* Yw = Y + (size_t)s0 * P * NCOL;
  const int rows = n * P;
  for (int idx = tid; idx < NCOL * NCOL; idx += nth) {
    const int i = idx / NCOL, j = idx % NCOL;
    if (j < i) continue;
    double sacc = 0.0;
    // right-separator columns are zero above the last 3 interior frames
    int r0 = 0;
    if ((i >= cR && i < cT) || (j >= cR && j < cT)) r0 = max(0, (n - 3) * P);
    for (int r = r0; r < rows; ++r) sacc = fma(Yw[(size_t)r * NCOL + i], Yw[(size_t)r * NCOL + j], sacc);
    S[i * NCOL + j] = sacc;
    S[j * NCOL + i] = sacc;
  }
}

// ---------------------------------------------------------------------------------------
// 4. reduced (separator + tau) system
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fte_reduced(FteDims d, const int* __restrict__ wstart,
                                                     const int* __restrict__ wlen, FteState* __restrict__ st,
                                                     int force, double lam_force, const double* __restrict__ Ab,
                                                     const double* __restrict__ gb, const double* __restrict__ Bt,
                                                     const double* __restrict__ Hloc,
                                                     const double* __restrict__ gloc,
                                                     const double* __restrict__ Sw,
                                                     const double* __restrict__ gmaxp, double* __restrict__ RA,
                                                     double* __restrict__ RL, double* __restrict__ LT,
                                                     double* __restrict__ ry, double* __restrict__ Rt,
                                                     double* __restrict__ rt, double* __restrict__ dS,
                                                     double* __restrict__ dtau, int* __restrict__ bad) {
  if (!force && st->status != 0) return;
  const int tid = threadIdx.x, nth = blockDim.x;
  const int P = d.P, PP = P * P, NCOL = d.NCOL, Cg = d.Cg, B = d.B, J = d.W - 1;
  const int cL = 0, cR = 3 * P, cT = 6 * P, cb = 6 * P + Cg;
  const double lam = force ? lam_force : st->lam;
  __shared__ double s_red[256];
  // gradient max (frames + tau border)
  {
    double mx = 0.0;
    for (int f = tid; f < d.M; f += nth) mx = fmax(mx, gmaxp[f]);
    for (int c = 1 + tid; c < Cg; c += nth) {
      double gt = 0.0;
      for (int k = 0; k < d.N; ++k) gt += gloc[(size_t)k * FTE_NZP + P + 6 + c];
      mx = fmax(mx, fabs(gt));
    }
    mx = block_max(mx, s_red);
    if (tid == 0 && !force) st->gmax = mx;
  }
  // tau block: Rt = sum_k Hloc_tt - sum_w Sw_tt (+ damping, tau_0 pinned); rt = -g_t - sum_w Sw_t,rhs
  for (int i = tid; i < Cg * Cg; i += nth) {
    const int r = i / Cg, c = i % Cg;
    double v = 0.0;
    for (int k = 0; k < d.N; ++k) v += Hloc[(size_t)k * FTE_NZP * FTE_NZP + (P + 6 + r) * FTE_NZP + P + 6 + c];
    if (r == c) v += lam * fmax(v, 1e-12);
    for (int w = 0; w < d.W; ++w) v -= Sw[(size_t)w * NCOL * NCOL + (cT + r) * NCOL + cT + c];
    if (r == 0 || c == 0) v = (r == c) ? 1.0 : 0.0;
    Rt[i] = v;
  }
  for (int r = tid; r < Cg; r += nth) {
    double v = 0.0;
    for (int k = 0; k < d.N; ++k) v += gloc[(size_t)k * FTE_NZP + P + 6 + r];
    v = -v;
    for (int w = 0; w < d.W; ++w) v -= Sw[(size_t)w * NCOL * NCOL + (cT + r) * NCOL + cb];
    rt[r] = (r == 0) ? 0.0 : v;
  }
  __syncthreads();
  // assemble separator blocks
  for (int j = 0; j < J; ++j) {
    const int e = wstart[j] + wlen[j];
    double* A = RA + (size_t)j * B * B;
    const double* SL = Sw + (size_t)j * NCOL * NCOL;        // window j: S_j is its right separator
    const double* SR = Sw + (size_t)(j + 1) * NCOL * NCOL;  // window j+1: S_j is its left separator
    for (int i = tid; i < B * B; i += nth) {
      const int r = i / B, c = i % B;
      const int fa = r / P, pa = r % P, fb = c / P, pb = c % P;
      double v;
      if (fa >= fb)
        v = Ab[(size_t)(e + fa) * 4 * PP + (fa - fb) * PP + pa * P + pb];
      else
        v = Ab[(size_t)(e + fb) * 4 * PP + (fb - fa) * PP + pb * P + pa];
      if (r == c) v += lam * fmax(v, 1e-12);
      v -= SL[(cR + r) * NCOL + cR + c];
      v -= SR[(cL + r) * NCOL + cL + c];
      A[i] = v;
    }
    if (j >= 1) {
      double* Lo = RL + (size_t)j * B * B;  // block (S_j, S_{j-1}) = -(window j) right x left
      for (int i = tid; i < B * B; i += nth) {
        const int r = i / B, c = i % B;
        Lo[i] = -SL[(cR + r) * NCOL + cL + c];
      }
    }
    double* T = LT + (size_t)j * Cg * B;  // border, stored transposed (Cg x B)
    for (int i = tid; i < Cg * B; i += nth) {
      const int c = i / B, r = i % B;
      const int fa = r / P, pa = r % P;
      double v = Bt[(size_t)(e + fa) * P * Cg + pa * Cg + c];
      v -= SL[(cR + r) * NCOL + cT + c];
      v -= SR[(cL + r) * NCOL + cT + c];
      T[i] = (c == 0) ? 0.0 : v;
    }
    for (int r = tid; r < B; r += nth) {
      const int fa = r / P, pa = r % P;
      double v = -gb[(size_t)(e + fa) * P + pa];
      v -= SL[(cR + r) * NCOL + cb];
      v -= SR[(cL + r) * NCOL + cb];
      ry[(size_t)j * B + r] = v;
    }
    __syncthreads();
  }
  // block Cholesky of the arrow matrix, forward substitution
  for (int j = 0; j < J; ++j) {
    double* A = RA + (size_t)j * B * B;
    double* T = LT + (size_t)j * Cg * B;
    double* y = ry + (size_t)j * B;
    if (j >= 1) {
      const double* Lo = RL + (size_t)j * B * B;
      wg_gemm<false, true>(A, B, Lo, B, Lo, B, B, B, B, -1.0);
      if (Cg) wg_gemm<false, true>(T, B, LT + (size_t)(j - 1) * Cg * B, B, Lo, B, Cg, B, B, -1.0);
      wg_gemm<false, false>(y, 1, Lo, B, ry + (size_t)(j - 1) * B, 1, B, 1, B, -1.0);
    }
    wg_chol(A, B, B, bad);
    wg_trsm_lln(y, 1, A, B, B, 1);
    if (Cg) {
      wg_trsm_rlt(T, B, A, B, Cg, B);
      wg_gemm<false, true>(Rt, Cg, T, B, T, B, Cg, Cg, B, -1.0);
      wg_gemm<false, false>(rt, 1, T, B, y, 1, Cg, 1, B, -1.0);
    }
    if (j + 1 < J) {
      // next sub-diagonal block must exist: assembled above; transform to L_{j+1,j}
      wg_trsm_rlt(RL + (size_t)(j + 1) * B * B, B, A, B, B, B);
    }
  }
  if (Cg) {
    // keep the pinned tau_0 row exact
    for (int i = tid; i < Cg; i += nth) {
      if (i != 0) {
        Rt[i] = 0.0;
        Rt[i * Cg] = 0.0;
      }
    }
    if (tid == 0) {
      Rt[0] = 1.0;
      rt[0] = 0.0;
    }
    __syncthreads();
    wg_chol(Rt, Cg, Cg, bad);
    wg_trsm_lln(rt, 1, Rt, Cg, Cg, 1);
    wg_trsm_llt(rt, 1, Rt, Cg, Cg, 1);
    for (int i = tid; i < Cg; i += nth) dtau[i] = rt[i];
    __syncthreads();
  }
  for (int j = J - 1; j >= 0; --j) {
    double* y = ry + (size_t)j * B;
    if (j + 1 < J) wg_gemm<true, false>(y, 1, RL + (size_t)(j + 1) * B * B, B, ry + (size_t)(j + 1) * B, 1, B, 1, B, -1.0);
    if (Cg) wg_gemm<true, false>(y, 1, LT + (size_t)j * Cg * B, B, rt, 1, B, 1, Cg, -1.0);
    wg_trsm_llt(y, 1, RA + (size_t)j * B * B, B, B, 1);
    for (int i = tid; i < B; i += nth) dS[(size_t)j * B + i] = y[i];
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// 5. back substitution + trial state
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fte_backsolve(FteDims d, const int* __restrict__ wstart,
                                                       const int* __restrict__ wlen, const FteState* __restrict__ st,
                                                       int force, const double* __restrict__ Lb,
                                                       const double* __restrict__ Y, const double* __restrict__ dS,
                                                       const double* __restrict__ dtau, double* __restrict__ delta,
                                                       double* __restrict__ Xbuf, double* __restrict__ taubuf,
                                                       double* __restrict__ normp) {
  if (!force && st->status != 0) return;
  const int w = blockIdx.x;
  const int tid = threadIdx.x, nth = blockDim.x;
  const int P = d.P, PP = P * P, NCOL = d.NCOL, Cg = d.Cg, B = d.B;
  const int s0 = wstart[w], n = wlen[w];
  const bool hasL = w > 0, hasR = w < d.W - 1;
  const int cL = 0, cR = 3 * P, cT = 6 * P, cb = 6 * P + Cg;
  __shared__ double s_red[256];
  // r = y_b - Y_L dS_{w-1} - Y_R dS_w - Y_T dtau
  for (int i = tid; i < n * P; i += nth) {
    const double* Yr = Y + ((size_t)s0 * P + i) * NCOL;
    double v = Yr[cb];
    if (hasL)
      for (int c = 0; c < B; ++c) v -= Yr[cL + c] * dS[(size_t)(w - 1) * B + c];
    if (hasR)
      for (int c = 0; c < B; ++c) v -= Yr[cR + c] * dS[(size_t)w * B + c];
    for (int c = 0; c < Cg; ++c) v -= Yr[cT + c] * dtau[c];
    delta[(size_t)s0 * P + i] = v;
  }
  __syncthreads();
  for (int j = n - 1; j >= 0; --j) {
    const int f = s0 + j;
    double* df = delta + (size_t)f * P;
    for (int dd = 1; dd <= 3; ++dd) {
      if (j + dd >= n) continue;
      // df -= L_{f+dd, f}^T delta_{f+dd}
      wg_gemm<true, false>(df, 1, Lb + (size_t)(f + dd) * 4 * PP + dd * PP, P, delta + (size_t)(f + dd) * P, 1, P, 1,
                           P, -1.0);
    }
    wg_trsm_llt(df, 1, Lb + (size_t)f * 4 * PP, P, P, 1);
  }
  if (hasR) {
    for (int i = tid; i < B; i += nth) delta[(size_t)(s0 + n) * P + i] = dS[(size_t)w * B + i];
  }
  __syncthreads();
  const int cur = force ? 0 : st->cur;
  const double* X = Xbuf + (size_t)cur * d.M * P;
  double* Xn = Xbuf + (size_t)(cur ^ 1) * d.M * P;
  const int span = (n + (hasR ? 3 : 0)) * P;
  double dn = 0.0, xn = 0.0;
  for (int i = tid; i < span; i += nth) {
    const size_t o = (size_t)s0 * P + i;
    const double x = X[o], dv = delta[o];
    Xn[o] = x + dv;
    dn += dv * dv;
    xn += x * x;
  }
  if (w == 0 && Cg) {
    const double* tau = taubuf + cur * d.C;
    double* taun = taubuf + (cur ^ 1) * d.C;
    for (int c = tid; c < d.C; c += nth) {
      const double dv = (c == 0) ? 0.0 : dtau[c];
      double v = (c == 0) ? 0.0 : tau[c] + dv;
      v = fmin(fmax(v, -d.Ts), d.Ts);
      taun[c] = v;
      dn += dv * dv;
      xn += tau[c] * tau[c];
    }
  }
  dn = block_sum(dn, s_red);
  xn = block_sum(xn, s_red);
  if (tid == 0) {
    normp[2 * w] = dn;
    normp[2 * w + 1] = xn;
  }
}

// ---------------------------------------------------------------------------------------
// 6. exact objective at a state (per-frame partials)
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_fte_cost(FteDims d, const int* __restrict__ I, const double* __restrict__ Rl,
                                                 const double* __restrict__ cams, const double* __restrict__ meas,
                                                 const double* __restrict__ wts, const double* __restrict__ Xbuf,
                                                 const double* __restrict__ taubuf, const double* __restrict__ qinv,
                                                 const FteState* __restrict__ st, int which /*0 cur, 1 trial*/,
                                                 double* __restrict__ Fm, double* __restrict__ Fq) {
  if (which == 1 && st->status != 0) return;
  const int k = blockIdx.x;
  const int tid = threadIdx.x;
  const int P = d.P, C = d.C, L = d.L;
  const int buf = which == 1 ? (st->cur ^ 1) : st->cur;
  const double* X = Xbuf + (size_t)buf * d.M * P;
  const double* tau = taubuf + buf * C;
  __shared__ FkShared fk;
  __shared__ double s_red[64];
  __shared__ double s_dx[3], s_ddx[3];
  const SkelView s = skel_view(I, Rl);
  const int f = k + 2;
  if (tid < 3) {
    const double x0 = X[f * P + tid], x1 = X[(f - 1) * P + tid], x2 = X[(f - 2) * P + tid];
    s_dx[tid] = (x0 - x1) / d.Ts;
    s_ddx[tid] = (x0 - 2.0 * x1 + x2) / (d.Ts * d.Ts);
  }
  fk_frame(s, X + f * P, fk, tid, blockDim.x);
  __syncthreads();
  double rho = 0.0;
  for (int o = tid; o < C * L; o += blockDim.x) {
    const int c = o / L, l = o - (o / L) * L;
    const int node = s.outn[l];
    const double tc = d.Cg ? tau[c] : 0.0;
    double p[3];
    for (int i = 0; i < 3; ++i) {
      p[i] = fk.pos[node][i];
      if (d.im >= 1) p[i] += s_dx[i] * tc;
      if (d.im == 2) p[i] += s_ddx[i] * (tc * tc);
    }
    ProjOut po;
    fisheye_project<false, true>(cams + c * ACS_CAM_STRIDE, p[0], p[1], p[2], po);
    const size_t mi = ((size_t)k * C + c) * L + l;
    const double wt = wts[mi];
    const double mu = wt != 0.0 ? meas[2 * mi] : 0.0, mv = wt != 0.0 ? meas[2 * mi + 1] : 0.0;
    rho += redescending(wt * (po.u - mu), d.la, d.lb, d.lc).f + redescending(wt * (po.v - mv), d.la, d.lb, d.lc).f;
  }
  double q = 0.0;
  if (k >= 1) {
    const double its2 = 1.0 / (d.Ts * d.Ts);
    for (int p = tid; p < P; p += blockDim.x) {
      const double sm = (X[f * P + p] - 3.0 * X[(f - 1) * P + p] + 3.0 * X[(f - 2) * P + p] - X[(f - 3) * P + p]) * its2;
      q += qinv[p] * sm * sm;
    }
  }
  rho = block_sum(rho, s_red);
  q = block_sum(q, s_red);
  if (tid == 0) {
    Fm[k] = rho;
    Fq[k] = q;
  }
}

// ---------------------------------------------------------------------------------------
// 7. LM control
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_fte_lm(FteDims d, FteState* __restrict__ st, FteOptsDev o, int init,
                                                const double* __restrict__ Fm, const double* __restrict__ Fq,
                                                const double* __restrict__ normp) {
  __shared__ double s_red[256];
  const int tid = threadIdx.x;
  double a = 0.0, b = 0.0;
  for (int k = tid; k < d.N; k += blockDim.x) {
    a += Fm[k];
    b += Fq[k];
  }
  const double fm = block_sum(a, s_red), fq = block_sum(b, s_red);
  if (init) {
    if (tid == 0) {
      st->F = st->F0 = fm + fq;
      st->Fmeas = fm;
      st->Fmodel = fq;
    }
    return;
  }
  if (st->status != 0) return;
  double dn = 0.0, xn = 0.0;
  for (int w = tid; w < d.W; w += blockDim.x) {
    dn += normp[2 * w];
    xn += normp[2 * w + 1];
  }
  dn = block_sum(dn, s_red);
  xn = block_sum(xn, s_red);
  if (tid != 0) return;
  if (st->gmax <= o.gtol) {
    st->status = ACS_STATUS_GTOL;
    return;
  }
  const double Fn = fm + fq;
  st->iters += 1;
  st->dnorm = sqrt(dn);
  st->xnorm = sqrt(xn);
  const bool small = sqrt(dn) <= o.xtol * (o.xtol + sqrt(xn));
  if (Fn < st->F) {
    const bool fconv = (st->F - Fn) <= o.ftol * fabs(st->F);
    st->nacc += 1;
    st->F = Fn;
    st->Fmeas = fm;
    st->Fmodel = fq;
    st->cur ^= 1;
    st->lam = fmax(st->lam * 0.1, 1e-15);
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

// =======================================================================================
// host side
// =======================================================================================
struct FteBuffers {
  int* I;
  double *Rl, *cams, *meas, *w, *qinv, *X, *tau;
  double *Hloc, *gloc, *Floc, *Ab, *gb, *Bt, *gmaxp, *Lb, *Y, *Sw, *RA, *RL, *LT, *ry, *Rt, *rt, *dS, *dtau, *delta,
      *normp, *Fm, *Fq;
  int *wstart, *wlen, *bad;
  FteState* st;
};

static void fte_windows(int M, int wl, std::vector<int>& ws, std::vector<int>& wn) {
  if (wl < 3) wl = 3;
  int W = (M + 3) / (wl + 3);
  if (W < 1) W = 1;
  while (W > 1 && M - 3 * (W - 1) < 3 * W) --W;
  const int interior = M - 3 * (W - 1);
  ws.resize(W);
  wn.resize(W);
  int pos = 0;
  for (int w = 0; w < W; ++w) {
    const int n = interior / W + (w < interior % W ? 1 : 0);
    ws[w] = pos;
    wn[w] = n;
    pos += n + 3;
  }
}

struct FteSetup {
  FteDims d;
  FteBuffers b;
  std::vector<int> ws, wn;
};

static int fte_setup(acs_ctx* ctx, FteSetup& S, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                     int64_t n_reals, const double* cams, int32_t n_cams, const double* meas, const double* w,
                     int32_t N, int32_t sd, double Ts, const double* qinv, int32_t intermode, const double* X,
                     const double* tau, int window, double la, double lb, double lc, uint32_t flags) {
  int hdr[FK_HDR];
  if (flags & ACS_DEVICE_PTRS)
    ACS_HIP(ctx, hipMemcpy(hdr, skel_ints, sizeof(hdr), hipMemcpyDeviceToHost));
  else
    std::memcpy(hdr, skel_ints, sizeof(hdr));
  const int Jn = hdr[0], K = hdr[1], P = hdr[2], L = hdr[3];
  ACS_CHECK(ctx, Jn > 0 && Jn <= FK_MAXJ && K <= FK_MAXN && P >= 3 && P <= FK_MAXP && L >= 1 && L <= K,
            "fte: skeleton table out of range");
  ACS_CHECK(ctx, n_ints == FK_HDR + 9 * Jn + 4 * K + L + 4 * P + K * P && n_reals == 3 * K, "fte: blob sizes");
  ACS_CHECK(ctx, N >= 2 && n_cams >= 1 && n_cams <= FTE_MAXC && Ts > 0, "fte: N=%d C=%d Ts=%g", N, n_cams, Ts);
  ACS_CHECK(ctx, intermode >= 0 && intermode <= 2 && (sd ? intermode >= 1 : intermode == 0),
            "fte: shutter_delay=%d needs intermode %s (got %d), as src/core/fte.py:44-48", sd,
            sd ? "vel/acc" : "pos", intermode);
  FteDims& d = S.d;
  d.N = N;
  d.M = N + 2;
  d.P = P;
  d.L = L;
  d.C = n_cams;
  d.Cg = sd ? n_cams : 0;
  d.NZ = P + 6 + d.Cg;
  ACS_CHECK(ctx, d.NZ <= FTE_NZP, "fte: P + 6 + C = %d exceeds %d", d.NZ, FTE_NZP);
  d.im = intermode;
  d.Ts = Ts;
  d.la = la;
  d.lb = lb;
  d.lc = lc;
  d.B = 3 * P;
  d.NCOL = 6 * P + d.Cg + 1;
  fte_windows(d.M, window, S.ws, S.wn);
  d.W = (int)S.ws.size();
  const int M = d.M, W = d.W, NCOL = d.NCOL, B = d.B, Cg = d.Cg, C = d.C;
  FteBuffers& b = S.b;
  int rc;
  void* p;
  if ((rc = acs_stage_in(ctx, WS_FTE0, skel_ints, sizeof(int32_t) * n_ints, flags, &p))) return rc;
  b.I = (int*)p;
  if ((rc = acs_stage_in(ctx, WS_FTE1, skel_reals, sizeof(double) * n_reals, flags, &p))) return rc;
  b.Rl = (double*)p;
  if ((rc = acs_stage_in(ctx, WS_CAMS, cams, sizeof(double) * ACS_CAM_STRIDE * C, flags, &p))) return rc;
  b.cams = (double*)p;
  if ((rc = acs_stage_in(ctx, WS_FTE2, meas, sizeof(double) * (size_t)N * C * L * 2, flags, &p))) return rc;
  b.meas = (double*)p;
  if ((rc = acs_stage_in(ctx, WS_FTE3, w, sizeof(double) * (size_t)N * C * L, flags, &p))) return rc;
  b.w = (double*)p;
  if ((rc = acs_stage_in(ctx, WS_FTE4, qinv, sizeof(double) * P, flags, &p))) return rc;
  b.qinv = (double*)p;
  // one arena for everything else
  size_t off = 0;
  auto take = [&](size_t n) {
    size_t o = off;
    off += ((n * sizeof(double) + 255) / 256) * 256 / sizeof(double);
    return o;
  };
  const size_t oX = take((size_t)2 * M * P), oT = take(2 * C), oH = take((size_t)N * FTE_NZP * FTE_NZP),
               og = take((size_t)N * FTE_NZP), oF = take(N), oAb = take((size_t)M * 4 * P * P),
               ogb = take((size_t)M * P), oBt = take((size_t)M * P * (Cg ? Cg : 1)), ogm = take(M),
               oLb = take((size_t)M * 4 * P * P), oY = take((size_t)M * P * NCOL),
               oSw = take((size_t)W * NCOL * NCOL), oRA = take((size_t)(W > 1 ? W - 1 : 1) * B * B),
               oRL = take((size_t)(W > 1 ? W - 1 : 1) * B * B), oLT = take((size_t)(W > 1 ? W - 1 : 1) * (Cg ? Cg : 1) * B),
               ory = take((size_t)(W > 1 ? W - 1 : 1) * B), oRt = take((Cg ? Cg : 1) * (Cg ? Cg : 1)),
               ort = take(Cg ? Cg : 1), odS = take((size_t)(W > 1 ? W - 1 : 1) * B), odt = take(Cg ? Cg : 1),
               odl = take((size_t)M * P), onp = take(2 * W), oFm = take(N), oFq = take(N), ost = take(16),
               oint = take(2 * W + 8);
  double* arena = (double*)acs_ws(ctx, WS_FTE5, off * sizeof(double));
  if (!arena) return ACS_E_NOMEM;
  b.X = arena + oX;
  b.tau = arena + oT;
  b.Hloc = arena + oH;
  b.gloc = arena + og;
  b.Floc = arena + oF;
  b.Ab = arena + oAb;
  b.gb = arena + ogb;
  b.Bt = arena + oBt;
  b.gmaxp = arena + ogm;
  b.Lb = arena + oLb;
  b.Y = arena + oY;
  b.Sw = arena + oSw;
  b.RA = arena + oRA;
  b.RL = arena + oRL;
  b.LT = arena + oLT;
  b.ry = arena + ory;
  b.Rt = arena + oRt;
  b.rt = arena + ort;
  b.dS = arena + odS;
  b.dtau = arena + odt;
  b.delta = arena + odl;
  b.normp = arena + onp;
  b.Fm = arena + oFm;
  b.Fq = arena + oFq;
  b.st = (FteState*)(arena + ost);
  int* ints = (int*)(arena + oint);
  b.wstart = ints;
  b.wlen = ints + W;
  b.bad = ints + 2 * W;
  hipStream_t s = ctx->stream;
  const hipMemcpyKind kin = (flags & ACS_DEVICE_PTRS) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  ACS_HIP(ctx, hipMemcpyAsync(b.X, X, sizeof(double) * M * P, kin, s));
  if (tau)
    ACS_HIP(ctx, hipMemcpyAsync(b.tau, tau, sizeof(double) * C, kin, s));
  else
    ACS_HIP(ctx, hipMemsetAsync(b.tau, 0, sizeof(double) * C, s));
  ACS_HIP(ctx, hipMemsetAsync(b.tau + C, 0, sizeof(double) * C, s));
  ACS_HIP(ctx, hipMemcpyAsync(b.X + (size_t)M * P, b.X, sizeof(double) * M * P, hipMemcpyDeviceToDevice, s));
  ACS_HIP(ctx, hipMemcpyAsync(b.wstart, S.ws.data(), sizeof(int) * W, hipMemcpyHostToDevice, s));
  ACS_HIP(ctx, hipMemcpyAsync(b.wlen, S.wn.data(), sizeof(int) * W, hipMemcpyHostToDevice, s));
  ACS_HIP(ctx, hipMemsetAsync(b.bad, 0, sizeof(int), s));
  ACS_HIP(ctx, hipStreamSynchronize(s));  // host vectors ws/wn must outlive the copies
  return ACS_OK;
}

static int fte_linearize_launch(acs_ctx* ctx, FteSetup& S, int force) {
  const FteDims& d = S.d;
  FteBuffers& b = S.b;
  hipStream_t s = ctx->stream;
  hipLaunchKernelGGL(k_fte_linearize, dim3(d.N), dim3(256), 0, s, d, b.I, b.Rl, b.cams, b.meas, b.w, b.X, b.tau,
                     b.st, force, b.Hloc, b.gloc, b.Floc);
  hipLaunchKernelGGL(k_fte_assemble, dim3(d.M), dim3(256), 0, s, d, b.X, b.qinv, b.st, force, b.Hloc, b.gloc, b.Ab,
                     b.gb, b.Bt, b.gmaxp);
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

static int fte_iteration(acs_ctx* ctx, FteSetup& S, const FteOptsDev& o) {
  const FteDims& d = S.d;
  FteBuffers& b = S.b;
  hipStream_t s = ctx->stream;
  int rc;
  if ((rc = fte_linearize_launch(ctx, S, 0))) return rc;
  hipLaunchKernelGGL(k_fte_window, dim3(d.W), dim3(256), 0, s, d, b.wstart, b.wlen, b.st, 0, 0.0, b.Ab, b.gb, b.Bt,
                     b.Lb, b.Y, b.Sw, b.bad);
  hipLaunchKernelGGL(k_fte_reduced, dim3(1), dim3(256), 0, s, d, b.wstart, b.wlen, b.st, 0, 0.0, b.Ab, b.gb, b.Bt,
                     b.Hloc, b.gloc, b.Sw, b.gmaxp, b.RA, b.RL, b.LT, b.ry, b.Rt, b.rt, b.dS, b.dtau, b.bad);
  hipLaunchKernelGGL(k_fte_backsolve, dim3(d.W), dim3(256), 0, s, d, b.wstart, b.wlen, b.st, 0, b.Lb, b.Y, b.dS,
                     b.dtau, b.delta, b.X, b.tau, b.normp);
  hipLaunchKernelGGL(k_fte_cost, dim3(d.N), dim3(64), 0, s, d, b.I, b.Rl, b.cams, b.meas, b.w, b.X, b.tau, b.qinv,
                     b.st, 1, b.Fm, b.Fq);
  hipLaunchKernelGGL(k_fte_lm, dim3(1), dim3(256), 0, s, d, b.st, o, 0, b.Fm, b.Fq, b.normp);
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

extern "C" {

void acs_fte_default_opts(acs_fte_opts* o) {
  o->max_iters = 200;
  o->window = 24;
  o->ftol = 1e-12;
  o->xtol = 1e-12;
  o->gtol = 1e-8;
  o->lambda0 = 1e-3;
  o->redesc_a = 3.0;
  o->redesc_b = 10.0;
  o->redesc_c = 20.0;
}

int acs_fte_solve(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals, int64_t n_reals,
                  const double* cams, int32_t n_cams, const double* meas, const double* w, int32_t n_frames,
                  int32_t shutter_delay, double Ts, const double* qinv, int32_t sd_mode, int32_t intermode, double* X,
                  double* tau, const acs_fte_opts* opts, acs_fte_report* report, uint32_t flags) {
  acs_fte_opts op;
  acs_fte_default_opts(&op);
  if (opts) op = *opts;
  ACS_CHECK(ctx, sd_mode == 0, "fte: only shutter_delay_mode='const' (0) is implemented");
  FteSetup S;
  int rc;
  if ((rc = fte_setup(ctx, S, skel_ints, n_ints, skel_reals, n_reals, cams, n_cams, meas, w, n_frames, shutter_delay,
                      Ts, qinv, intermode, X, tau, op.window, op.redesc_a, op.redesc_b, op.redesc_c, flags)))
    return rc;
  const FteDims& d = S.d;
  FteBuffers& b = S.b;
  hipStream_t s = ctx->stream;
  FteState st0;
  std::memset(&st0, 0, sizeof(st0));
  st0.lam = op.lambda0;
  st0.relin = 1;
  ACS_HIP(ctx, hipMemcpyAsync(b.st, &st0, sizeof(st0), hipMemcpyHostToDevice, s));
  FteOptsDev o{op.max_iters, op.ftol, op.xtol, op.gtol};
  hipLaunchKernelGGL(k_fte_cost, dim3(d.N), dim3(64), 0, s, d, b.I, b.Rl, b.cams, b.meas, b.w, b.X, b.tau, b.qinv,
                     b.st, 0, b.Fm, b.Fq);
  hipLaunchKernelGGL(k_fte_lm, dim3(1), dim3(256), 0, s, d, b.st, o, 1, b.Fm, b.Fq, b.normp);
  ACS_HIP(ctx, hipGetLastError());
  FteState hs;
  const int chunk = 4;  // iterations enqueued between host polls of the device status
  for (int it = 0; it < op.max_iters + 1; it += chunk) {
    for (int c = 0; c < chunk; ++c)
      if ((rc = fte_iteration(ctx, S, o))) return rc;
    ACS_HIP(ctx, hipMemcpyAsync(&hs, b.st, sizeof(hs), hipMemcpyDeviceToHost, s));
    ACS_HIP(ctx, hipStreamSynchronize(s));
    if (hs.status != 0) break;
  }
  // outputs: current state
  const hipMemcpyKind kout = (flags & ACS_DEVICE_PTRS) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  ACS_HIP(ctx, hipMemcpyAsync(X, b.X + (size_t)hs.cur * d.M * d.P, sizeof(double) * d.M * d.P, kout, s));
  if (tau) ACS_HIP(ctx, hipMemcpyAsync(tau, b.tau + hs.cur * d.C, sizeof(double) * d.C, kout, s));
  int nbad = 0;
  ACS_HIP(ctx, hipMemcpyAsync(&nbad, b.bad, sizeof(int), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipStreamSynchronize(s));
  if (report) {
    report->status = hs.status;
    report->iters = hs.iters;
    report->n_accepted = hs.nacc;
    report->n_bad_pivots = nbad;
    report->cost_before = hs.F0;
    report->cost_after = hs.F;
    report->cost_meas = hs.Fmeas;
    report->cost_model = hs.Fmodel;
    report->grad_max = hs.gmax;
    report->lambda_final = hs.lam;
  }
  return ACS_OK;
}

// Cost, gradient and (optionally) the dense undamped normal matrix at (X, tau): the
// linearisation the solver uses, exported for parity tests.
int acs_fte_eval(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals, int64_t n_reals,
                 const double* cams, int32_t n_cams, const double* meas, const double* w, int32_t n_frames,
                 int32_t shutter_delay, double Ts, const double* qinv, int32_t sd_mode, int32_t intermode,
                 const double* X, const double* tau, double* cost3, double* grad, double* H, uint32_t flags) {
  ACS_CHECK(ctx, sd_mode == 0, "fte: only shutter_delay_mode='const' (0) is implemented");
  ACS_CHECK(ctx, !(flags & ACS_DEVICE_PTRS), "acs_fte_eval takes host pointers");
  FteSetup S;
  int rc;
  if ((rc = fte_setup(ctx, S, skel_ints, n_ints, skel_reals, n_reals, cams, n_cams, meas, w, n_frames, shutter_delay,
                      Ts, qinv, intermode, X, tau, 1 << 20, 3.0, 10.0, 20.0, 0)))
    return rc;
  const FteDims& d = S.d;
  FteBuffers& b = S.b;
  hipStream_t s = ctx->stream;
  FteState st0;
  std::memset(&st0, 0, sizeof(st0));
  st0.relin = 1;
  ACS_HIP(ctx, hipMemcpyAsync(b.st, &st0, sizeof(st0), hipMemcpyHostToDevice, s));
  if ((rc = fte_linearize_launch(ctx, S, 1))) return rc;
  hipLaunchKernelGGL(k_fte_cost, dim3(d.N), dim3(64), 0, s, d, b.I, b.Rl, b.cams, b.meas, b.w, b.X, b.tau, b.qinv,
                     b.st, 0, b.Fm, b.Fq);
  ACS_HIP(ctx, hipGetLastError());
  const int M = d.M, P = d.P, Cg = d.Cg, N = d.N, PP = P * P;
  std::vector<double> Ab((size_t)M * 4 * PP), gb((size_t)M * P), Bt((size_t)M * P * (Cg ? Cg : 1)),
      Hl((size_t)N * FTE_NZP * FTE_NZP), gl((size_t)N * FTE_NZP), Fm(N), Fq(N);
  ACS_HIP(ctx, hipMemcpyAsync(Ab.data(), b.Ab, sizeof(double) * Ab.size(), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipMemcpyAsync(gb.data(), b.gb, sizeof(double) * gb.size(), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipMemcpyAsync(Bt.data(), b.Bt, sizeof(double) * Bt.size(), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipMemcpyAsync(Hl.data(), b.Hloc, sizeof(double) * Hl.size(), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipMemcpyAsync(gl.data(), b.gloc, sizeof(double) * gl.size(), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipMemcpyAsync(Fm.data(), b.Fm, sizeof(double) * N, hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipMemcpyAsync(Fq.data(), b.Fq, sizeof(double) * N, hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipStreamSynchronize(s));
  const int nv = M * P + Cg;
  double fm = 0.0, fq = 0.0;
  for (int k = 0; k < N; ++k) {
    fm += Fm[k];
    fq += Fq[k];
  }
  if (cost3) {
    cost3[0] = fm + fq;
    cost3[1] = fm;
    cost3[2] = fq;
  }
  if (grad) {
    for (int i = 0; i < M * P; ++i) grad[i] = gb[i];
    for (int c = 0; c < Cg; ++c) {
      double v = 0.0;
      for (int k = 0; k < N; ++k) v += gl[(size_t)k * FTE_NZP + P + 6 + c];
      grad[M * P + c] = v;
    }
  }
  if (H) {
    std::memset(H, 0, sizeof(double) * (size_t)nv * nv);
    for (int f = 0; f < M; ++f)
      for (int dd = 0; dd < 4 && f - dd >= 0; ++dd)
        for (int r = 0; r < P; ++r)
          for (int c = 0; c < P; ++c) {
            const double v = Ab[(size_t)f * 4 * PP + dd * PP + r * P + c];
            H[(size_t)(f * P + r) * nv + (f - dd) * P + c] = v;
            H[(size_t)((f - dd) * P + c) * nv + f * P + r] = v;
          }
    for (int f = 0; f < M; ++f)
      for (int r = 0; r < P; ++r)
        for (int c = 0; c < Cg; ++c) {
          const double v = Bt[(size_t)f * P * Cg + r * Cg + c];
          H[(size_t)(f * P + r) * nv + M * P + c] = v;
          H[(size_t)(M * P + c) * nv + f * P + r] = v;
        }
    for (int r = 0; r < Cg; ++r)
      for (int c = 0; c < Cg; ++c) {
        double v = 0.0;
        for (int k = 0; k < N; ++k) v += Hl[(size_t)k * FTE_NZP * FTE_NZP + (P + 6 + r) * FTE_NZP + P + 6 + c];
        H[(size_t)(M * P + r) * nv + M * P + c] = v;
      }
  }
  return ACS_OK;
}

}  // extern "C"
