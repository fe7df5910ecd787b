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
// One LM iteration (one hipGraph replay, the next one queued behind it; the host polls a
// pinned status word one iteration late, fte_snapshot / fte_wait_snapshot):
//   k_cr_assemble_build [n blocks]  block-banded normal matrix (bandwidth 3) + tau border +
//                                exact model term, gathered into 3-frame super-blocks (block
//                                tridiagonal) + LM damping
//   k_cr_level       [log2 n levels]  block cyclic reduction, one launch per level:
//                                register-tiled Gauss-Jordan on [D | couplings | rhs] and the
//                                neighbours' Schur terms, all on f64 MFMA tiles
//   k_cr_tau_partial, k_cr_top [1 block]  last block + tau border, block 0's trial rows
//   k_cr_back_all    [n - 1 blocks]  every back-substitution level in one launch (ticket-
//                                ordered workgroups, granule hand-offs) + the trial state
//   k_fte_linearize  [N blocks]  at the trial state, speculatively: FK + analytic FK
//                                Jacobian (fk.hpp), fisheye projection and its Jacobian, loss
//                                derivatives, per-frame J^T W J on v_mfma_f64_16x16x4f64,
//                                gradient and the exact objective (per-frame partials)
//   k_fte_lm         [1 block ]  fixed-order reduction, accept/reject, lambda, stop tests
#include <climits>

#ifdef FTE_PROFILE
__device__ unsigned long long g_fte_prof[64];  // wall-clock ticks (100 MHz) of block 0 phases
// k_cr_back_all per ticket: {entry, inputs ready, done, level} (tools/prof_back_all.py)
#define FTE_BACK_TRACE 8192
__device__ unsigned long long g_back_trace[4 * FTE_BACK_TRACE];
// fk_frame phase marks (slots 24..28): thread 0 of block 0, time since fk_frame started
#define FK_MARK_T0 const unsigned long long fk_t0 = wall_clock64();
#define FK_MARK(slot)                                                                  \
  do {                                                                                 \
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_fte_prof[slot], wall_clock64() - fk_t0); \
  } while (0)
#endif
#include "fk.hpp"
#include "mfma64.hpp"

#define FTE_NZP 64
#define FTE_MAXC 16
#define FTE_CH 32  // observations per LDS chunk (64 Jacobian rows)


// Shutter delays: const mode (src/core/fte.py:236) has C unknowns tau_c, the border Cg = C
// of the normal matrix; variable mode (:238) has N*C unknowns tau[k, c] (NT values, frame
// major), each touching frame k's measurements only, so they are eliminated per frame
// (Ct = C tau columns in the local blocks, no border: Cg = 0).
struct FteDims {
  int N, M, P, L, C, Cg, NZ, im, nblk, BP, GR, nlev;
  int var, Ct, NT, nint, nreal, pad_;  // nint / nreal: the skeleton table's sizes
  double Ts, la, lb, lc;
};

struct FteState {
  double F, F0, lam, gmax, Fmeas, Fmodel, dnorm, xnorm;
  int cur, status, iters, nacc, relin, bad, pad0, pad1;
  // frame-window rounds (acs_fte_dist_round): a step awaiting its summed trial cost, the
  // first round (initial cost), and the state swapped for the speculative reduced system
  int pending, first, spec_on, save_cur;
  double save_lam;
  int launch, pad2;  // iterations run by the solve loop (its host snapshot slot is launch & 1)
};
// transient status of a round whose step was rejected: its solve / step / trial kernels
// (which all stop on status != 0) are skipped, then the status returns to 0
#define FTE_STATUS_SKIP 100

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

// A shutter delay held out of an LM step (oracle/fte.py solve / active_bounds): camera 0
// (tau = 0, src/core/fte.py:304-308) and a delay at a bound of [-Ts, Ts] (:310-314) whose
// descent direction -g points out of the box.
__device__ __forceinline__ bool tau_held(double t, double g, double Ts, int c) {
  return c == 0 || (t >= Ts && g < 0.0) || (t <= -Ts && g > 0.0);
}

__device__ __forceinline__ double loss_curv(double e, const LossOut& l) {
  double c = l.d2;
  if (e != 0.0) c = fmax(c, l.d1 / e);
  return fmax(c, 0.0);
}

// fixed-order block sum (blockDim.x must be a power of two <= 256)
// Sum over the workgroup (blockDim a power of two, 64..1024) in the fixed order of the
// halving tree s[t] += s[t + h], h = n/2 .. 1. The levels h >= 128 go through LDS; then
// every wave evaluates the last seven levels itself (s[l] + s[l + 64], then shuffles down
// 32 .. 1: lane l < h adds lane l + h, the tree's own operands), so each wave ends with the
// tree's bits in lane 0 without a broadcast round trip: 3 barriers at 256 threads, was 10.
__device__ double block_sum(double v, double* s_red) {
  const int t = threadIdx.x, n = blockDim.x, l = t & 63;
  double r = v;
  if (n > 64) {
    s_red[t] = v;
    __syncthreads();
    for (int h = n / 2; h >= 128; h >>= 1) {
      if (t < h) s_red[t] += s_red[t + h];
      __syncthreads();
    }
    r = s_red[l] + s_red[l + 64];
  }
#pragma unroll
  for (int h = 32; h > 0; h >>= 1) r += __shfl_down(r, h, 64);
  r = __shfl(r, 0, 64);
  if (n > 64) __syncthreads();  // s_red is free for the caller's next reduction
  return r;
}
// block_sum of NV values at once (the same tree per value, so each result is bit-identical
// to its own block_sum; one set of barriers instead of NV). s_red: NV x blockDim doubles.
template <int NV>
__device__ void block_sums(double (&v)[NV], double* s_red) {
  const int t = threadIdx.x, n = blockDim.x, l = t & 63;
  double r[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) r[j] = v[j];
  if (n > 64) {
#pragma unroll
    for (int j = 0; j < NV; ++j) s_red[j * n + t] = v[j];
    __syncthreads();
    for (int h = n / 2; h >= 128; h >>= 1) {
      if (t < h) {
#pragma unroll
        for (int j = 0; j < NV; ++j) s_red[j * n + t] += s_red[j * n + t + h];
      }
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < NV; ++j) r[j] = s_red[j * n + l] + s_red[j * n + l + 64];
  }
#pragma unroll
  for (int h = 32; h > 0; h >>= 1)
#pragma unroll
    for (int j = 0; j < NV; ++j) r[j] += __shfl_down(r[j], h, 64);
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = __shfl(r[j], 0, 64);
  if (n > 64) __syncthreads();
}
// acc[s] += x[s][es * k] for k = k0, k0 + st, .. < k1 in that order (the plain strided
// loop's sums, bit for bit), with eight strides' loads of every stream issued before the
// first add instead of one dependent round trip per stride
template <int NS>
__device__ __forceinline__ void strided_sums(const double* const (&x)[NS], int es, int k0, int k1, int st,
                                             double* acc) {
  int k = k0;
  for (; k + 7 * st < k1; k += 8 * st) {
    double v[NS][8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int s = 0; s < NS; ++s) v[s][j] = x[s][(size_t)es * (k + j * st)];
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int s = 0; s < NS; ++s) acc[s] += v[s][j];
  }
  for (; k < k1; k += st)
#pragma unroll
    for (int s = 0; s < NS; ++s) acc[s] += x[s][(size_t)es * k];
}

// max(m, x[k]) over k = k0, k0 + st, .. < k1 with eight loads in flight (max is exact, so
// any grouping gives the same value)
__device__ __forceinline__ double strided_max(const double* __restrict__ x, int k0, int k1, int st, double m) {
  int k = k0;
  for (; k + 7 * st < k1; k += 8 * st) {
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = x[k + j * st];
#pragma unroll
    for (int j = 0; j < 8; ++j) m = fmax(m, v[j]);
  }
  for (; k < k1; k += st) m = fmax(m, x[k]);
  return m;
}

// any blockDim (max is exact: the fold order does not change the value)
__device__ double block_max(double v, double* s_red) {
  const int t = threadIdx.x, n = blockDim.x;
  s_red[t] = v;
  __syncthreads();
  int w = n;
  while (w > 1) {
    const int h = (w + 1) >> 1;
    if (t < w - h) s_red[t] = fmax(s_red[t], s_red[t + h]);
    w = h;
    __syncthreads();
  }
  const double r = s_red[0];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------------------
// 1. per-frame linearisation
//
// Observation o = (camera c, marker l) has the 2 x NZ Jacobian Jp_o (2x3, the fisheye
// projection derivative scaled by the weight) times D_o (3 x NZ, the derivative of the
// shifted marker position), and D_o = D_l + S_c splits into the camera-independent FK part
// D_l (columns < P, fk_dpos) and the shutter-delay part S_c = [own_c I (x_0..z_0) | prev_c I
// | prev2_c I | v_c (tau column of camera c)] that is the same for every marker. With the
// 3x3 curvature blocks Z_o = Jp_o^T diag(curv) Jp_o and gradient vectors r_o = Jp_o^T rho',
//   H = sum_o D_o^T Z_o D_o
//     = sum_l [D_l ; Q_l]^T [Z_l D_l + Q_l ; D_l]  +  sum_c S_c^T Z_c S_c,
//   g = sum_l D_l^T r_l + sum_c S_c^T r_c,
// with Z_l = sum_c Z_o, Q_l = sum_c Z_o S_c, Z_c = sum_l Z_o (and r likewise). The first
// term is one MFMA product with K = 6L rows instead of the 2CL rows of the stacked
// Jacobian (C times fewer FK derivatives, 2C/2 = C times fewer MFMA K-steps); the second
// touches only the 9 + C shift / delay columns and is added when H is stored.
// ---------------------------------------------------------------------------------------
#ifdef FTE_PROFILE
// k_fte_linearize phases (block 0, thread 0, after a barrier), slots 56..61
#define LPROF(slot)                                                          \
  do {                                                                     \
    __syncthreads();                                                       \
    if (blockIdx.x == 0 && threadIdx.x == 0)                               \
      atomicAdd(&g_fte_prof[slot], wall_clock64() - lprof_t0);             \
  } while (0)
#define LPROF_T0 const unsigned long long lprof_t0 = wall_clock64();
#else
#define LPROF(slot)
#define LPROF_T0
#endif
#define LIN_OCH 128  // observations per aggregation chunk (<= blockDim)
#define LIN_MC 4     // markers per MFMA chunk (3 * LIN_MC operand rows)

// compact per-frame tau border of the local normal matrix: Cg x Cg block, then Cg gradient
__host__ __device__ __forceinline__ int tc_stride(int Cg) { return Cg * Cg + Cg; }

struct LinLds {
  int cam, am, qt, ac, cf, uni, xr, tabR, tabI, total;
};
// dynamic LDS of k_fte_linearize (doubles): QW = the compact width of the Q rows (the
// shift / delay columns 0..2 and P..NZ-1), nint / nreal the skeleton table's sizes
__host__ __device__ __forceinline__ LinLds lin_lds(int C, int L, int P, int NZP, int QW, int nint, int nreal) {
  LinLds o;
  int p = 0;
  o.cam = p;
  p += C * ACS_CAM_STRIDE;
  o.am = p;  // per marker: Z_l, sum own Z, sum prev Z, sum prev2 Z (6 each), r_l (3)
  p += 27 * L;
  o.qt = p;  // per (marker, camera): Z_o v_c (tau column of Q_l)
  p += 3 * C * L;
  o.ac = p;  // per camera: Z_c (6), r_c (3)
  p += 9 * C;
  o.cf = p;  // per camera: own, prev, prev2, v_c (3), tau_c
  p += 7 * C;
  o.uni = p;  // observation chunk (9 per obs) | operand rows D, B (3 LIN_MC x (NZP + 1)) and
              // Q (3 LIN_MC x QW) | the block sums' scratch (256)
  const int a = 9 * LIN_OCH, b = 3 * LIN_MC * (2 * (NZP + 1) + QW);
  p += a > b ? (a > 256 ? a : 256) : (b > 256 ? b : 256);
  o.xr = p;  // the frame's pose stencil: rows f - 3 .. f of X (FK reads row f, the model term all four)
  p += 4 * P;
  o.tabR = p;  // skeleton table: reals, then ints
  p += nreal;
  o.tabI = p;
  p += (nint + 1) / 2;
  o.total = p;
  return o;
}

__device__ __forceinline__ int sym3(int i, int j) {
  // [xx xy xz yy yz zz]
  return i <= j ? (i == 0 ? j : (i == 1 ? 2 + j : 5)) : (j == 0 ? i : (j == 1 ? 2 + i : 5));
}

// shift / delay column class: 0..2 = own (x_0..z_0), prev, prev2 with component *i;
// 3 = tau column of camera *i; -1 = FK-only column
__device__ __forceinline__ int lin_tcol(int x, int P, int NZ, int* i) {
  if (x < 3) {
    *i = x;
    return 0;
  }
  if (x >= P && x < P + 6) {
    *i = (x - P) % 3;
    return 1 + (x - P) / 3;
  }
  if (x >= P + 6 && x < NZ) {
    *i = x - P - 6;
    return 3;
  }
  return -1;
}

// WPC: the workgroups per CU the register budget is set for (256 threads each). The kernel is
// bound by its dependent LDS chains, so with more frames than fit the chip at once the frames
// in flight per CU set its throughput: 5 per CU (the LDS, ~30 KB per workgroup at 6 cameras,
// allows it; 96 VGPRs with a few spilled) took 10,000 frames 357 -> 326 us, while a grid that
// fits in one wave of workgroups at 4 per CU is latency-bound and the spills cost it (1,000
// frames 42.3 -> 45.8 us; profiles/r05/seq*_lin4.log). lin_kernel picks the instance.
template <int WPC>
__global__ __launch_bounds__(256, WPC) void k_fte_linearize(FteDims d, const int* __restrict__ I,
                                                       const double* __restrict__ Rl,
                                                       const double* __restrict__ cams,
                                                       const double* __restrict__ meas,
                                                       const double* __restrict__ wts,
                                                       const double* __restrict__ Xbuf,
                                                       const double* __restrict__ taubuf,
                                                       const FteState* __restrict__ st, int force, int k0,
                                                       double* __restrict__ Hloc, double* __restrict__ gloc,
                                                       double* __restrict__ Floc, int spec,
                                                       double* __restrict__ Fq, const double* __restrict__ qinv,
                                                       double* __restrict__ Tc) {
  // spec: speculative linearisation at the trial state X[cur ^ 1] into the second
  // Hloc / gloc / Floc buffer, with the model cost of the frame's stencil in Fq: it is the
  // trial cost for k_fte_lm, and an accepted step (cur ^= 1) needs no new linearisation
  if (spec ? st->status != 0 : (!force && (st->status != 0 || !st->relin))) return;
  {
    const size_t hb = spec ? (size_t)(st->cur ^ 1) : 0;
    Hloc += hb * d.N * FTE_NZP * FTE_NZP;
    gloc += hb * d.N * FTE_NZP;
    Floc += hb * d.N;
    Tc += hb * d.N * tc_stride(d.Cg);
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lk = lane >> 4;
  const int P = d.P, C = d.C, L = d.L, NZ = d.NZ;
  const int NZP = (NZ + 15) & ~15, LD = NZP + 1, NT = NZP >> 4;
  const int cur = force ? 0 : (spec ? st->cur ^ 1 : st->cur);
  const double* X = Xbuf + (size_t)cur * d.M * P;
  extern __shared__ double lds[];
  const int QW = 3 + NZ - P;  // compact Q rows: columns 0..2 and P..NZ-1
  const LinLds lo = lin_lds(C, L, P, NZP, QW, d.nint, d.nreal);
  double *s_cam = lds + lo.cam, *s_am = lds + lo.am, *s_qt = lds + lo.qt, *s_ac = lds + lo.ac, *s_cf = lds + lo.cf,
         *s_u = lds + lo.uni, *s_xr = lds + lo.xr;
  double* s_red = s_u;  // the block sums at the end (the operand rows are dead by then)
  int* s_tabI = reinterpret_cast<int*>(lds + lo.tabI);
  double* s_tabR = lds + lo.tabR;
  __shared__ FkShared fk;
  __shared__ FkDeriv fkd;
  __shared__ double s_dx[3], s_ddx[3];
  LPROF_T0
  // every input load in flight before the first LDS store and the one barrier: the skeleton
  // table (sizes from the host: no dependent header load), the cameras, the frame's pose stencil
  // rows f - 3 .. f (an LDS copy: FK reads row f, the model term all four; from global memory
  // their round trip sat at FK's start and again before the closing sums), the root's velocity /
  // acceleration and the shutter delays (slot 6 of each camera's coefficients; after FK they
  // were a round trip of their own). Each thread gathers its elements into registers first:
  // copy loops of the form `for (i = tid; ..) lds[i] = g[i]` waited for every load before the
  // next loop's were issued, a chain of global round trips (2.4-3.3 us to the table staged,
  // profiles/r06/lin_phases_r06v_*.log). blockDim = 256.
  const int k = blockIdx.x + k0;
  const double* tau = taubuf + (size_t)cur * d.NT + (d.var ? (size_t)k * C : 0);
  const int f = k + 2;
  constexpr int NTH = 256, NIQ = (FK_MAX_INTS + NTH - 1) / NTH, NCQ = (FTE_MAXC * ACS_CAM_STRIDE + NTH - 1) / NTH;
  static_assert(3 * FK_MAXN <= NTH && 4 * FK_MAXP <= NTH && FTE_MAXC <= NTH, "one element per thread");
  int iv[NIQ];
  double cv[NCQ], rv = 0.0, xv = 0.0, tv = 0.0, x0 = 0.0, x1 = 0.0, x2 = 0.0;
#pragma unroll
  for (int q = 0; q < NIQ; ++q) iv[q] = tid + NTH * q < d.nint ? I[tid + NTH * q] : 0;
  if (tid < d.nreal) rv = Rl[tid];
#pragma unroll
  for (int q = 0; q < NCQ; ++q) cv[q] = tid + NTH * q < C * ACS_CAM_STRIDE ? cams[tid + NTH * q] : 0.0;
  const int fr = f - 3 + tid / P;  // row f - 3 is read by the model term only (k >= 1)
  if (tid < 4 * P && fr >= 0) xv = X[(size_t)fr * P + tid % P];
  if (tid < C && d.Ct) tv = tau[tid];
  if (tid < 3) {
    x0 = X[f * P + tid];
    x1 = X[(f - 1) * P + tid];
    x2 = X[(f - 2) * P + tid];
  }
  for (int i = lo.am + tid; i < lo.cf; i += blockDim.x) lds[i] = 0.0;
#pragma unroll
  for (int q = 0; q < NIQ; ++q)
    if (tid + NTH * q < d.nint) s_tabI[tid + NTH * q] = iv[q];
  if (tid < d.nreal) s_tabR[tid] = rv;
#pragma unroll
  for (int q = 0; q < NCQ; ++q)
    if (tid + NTH * q < C * ACS_CAM_STRIDE) s_cam[tid + NTH * q] = cv[q];
  if (tid < 4 * P) s_xr[tid] = xv;
  if (tid < C) s_cf[7 * tid + 6] = tv;
  if (tid < 3) {
    s_dx[tid] = (x0 - x1) / d.Ts;
    s_ddx[tid] = (x0 - 2.0 * x1 + x2) / (d.Ts * d.Ts);
  }
  __syncthreads();
  const SkelView s = skel_view(s_tabI, s_tabR);
  LPROF(61);
  LPROF(62);
  fk_frame(s, s_xr + 3 * P, fk, tid, blockDim.x);
  __syncthreads();
  if (tid < P) fk_deriv_prep(s, fk, fkd, tid);  // read after the barriers of phase (a)
  LPROF(56);
  if (tid < C) {
    const double tc = s_cf[7 * tid + 6];
    const ShiftCoef sc = shift_coef(d.im, tc, d.Ts);
    double* cf = s_cf + 7 * tid;
    cf[0] = sc.own;
    cf[1] = sc.prev;
    cf[2] = sc.prev2;
    const bool tcol = d.Ct && tid > 0;
    for (int i = 0; i < 3; ++i) cf[3 + i] = tcol ? s_dx[i] + (d.im == 2 ? 2.0 * tc * s_ddx[i] : 0.0) : 0.0;
    cf[6] = tc;
  }
  __syncthreads();

  // (a) one observation per thread: projection, loss, Z_o, r_o; then the fixed-order sums
  double rho = 0.0;
  const int nobs = C * L;
  // one chunk's observations (LIN_OCH per chunk); a frame whose observations fit one chunk
  // (6 cameras x 20 markers) runs it as straight-line code: in the loop, the compiler hoisted
  // the projection's and the loss's f64 constants into VGPRs ahead of it and spilled them, 80 B
  // of scratch per thread written back to HBM (205 MB per launch at 10,000 frames)
  auto obs_chunk = [&](int ch) {
    const int no = min(LIN_OCH, nobs - ch);
    if (tid < no) {
      const int o = ch + tid, c = o / L, l = o - c * L;
      const double* p = fk.pos[s.outn[l]];
      const double tc = s_cf[7 * c + 6];
      double sh[3];
      for (int i = 0; i < 3; ++i) {
        sh[i] = 0.0;
        if (d.im >= 1) sh[i] += s_dx[i] * tc;
        if (d.im == 2) sh[i] += s_ddx[i] * (tc * tc);
      }
      // the weight and both measurements in one round trip, issued before the projection (the
      // measurements loaded only where the weight is nonzero waited for the weight's load first;
      // the select gives the same values)
      const size_t mi = ((size_t)k * C + c) * L + l;
      const double wt = wts[mi], mu0 = meas[2 * mi], mv0 = meas[2 * mi + 1];
      ProjOut po;
      fisheye_project<true, true>(s_cam + c * ACS_CAM_STRIDE, p[0] + sh[0], p[1] + sh[1], p[2] + sh[2], po);
      const double mu = wt != 0.0 ? mu0 : 0.0, mv = wt != 0.0 ? mv0 : 0.0;
      const bool ok = wt != 0.0;
      double* z = s_u + 9 * tid;
      for (int i = 0; i < 9; ++i) z[i] = 0.0;
      // u then v (one loss evaluation live at a time)
#pragma unroll 1
      for (int side = 0; side < 2; ++side) {
        const double e = wt * ((side ? po.v : po.u) - (side ? mv : mu));
        const LossOut ls = redescending(e, d.la, d.lb, d.lc);
        rho += ls.f;
        if (ok) {
          const double cw = wt * wt * loss_curv(e, ls), gw = wt * ls.d1;
          // selects, not po.J[3 * side]: a dynamic index would put the whole ProjOut in scratch
          const double j0 = side ? po.J[3] : po.J[0], j1 = side ? po.J[4] : po.J[1], j2 = side ? po.J[5] : po.J[2];
          z[0] += cw * j0 * j0;
          z[1] += cw * j0 * j1;
          z[2] += cw * j0 * j2;
          z[3] += cw * j1 * j1;
          z[4] += cw * j1 * j2;
          z[5] += cw * j2 * j2;
          z[6] += gw * j0;
          z[7] += gw * j1;
          z[8] += gw * j2;
        }
      }
    }
    __syncthreads();
    // per marker (cameras in order): Z_l, sum_c coef_c Z_o (own, prev, prev2), r_l
    for (int e = tid; e < 27 * L; e += blockDim.x) {
      const int l = e / 27, j = e - 27 * l;
      double v = 0.0;
      for (int c = 0; c < C; ++c) {
        const int oo = c * L + l - ch;
        if (oo < 0 || oo >= no) continue;
        const double* z = s_u + 9 * oo;
        if (j < 6)
          v += z[j];
        else if (j < 24)
          v += s_cf[7 * c + (j - 6) / 6] * z[(j - 6) % 6];
        else
          v += z[j - 18];
      }
      s_am[e] += v;
    }
    // per camera (markers in order): Z_c, r_c
    for (int e = tid; e < 9 * C; e += blockDim.x) {
      const int c = e / 9, j = e - 9 * c;
      double v = 0.0;
      for (int l = 0; l < L; ++l) {
        const int oo = c * L + l - ch;
        if (oo >= 0 && oo < no) v += s_u[9 * oo + j];
      }
      s_ac[e] += v;
    }
    // per observation: Z_o v_c
    for (int e = tid; e < 3 * no; e += blockDim.x) {
      const int oo = e / 3, i = e - 3 * oo, o = ch + oo, c = o / L, l = o - c * L;
      const double* z = s_u + 9 * oo;
      const double* v = s_cf + 7 * c + 3;
      s_qt[(l * C + c) * 3 + i] = z[sym3(i, 0)] * v[0] + z[sym3(i, 1)] * v[1] + z[sym3(i, 2)] * v[2];
    }
    __syncthreads();
  };
  if (nobs <= LIN_OCH) {
    obs_chunk(0);
  } else {
    for (int ch = 0; ch < nobs; ch += LIN_OCH) obs_chunk(ch);
  }

  LPROF(57);
  // (b) H = sum_l [D_l ; Q_l]^T [Z_l D_l + Q_l ; D_l] on v_mfma_f64_16x16x4f64: upper-triangle
  //     tiles of NT x NT, tile t on wave t % 4
  // tile t = wave + 4q (q = 0..2) of the NT (NT + 1) / 2 upper-triangle tiles, row-major
  const int ntile = NT * (NT + 1) / 2;
  // tile of this wave's q-th accumulator (-1: none): tile wave + 4q. (Dealing the
  // products that survive the zero-tile skip as two 3-step chains per wave, with the
  // gradient on wave 0, was slower in r03n: the gradient's dependent LDS chain then sits on
  // a wave with a full MFMA share.)
  auto tile_of = [&](int q) -> int {
    const int t = wave + 4 * q;
    return t < ntile ? t : -1;
  };
  auto tile_ab = [&](int t, int& a, int& b) {
    a = 0;
    while (t >= NT - a) {
      t -= NT - a;
      ++a;
    }
    b = a + t;
  };
  dbl4 acc[3];
  for (int q = 0; q < 3; ++q) acc[q] = dbl4{0.0, 0.0, 0.0, 0.0};
  double gacc = 0.0;
  const int gi = tid - 128;
  constexpr int RC = 3 * LIN_MC;
  double* sD = s_u;            // D_l rows
  double* sB = s_u + RC * LD;  // Z_l D_l + Q_l rows
  double* sQ = sB + RC * LD;   // Q_l rows, compact (RC x QW): zero outside the shift / delay columns
  auto qcol = [&](int x) { return x < 3 ? x : (x >= P && x < NZ ? 3 + x - P : -1); };
  for (int l0 = 0; l0 < L; l0 += LIN_MC) {
#ifdef FTE_PROFILE
    unsigned long long tb = wall_clock64();
#endif
    for (int e = tid; e < LIN_MC * NZP; e += blockDim.x) {
      const int m = e / NZP, q = e - m * NZP, l = l0 + m;
      double dp[3] = {0.0, 0.0, 0.0}, qv[3] = {0.0, 0.0, 0.0};
      const double* am = s_am + 27 * (l < L ? l : 0);
      if (l < L) {
        if (q < P) fk_dpos_fast(s, fk, fkd, s.outn[l], q, dp);
        int i0;
        const int cls = lin_tcol(q, P, NZ, &i0);
        if (cls >= 0 && cls < 3) {
          for (int i = 0; i < 3; ++i) qv[i] = am[6 + 6 * cls + sym3(i, i0)];
        } else if (cls == 3) {
          for (int i = 0; i < 3; ++i) qv[i] = s_qt[(l * C + i0) * 3 + i];
        }
      }
      const int cq = qcol(q);
      for (int i = 0; i < 3; ++i) {
        const int r = (3 * m + i) * LD + q;
        sD[r] = dp[i];
        sB[r] = (l < L) ? am[sym3(i, 0)] * dp[0] + am[sym3(i, 1)] * dp[1] + am[sym3(i, 2)] * dp[2] + qv[i] : 0.0;
        if (cq >= 0) sQ[(3 * m + i) * QW + cq] = qv[i];
      }
    }
    __syncthreads();
#ifdef FTE_PROFILE
    if (blockIdx.x == 0 && tid == 0) {  // operand rows built (slot 14), MFMA + barrier (slot 15)
      const unsigned long long t1 = wall_clock64();
      atomicAdd(&g_fte_prof[14], t1 - tb);
      tb = t1;
    }
#endif
    // gradient column gi = tid - 128 on wave 2, which carries one MFMA tile fewer than
    // waves 0 and 1 (NT = 3: tiles 0-5 on waves 0, 1, 2, 3, 0, 1)
    if (gi >= 0 && gi < NZP) {
      const int nr = 3 * min(LIN_MC, L - l0);
      for (int r = 0; r < nr; ++r) gacc = fma(sD[r * LD + gi], s_am[27 * (l0 + r / 3) + 24 + r % 3], gacc);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const int t = tile_of(q);
      if (t < 0) continue;
      int ta, tb;
      tile_ab(t, ta, tb);
      const int ci = ta * 16 + li, cj = tb * 16 + li;
      // D rows are zero past column P (FK columns only) and Q rows are zero outside the
      // own-shift (0..2) and shift / delay (P..NZ-1) columns: a product whose operand tile
      // is all zero adds exact zeros and is skipped (at P = 26, NZ = 38: 12 of the 36 MFMAs
      // per marker chunk; tile (2, 2) is the delay block, tpart only)
      if (ta * 16 < P) {
#pragma unroll
        for (int r0 = 0; r0 < RC; r0 += 4) {
          const int r = (r0 + lk) * LD;
          acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(sD[r + ci], sB[r + cj], acc[q], 0, 0, 0);
        }
      }
      if (tb * 16 < P && (ta == 0 || (ta * 16 + 15 >= P && ta * 16 < NZ))) {
        const int cq = qcol(ci);
#pragma unroll
        for (int r0 = 0; r0 < RC; r0 += 4) {
          const int r = (r0 + lk) * LD;
          const double qa = cq >= 0 ? sQ[(r0 + lk) * QW + (cq >= 0 ? cq : 0)] : 0.0;
          acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(qa, sD[r + cj], acc[q], 0, 0, 0);
        }
      }
    }
    __syncthreads();
#ifdef FTE_PROFILE
    if (blockIdx.x == 0 && tid == 0) atomicAdd(&g_fte_prof[15], wall_clock64() - tb);
#endif
  }

  LPROF(58);
  // (c) sum_c S_c^T Z_c S_c and sum_c S_c^T r_c (shift / delay columns), store
  auto zc_v = [&](int c, int i) {  // (Z_c v_c)[i]
    const double* z = s_ac + 9 * c;
    const double* v = s_cf + 7 * c + 3;
    return z[sym3(i, 0)] * v[0] + z[sym3(i, 1)] * v[1] + z[sym3(i, 2)] * v[2];
  };
  auto tpart = [&](int row, int col) {
    int i, j;
    const int a = lin_tcol(row, P, NZ, &i), b = lin_tcol(col, P, NZ, &j);
    if (a < 0 || b < 0) return 0.0;
    double v = 0.0;
    if (a < 3 && b < 3) {
      for (int c = 0; c < C; ++c) v += s_cf[7 * c + a] * s_cf[7 * c + b] * s_ac[9 * c + sym3(i, j)];
    } else if (a < 3) {
      v = s_cf[7 * j + a] * zc_v(j, i);
    } else if (b < 3) {
      v = s_cf[7 * i + b] * zc_v(i, j);
    } else if (i == j) {
      const double* vv = s_cf + 7 * i + 3;
      v = vv[0] * zc_v(i, 0) + vv[1] * zc_v(i, 1) + vv[2] * zc_v(i, 2);
    }
    return v;
  };
  double* H = Hloc + (size_t)k * FTE_NZP * FTE_NZP;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int t = tile_of(q);
    if (t < 0) continue;
    int ta, tb;
    tile_ab(t, ta, tb);
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      const int row = ta * 16 + lk + 4 * rg, col = tb * 16 + li;
      if (row > col) continue;  // diagonal tiles: the (row <= col) element writes both
      const double v = acc[q][rg] + tpart(row, col);
      H[row * FTE_NZP + col] = v;
      H[col * FTE_NZP + row] = v;
      // the tau border block again, compact (k_cr_tau_partial reads it contiguously)
      const int tr = row - (P + 6), tq = col - (P + 6);
      if (tr >= 0 && tq < d.Cg) {
        double* T = Tc + (size_t)k * tc_stride(d.Cg);
        T[tr * d.Cg + tq] = v;
        T[tq * d.Cg + tr] = v;
      }
    }
  }
  if (gi >= 0 && gi < NZP) {
    int i;
    const int a = lin_tcol(gi, P, NZ, &i);
    if (a >= 0 && a < 3) {
      for (int c = 0; c < C; ++c) gacc += s_cf[7 * c + a] * s_ac[9 * c + 6 + i];
    } else if (a == 3) {
      const double* v = s_cf + 7 * i + 3;
      const double* r = s_ac + 9 * i + 6;
      gacc += v[0] * r[0] + v[1] * r[1] + v[2] * r[2];
    }
    gloc[(size_t)k * FTE_NZP + gi] = gacc;
    const int ti = gi - (P + 6);
    if (ti >= 0 && ti < d.Cg) Tc[(size_t)k * tc_stride(d.Cg) + d.Cg * d.Cg + ti] = gacc;
  }
  if (Fq) {  // the model stencil ending at row k + 2 (rows k-1 .. k+2), as k_fte_cost
    double q = 0.0;
    if (k >= 1) {
      const double its2 = 1.0 / (d.Ts * d.Ts);
      for (int p = tid; p < P; p += blockDim.x) {
        const double sm = (s_xr[3 * P + p] - 3.0 * s_xr[2 * P + p] + 3.0 * s_xr[P + p] - s_xr[p]) * its2;
        q += qinv[p] * sm * sm;
      }
    }
    double v[2] = {rho, q};  // both sums on one set of barriers (each bit-identical to its block_sum)
    block_sums<2>(v, s_red);
    if (tid == 0) {
      Floc[k] = v[0];
      Fq[k] = v[1];
    }
  } else {
    const double tot = block_sum(rho, s_red);
    if (tid == 0) Floc[k] = tot;
  }
  LPROF(59);
#ifdef FTE_PROFILE
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_fte_prof[60], 1ull);
#endif
}

typedef void (*LinKernel)(FteDims, const int*, const double*, const double*, const double*, const double*,
                          const double*, const double*, const FteState*, int, int, double*, double*, double*, int,
                          double*, const double*, double*);
static LinKernel lin_kernel(int nwg) { return nwg > 4 * 256 ? k_fte_linearize<5> : k_fte_linearize<4>; }

static size_t lin_lds_bytes(const FteDims& d) {
  return sizeof(double) * (size_t)lin_lds(d.C, d.L, d.P, (d.NZ + 15) & ~15, 3 + d.NZ - d.P, d.nint, d.nreal).total;
}

// ---------------------------------------------------------------------------------------
// 2. assembly of the banded normal matrix (row f: blocks (f, f-d), d = 0..3)
// ---------------------------------------------------------------------------------------
// Row f: A = blocks (f, f-dd), dd = 0..3 (4 P x P), g (P) and the tau border B (P x Cg),
// from the local blocks of frames f-2 (own rows), f-1 (prev) and f (prev2) that are owned
// (lo <= k < hi), plus the exact third-difference model term of the stencils starting in
// [lo, hi). Threads t < nth of the calling group work; every thread of the workgroup must
// call it (it holds barriers). Fixed accumulation order per element: 0 + own + prev + prev2 +
// model (a term that is not owned adds +0.0, which is exact: no partial sum is -0.0).
// Every global load (own / prev / prev2 blocks, gradients, the stencil rows of X) is issued in
// one round. Each element's own term is added where it is stored; after one barrier, thread
// p < P finishes the diagonal entries of row p (prev / prev2 for p < 3, then the model term)
// and the next threads the other entries that prev / prev2 touch (rows < 3 of blocks dd = 0, 1
// and of B), with the terms they loaded in that round. (It was zero-fill, then one barrier and
// one dependent global round trip per term: own, prev, prev2, model.)
// Compact row storage (CMP, k_cr_assemble_build's LDS rows): blocks 1 and 2 are zero outside their
// columns < 3 and the diagonal, block 3 outside the diagonal, so a row keeps block 0 whole, the
// columns < 3 of blocks 1, 2 (P x 3 each), and the diagonals of blocks 1..3 (rows >= 3 of blocks
// 1, 2 and all of block 3 are read from there): PP + 9P doubles instead of 4 PP.
struct RowCmp {
  static __host__ __device__ __forceinline__ int size(int P) { return P * P + 9 * P; }
  // entry (dd, r, c) of a compact row, or -1 for a structural zero
  static __device__ __forceinline__ int at(int P, int dd, int r, int c) {
    if (dd == 0) return r * P + c;
    if (dd <= 2 && c < 3) return P * P + 3 * P * (dd - 1) + 3 * r + c;
    if (r == c && (dd == 3 || r >= 3)) return P * P + 6 * P + P * (dd - 1) + r;
    return -1;
  }
};
template <bool CMP>
__device__ void assemble_row(const FteDims& d, int f, const double* __restrict__ X, const double* __restrict__ qinv,
                             int lo, int hi, const double* __restrict__ Hloc, const double* __restrict__ gloc,
                             double* A, double* g, double* B, int t, int nth) {
  const int P = d.P, Cg = d.Cg, N = d.N, PP = P * P;
  const int kown = f - 2, kprev = f - 1, kprev2 = f;
  auto owned = [&](int k) { return k >= 0 && k < N && k >= lo && k < hi; };
  const bool oo = owned(kown), op = owned(kprev), op2 = owned(kprev2);
  const double* Ho = Hloc + (size_t)(oo ? kown : 0) * FTE_NZP * FTE_NZP;
  const double* Hp = Hloc + (size_t)(op ? kprev : 0) * FTE_NZP * FTE_NZP;
  const double* Hp2 = Hloc + (size_t)(op2 ? kprev2 : 0) * FTE_NZP * FTE_NZP;
  const double cf[4] = {1.0, -3.0, 3.0, -1.0};
  const double its2 = 1.0 / (d.Ts * d.Ts);
  // model stencil m = f + i (rows m-3 .. m) is in the row's sums iff 3 <= m <= M-1, lo <= m-3 < hi
  auto mvalid = [&](int i) {
    const int m = f + i;
    return !(m < 3 || m > d.M - 1 || m - 3 < lo || m - 3 >= hi);
  };
  // the second-round work of this thread and its loads: t < P the gradient entry and the
  // diagonal of row t; then the off-diagonal entries (r, c < 3) of blocks dd = 0, 1 (6 each),
  // then rows < 3 of B (3 Cg)
  double sg[3] = {0.0, 0.0, 0.0}, dg[3] = {0.0, 0.0, 0.0}, sq = 0.0, sx[7];
#pragma unroll
  for (int j = 0; j < 7; ++j) sx[j] = 0.0;
  int se = -1;  // the entry of A (< 4 PP) or B (>= 4 PP) a second-round thread finishes
  if constexpr (CMP) {
    // The gradient specials are threads t < P (the first wave of the row's group); the others
    // start at the second wave (S0), each with one load pair at offsets formed by selects, so no
    // wave holds two of these load branches (the compiler waited for a branch's loads before the
    // next branch's, a round trip per branch of one wave).
    constexpr int S0 = 64;
    const int nS1 = 12 + 3 * Cg;  // nth >= S0 + nS1 (<= 124: 16 delays)
    if (t < P) {
      // every load unconditional (valid clamped addresses), the terms that do not apply selected
      // to zero after: nested load branches were waited for one after the other
      const int t3 = t < 3 ? t : 0;
      const size_t ko = oo ? kown : 0, kp = op ? kprev : 0, kp2 = op2 ? kprev2 : 0;
      const double g0 = gloc[ko * FTE_NZP + t], g1 = gloc[kp * FTE_NZP + P + t3], g2 = gloc[kp2 * FTE_NZP + P + 3 + t3];
      const double h0 = Hp[(P + t3) * FTE_NZP + P + t3];           // block 0, prev
      const double h1 = Hp2[(P + 3 + t3) * FTE_NZP + P + 3 + t3];  // block 0, prev2
      const double h2 = Hp[(P + t3) * FTE_NZP + P + 3 + t3];       // block 1, prev
      sq = qinv[t];
      double xr[7];
#pragma unroll
      for (int j = 0; j < 7; ++j) {  // rows f - 3 .. f + 3
        const int row = f - 3 + j;
        xr[j] = X[(size_t)(row < 0 ? 0 : (row > d.M - 1 ? d.M - 1 : row)) * P + t];
      }
      sg[0] = oo ? g0 : 0.0;
      sg[1] = (op && t < 3) ? g1 : 0.0;
      sg[2] = (op2 && t < 3) ? g2 : 0.0;
      dg[0] = (op && t < 3) ? h0 : 0.0;
      dg[1] = (op2 && t < 3) ? h1 : 0.0;
      dg[2] = (op && t < 3) ? h2 : 0.0;
#pragma unroll
      for (int j = 0; j < 7; ++j) {
        const int row = f - 3 + j;
        sx[j] = (row >= 0 && row <= d.M - 1) ? xr[j] : 0.0;
      }
    } else if (t >= S0 && t < S0 + nS1) {
      // off-diagonal entries (r, c < 3, c != r) of block dd = 0 (prev and prev2 terms) and dd = 1
      // (prev), then rows < 3 of B (prev and prev2): prev at column P + ca of row P + r, prev2 at
      // column P + cb of row P + 3 + r
      const int w = t - S0;
      int r, ca, cb;
      bool p2on;
      if (w < 12) {
        const int dd = w / 6, ww = w % 6;
        r = ww / 2;
        const int c = (ww % 2 < r) ? ww % 2 : ww % 2 + 1;  // c != r
        se = dd * PP + r * P + c;
        ca = dd == 0 ? c : 3 + c;
        cb = 3 + c;
        p2on = dd == 0;
      } else {
        const int wb = w - 12;
        r = wb / Cg;
        const int c = wb - r * Cg;
        se = 4 * PP + wb;
        ca = 6 + c;
        cb = 6 + c;
        p2on = true;
      }
      const double a1 = Hp[(P + r) * FTE_NZP + P + ca], a2 = Hp2[(P + 3 + r) * FTE_NZP + P + cb];
      dg[0] = op ? a1 : 0.0;
      dg[1] = (op2 && p2on) ? a2 : 0.0;
    }
  } else {
    // the 1,024-thread rows (and k_fte_assemble) keep the branch per special kind: the
    // regrouped form above costs them 6 spilled VGPRs within 64, and 17.3 -> 17.9 us at 1,000
    // frames (profiles/r06/fte_kernel_totals_*_r06ze.log)
    const int nOff = P + 12, nS = nOff + 3 * Cg;
    if (t < P) {
      sg[0] = oo ? gloc[(size_t)kown * FTE_NZP + t] : 0.0;
      if (t < 3) {
        sg[1] = op ? gloc[(size_t)kprev * FTE_NZP + P + t] : 0.0;
        sg[2] = op2 ? gloc[(size_t)kprev2 * FTE_NZP + P + 3 + t] : 0.0;
        dg[0] = op ? Hp[(P + t) * FTE_NZP + P + t] : 0.0;           // block 0, prev
        dg[1] = op2 ? Hp2[(P + 3 + t) * FTE_NZP + P + 3 + t] : 0.0;  // block 0, prev2
        dg[2] = op ? Hp[(P + t) * FTE_NZP + P + 3 + t] : 0.0;       // block 1, prev
      }
      sq = qinv[t];
#pragma unroll
      for (int j = 0; j < 7; ++j) {  // rows f - 3 .. f + 3
        const int row = f - 3 + j;
        sx[j] = (row >= 0 && row <= d.M - 1) ? X[(size_t)row * P + t] : 0.0;
      }
    } else if (t < nOff) {
      const int dd = (t - P) / 6, w = (t - P) % 6, r = w / 2, c = (w % 2 < r) ? w % 2 : w % 2 + 1;  // c != r
      se = dd * PP + r * P + c;
      if (dd == 0) {
        dg[0] = op ? Hp[(P + r) * FTE_NZP + P + c] : 0.0;
        dg[1] = op2 ? Hp2[(P + 3 + r) * FTE_NZP + P + 3 + c] : 0.0;
      } else {
        dg[0] = op ? Hp[(P + r) * FTE_NZP + P + 3 + c] : 0.0;
      }
    } else if (t < nS) {
      const int w = t - nOff, r = w / Cg, c = w % Cg;
      se = 4 * PP + w;
      dg[0] = op ? Hp[(P + r) * FTE_NZP + P + 6 + c] : 0.0;
      dg[1] = op2 ? Hp2[(P + 3 + r) * FTE_NZP + P + 6 + c] : 0.0;
    }
  }
  // entries with an own term (block 0, columns < 3 of blocks 1, 2, and B): loads of a batch
  // before its stores (k_fte_assemble's A is global memory)
  const int n1 = PP + 6 * P, n2 = n1 + P * Cg;
  constexpr int NBT = 4;
  for (int e0 = t; e0 < n2; e0 += NBT * nth) {
    double ov[NBT];
#pragma unroll
    for (int j = 0; j < NBT; ++j) {
      // the entry's offset in the own block by selects, then one unconditional load from a valid
      // address (frame 0's block when not owned, offset 0 past the row's entries) and a select:
      // a load per branch made the compiler wait for each before the next (k_cr_assemble_build's
      // ISA), four round trips per batch instead of one
      const int u = e0 + j * nth;
      int r, col;
      if (u < PP) {
        r = u / P;
        col = u - r * P;
      } else if (u < n1) {
        const int w = u - PP;  // block 1 + cc / 3, column cc % 3
        r = w / 6;
        col = P + (w - 6 * r);
      } else {
        const int w = u - n1;
        r = w / (Cg > 0 ? Cg : 1);
        col = P + 6 + (w - r * Cg);
      }
      ov[j] = Ho[u < n2 ? r * FTE_NZP + col : 0];
    }
    // every load of the batch issued before the first use: the compiler otherwise moved each
    // load under its select's condition and waited for it there (the compact-row instance only:
    // the 1,024-thread rows measured 17.1 -> 17.5 us at 1,000 frames with it, r06ze2)
    if constexpr (CMP) {
#pragma unroll
      for (int j = 0; j < NBT; ++j) asm volatile("" ::"v"(ov[j]));
    }
#pragma unroll
    for (int j = 0; j < NBT; ++j) ov[j] = (oo && e0 + j * nth < n2) ? ov[j] : 0.0;
#pragma unroll
    for (int j = 0; j < NBT; ++j) {
      const int u = e0 + j * nth;
      if (u >= n2) break;
      double v = 0.0;
      v += ov[j];
      if (u < PP) {
        A[u] = v;
      } else if (u < n1) {
        const int w = u - PP, r = w / 6, cc = w - 6 * r;
        if constexpr (CMP)
          A[PP + 3 * P * (cc / 3) + 3 * r + cc % 3] = v;
        else
          A[(1 + cc / 3) * PP + r * P + cc % 3] = v;
      } else {
        B[u - n1] = v;
      }
    }
  }
  // entries with no own term: columns >= 3 of blocks 1, 2, and block 3 (the compact rows keep
  // only their diagonals, which the second round writes)
  const int Q = P * (P - 3), n3 = CMP ? 0 : 2 * Q + PP;
  for (int u = t; u < n3; u += nth) {
    int e;
    if (u < 2 * Q) {
      const int dd = 1 + u / Q, w = u - (dd - 1) * Q, r = w / (P - 3), c = 3 + w - r * (P - 3);
      e = dd * PP + r * P + c;
    } else {
      e = 3 * PP + (u - 2 * Q);
    }
    A[e] = 0.0;
  }
  if (t < P) {  // the gradient entry: own, prev, prev2, then the model term's stencils
    double gm = 0.0;
    for (int i = 0; i < 4; ++i) {
      if (!mvalid(i)) continue;
      // stencil m = f + i reads rows m .. m - 3 = sx[i + 3] .. sx[i]
      const double sm = (sx[i + 3] - 3.0 * sx[i + 2] + 3.0 * sx[i + 1] - sx[i]) * its2;
      gm += 2.0 * sq * cf[i] * its2 * sm;
    }
    double v = 0.0;
    v += sg[0];
    v += sg[1];
    v += sg[2];
    v += gm;
    g[t] = v;
  }
  __syncthreads();
  if (t < P) {
#pragma unroll
    for (int dd = 0; dd < 4; ++dd) {
      double* a = A + (CMP ? RowCmp::at(P, dd, t, t) : dd * PP + t * P + t);
      // (compact rows: the diagonal of blocks 1, 2 past row 2 and of block 3 was not stored)
      double v = (CMP && dd > 0 && (dd == 3 || t >= 3)) ? 0.0 : *a;
      if (dd == 0) {
        v += dg[0];
        v += dg[1];
      } else if (dd == 1) {
        v += dg[2];
      }
      double h = 0.0;  // the model term's diagonal entry (stencils in ascending order)
      for (int i = 0; i + dd < 4; ++i)
        if (mvalid(i)) h += 2.0 * sq * cf[i] * cf[i + dd] * its2 * its2;
      v += h;
      *a = v;
    }
  } else if (se >= 0) {
    int ea = se;
    if (CMP && se < 4 * PP) {
      const int dd = se / PP, r = (se - dd * PP) / P;
      ea = RowCmp::at(P, dd, r, se - dd * PP - r * P);
    }
    double* a = se < 4 * PP ? A + ea : B + (se - 4 * PP);
    double v = *a;
    v += dg[0];
    v += dg[1];
    *a = v;
  }
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_fte_assemble(FteDims d, const double* __restrict__ Xbuf,
                                                      const double* __restrict__ taubuf,
                                                      const double* __restrict__ qinv,
                                                      const FteState* __restrict__ st, int force, int f0, int lo,
                                                      int hi, const double* __restrict__ Hloc,
                                                      const double* __restrict__ gloc, double* __restrict__ Ab,
                                                      double* __restrict__ gb, double* __restrict__ Bt,
                                                      double* __restrict__ gmaxp, double* __restrict__ Adiag,
                                                      int hsel, double* __restrict__ graw = nullptr,
                                                      double* __restrict__ gmaxt = nullptr) {
  // Terms are owned by the lowest X row they touch: frame k (rows k..k+2) iff lo <= k < hi,
  // model stencil m (rows m-3..m) iff lo <= m-3 < hi. The single-GPU solve owns all terms;
  // a frame-window rank owns the terms starting in its window (dist path below).
  // Variable shutter delay (force == 0): the per-frame delays are eliminated here, every
  // iteration (the damping changes): block (f, f') -= sum_c h_c h_c'^T / T_c and
  // g_f -= sum_c h_c g_c / T_c over the frames touching row f, T_c = H_cc + lam max(H_cc,
  // 1e-12) (oracle damping), held delays skipped; Adiag keeps the raw diagonal for k_cr_build.
  // (The single-GPU const / no-delay solve assembles inside k_cr_assemble_build instead.)
  const bool elim = d.var && !force;
  if (!force && (st->status != 0 || (!st->relin && !elim))) return;
  if (hsel) {  // the linearisation of X[cur] (double-buffered by the speculative solve)
    Hloc += (size_t)st->cur * d.N * FTE_NZP * FTE_NZP;
    gloc += (size_t)st->cur * d.N * FTE_NZP;
  }
  const int f = blockIdx.x + f0;
  const int tid = threadIdx.x, nth = blockDim.x;
  const int P = d.P, Cg = d.Cg, N = d.N, C = d.C;
  const int cur = force ? 0 : st->cur;
  const double* X = Xbuf + (size_t)cur * d.M * P;
  double* A = Ab + (size_t)f * 4 * P * P;
  double* g = gb + (size_t)f * P;
  double* B = Bt + (size_t)f * P * Cg;
  __shared__ double s_red[256];
  __shared__ double s_ti[3][FTE_MAXC], s_tg[3][FTE_MAXC];
  auto owned = [&](int k) { return k >= 0 && k < N && k >= lo && k < hi; };
  const int kown = f - 2, kprev = f - 1, kprev2 = f;
  if (d.var && tid < 3 * C) {
    // j = 0, 1, 2: frames kown, kprev, kprev2
    const int j = tid / C, c = tid - j * C, k = f - 2 + j;
    double ti = 0.0, tg = 0.0;
    if (owned(k)) {
      const double* H = Hloc + (size_t)k * FTE_NZP * FTE_NZP;
      const double t = taubuf[(size_t)cur * d.NT + (size_t)k * C + c];
      tg = gloc[(size_t)k * FTE_NZP + P + 6 + c];
      if (tau_held(t, tg, d.Ts, c)) {
        tg = 0.0;
      } else if (elim) {
        const double h = H[(P + 6 + c) * FTE_NZP + P + 6 + c];
        ti = 1.0 / (h + st->lam * fmax(h, 1e-12));
      }
    }
    s_ti[j][c] = ti;
    s_tg[j][c] = tg;
  }
  assemble_row<false>(d, f, X, qinv, lo, hi, Hloc, gloc, A, g, B, tid, nth);
  double mx = 0.0;
  for (int i = tid; i < P; i += nth) mx = fmax(mx, fabs(g[i]));
  double mt = 0.0;
  if (d.var)
    for (int c = tid; c < C; c += nth) mt = fmax(mt, fabs(s_tg[0][c]));  // each frame once (kown)
  mx = block_max(fmax(mx, mt), s_red);
  if (tid == 0) gmaxp[f] = mx;
  if (gmaxt) {
    mt = block_max(mt, s_red);
    if (tid == 0) gmaxt[f] = mt;
  }
  if (graw)
    for (int i = tid; i < P; i += nth) graw[(size_t)f * P + i] = g[i];
  if (!elim) return;
  for (int i = tid; i < P; i += nth) Adiag[(size_t)f * P + i] = A[i * P + i];
  __syncthreads();
  // Schur terms of the delays of frame k: rows / columns i, j of its local block
  auto corr = [&](const double* H, int jj, int i, int j) {
    double v = 0.0;
    for (int c = 1; c < C; ++c) v += s_ti[jj][c] * H[i * FTE_NZP + P + 6 + c] * H[j * FTE_NZP + P + 6 + c];
    return v;
  };
  auto gcorr = [&](const double* H, int jj, int i) {
    double v = 0.0;
    for (int c = 1; c < C; ++c) v += s_ti[jj][c] * H[i * FTE_NZP + P + 6 + c] * s_tg[jj][c];
    return v;
  };
  if (owned(kown)) {
    const double* H = Hloc + (size_t)kown * FTE_NZP * FTE_NZP;
    for (int i = tid; i < P * P; i += nth) {
      const int r = i / P, c = i % P;
      A[r * P + c] -= corr(H, 0, r, c);
    }
    for (int i = tid; i < P * 3; i += nth) {
      const int r = i / 3, c = i % 3;
      A[1 * P * P + r * P + c] -= corr(H, 0, r, P + c);
      A[2 * P * P + r * P + c] -= corr(H, 0, r, P + 3 + c);
    }
    for (int i = tid; i < P; i += nth) g[i] -= gcorr(H, 0, i);
  }
  __syncthreads();
  if (owned(kprev)) {
    const double* H = Hloc + (size_t)kprev * FTE_NZP * FTE_NZP;
    for (int i = tid; i < 9; i += nth) {
      const int r = i / 3, c = i % 3;
      A[r * P + c] -= corr(H, 1, P + r, P + c);
      A[1 * P * P + r * P + c] -= corr(H, 1, P + r, P + 3 + c);
    }
    for (int i = tid; i < 3; i += nth) g[i] -= gcorr(H, 1, P + i);
  }
  __syncthreads();
  if (owned(kprev2)) {
    const double* H = Hloc + (size_t)kprev2 * FTE_NZP * FTE_NZP;
    for (int i = tid; i < 9; i += nth) {
      const int r = i / 3, c = i % 3;
      A[r * P + c] -= corr(H, 2, P + 3 + r, P + 3 + c);
    }
    for (int i = tid; i < 3; i += nth) g[i] -= gcorr(H, 2, P + 3 + i);
  }
}

// ---------------------------------------------------------------------------------------
// 3-6. block cyclic reduction on 3-frame super-blocks
//
// Frames are grouped into n = ceil(M/3) super-blocks of B = 3P unknowns (padded to BP, a
// multiple of 16; padding rows are identity). With bandwidth 3 the normal matrix is block
// tridiagonal in super-blocks: D_i (diagonal) and E_i = T(i, i-1), plus the tau border
// G_i and rhs b_i = -g_i packed as GB_i = [G_i | b_i] (BP x GR). Level s (= 1, 2, 4, ..)
// eliminates the active blocks i = s(2m+1) in parallel (k_cr_level):
//   W_i = D_i^-1 [E_i | E_{i+s}^T | GB_i]      (register-tiled Gauss-Jordan, MFMA)
// and every survivor j = 2sm receives the Schur terms of its eliminated neighbours
// a = j - s and c = j + s:
//   D_j -= E_j W_r(a) + E_c^T W_l(c),  GB_j -= E_j W_gb(a) + E_c^T W_gb(c),
//   E_j <- -E_j W_l(a)   (new coupling to the next active block on the left)
// (formed by the eliminating workgroups, applied when j is next loaded) until only block 0
// is left; k_cr_top solves block 0 with the tau border (tau Schur sum
// over every eliminated block, fixed order), and k_cr_back substitutes the levels back:
//   delta_i = W_b(i) - W_l(i) delta_{i-s} - W_r(i) delta_{i+s} - W_g(i) delta_tau.
// All sums are in a fixed order, so the solve is deterministic run to run.
// ---------------------------------------------------------------------------------------
#define CR_MAXBP 96

#ifdef FTE_PROFILE  // per-phase wall-clock ticks (100 MHz) of block 0 (tools/prof_fte_phases.py)
// the timeline (PROFA) of the deep levels, or with -DFTE_PROF_WIDE=n of the levels with at
// least n elimination workgroups (tools/prof_cr_timeline.py)
#ifdef FTE_PROF_WIDE
#ifndef FTE_PROF_WIDE_MAX
#define FTE_PROF_WIDE_MAX 1000000
#endif
#define PROF_ON_LEVEL(nwg) ((nwg) >= FTE_PROF_WIDE && (nwg) <= FTE_PROF_WIDE_MAX)
#else
#define PROF_ON_LEVEL(nwg) ((nwg) <= 12)
#endif
#define PROF_T0 unsigned long long t_prof = wall_clock64(); const unsigned long long t_start = t_prof; \
  const bool prof_on = ne > 0 && PROF_ON_LEVEL(ne * nsplit);
// timeline event: wave w of block 0 at time since the kernel start (deep levels only)
#define PROFA(slot, w)                                                      \
  do {                                                                      \
    if (prof_on && blockIdx.x == 0 && threadIdx.x == 64 * (w))              \
      atomicAdd(&g_fte_prof[slot], wall_clock64() - t_start);               \
  } while (0)
#define PROF(slot)                                                          \
  do {                                                                      \
    __syncthreads();                                                        \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                              \
      const unsigned long long t_now = wall_clock64();                      \
      atomicAdd(&g_fte_prof[slot], t_now - t_prof);                         \
      t_prof = t_now;                                                       \
    }                                                                       \
  } while (0)
// no barrier: lane 0 of wave w of block 0 (time since its own previous mark)
#define PROFW(slot, w)                                                      \
  do {                                                                      \
    if (blockIdx.x == 0 && threadIdx.x == 64 * (w)) {                       \
      const unsigned long long t_now = wall_clock64();                      \
      atomicAdd(&g_fte_prof[slot], t_now - t_prof);                         \
      t_prof = t_now;                                                       \
    }                                                                       \
  } while (0)
#else
#define PROF_T0
#define PROF(slot)
#define PROFW(slot, w)
#define PROFA(slot, w)
#endif

template <int NB>
__global__ __launch_bounds__(1024) void k_cr_build(FteDims d, const FteState* __restrict__ st,
                                                   const double* __restrict__ Ab, const double* __restrict__ gb,
                                                   const double* __restrict__ Bt, double* __restrict__ Dc,
                                                   double* __restrict__ Ec, double* __restrict__ GBc, int b0,
                                                   int end_l, int end_r, const double* __restrict__ Adiag) {
  if (st->status != 0) return;
  constexpr int BP = 16 * NB, NE = (BP * BP + 1023) / 1024;
  const int i = blockIdx.x + b0, tid = threadIdx.x;
  const bool damp = i != end_l && i != end_r;  // chain ends are damped in the reduced system
  const int P = d.P, PP = P * P, GR = d.GR, Cg = d.Cg;
  const double lam = st->lam;
  double* D = Dc + (size_t)i * BP * BP;
  double* E = Ec + (size_t)i * BP * BP;
  double* G = GBc + (size_t)i * BP * GR;
  __shared__ int s_a[BP], s_p[BP];  // super-block row/col -> (frame in block, parameter)
  if (tid < BP) {
    s_a[tid] = tid / P;
    s_p[tid] = tid - (tid / P) * P;
  }
  __syncthreads();
  double dv[NE], ev[NE];
#pragma unroll
  for (int q = 0; q < NE; ++q) {
    const int e = tid + 1024 * q;
    const int r = e / BP, c = e - (e / BP) * BP;
    dv[q] = 0.0;
    ev[q] = 0.0;
    if (e >= BP * BP) continue;
    const int ar = s_a[r], pr = s_p[r], ac = s_a[c], pc = s_p[c];
    const int fr = 3 * i + ar, fc = 3 * i + ac;
    const bool rin = r < 3 * P && fr < d.M, cin = c < 3 * P && fc < d.M;
    if (rin && cin) {
      double v = (ar >= ac) ? Ab[(size_t)fr * 4 * PP + (ar - ac) * PP + pr * P + pc]
                            : Ab[(size_t)fc * 4 * PP + (ac - ar) * PP + pc * P + pr];
      if (r == c && damp) v += lam * fmax(Adiag ? Adiag[(size_t)fr * P + pr] : v, 1e-12);
      dv[q] = v;
    } else if (r == c) {
      dv[q] = 1.0;  // padding: identity
    }
    // E_i = T(block i, block i-1): frames 3i+ar vs 3(i-1)+ac, distance 3 + ar - ac <= 3
    const int fe = 3 * (i - 1) + ac;
    if (i > 0 && rin && c < 3 * P && fe < d.M) {
      const int dist = 3 + ar - ac;
      if (dist <= 3) ev[q] = Ab[(size_t)fr * 4 * PP + dist * PP + pr * P + pc];
    }
  }
#pragma unroll
  for (int q = 0; q < NE; ++q) {
    const int e = tid + 1024 * q;
    if (e < BP * BP) {
      D[e] = dv[q];
      E[e] = ev[q];
    }
  }
  for (int e = tid; e < BP * GR; e += blockDim.x) {
    const int r = e / GR, c = e - (e / GR) * GR;
    const int pr = s_p[r], fr = 3 * i + s_a[r];
    double v = 0.0;
    if (r < 3 * P && fr < d.M) {
      if (c < Cg)
        v = Bt[(size_t)fr * P * Cg + pr * Cg + c];
      else if (c == Cg)
        v = -gb[(size_t)fr * P + pr];
    }
    G[e] = v;
  }
}

// k_fte_assemble + k_cr_build in one pass for the single-GPU solve without per-frame delays
// (d.var == 0): super-block i assembles its three banded rows f = 3i + a (one group of 320
// threads per row) into LDS and builds D_i, E_i, GB_i from there, so the banded rows never
// make an HBM round trip. Same arithmetic and order as the two kernels, so the same bits.
// Runs every iteration (the damping changes on a rejected step; the rows are then
// re-assembled from the unchanged linearisation).
// Frame-window ranks (dist path): blocks b0 + blockIdx.x of the chain, only the terms the
// rank owns (lowest row in [lo, hi)), the chain ends end_l / end_r left undamped (they are
// damped in the reduced system with the summed raw diagonals), and the raw diagonal and
// gradient of every row written to rdiag / graw (row layout f P + p) for the payload.
// TH threads per block (16 x 16 TH / 1024 waves per SIMD's register budget): 1024 when the grid
// fits the chip in one round of two blocks per CU (each row assembled by 320 threads: the
// shortest block), 512 for larger grids (four blocks per CU hide each other's latency:
// 10,000 frames 111.8 -> 99.4 us; at 1,000 frames the 512-thread block takes 21.9 us against
// 17.8, profiles/r06/fte_kernel_totals_*_r06y.log)
template <int NB, int TH>
__global__ __launch_bounds__(TH) __attribute__((amdgpu_waves_per_eu(8))) void k_cr_assemble_build(
    FteDims d, const double* __restrict__ Xbuf, const double* __restrict__ qinv, const FteState* __restrict__ st,
    const double* __restrict__ Hloc, const double* __restrict__ gloc, double* __restrict__ Dc,
    double* __restrict__ Ec, double* __restrict__ GBc, double* __restrict__ gmaxp, int b0, int lo, int hi,
    int end_l, int end_r, double* __restrict__ rdiag, double* __restrict__ graw, int d_full) {
  if (st->status != 0) return;
  constexpr int BP = 16 * NB;
  const int i = blockIdx.x + b0, tid = threadIdx.x;
  const bool damp = i != end_l && i != end_r;
  const int P = d.P, GR = d.GR, Cg = d.Cg;
  const int cur = st->cur;
  Hloc += (size_t)cur * d.N * FTE_NZP * FTE_NZP;
  gloc += (size_t)cur * d.N * FTE_NZP;
  const double* X = Xbuf + (size_t)cur * d.M * P;
  const double lam = st->lam;
  extern __shared__ double lds[];
  // per row: A (4 P x P; CMP: the compact layout, RowCmp), g (P), B (P x Cg). CMP (the 512-thread
  // instance): 26 KB for the three rows at P = 26, six cameras instead of 69 KB, so four blocks
  // share a CU. The 1024-thread instance keeps the full rows: the compact layout's index
  // arithmetic cost it 17.3 -> 19.5 us per block (profiles/r06/fte_kernel_totals_*_r06z.log).
  constexpr bool CMP = TH < 1024;
  const int asz = CMP ? RowCmp::size(P) : 4 * P * P;
  const int rowsz = asz + P + P * Cg;
  auto rowA = [&](int a) { return lds + (size_t)a * rowsz; };
  auto rowg = [&](int a) { return lds + (size_t)a * rowsz + asz; };
  auto rowB = [&](int a) { return lds + (size_t)a * rowsz + asz + P; };
  // block (dd) entry (r, c) of row a (zero where the compact layout stores nothing)
  auto rowAt = [&](int a, int dd, int r, int c) {
    if constexpr (CMP) {
      const int e = RowCmp::at(P, dd, r, c);
      return e >= 0 ? rowA(a)[e] : 0.0;
    } else {
      return rowA(a)[dd * P * P + r * P + c];
    }
  };
  __shared__ int s_a[BP], s_p[BP];
  for (int r = tid; r < BP; r += blockDim.x) {
    s_a[r] = r / P;
    s_p[r] = r - (r / P) * P;
  }
  {
    constexpr int GT = TH / 3 / 32 * 32;  // threads per row (320, 160)
    const int grp = tid / GT, a = grp < 3 ? grp : 0;
    const int f = 3 * i + a;
    const bool act = grp < 3 && f < d.M;
    // inactive threads (the spare ones, rows past the sequence) start past every loop
    assemble_row<CMP>(d, f, X, qinv, lo, hi, Hloc, gloc, rowA(a), rowg(a), rowB(a), act ? tid - GT * grp : 1 << 30,
                      GT);
  }
  if (rdiag && tid < 3 * d.P) {
    const int a = tid / d.P, p = tid - a * d.P, f = 3 * i + a;
    if (f < d.M) {
      rdiag[(size_t)f * d.P + p] = rowA(a)[p * d.P + p];
      graw[(size_t)f * d.P + p] = rowg(a)[p];
    }
  }
  // |g| max of each row (max is order-free): wave a < 3 takes row 3i + a
  if (tid < 192) {
    const int a = tid >> 6, lane = tid & 63, f = 3 * i + a;
    double mx = 0.0;
    for (int p = lane; p < P; p += 64) mx = fmax(mx, fabs(rowg(a)[p]));
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
    if (lane == 0 && f < d.M) gmaxp[f] = mx;
  }
  double* D = Dc + (size_t)i * BP * BP;
  double* E = Ec + (size_t)i * BP * BP;
  double* G = GBc + (size_t)i * BP * GR;
  constexpr int NE = (BP * BP + TH - 1) / TH;
#pragma unroll
  for (int q = 0; q < NE; ++q) {
    const int e = tid + TH * q;
    if (e >= BP * BP) continue;
    const int r = e / BP, c = e - (e / BP) * BP;
    const int ar = s_a[r], pr = s_p[r], ac = s_a[c], pc = s_p[c];
    const int fr = 3 * i + ar, fc = 3 * i + ac;
    const bool rin = r < 3 * P && fr < d.M, cin = c < 3 * P && fc < d.M;
    double dv = 0.0, ev = 0.0;
    if (rin && cin) {
      double v = (ar >= ac) ? rowAt(ar, ar - ac, pr, pc) : rowAt(ac, ac - ar, pc, pr);
      if (r == c && damp) v += lam * fmax(v, 1e-12);
      dv = v;
    } else if (r == c) {
      dv = 1.0;  // padding: identity
    }
    // E_i = T(block i, block i-1): frames 3i+ar vs 3(i-1)+ac, distance 3 + ar - ac <= 3
    const int fe = 3 * (i - 1) + ac;
    if (i > 0 && rin && c < 3 * P && fe < d.M) {
      const int dist = 3 + ar - ac;
      if (dist <= 3) ev = rowAt(ar, dist, pr, pc);
    }
    // D is symmetric by construction (element (r, c) and (c, r) are the same row-block entry):
    // the single-GPU solve stores its upper 16 x 16 tiles only and the levels that read it as
    // assembled (k_cr_level d_up) take the lower ones from the transposed tile; the frame-window
    // ranks (rdiag set: k_dist_pack copies chain ends whole) and d_full store every tile
    if (rdiag || d_full || (r >> 4) <= (c >> 4)) D[e] = dv;
    // E_i is upper triangular (frame distance 3 + ar - ac <= 3, and the distance-3 blocks are
    // the model term's diagonal): in the single-GPU solve its strictly lower 16 x 16 tiles are
    // not stored; level 0 of k_cr_level, their only reader there, takes them as zeros
    // (cr_reduce's e_upper). The frame-window ranks (rdiag set) store every tile: k_dist_pack
    // copies a chain end's E as it is.
    if (rdiag || (r >> 4) <= (c >> 4)) E[e] = ev;
  }
  for (int e = tid; e < BP * GR; e += blockDim.x) {
    const int r = e / GR, c = e - (e / GR) * GR;
    const int pr = s_p[r], ar = s_a[r], fr = 3 * i + ar;
    double v = 0.0;
    if (r < 3 * P && fr < d.M) {
      if (c < Cg)
        v = rowB(ar)[pr * Cg + c];
      else if (c == Cg)
        v = -rowg(ar)[pr];
    }
    G[e] = v;
  }
}

static size_t asm_build_lds_bytes(const FteDims& d, bool cmp) {
  return sizeof(double) * 3 * (size_t)((cmp ? RowCmp::size(d.P) : 4 * d.P * d.P) + d.P + d.P * d.Cg);
}

static void cr_launch_build(const FteDims& d, hipStream_t s, int nblk, const FteState* st, const double* Ab,
                            const double* gb, const double* Bt, double* Dc, double* Ec, double* GBc, int b0,
                            int end_l, int end_r, const double* Adiag) {
  if (nblk <= 0) return;
#define CR_BUILD(nb)                                                                                          \
  hipLaunchKernelGGL((k_cr_build<nb>), dim3(nblk), dim3(1024), 0, s, d, st, Ab, gb, Bt, Dc, Ec, GBc, b0, end_l, \
                     end_r, Adiag)
  switch (d.BP >> 4) {
    case 1: CR_BUILD(1); break;
    case 2: CR_BUILD(2); break;
    case 3: CR_BUILD(3); break;
    case 4: CR_BUILD(4); break;
    case 5: CR_BUILD(5); break;
    default: CR_BUILD(6); break;
  }
#undef CR_BUILD
}

// Fixed-order partial sums feeding the tau border (parallel over chunks, summed in chunk
// order by k_cr_top): per-frame tau blocks of the normal matrix / gradient, and the tau
// Schur contributions of every eliminated super-block.
#define CR_NCHUNK 64
// chunk `ch` of the partial sums; `store(e, v)` writes element e of the chunk's row of `part`
template <typename Store>
__device__ __forceinline__ void cr_tau_partial_chunk(const FteDims& d, const FteState* __restrict__ st,
                                                     const double* __restrict__ Hloc, const double* __restrict__ gloc,
                                                     const double* __restrict__ Tau, int k_lo, int k_hi, int b_lo,
                                                     int b_hi, int hsel, const double* __restrict__ Tc, int ch,
                                                     Store store) {
  // frames [k_lo, k_hi) (tau blocks of their normal matrices / gradients) and eliminated
  // super-blocks [b_lo, b_hi) (tau Schur terms), each range cut into CR_NCHUNK chunks
  if (hsel) {
    Hloc += (size_t)st->cur * d.N * FTE_NZP * FTE_NZP;
    gloc += (size_t)st->cur * d.N * FTE_NZP;
    if (Tc) Tc += (size_t)st->cur * d.N * tc_stride(d.Cg);
  }
  const int P = d.P, Cg = d.Cg, GR = d.GR;
  const int nH = Cg * Cg, nE = nH + Cg + GR * GR;
  const int nf = max(0, k_hi - k_lo), nb = max(0, b_hi - b_lo);
  const int fc = (nf + CR_NCHUNK - 1) / CR_NCHUNK, bc = (nb + CR_NCHUNK - 1) / CR_NCHUNK;
  const int k0 = k_lo + ch * fc, k1 = min(k_hi, k0 + fc);
  const int b0 = b_lo + ch * bc, b1 = min(b_hi, b0 + bc);
  // 16 loads in flight per thread (the frame / block loops are strided gathers: at 10,000
  // frames a chunk's 157 frames took 20 rounds of 8, ~22 us), summed in index order (the
  // same bits as any batch size)
  auto sum8 = [](const double* base, size_t stride, int lo, int hi) {
    double v = 0.0;
    for (int k = lo; k < hi; k += 16) {
      double t[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) t[q] = k + q < hi ? base[(size_t)(k + q) * stride] : 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q) v += t[q];
    }
    return v;
  };
  for (int e = threadIdx.x; e < nE; e += blockDim.x) {
    double v;
    if (Tc && e < nH + Cg) {
      v = sum8(Tc + e, (size_t)tc_stride(Cg), k0, k1);  // compact copy from k_fte_linearize
    } else if (e < nH) {
      const int r = e / Cg, c = e % Cg;
      v = sum8(Hloc + (P + 6 + r) * FTE_NZP + P + 6 + c, (size_t)FTE_NZP * FTE_NZP, k0, k1);
    } else if (e < nH + Cg) {
      v = sum8(gloc + P + 6 + (e - nH), FTE_NZP, k0, k1);
    } else {
      v = sum8(Tau + (e - nH - Cg), (size_t)GR * GR, b0, b1);
    }
    store(e, v);
  }
}

// the top level's extra workgroups (cr_launch_top with partials): the tau partial sums of the
// single-GPU solve, computed while the top block is eliminated (k_cr_back_all's top then
// adds the top block's own Tau last)
struct CrTauSrc {
  const double* Tc;
  const double* gmaxp;
  double* part;
};

// the top level's extra workgroups (k_cr_level, top_mode, blockIdx.x = 1 + chunk): chunk
// `ch` of the tau partial sums (every frame, every eliminated block but the top one, a0 = 0;
// consecutive threads read consecutive elements) and of the frames' |g| max, as row ch of
// part (nE + 1 wide). (One wave per element, lanes over the frames, took 130 us at 10,000
// frames: every load instruction touched 64 lines.)
__device__ __forceinline__ void cr_top_border_sums(const FteDims& d, const FteState* __restrict__ st,
                                                   const double* __restrict__ Tau, const CrTauSrc& tsrc) {
  const int ch = (int)blockIdx.x - 1, nE = d.Cg * d.Cg + d.Cg + d.GR * d.GR;
  double* row = tsrc.part + (size_t)ch * (nE + 1);
  cr_tau_partial_chunk(d, st, nullptr, nullptr, Tau, 0, d.N, 1, d.nblk, 1, tsrc.Tc, ch,
                       [&](int e, double v) { row[e] = v; });
  if (threadIdx.x < 64) {
    const int fm = (d.M + CR_NCHUNK - 1) / CR_NCHUNK, f0 = ch * fm, f1 = min(d.M, f0 + fm);
    double mx = strided_max(tsrc.gmaxp, f0 + (int)threadIdx.x, f1, 64, 0.0);
#pragma unroll
    for (int h = 32; h > 0; h >>= 1) mx = fmax(mx, __shfl_xor(mx, h, 64));
    if (threadIdx.x == 0) row[nE] = mx;
  }
}

// One reduction level: workgroups [0, ne * nsplit) eliminate the blocks i = a0 + s(2m+1)
// (< iend), workgroups after them apply the pending Schur terms to the survivors
// j = a0 + astep m (<= top). Pending terms are applied lazily, and at the wide levels not at
// every level: the terms of the levels with steps lo_s, 2 lo_s, .., s/2 have not reached the
// blocks yet (no survivor workgroups were launched for them: they would have cost whole
// extra rounds of 1024-thread workgroups), so an eliminated block or a survivor subtracts
// them all, level by level in ascending order (symmask bit l: the level of step 2^l stored its
// D parts as upper tiles). 1024 threads = 16 waves, register-tiled (16x16 f64 MFMA tiles):
//   waves 0 .. NB-1  hold the row-blocks of D_i,
//   waves NB ..      hold one column-block each of [E_i | E_r^T | GB_i] (r = i + s);
// Gauss-Jordan elimination on that augmented matrix leaves W_i = D_i^-1 [E_i | E_r^T | GB_i]
// in the column waves' registers after NB steps, one barrier per step (the pivot inverse,
// the new pivot row and the old pivot column travel through double-buffered LDS).
// `nsplit` workgroups share one block: each repeats the (cheap) D part and owns the
// column-blocks J = part mod nsplit, which spreads the MFMA work of the few blocks of the
// deep levels over more CUs (and is required when 2NB + GR/16 > 16 - NB).
// The column waves then form this block's Schur terms for its neighbours (MFMA, A operand
// from LDS copies of the coupling blocks, B operand = the W tiles in registers); every
// output column depends on one W column only:
//   dL_i = E_i^T [W_l | W_gb]  (-> left survivor l = i - s),
//   dR_i = E_r   [W_r | W_gb]  (-> right survivor r),   E_r <- -E_r W_l  (next level's E),
//   Tau_i = GB_i^T W_gb.
// Survivors accumulate them lazily: a block applies dR_{j-s/2} + dL_{j+s/2} when it is
// loaded at the next level (or by an apply workgroup), so a level is one launch.
// E_r staged in LDS beside E_i: room for both coupling copies only up to BP = 80 with one
// column-block of GB (GR = 16: up to 15 cameras with a constant shutter delay); otherwise
// E_r is read from global memory (k_cr_level's sEr == nullptr path)
__host__ __device__ __forceinline__ bool cr_er_lds(int NB, int GR) { return NB <= 5 && GR <= 16; }
__host__ __device__ __forceinline__ size_t cr_level_lds_doubles(int BP, int GR) {
  return 2 * (16 * 17 + 16 * (size_t)BP + 17 * (size_t)BP) + (size_t)BP * GR +
         (cr_er_lds(BP >> 4, GR) ? 2 * (size_t)BP + 1 : (size_t)BP) * BP;
}

// GB2: the instance for two GB column-blocks (GR = 32, 16 constant delays; the host picks it
// by d.GR), so the GR = 16 instances carry none of its code
// Wave-to-wave hand-off inside a workgroup through an LDS word: the producer's LDS stores land
// (lgkmcnt 0) before the flag; the consumer spins on the flag, then reads (LDS ops of a wave
// execute in order).
__device__ __forceinline__ void cr_flag_set(int* f, int v) {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt / expcnt not waited for
  __hip_atomic_store(f, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void cr_flag_wait(const int* f, int v) {
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != v) __builtin_amdgcn_s_sleep(1);
}
// s_barrier after this wave's LDS stores have landed, without waiting for its global loads
__device__ __forceinline__ void cr_lds_barrier() {
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
}

// DUP: D as k_cr_assemble_build stores it, upper tiles only (levels 0 and 1 of the single-GPU
// solve, and its top block when nlev <= 1): a compile-time switch, as a run-time one made the
// kernel spill
template <int NB, bool GB2 = false, bool DUP = false>
__global__ __launch_bounds__(1024) void k_cr_level(FteDims d, int s, int a0, int iend, int top, int ne, int astep,
                                                   int nsplit, unsigned symmask, int lo_s, int top_mode, int l0,
                                                   const FteState* __restrict__ st,
                                                   double* __restrict__ Dc, const double* __restrict__ Ein,
                                                   double* __restrict__ Eout, double* __restrict__ GBc,
                                                   double* __restrict__ Wc, double* __restrict__ Tau,
                                                   double* __restrict__ dL, double* __restrict__ dR,
                                                   int* __restrict__ bad, CrTauSrc tsrc) {
  if (st->status != 0) return;
  if (top_mode && blockIdx.x >= 1) {
    cr_top_border_sums(d, st, Tau, tsrc);
    return;
  }
  // pivot tiles in LDS with row stride 17 doubles: the 16 rows an A fragment reads land on
  // distinct banks
  constexpr int BP = 16 * NB, TS = 17, BUF = 16 * TS + 16 * BP + BP * TS;
  constexpr bool ER_LDS = NB <= 5 && !GB2;  // room for both coupling copies (cr_er_lds)
  const int GR = d.GR, GRB = GR >> 4, WL = 2 * BP + GR, LDD = BP + GR, NBB = 2 * NB + GRB;
  const int hs = s >> 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 15, lk = lane >> 4;
  if ((int)blockIdx.x >= ne * nsplit) {
    // survivor: D_j -= sum over the pending levels sp of dR_{j-sp} + dL_{j+sp},  GB_j likewise
    if (!hs) return;
    const int j = a0 + astep * ((int)blockIdx.x - ne * nsplit);
    double* D = Dc + (size_t)j * BP * BP;
    double* G = GBc + (size_t)j * BP * GR;
    // every load of a level in flight before it is summed, the block's own loads first
    // (blockDim = 1024; the loop form waited for each round of loads: ~15 us per survivor)
    constexpr int NQ = (BP * (BP + 32) + 1023) / 1024;  // GR <= 32
    const int n = BP * LDD;
    double vd[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int e = tid + 1024 * q;
      const int r = e / LDD, c = e - r * LDD;
      // d_up: D as k_cr_assemble_build stored it, upper 16 x 16 tiles only (the lower ones from
      // the transposed tile); the survivors write it back whole
      vd[q] = e < n ? (c < BP ? (DUP && (r >> 4) > (c >> 4) ? D[c * BP + r] : D[r * BP + c]) : G[r * GR + c - BP])
                    : 0.0;
    }
    // one pending term per trip (dR then dL of each level, ascending)
#pragma unroll 1
    for (int k = 0; (lo_s << (k >> 1)) <= hs; ++k) {
      const int sp = lo_s << (k >> 1);
      const bool sy = (symmask >> (__ffs(sp) - 1)) & 1u;
      const double* pq = (k & 1) ? ((j + sp < iend) ? dL + (size_t)(j + sp) * BP * LDD : nullptr)
                                 : ((j - sp >= a0) ? dR + (size_t)(j - sp) * BP * LDD : nullptr);
      if (!pq) continue;
      double v[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int e = tid + 1024 * q;
        const int r = e / LDD, c = e - r * LDD;
        // D parts of the pending terms of a one-wave-per-column-block level (sy) hold their
        // upper tiles only; the deep path writes full tiles
        const int es = (sy && c < BP && (r >> 4) > (c >> 4)) ? c * LDD + r : e;
        v[q] = e < n ? pq[es] : 0.0;
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) vd[q] -= v[q];
    }
    // DUP: the lower tiles were read from the upper ones, which other waves of this workgroup
    // are about to overwrite: every read lands before the first store
    if constexpr (DUP) __syncthreads();
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int e = tid + 1024 * q;
      if (e >= n) continue;
      const int r = e / LDD, c = e - r * LDD;
      if (c < BP)
        D[r * BP + c] = vd[q];
      else
        G[r * GR + c - BP] = vd[q];
    }
    return;
  }
  const int part = (int)blockIdx.x % nsplit;
  // pivot-row hand-off flags (R_kK of step k carries stamp k + 1; double-buffered like the
  // pivot buffers): cleared before any wave can read them (LDS-only barrier: the global loads
  // issued below are not waited for)
  __shared__ int s_rflag[2][8];
  if (tid < 16) s_rflag[tid >> 3][tid & 7] = -1;
  cr_lds_barrier();
  // top_mode: the last surviving block a0 itself (no neighbours, only its GB column-blocks:
  // W_gb = D^-1 GB and Tau = GB^T W_gb for k_cr_top), after its pending terms
  const int i = top_mode ? a0 : a0 + s * (2 * ((int)blockIdx.x / nsplit) + 1);
  const int r = (!top_mode && i + s <= top) ? i + s : -1;
  // pending terms of the levels lo_s .. hs: dR of the left neighbour i - sp (none for the top
  // block) and dL of the right one i + sp (when it was eliminated, < iend)
  auto qR_at = [&](int sp) { return !top_mode ? dR + (size_t)(i - sp) * BP * LDD : (const double*)nullptr; };
  auto qL_at = [&](int sp) { return i + sp < iend ? dL + (size_t)(i + sp) * BP * LDD : (const double*)nullptr; };
  const double* Ei = top_mode ? nullptr : Ein + (size_t)i * BP * BP;
  const double* Er = r >= 0 ? Ein + (size_t)r * BP * BP : nullptr;
  extern __shared__ double lds[];
  double* G0 = lds + 2 * BUF;  // GB_i (pending applied), BP x GR, for Tau
  // LDS copies of the coupling blocks (A operands of the Schur terms): E_i (row major BP x
  // BP) and E_r (row stride BP + 1: the 16 rows of a fragment spread over the banks); E_r is
  // read from global memory when BP = 96 or GR = 32 leaves no room (cr_er_lds)
  double* sEi = G0 + BP * GR;
  double* sEr = ER_LDS && Er ? sEi + BP * BP : nullptr;
  const bool dwave = wave < NB;
  // this wave's column-block J (0..NB-1 E_i, NB..2NB-1 E_r^T, 2NB.. GB_i): the p-th of the
  // column-blocks J = part (mod nsplit)
  int J = -1;
  if (!dwave) {
    const int jj = part + nsplit * (wave - NB);
    if (jj < NBB) J = jj;
    if (top_mode) {
      J = (wave - NB < GRB) ? 2 * NB + (wave - NB) : -1;
    } else if (nsplit == 1 && NB == 5 && NBB == 11) {
      // one workgroup holds all 11 column-blocks: deal them so that the four SIMDs (wave
      // w runs on SIMD w % 4) carry about the same MFMA work (GJ 5 + Schur tiles, in units
      // of 4-MFMA chains: J0-4: 6..10 + 5, J5-9: 1..5 + 5, J10: 11 + 5)
      constexpr int perm[11] = {4, 3, 2, 10, 8, 1, 0, 9, 6, 5, 7};
      J = perm[wave - NB];
    } else if (nsplit == 2 && NB == 5 && NBB == 11) {
      // two workgroups per block (even / odd column-blocks), the same balancing
      constexpr int perm2[2][11] = {{4, 2, 0, 10, -1, 8, 6, -1, -1, -1, -1},
                                    {1, 9, 7, 3, -1, 5, -1, -1, -1, -1, -1}};
      J = perm2[part][wave - NB];
    }
  }
  PROF_T0
  // one workgroup holding every column block (the wide levels): the column waves' own E_i and
  // E_r^T blocks ARE the LDS copies, stored from their registers below; otherwise the column
  // waves copy the two coupling blocks from global memory first (HBM-bound when every CU
  // starts a level at once: 265 KB per block with the copies, 163 KB without)
  const bool own_all = nsplit == 1 && 16 - NB >= NBB && !top_mode;
  if (!dwave && !own_all) {
    // the column waves copy the coupling blocks (read only in the Schur phase, after the
    // pivot steps' barriers); the row waves go straight to their loads: wave 0's first
    // pivot tile no longer waits behind this copy's round trip. Every load in flight
    // before the LDS stores (blockDim = 1024).
    constexpr int CN = 1024 - 64 * NB, NCP = (BP * BP + CN - 1) / CN;
    const int ct = tid - 64 * NB;
    double ve[NCP], vr[NCP];
#pragma unroll
    for (int q = 0; q < NCP; ++q) {
      const int e = ct + CN * q;
      // level 0: the strictly lower tiles of E are zero and not stored (k_cr_assemble_build)
      const bool ez = l0 && ((e / BP) >> 4) > ((e % BP) >> 4);
      ve[q] = (Ei && e < BP * BP && !ez) ? Ei[e] : 0.0;
      vr[q] = (sEr && e < BP * BP && !ez) ? Er[e] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < NCP; ++q) {
      const int e = ct + CN * q;
      if (e < BP * BP) {
        sEi[e] = ve[q];
        if (sEr) sEr[(e / BP) * (BP + 1) + e % BP] = vr[q];
      }
    }
  }
  dbl4 t[NB];
  // loads: one branch-free unrolled batch per source so that they all issue back to back
  auto load_rows = [&](const double* src, int ld, int r0) {
#pragma unroll
    for (int K = 0; K < NB; ++K)
#pragma unroll
      for (int q = 0; q < 4; ++q) t[K][q] = src[(r0 + lk + 4 * q) * ld + K * 16 + li];
  };
  // pending D terms of a level that took the one-wave-per-column-block path (its symmask bit) are
  // stored as upper tiles: tile (r0/16, K) with K < r0/16 is the transpose of tile (K, r0/16);
  // the deep path writes full tiles (rows read contiguously). (Reading every pending term as its
  // mirrored upper triangle makes each factored D bitwise symmetric, but moves the rounding of
  // the single-GPU and frame-window reductions apart: measured in r06c, the head-model 3-rank
  // solve then took 14 LM iterations against the single GPU's 12 at the same cost. Not kept.)
  auto sub_rows = [&](const double* src, int ld, int r0, bool sy) {
    double v[NB][4];
#pragma unroll
    for (int K = 0; K < NB; ++K)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        v[K][q] = (sy && K * 16 < r0) ? src[(K * 16 + li) * ld + r0 + lk + 4 * q]
                                      : src[(r0 + lk + 4 * q) * ld + K * 16 + li];
#pragma unroll
    for (int K = 0; K < NB; ++K)
#pragma unroll
      for (int q = 0; q < 4; ++q) t[K][q] -= v[K][q];
  };
  // column-block loads: element (K*16 + lk + 4q, c0 + li) of a row-major source
  auto load_cols = [&](const double* src, int ld, int c0) {
#pragma unroll
    for (int K = 0; K < NB; ++K)
#pragma unroll
      for (int q = 0; q < 4; ++q) t[K][q] = src[(K * 16 + lk + 4 * q) * ld + c0 + li];
  };
  auto sub_cols = [&](const double* src, int ld, int c0) {
    double v[NB][4];
#pragma unroll
    for (int K = 0; K < NB; ++K)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[K][q] = src[(K * 16 + lk + 4 * q) * ld + c0 + li];
#pragma unroll
    for (int K = 0; K < NB; ++K)
#pragma unroll
      for (int q = 0; q < 4; ++q) t[K][q] -= v[K][q];
  };
  if (dwave) {
    if constexpr (DUP) {
      // D as assembled: upper tiles only; tile (wave, K < wave) is the transpose of (K, wave)
      // (one base and stride per tile, selected: the per-element form kept both address sets
      // live and spilled)
      const double* src = Dc + (size_t)i * BP * BP;
      const int r0 = wave * 16;
#pragma unroll
      for (int K = 0; K < NB; ++K) {
        const bool tr = K * 16 < r0;
        const double* b = src + (tr ? (K * 16 + li) * BP + r0 + lk : (r0 + lk) * BP + K * 16 + li);
        const int st = tr ? 4 : 4 * BP;
#pragma unroll
        for (int q = 0; q < 4; ++q) t[K][q] = b[q * st];
      }
    } else {
      load_rows(Dc + (size_t)i * BP * BP, BP, wave * 16);
    }
    // dR then dL of each level; both terms' loads in flight at once where the registers allow
    // (NB <= 5), one at a time at NB = 6
#pragma unroll 1
    for (int sp = lo_s; sp <= hs; sp <<= 1) {
      const bool sy = (symmask >> (__ffs(sp) - 1)) & 1u;
      const double *qR = qR_at(sp), *qL = qL_at(sp);
      if constexpr (NB <= 5) {
        if (qR) sub_rows(qR, LDD, wave * 16, sy);
        if (qL) sub_rows(qL, LDD, wave * 16, sy);
      } else {
        if (qR) sub_rows(qR, LDD, wave * 16, sy);
        __builtin_amdgcn_sched_barrier(0);
        if (qL) sub_rows(qL, LDD, wave * 16, sy);
      }
    }
  } else if (J >= 0 && J < NB) {
    if (l0) {  // level 0: tiles (K > J) of E_i are zero and not stored (k_cr_assemble_build)
#pragma unroll
      for (int K = 0; K < NB; ++K)
#pragma unroll
        for (int q = 0; q < 4; ++q) t[K][q] = K > J ? 0.0 : Ei[(K * 16 + lk + 4 * q) * BP + J * 16 + li];
    } else {
      load_cols(Ei, BP, J * 16);
    }
    if (own_all)
#pragma unroll
      for (int K = 0; K < NB; ++K)
#pragma unroll
        for (int q = 0; q < 4; ++q) sEi[(K * 16 + lk + 4 * q) * BP + J * 16 + li] = t[K][q];
  } else if (J >= NB && J < 2 * NB) {
    if (Er) {
      // E_r^T: element (K*16 + lk + 4q, li) = E_r[(J-NB)*16 + li][K*16 + lk + 4q]
      const double* src = Er + (size_t)((J - NB) * 16 + li) * BP;
#pragma unroll
      for (int K = 0; K < NB; ++K)
#pragma unroll
        for (int q = 0; q < 4; ++q) t[K][q] = (l0 && K < J - NB) ? 0.0 : src[K * 16 + lk + 4 * q];
      if (own_all && sEr)
#pragma unroll
        for (int K = 0; K < NB; ++K)
#pragma unroll
          for (int q = 0; q < 4; ++q) sEr[((J - NB) * 16 + li) * (BP + 1) + K * 16 + lk + 4 * q] = t[K][q];
    } else {
#pragma unroll
      for (int K = 0; K < NB; ++K) t[K] = dbl4{0.0, 0.0, 0.0, 0.0};
    }
  } else if (J >= 2 * NB) {
    const int c0 = (J - 2 * NB) * 16;
    load_cols(GBc + (size_t)i * BP * GR, GR, c0);
#pragma unroll 1
    for (int k = 0; (lo_s << (k >> 1)) <= hs; ++k) {
      const int sp = lo_s << (k >> 1);
      const double* q = (k & 1) ? qL_at(sp) : qR_at(sp);
      if (q) sub_cols(q + BP, LDD, c0);
    }
#pragma unroll
    for (int K = 0; K < NB; ++K)
#pragma unroll
      for (int q = 0; q < 4; ++q) G0[(K * 16 + lk + 4 * q) * GR + c0 + li] = t[K][q];
  } else if (GB2 && nsplit > 1 && !dwave && !top_mode) {
    // Two GB column-blocks (GR = 32: 16 delays) dealt over the nsplit workgroups of a block:
    // Tau_i = GB_i^T W_gb (below) still reads all of GB_i from G0, so idle wave k (k = 0, 1)
    // loads GB column-block k when another workgroup owns it, with the owner's loads and
    // sums (the same bits), into G0 only (cr_nsplit leaves at least GRB idle waves)
    const int k = wave - NB - (NBB - part + nsplit - 1) / nsplit;
    if (k >= 0 && k < GRB && (2 * NB + k) % nsplit != part) {
      const int c0 = k * 16;
      load_cols(GBc + (size_t)i * BP * GR, GR, c0);
#pragma unroll 1
      for (int kk = 0; (lo_s << (kk >> 1)) <= hs; ++kk) {
        const int sp = lo_s << (kk >> 1);
        const double* q = (kk & 1) ? qL_at(sp) : qR_at(sp);
        if (q) sub_cols(q + BP, LDD, c0);
      }
#pragma unroll
      for (int K = 0; K < NB; ++K)
#pragma unroll
        for (int q = 0; q < 4; ++q) G0[(K * 16 + lk + 4 * q) * GR + c0 + li] = t[K][q];
    }
  }
  PROFA(32, 0);
  PROFA(33, NB);
#ifdef FTE_PROFILE
  if (prof_on && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&g_fte_prof[63], 1ull);
#endif
  PROF(0);
  // Gauss-Jordan elimination, pivot block k
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    double* Pk = lds + (k & 1) * BUF;  // D_kk^-1, 16 x 16 (stride TS)
    double* Rk = Pk + 16 * TS;         // new pivot row-block of D, 16 x BP
    double* Ck = Rk + 16 * BP;         // old pivot column-block of D, BP x 16 (stride TS)
    if (dwave) {
      if (wave == k) {
        // pivot tile inverse: pivot 0 here, pivot k > 0 already inverted by this wave at the
        // end of step k-1 (overlapped with its remaining row updates)
        if (k == 0) {
          double v[4] = {t[0][0], t[0][1], t[0][2], t[0][3]};
          tile16_gj_inverse<true>(v, lane, part ? nullptr : bad);
#pragma unroll
          for (int q = 0; q < 4; ++q) t[0][q] = v[q];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) Pk[(lk + 4 * q) * TS + li] = t[k][q];
        // R_kK = D_kk^-1 D_kK. The A operand is read back from Pk (row li, column 4ks + lk):
        // the computed inverse is not exactly symmetric, and its transpose (register ks of
        // the tile) costs accuracy on ill-conditioned blocks (the last, most reduced one)
#pragma unroll
        for (int K = k + 1; K < NB; ++K) {
          dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) acc = mfma64(Pk[li * TS + 4 * ks + lk], t[K][ks], acc);
          t[K] = acc;
#pragma unroll
          for (int q = 0; q < 4; ++q) Rk[(lk + 4 * q) * BP + K * 16 + li] = acc[q];
          // hand R_kK to the next pivot wave now, not at the barrier (cr_flag_*)
          if (k + 1 < NB) cr_flag_set(&s_rflag[k & 1][K], k + 1);
        }
        PROFA(34 + k, k);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) Ck[(wave * 16 + lk + 4 * q) * TS + li] = t[k][q];
      }
    }
    // The next pivot's wave (k + 1) does not wait here for the whole pivot row: it starts its
    // diagonal update and tile inverse as soon as R_k,k+1 is flagged, takes each later R_kK at
    // its flag, and arrives at this step's barrier inside its inverse (after 4 scalar steps),
    // when the pivot wave's row panel is done. Every wave still passes one barrier per step.
#ifndef CR_EARLY_PIVOT
#define CR_EARLY_PIVOT 1
#endif
    const bool early = CR_EARLY_PIVOT && dwave && wave == k + 1;
    if (!early) __syncthreads();
    if (dwave) {
      if (wave == k + 1) {
        // next pivot: its diagonal tile first, then its inverse with the remaining row
        // updates (MFMA) slotted between the pivot steps (VALU)
        PROFA(44 + k, k + 1);
        if (CR_EARLY_PIVOT) cr_flag_wait(&s_rflag[k & 1][k + 1], k + 1);
        {
          dbl4 acc = t[k + 1];
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            acc = mfma64(-Ck[(wave * 16 + li) * TS + 4 * ks + lk], Rk[(4 * ks + lk) * BP + (k + 1) * 16 + li], acc);
          t[k + 1] = acc;
        }
        double v[4] = {t[k + 1][0], t[k + 1][1], t[k + 1][2], t[k + 1][3]};
        tile16_gj_inverse_hook<true>(v, lane, part ? nullptr : bad, [&](auto sc) {
          constexpr int S = decltype(sc)::value;
          const int K = k + 2 + S / 4, ks = S % 4;  // constants once the k loop is unrolled
          if (K < NB) {
            if (CR_EARLY_PIVOT && ks == 0) cr_flag_wait(&s_rflag[k & 1][K], k + 1);
            t[K] = mfma64(-Ck[(wave * 16 + li) * TS + 4 * ks + lk], Rk[(4 * ks + lk) * BP + K * 16 + li], t[K]);
          }
          if constexpr (CR_EARLY_PIVOT && S == 3) __syncthreads();  // this wave's arrival at step k's barrier
        });
#pragma unroll
        for (int q = 0; q < 4; ++q) t[k + 1][q] = v[q];
        PROFA(50 + k, k + 1);
      } else if (wave != k) {
#pragma unroll
        for (int K = k + 1; K < NB; ++K) {
          dbl4 acc = t[K];
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
            acc = mfma64(-Ck[(wave * 16 + li) * TS + 4 * ks + lk], Rk[(4 * ks + lk) * BP + K * 16 + li], acc);
          t[K] = acc;
        }
      }
    } else if (J >= 0 && !(l0 && J >= NB && J < 2 * NB && k < J - NB)) {
      // (l0: level 0, where every E is upper triangular: column-block m = J - NB of E_r^T is
      // zero in row-blocks < m, so its first m pivot steps only add zeros and are skipped)
      dbl4 nk = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) nk = mfma64(Pk[li * TS + 4 * ks + lk], t[k][ks], nk);
      t[k] = nk;
#pragma unroll
      for (int I = 0; I < NB; ++I) {
        if (I == k) continue;
        dbl4 acc = t[I];
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc = mfma64(-Ck[(I * 16 + li) * TS + 4 * ks + lk], nk[ks], acc);
        t[I] = acc;
      }
    }
  }
  PROFA(40, NB);
  PROFA(29, 15);
  PROFA(31, 0);
  PROF(1);
  if (nsplit >= 3 && ((NBB + nsplit - 1) / nsplit) * BP * 16 <= 2 * BUF) {
    // Deep levels (few column-blocks per workgroup): the Schur terms are dealt out to all 16
    // waves instead of each column wave forming its own 2 NB output tiles, which would
    // serialise on one SIMD's matrix core. The W column-blocks go to LDS (the pivot buffers
    // are free once every wave is past the last pivot step) and to global memory.
    const int nJ = (NBB - part + nsplit - 1) / nsplit;
    double* sWl = lds;  // nJ x (BP x 16)
    __syncthreads();
    if (!dwave && J >= 0) {
      const int jl = wave - NB;
      double* W = Wc + (size_t)i * BP * WL;
      const int wcol = J < NB ? J * 16 : (J < 2 * NB ? BP + (J - NB) * 16 : 2 * BP + (J - 2 * NB) * 16);
#pragma unroll
      for (int K = 0; K < NB; ++K)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          W[(size_t)(K * 16 + lk + 4 * q) * WL + wcol + li] = t[K][q];
          sWl[(size_t)jl * BP * 16 + (K * 16 + lk + 4 * q) * 16 + li] = t[K][q];
        }
    }
    __syncthreads();
    const int per = 2 * NB + 1;
    for (int task = wave; task < nJ * per; task += 16) {
      const int jl = task / per, rr = task - jl * per;
      const int Jt = part + nsplit * jl;
      const double* w = sWl + (size_t)jl * BP * 16;
      const int ocol = Jt < NB ? Jt * 16 : (Jt < 2 * NB ? (Jt - NB) * 16 : BP + (Jt - 2 * NB) * 16);
      auto chain = [&](auto aop, int I) {
        dbl4 a0 = {0.0, 0.0, 0.0, 0.0}, a1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int K = 0; K < NB; K += 2) {
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            a0 = mfma64(aop(I, K, ks), w[(K * 16 + 4 * ks + lk) * 16 + li], a0);
            if (K + 1 < NB) a1 = mfma64(aop(I, K + 1, ks), w[((K + 1) * 16 + 4 * ks + lk) * 16 + li], a1);
          }
        }
        return a0 + a1;
      };
      if (rr < NB) {  // left term E_i^T [W_l | W_gb], output tile I
        if (Jt >= NB && Jt < 2 * NB) continue;
        const dbl4 acc = chain([&](int I, int K, int ks) { return sEi[(K * 16 + 4 * ks + lk) * BP + I * 16 + li]; }, rr);
        double* o = dL + (size_t)i * BP * LDD;
#pragma unroll
        for (int q = 0; q < 4; ++q) o[(size_t)(rr * 16 + lk + 4 * q) * LDD + ocol + li] = acc[q];
      } else if (rr < 2 * NB) {  // right term E_r [W_r | W_gb] and the new coupling -E_r W_l
        if (!Er) continue;
        const int I = rr - NB;
        const dbl4 acc = sEr ? chain([&](int I_, int K, int ks) { return sEr[(I_ * 16 + li) * (BP + 1) + K * 16 + 4 * ks + lk]; }, I)
                             : chain([&](int I_, int K, int ks) {
                                 return (l0 && K < I_) ? 0.0 : Er[(I_ * 16 + li) * BP + K * 16 + 4 * ks + lk];
                               }, I);
        if (Jt < NB) {
          double* o = Eout + (size_t)r * BP * BP;
#pragma unroll
          for (int q = 0; q < 4; ++q) o[(size_t)(I * 16 + lk + 4 * q) * BP + Jt * 16 + li] = -acc[q];
        } else {
          double* o = dR + (size_t)i * BP * LDD;
#pragma unroll
          for (int q = 0; q < 4; ++q) o[(size_t)(I * 16 + lk + 4 * q) * LDD + ocol + li] = acc[q];
        }
      } else {  // Tau_i = GB_i^T W_gb
        if (Jt < 2 * NB) continue;
        const int g = Jt - 2 * NB;
        for (int g2 = 0; g2 < GRB; ++g2) {
          dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int K = 0; K < NB; ++K)
#pragma unroll
            for (int ks = 0; ks < 4; ++ks)
              acc = mfma64(G0[(K * 16 + 4 * ks + lk) * GR + g2 * 16 + li], w[(K * 16 + 4 * ks + lk) * 16 + li], acc);
#pragma unroll
          for (int q = 0; q < 4; ++q) Tau[(size_t)i * GR * GR + (g2 * 16 + lk + 4 * q) * GR + g * 16 + li] = acc[q];
        }
      }
    }
    PROFA(43, 0);
    return;
  }
  if (dwave || J < 0) return;
  // W_i (back substitution), Schur terms for the neighbours, Tau_i
  double* W = Wc + (size_t)i * BP * WL;
  double* oL = dL + (size_t)i * BP * LDD;
  double* oR = dR + (size_t)i * BP * LDD;
  double* Er_out = r >= 0 ? Eout + (size_t)r * BP * BP : nullptr;
  const int wcol = J < NB ? J * 16 : (J < 2 * NB ? BP + (J - NB) * 16 : 2 * BP + (J - 2 * NB) * 16);
#pragma unroll
  for (int K = 0; K < NB; ++K)
#pragma unroll
    for (int q = 0; q < 4; ++q) W[(size_t)(K * 16 + lk + 4 * q) * WL + wcol + li] = t[K][q];
  const int ocol = J < NB ? J * 16 : (J < 2 * NB ? (J - NB) * 16 : BP + (J - 2 * NB) * 16);
  // out tile I = sum_K A(I, K) W(K): two independent MFMA chains (even / odd K). tri (level 0,
  // every E upper triangular): 1 = A(I, K) is zero for K > I (E_i^T), 2 = zero for K < I (E_r);
  // those products add exact zeros and are skipped (1320 -> 800 MFMAs per block)
  auto term = [&](auto aop, auto store, int Imax, int tri) {  // output tiles I = 0 .. Imax
#pragma unroll 1
    for (int I = 0; I <= Imax; ++I) {
      dbl4 a0 = {0.0, 0.0, 0.0, 0.0}, a1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int K = 0; K < NB; K += 2) {
        const bool z0 = (tri == 1 && K > I) || (tri == 2 && K < I);
        const bool z1 = K + 1 >= NB || (tri == 1 && K + 1 > I) || (tri == 2 && K + 1 < I);
        if (!z0)
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) a0 = mfma64(aop(I, K, ks), t[K][ks], a0);
        if (!z1)
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) a1 = mfma64(aop(I, K + 1, ks), t[K + 1][ks], a1);
      }
      store(I, a0 + a1);
    }
  };
  // A operands (lane: row li, column 4 ks + lk of tile (I, K))
  auto aEiT = [&](int I, int K, int ks) { return sEi[(K * 16 + 4 * ks + lk) * BP + I * 16 + li]; };
  auto aEr_lds = [&](int I, int K, int ks) { return sEr[(I * 16 + li) * (BP + 1) + K * 16 + 4 * ks + lk]; };
  auto aEr_glb = [&](int I, int K, int ks) { return Er[(I * 16 + li) * BP + K * 16 + 4 * ks + lk]; };
  auto put_L = [&](int I, dbl4 acc) {
#pragma unroll
    for (int q = 0; q < 4; ++q) oL[(size_t)(I * 16 + lk + 4 * q) * LDD + ocol + li] = acc[q];
  };
  auto put_R = [&](int I, dbl4 acc) {
#pragma unroll
    for (int q = 0; q < 4; ++q) oR[(size_t)(I * 16 + lk + 4 * q) * LDD + ocol + li] = acc[q];
  };
  auto put_E = [&](int I, dbl4 acc) {
#pragma unroll
    for (int q = 0; q < 4; ++q) Er_out[(size_t)(I * 16 + lk + 4 * q) * BP + J * 16 + li] = -acc[q];
  };
  // left term E_i^T W (columns W_l and W_gb); E_i^T W_l is symmetric: upper tiles only
  if (!top_mode && (J < NB || J >= 2 * NB)) term(aEiT, put_L, J < NB ? J : NB - 1, l0 ? 1 : 0);
  PROFA(41, NB);
  PROFW(3, NB);
  PROFW(3 + 8, 15);
  // right term E_r W (columns W_r and W_gb) and the new coupling -E_r W_l
  if (Er) {
    if (J < NB) {
      if (sEr)
        term(aEr_lds, put_E, NB - 1, l0 ? 2 : 0);
      else
        term(aEr_glb, put_E, NB - 1, l0 ? 2 : 0);
    } else {
      // E_r W_r is symmetric: upper tiles only
      const int Imax = J < 2 * NB ? J - NB : NB - 1;
      if (sEr)
        term(aEr_lds, put_R, Imax, l0 ? 2 : 0);
      else
        term(aEr_glb, put_R, Imax, l0 ? 2 : 0);
    }
  }
  PROFA(42, NB);
  PROFW(4, NB);
  PROFW(4 + 8, 15);
  if (J >= 2 * NB) {
    const int g = J - 2 * NB;
    for (int g2 = 0; g2 < GRB; ++g2) {
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int K = 0; K < NB; ++K)
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) acc = mfma64(G0[(K * 16 + 4 * ks + lk) * GR + g2 * 16 + li], t[K][ks], acc);
#pragma unroll
      for (int q = 0; q < 4; ++q) Tau[(size_t)i * GR * GR + (g2 * 16 + lk + 4 * q) * GR + g * 16 + li] = acc[q];
    }
  }
  PROFW(5 + 8, 15);
  PROFA(43, NB);
  PROFA(30, 15);
}

__global__ __launch_bounds__(512) void k_cr_tau_partial(FteDims d, const FteState* __restrict__ st,
                                                        const double* __restrict__ Hloc,
                                                        const double* __restrict__ gloc,
                                                        const double* __restrict__ Tau, double* __restrict__ part,
                                                        int k_lo, int k_hi, int b_lo, int b_hi, int hsel,
                                                        const double* __restrict__ Tc) {
  if (st->status != 0) return;
  const int ch = blockIdx.x, nE = d.Cg * d.Cg + d.Cg + d.GR * d.GR;
  cr_tau_partial_chunk(d, st, Hloc, gloc, Tau, k_lo, k_hi, b_lo, b_hi, hsel, Tc, ch,
                       [&](int e, double v) { part[(size_t)ch * nE + e] = v; });
}

// Trial state of super-block i (frames 3i..3i+2: X[cur ^ 1] = X[cur] + dv) and the
// constant-mode delays when `taus` (block 0), with the block's step / state norm partials.
// Thread e < 3P holds row e of the step (`dv`); thread c < C steps delay c. The sums are
// k_cr_trial's bit for bit: the same per-thread terms in the same order, and block_sum's
// tree over 1024 threads first folds threads >= 256 (zeros) exactly.
// this thread's current-state element of block i (issued early by the callers: its load
// latency then hides behind their work)
__device__ __forceinline__ double cr_trial_x(const FteDims& d, const FteState* st, int i,
                                             const double* __restrict__ Xbuf) {
  const int P = d.P, e = threadIdx.x;
  if (!Xbuf || e >= 3 * P || 3 * i + e / P >= d.M) return 0.0;
  return Xbuf[(size_t)st->cur * d.M * P + (size_t)(3 * i + e / P) * P + e % P];
}
// block_sum of a and b where only threads < 128 hold nonzero terms, all >= +0: every level
// of block_sum's tree above 128 then adds exact zeros, so its result is the wave tree over
// s[l] + s[l + 64] - computed here with one exchange and two barriers instead of ten
// (bit-identical). blockDim.x >= 128; s_red: 256 doubles.
__device__ __forceinline__ void block_sum2_lo128(double& a, double& b, double* s_red) {
  const int t = threadIdx.x, l = t & 63;
  if (t < 128) {
    s_red[t] = a;
    s_red[128 + t] = b;
  }
  __syncthreads();
  double ra = s_red[l] + s_red[l + 64], rb = s_red[128 + l] + s_red[128 + l + 64];
#pragma unroll
  for (int h = 32; h > 0; h >>= 1) {
    ra += __shfl_down(ra, h, 64);
    rb += __shfl_down(rb, h, 64);
  }
  a = __shfl(ra, 0, 64);
  b = __shfl(rb, 0, 64);
  __syncthreads();
}
__device__ __forceinline__ void cr_trial_rows(const FteDims& d, const FteState* st, int i, double dv, double x,
                                              const double* __restrict__ dtau, double* __restrict__ Xbuf,
                                              double* __restrict__ taubuf, double* __restrict__ normp, bool taus,
                                              double* s_red, bool tau_norm = true) {
  const int P = d.P, e = threadIdx.x, cur = st->cur;
  double dn = 0.0, xn = 0.0;
  if (e < 3 * P) {
    const int f = 3 * i + e / P, p = e % P;
    if (f < d.M) {
      const size_t o = (size_t)f * P + p;
      Xbuf[(size_t)(cur ^ 1) * d.M * P + o] = x + dv;
      dn += dv * dv;
      xn += x * x;
    }
  }
  if (taus && e < d.C) {
    const double* tau = taubuf + cur * d.NT;
    double* taun = taubuf + (cur ^ 1) * d.NT;
    const double t = (e == 0) ? 0.0 : dtau[e];
    taun[e] = (e == 0) ? 0.0 : fmin(fmax(tau[e] + t, -d.Ts), d.Ts);
    if (tau_norm) {  // the replicated delays count once over the frame-window ranks (rank 0)
      dn += t * t;
      xn += tau[e] * tau[e];
    }
  }
  if (3 * P <= 128 && d.C <= 128 && blockDim.x >= 128) {
    block_sum2_lo128(dn, xn, s_red);
  } else {
    dn = block_sum(dn, s_red);
    xn = block_sum(xn, s_red);
  }
  if (threadIdx.x == 0) {
    normp[2 * i] = dn;
    normp[2 * i + 1] = xn;
  }
}

// k_cr_top's work (blockDim 1024, or k_cr_back_all's 8 BP; every thread, nth >= 8 BP):
// `loadp(i)` reads element i of the CR_NCHUNK chunk partials, rows nE wide; fused (the rows
// of cr_launch_top with_partials): rows nE + 1 wide, the chunk's frame |g| max last;
// `pub_tau(c, v)` (c < 32) and `pub_row(r, v)` (r < BP) hand dtau and block 0's step on to
// the back substitution (besides the plain dtau / dcv stores); tau0: the top block's own Tau
// term when the sums leave it out
template <typename LoadPart, typename PubTau, typename PubRow>
__device__ __forceinline__ void cr_top_body(const FteDims& d, FteState* __restrict__ st, const double* __restrict__ W0,
                                            const double* __restrict__ gmaxp, double* __restrict__ taubuf,
                                            double* __restrict__ dcv, double* __restrict__ dtau, int* __restrict__ bad,
                                            double* __restrict__ Xbuf, double* __restrict__ normp, LoadPart loadp,
                                            PubTau pub_tau, PubRow pub_row, bool fused = false,
                                            const double* __restrict__ tau0 = nullptr) {
  // block 0 has been eliminated by k_cr_level (top_mode): W0 = its W (BP x WL), its tau Schur
  // term is in the Tau sums like every other block's (or in tau0)
  const int tid = threadIdx.x, nth = blockDim.x;
  const int BP = d.BP, GR = d.GR, Cg = d.Cg, WL = 2 * BP + GR;
  const double lam = st->lam;
  const double xpre = cr_trial_x(d, st, 0, Xbuf);
  // block 0's step rows = rhs - W_tau dtau, 8 lanes per row: this lane's W_tau entries and the
  // rhs loaded first (they were dependent loads after the tau solve)
  const int wrow = tid >> 3, wj = tid & 7;
  const bool wlive = wrow < BP;
  double wq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = wj + 8 * q;
    wq[q] = (wlive && c < Cg) ? W0[(size_t)wrow * WL + 2 * BP + c] : 0.0;
  }
  const double wrhs = (wlive && wj == 0) ? W0[(size_t)wrow * WL + 2 * BP + Cg] : 0.0;
  __shared__ double sS[32 * 32];
  __shared__ double sr[32];
  __shared__ double tmp[512];
  __shared__ double s_red[1024];
  __shared__ double s_dt[32];
  // chunk partials -> sums (fixed order)
  const int nH = Cg * Cg, nE = nH + Cg + GR * GR;
  __shared__ double s_sum[16 * 16 + 16 + 32 * 32];
  __shared__ int s_held[32];
  const int pw = fused ? nE + 1 : nE;
  __shared__ double s_gm;
  for (int e = tid; e < (fused ? nE + 1 : nE); e += nth) {
    // 16 loads in flight at a time, summed in chunk order (one CU streams the 64 x nE
    // partials from L2: splitting the chunks over more threads did not help, r03j)
    double v = 0.0;
    for (int c0 = 0; c0 < CR_NCHUNK; c0 += 16) {
      double pv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) pv[q] = loadp((size_t)(c0 + q) * pw + e);
#pragma unroll
      for (int q = 0; q < 16; ++q) v = e < nE ? v + pv[q] : fmax(v, pv[q]);
    }
    if (e == nE) {
      s_gm = v;  // fused: the frames' |g| max
      continue;
    }
    if (tau0 && e >= nH + Cg) v += tau0[e - nH - Cg];
    s_sum[e] = v;
  }
  __syncthreads();
  if (tid < 32) s_held[tid] = tid >= Cg || tau_held(taubuf[(size_t)st->cur * d.NT + tid], s_sum[nH + tid], d.Ts, tid);
  __syncthreads();
  // gradient max (frames + free tau border)
  if (fused) {
    if (tid == 0) {
      double mx = s_gm;
      for (int c = 0; c < Cg; ++c)
        if (!s_held[c]) mx = fmax(mx, fabs(s_sum[nH + c]));
      st->gmax = mx;
    }
  } else {
    double mx = 0.0;
    mx = strided_max(gmaxp, tid, d.M, nth, mx);
    for (int c = tid; c < Cg; c += nth)
      if (!s_held[c]) mx = fmax(mx, fabs(s_sum[nH + c]));
    mx = block_max(mx, s_red);
    if (tid == 0) st->gmax = mx;
  }
  if (tid < 32) s_dt[tid] = 0.0;
  if (Cg) {
    // S = D_tau - sum_i Tau_i ;  rhs = b_tau - sum_i Tau_i[:, Cg]   (GR x GR, padded)
    for (int e = tid; e < GR * GR; e += nth) {
      const int r = e / GR, c = e % GR;
      double h = 0.0;
      if (r < Cg && c <= Cg) {
        if (c < Cg) {
          h = s_sum[r * Cg + c];
          if (r == c) h += lam * fmax(h, 1e-12);
        } else {
          h = -s_sum[nH + r];
        }
        h -= s_sum[nH + Cg + r * GR + c];
      }
      sS[e] = h;
    }
    __syncthreads();
    if (tid < GR) sr[tid] = (tid < Cg && !s_held[tid]) ? sS[tid * GR + Cg] : 0.0;
    __syncthreads();
    // pin tau_0, the held delays and the padding (identity rows / columns)
    for (int e = tid; e < GR * GR; e += nth) {
      const int r = e / GR, c = e % GR;
      if (r >= Cg || c >= Cg || s_held[r] || s_held[c]) sS[e] = (r == c) ? 1.0 : 0.0;
    }
    __syncthreads();
    wg_gj_inverse_body<true>(sS, GR, GR >> 4, tmp, bad);  // inlined: k_cr_back_all's VGPR budget
    if (tid < GR) {
      double v = 0.0;
      for (int c = 0; c < GR; ++c) v += sS[tid * GR + c] * sr[c];
      const double dt = (tid < Cg && !s_held[tid]) ? v : 0.0;
      dtau[tid] = dt;
      if (tid < 32) {
        pub_tau(tid, dt);
        s_dt[tid] = dt;
      }
    }
  }
  if (tid < 32 && (!Cg || tid >= GR)) pub_tau(tid, 0.0);
  __syncthreads();
  // block 0's step: row wrow = rhs - sum_c W[wrow][2 BP + c] dtau_c (a 3-step DPP sum)
  double vp = 0.0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int c = wj + 8 * q;
    if (c < 32) vp = fma(wq[q], s_dt[c], vp);
  }
  vp = group_sum<8>(vp);
  if (wlive && wj == 0) {
    const double v = wrhs - vp;
    dcv[wrow] = v;
    pub_row(wrow, v);
    tmp[wrow] = v;
  }
  __syncthreads();
  // the single-GPU solve steps block 0 (and the constant delays) here: no k_cr_trial launch
  if (Xbuf) cr_trial_rows(d, st, 0, tid < BP ? tmp[tid] : 0.0, xpre, dtau, Xbuf, taubuf, normp, d.Cg != 0, s_red);
}

__global__ __launch_bounds__(1024) void k_cr_top(FteDims d, FteState* __restrict__ st, const double* __restrict__ W0,
                                                const double* __restrict__ part, const double* __restrict__ gmaxp,
                                                double* __restrict__ taubuf, double* __restrict__ dcv,
                                                double* __restrict__ dtau, int* __restrict__ bad,
                                                double* __restrict__ Xbuf = nullptr,
                                                double* __restrict__ normp = nullptr) {
  if (st->status != 0) return;
  cr_top_body(
      d, st, W0, gmaxp, taubuf, dcv, dtau, bad, Xbuf, normp, [&](size_t i) { return part[i]; },
      [](int, double) {}, [](int, double) {});
}

// back substitution of eliminated block i at level s (blockDim >= 8 BP; every thread calls it).
// `fetch(l, r)` runs after the W loads are issued and fills sl / sr_ (threads < BP) with the
// survivors' rows and st_ (threads < 32) with dtau (zero past Cg); `publish(row, value)`
// stores one row of the block's step.
// NQ = BP / 8 and NTQ = GR / 8 columns per lane (the kernels' template sizes; CR_MAXBP / 8
// and 4 cover every size)
template <int NQ = CR_MAXBP / 8, int NTQ = 4, typename Fetch, typename Publish>
__device__ __forceinline__ void cr_back_block(const FteDims& d, int i, int s, int bend, const double* __restrict__ Wc,
                                              double* sl, double* sr_, double* st_,
                                              Fetch fetch, Publish publish, bool late = false) {
  const int l = i - s, r = (i + s <= bend && i + s < d.nblk) ? i + s : -1;
  const int BP = d.BP, GR = d.GR, Cg = d.Cg, WL = 2 * BP + GR;
  const double* W = Wc + (size_t)i * BP * WL;
  const int tid = threadIdx.x;
  // one row per aligned group of 8 lanes (BP <= 96 < 128 groups): the W loads of every
  // row are issued together, then an FMA chain per lane and a 3-step DPP sum
  const int row = tid >> 3, j = tid & 7;
  const bool live = row < BP;
  const double* w = W + (size_t)(live ? row : 0) * WL;
  // late: the inputs first, then the W loads (they then stay out of the memory queues while
  // the blocks the inputs come from are still being formed)
  if (late) fetch(l, r);
  double a[NQ], b[NQ], t[NTQ];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int c = j + 8 * q;
    a[q] = (live && c < BP) ? w[c] : 0.0;
    b[q] = (live && r >= 0 && c < BP) ? w[BP + c] : 0.0;
  }
#pragma unroll
  for (int q = 0; q < NTQ; ++q) {
    const int c = j + 8 * q;
    t[q] = (live && c < Cg) ? w[2 * BP + c] : 0.0;
  }
  const double rhs = live ? w[2 * BP + Cg] : 0.0;
  if (!late) fetch(l, r);
  __syncthreads();
  double v = 0.0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int c = j + 8 * q;
    if (c < BP) v = fma(a[q], sl[c], fma(b[q], sr_[c], v));
  }
#pragma unroll
  for (int q = 0; q < NTQ; ++q) {
    const int c = j + 8 * q;
    if (c < 32) v = fma(t[q], st_[c], v);
  }
  v = group_sum<8>(v);
  if (live && j == 0) publish(row, rhs - v);
}

__global__ __launch_bounds__(1024) void k_cr_back(FteDims d, int s, int a0, int bend,
                                                  const FteState* __restrict__ st,
                                                  const double* __restrict__ Wc, const double* __restrict__ dtau,
                                                  double* __restrict__ dcv) {
  if (st->status != 0) return;
  __shared__ double sl[CR_MAXBP], sr_[CR_MAXBP], st_[32];
  const int i = a0 + s * (2 * blockIdx.x + 1), BP = d.BP;
  cr_back_block(
      d, i, s, bend, Wc, sl, sr_, st_,
      [&](int l, int r) {
        if ((int)threadIdx.x < BP) {
          sl[threadIdx.x] = dcv[(size_t)l * BP + threadIdx.x];
          sr_[threadIdx.x] = r >= 0 ? dcv[(size_t)r * BP + threadIdx.x] : 0.0;
        }
        if (threadIdx.x < 32) st_[threadIdx.x] = (int)threadIdx.x < d.Cg ? dtau[threadIdx.x] : 0.0;
      },
      [&](int row, double v) { dcv[(size_t)i * BP + row] = v; });
}

// The end of the single-GPU solve's reduction in one launch: the top block with the tau
// border (k_cr_top's work, one workgroup) and every back-substitution level (nblk - 1
// workgroups, one per eliminated block). A workgroup takes a ticket at entry; tickets are
// dealt top first, then the back blocks coarse level first, so a workgroup only ever waits
// for workgroups of lower tickets, which have already started: the grid drains whatever the
// residency (two 8 BP-thread workgroups per CU). The tau partial sums come from the top
// level's launch (cr_launch_top with_partials: its 64 extra workgroups run beside the top
// block's elimination). Until r05 they were 64 workgroups of this launch, and the top waited
// for them behind the W loads of ~450 resident back blocks: 45 us to dtau at 10,000 frames
// (profiles/r05/back_all_timeline_10k_r05m.log). Hand-off (MI355X_MICROARCH.md, inter-
// workgroup visibility, first table row / handoff-1to1): the data is the flag
// (cdna_hip_programming.md §6 Guideline 16, R2): every row of a step and every dtau entry
// goes out as two 8-byte granules {stamp, high word} {stamp, low word}, each ONE sc1 store,
// and each consumer thread re-reads its granules with sc1 loads until all carry this
// launch's stamp. Stamps count launches (ticket / nwork + 1; bk[0] the ticket counter, the
// granules `gdcv` (rows, then 32 x 2 for dtau), all zeroed by fte_setup). The plain dcv /
// dtau are written too (k_cr_trial of the per-frame-delay mode reads them). A spin that
// outlives ~0.3 s gives up and counts into *bad (the solve then reports a failed
// factorisation, not a hang). Folding the top into this launch removed a kernel boundary (r03).
__device__ __forceinline__ void cr_publish_granules(unsigned long long* g, unsigned long long stamp, double v) {
  const unsigned long long bits = (unsigned long long)__double_as_longlong(v);
  __hip_atomic_store(g, (stamp << 32) | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(g + 1, (stamp << 32) | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NB, int GRB>
__global__ __launch_bounds__(768) __attribute__((amdgpu_waves_per_eu(5))) void k_cr_back_all(FteDims d, int bend, FteState* __restrict__ st,
                                                      const double* __restrict__ Wc, const double* __restrict__ Tau,
                                                      const double* __restrict__ part,
                                                      const double* __restrict__ gmaxp, double* __restrict__ taubuf,
                                                      double* __restrict__ dtau, double* __restrict__ dcv,
                                                      int* __restrict__ bk, unsigned long long* __restrict__ gdcv,
                                                      int* __restrict__ bad, double* __restrict__ Xbuf,
                                                      double* __restrict__ normp, int late_lv) {
  __shared__ double sl[CR_MAXBP], sr_[CR_MAXBP], st_[32], sdv[CR_MAXBP], s_red[1024];
  __shared__ int s_tk;
  const int nwork = d.nblk;  // top, nblk - 1 back blocks
#ifdef FTE_PROFILE
  const unsigned long long tb_entry = wall_clock64();
  unsigned long long tb_ready = 0;
#define BACK_TRACE(w_, lv_)                                                      \
  do {                                                                           \
    if (threadIdx.x == 0 && (w_) < FTE_BACK_TRACE) {                              \
      g_back_trace[4 * (w_)] = tb_entry;                                         \
      g_back_trace[4 * (w_) + 1] = tb_ready;                                     \
      g_back_trace[4 * (w_) + 2] = wall_clock64();                               \
      g_back_trace[4 * (w_) + 3] = (unsigned long long)(lv_);                    \
    }                                                                            \
  } while (0)
#else
#define BACK_TRACE(w_, lv_)
#endif
  if (threadIdx.x == 0) s_tk = atomicAdd(bk, 1);
  __syncthreads();
  const unsigned tk = (unsigned)s_tk;
  if (st->status != 0) return;
  const unsigned long long stamp = tk / (unsigned)nwork + 1u;
  int w = (int)(tk % (unsigned)nwork);
  const int BP = d.BP;
  unsigned long long* gtau = gdcv + (size_t)d.nblk * BP * 2;
  if (w == 0) {
    // the tau border partial sums and the frames' |g| max come from the top level's launch
    // (cr_launch_top with_partials), without the top block's own Tau term: added last here
    cr_top_body(
        d, st, Wc, gmaxp, taubuf, dcv, dtau, bad, Xbuf, normp, [&](size_t e) { return part[e]; },
        [&](int c, double v) { cr_publish_granules(gtau + 2 * c, stamp, v); },
        [&](int r, double v) { cr_publish_granules(gdcv + 2 * r, stamp, v); }, true, Tau);
    BACK_TRACE(w, 101);
    return;
  }
#ifdef FTE_PROFILE
  const int w_tr = w;
  int lv_tr = -1;
#endif
  w -= 1;
  int s = 1, i = 1;
  for (int lv = d.nlev - 1; lv >= 0; --lv) {
    const int sv = 1 << lv, ne = (d.nblk - sv + 2 * sv - 1) / (2 * sv);
    if (w < ne) {
      s = sv;
      i = sv * (2 * w + 1);
#ifdef FTE_PROFILE
      lv_tr = lv;
#endif
      break;
    }
    w -= ne;
  }
  const double xpre = cr_trial_x(d, st, i, Xbuf);
  cr_back_block<2 * NB, 2 * GRB>(
      d, i, s, bend, Wc, sl, sr_, st_,
      [&](int l, int r) {
        const int t = threadIdx.x;
        if (t >= BP && t >= 32) return;
        const bool wl = t < BP, wr = t < BP && r > 0, wt = t < 32;
        const unsigned long long* gl = gdcv + ((size_t)l * BP + (wl ? t : 0)) * 2;
        const unsigned long long* gr = gdcv + ((size_t)(r > 0 ? r : l) * BP + (wl ? t : 0)) * 2;
        const unsigned long long* gt = gtau + 2 * (wt ? t : 0);
        const unsigned long long t0 = wall_clock64();
        unsigned long long a0 = 0, a1 = 0, b0 = 0, b1 = 0, c0 = 0, c1 = 0;
        for (;;) {
          if (wl) {
            a0 = __hip_atomic_load(gl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            a1 = __hip_atomic_load(gl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          if (wr) {
            b0 = __hip_atomic_load(gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            b1 = __hip_atomic_load(gr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          if (wt) {
            c0 = __hip_atomic_load(gt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            c1 = __hip_atomic_load(gt + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          const bool ok = (!wl || ((a0 >> 32) == stamp && (a1 >> 32) == stamp)) &&
                          (!wr || ((b0 >> 32) == stamp && (b1 >> 32) == stamp)) &&
                          (!wt || ((c0 >> 32) == stamp && (c1 >> 32) == stamp));
          if (ok) break;
          if (wall_clock64() - t0 > 30000000ull) {
            atomicAdd(bad, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (wl) sl[t] = __hiloint2double((int)(unsigned)a0, (int)(unsigned)a1);
        if (wl) sr_[t] = wr ? __hiloint2double((int)(unsigned)b0, (int)(unsigned)b1) : 0.0;
        if (wt) st_[t] = __hiloint2double((int)(unsigned)c0, (int)(unsigned)c1);
#ifdef FTE_PROFILE
        tb_ready = wall_clock64();
#endif
      },
      [&](int row, double v) {
        const size_t e = (size_t)i * BP + row;
        cr_publish_granules(gdcv + 2 * e, stamp, v);
        dcv[e] = v;
        sdv[row] = v;
      },
      s >= (1 << late_lv));
  __syncthreads();
  // constant / no delays: this block's trial state and norms (k_cr_trial's work)
  if (Xbuf) cr_trial_rows(d, st, i, (int)threadIdx.x < BP ? sdv[threadIdx.x] : 0.0, xpre, dtau, Xbuf, nullptr, normp, false,
                          s_red);
  BACK_TRACE(w_tr, lv_tr);
}
#undef BACK_TRACE

// A frame-window rank's chain back substitution in one launch (the rank-round counterpart of
// k_cr_back_all, for the constant / no-delay modes): the chain ends a0 and bend (< nblk) have
// their step rows from the reduced solve (k_dist_scatter, plain dcv) and dtau from k_cr_top;
// the interior blocks a0 + s(2m + 1) < min(bend, nblk) are substituted coarse level first,
// ticket-ordered as k_cr_back_all (a workgroup only waits for lower tickets, which have
// started), each publishing its rows as {stamp, word} granules; every block, ends included,
// then forms its trial rows and norm partials (k_cr_trial's work; the replicated delays by
// block a0's workgroup, their norms counted on rank 0 only). Replaces klev k_cr_back launches
// and k_cr_trial: the same sums in the same order, so the same bits.
template <int NB, int GRB>
__global__ __launch_bounds__(768) __attribute__((amdgpu_waves_per_eu(5))) void k_cr_back_chain(
    FteDims d, int a0, int bend, int klev, int tau_norm, const FteState* __restrict__ st, const double* __restrict__ Wc,
    const double* __restrict__ dtau, double* __restrict__ dcv, int* __restrict__ bk,
    unsigned long long* __restrict__ gdcv, int* __restrict__ bad, double* __restrict__ Xbuf,
    double* __restrict__ taubuf, double* __restrict__ normp) {
  __shared__ double sl[CR_MAXBP], sr_[CR_MAXBP], st_[32], sdv[CR_MAXBP], s_red[1024];
  __shared__ int s_tk;
  const int iend = min(bend, d.nblk), nends = bend < d.nblk ? 2 : 1;
  int nint = 0;
  for (int lv = klev - 1; lv >= 0; --lv) {
    const int sv = 1 << lv;
    nint += max(0, (iend - a0 - sv + 2 * sv - 1) / (2 * sv));
  }
  const int nwork = nends + nint;
  if (threadIdx.x == 0) s_tk = atomicAdd(bk, 1);
  __syncthreads();
  const unsigned tk = (unsigned)s_tk;
  if (st->status != 0) return;
  const unsigned long long stamp = tk / (unsigned)nwork + 1u;
  int w = (int)(tk % (unsigned)nwork);
  const int BP = d.BP, t = threadIdx.x;
  if (w < nends) {
    // a chain end: its rows came from the reduced solve
    const int e = w == 0 ? a0 : bend;
    const double xpre = cr_trial_x(d, st, e, Xbuf);
    const double v = t < BP ? dcv[(size_t)e * BP + t] : 0.0;
    cr_trial_rows(d, st, e, v, xpre, dtau, Xbuf, taubuf, normp, e == a0 && d.Cg != 0, s_red, tau_norm != 0);
    return;
  }
  w -= nends;
  int s = 1, i = a0 + 1;
  for (int lv = klev - 1; lv >= 0; --lv) {
    const int sv = 1 << lv, ne = max(0, (iend - a0 - sv + 2 * sv - 1) / (2 * sv));
    if (w < ne) {
      s = sv;
      i = a0 + sv * (2 * w + 1);
      break;
    }
    w -= ne;
  }
  const double xpre = cr_trial_x(d, st, i, Xbuf);
  cr_back_block<2 * NB, 2 * GRB>(
      d, i, s, bend, Wc, sl, sr_, st_,
      [&](int l, int r) {
        if (t >= BP && t >= 32) return;
        const bool wl = t < BP, wr = t < BP && r > 0, wt = t < 32;
        // a neighbour that is a chain end is read from dcv; an interior one from its granules
        const bool gl_on = wl && l != a0, gr_on = wr && r != bend;
        const unsigned long long* gl = gdcv + ((size_t)l * BP + (wl ? t : 0)) * 2;
        const unsigned long long* gr = gdcv + ((size_t)(r > 0 ? r : l) * BP + (wl ? t : 0)) * 2;
        const unsigned long long t0 = wall_clock64();
        unsigned long long a0w = 0, a1w = 0, b0w = 0, b1w = 0;
        for (;;) {
          if (gl_on) {
            a0w = __hip_atomic_load(gl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            a1w = __hip_atomic_load(gl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          if (gr_on) {
            b0w = __hip_atomic_load(gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            b1w = __hip_atomic_load(gr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          const bool ok = (!gl_on || ((a0w >> 32) == stamp && (a1w >> 32) == stamp)) &&
                          (!gr_on || ((b0w >> 32) == stamp && (b1w >> 32) == stamp));
          if (ok) break;
          if (wall_clock64() - t0 > 30000000ull) {
            atomicAdd(bad, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        if (wl) sl[t] = gl_on ? __hiloint2double((int)(unsigned)a0w, (int)(unsigned)a1w) : dcv[(size_t)l * BP + t];
        if (wl)
          sr_[t] = !wr ? 0.0 : (gr_on ? __hiloint2double((int)(unsigned)b0w, (int)(unsigned)b1w) : dcv[(size_t)r * BP + t]);
        if (wt) st_[t] = t < d.Cg ? dtau[t] : 0.0;
      },
      [&](int row, double v) {
        const size_t e = (size_t)i * BP + row;
        cr_publish_granules(gdcv + 2 * e, stamp, v);
        dcv[e] = v;
        sdv[row] = v;
      });
  __syncthreads();
  cr_trial_rows(d, st, i, t < BP ? sdv[t] : 0.0, xpre, dtau, Xbuf, nullptr, normp, false, s_red);
}

// trial state X + delta, tau + dtau (clipped), norm partials per super-block. Variable
// shutter delay: block i back-substitutes the delays of frames 3i-2..3i (X rows 3i..3i+2),
// dtau[k, c] = -(g_c + h_c^T dx_k) / T_c over the local unknowns of frame k.
// Blocks b0 + blockIdx.x. The (replicated) const-mode delays are stepped by the first
// workgroup; their norm terms count only where tau_norm (once over the ranks).
// Frame-window ranks (normt != null): only the delays of the owned frames [klo, khi) are
// stepped (the others are copied: this rank's terms never read them); their norm terms go to
// normt so that they count over every block of the chain, not only the published rows'.
__global__ __launch_bounds__(256) void k_cr_trial(FteDims d, const FteState* __restrict__ st,
                                                  const double* __restrict__ dcv, const double* __restrict__ dtau,
                                                  const double* __restrict__ Hloc, const double* __restrict__ gloc,
                                                  double* __restrict__ Xbuf, double* __restrict__ taubuf,
                                                  double* __restrict__ normp, int hsel, int b0, int tau_norm,
                                                  int klo = 0, int khi = INT_MAX, double* __restrict__ normt = nullptr) {
  if (st->status != 0) return;
  if (hsel) {
    Hloc += (size_t)st->cur * d.N * FTE_NZP * FTE_NZP;
    gloc += (size_t)st->cur * d.N * FTE_NZP;
  }
  const int i = blockIdx.x + b0;
  const int P = d.P, BP = d.BP;
  __shared__ double s_red[256];
  const int cur = st->cur;
  const double* X = Xbuf + (size_t)cur * d.M * P;
  double* Xn = Xbuf + (size_t)(cur ^ 1) * d.M * P;
  double dn = 0.0, xn = 0.0;
  for (int e = threadIdx.x; e < 3 * P; e += blockDim.x) {
    const int f = 3 * i + e / P, p = e % P;
    if (f >= d.M) continue;
    const size_t o = (size_t)f * P + p;
    const double dv = dcv[(size_t)i * BP + e], x = X[o];
    Xn[o] = x + dv;
    dn += dv * dv;
    xn += x * x;
  }
  if (blockIdx.x == 0 && d.Cg) {
    const double* tau = taubuf + cur * d.NT;
    double* taun = taubuf + (cur ^ 1) * d.NT;
    for (int c = threadIdx.x; c < d.C; c += blockDim.x) {
      const double dv = (c == 0) ? 0.0 : dtau[c];
      taun[c] = (c == 0) ? 0.0 : fmin(fmax(tau[c] + dv, -d.Ts), d.Ts);
      if (tau_norm) {
        dn += dv * dv;
        xn += tau[c] * tau[c];
      }
    }
  }
  double dnt = 0.0, xnt = 0.0;
  if (d.var) {
    const int C = d.C;
    const double* tau = taubuf + (size_t)cur * d.NT;
    double* taun = taubuf + (size_t)(cur ^ 1) * d.NT;
    const double lam = st->lam;
    for (int e = threadIdx.x; e < 3 * C; e += blockDim.x) {
      const int k = 3 * i - 2 + e / C, c = e % C;
      if (k < 0 || k >= d.N) continue;
      if (k < klo || k >= khi) {
        taun[(size_t)k * C + c] = tau[(size_t)k * C + c];
        continue;
      }
      const double* H = Hloc + (size_t)k * FTE_NZP * FTE_NZP + (size_t)(P + 6 + c) * FTE_NZP;
      const double t = tau[(size_t)k * C + c], gc = gloc[(size_t)k * FTE_NZP + P + 6 + c];
      double dv = 0.0;
      if (!tau_held(t, gc, d.Ts, c)) {
        const int f = k + 2;
        double v = gc;
        for (int j = 0; j < P + 6; ++j) {
          const int row = j < P ? f : (j < P + 3 ? f - 1 : f - 2);
          const int p = j < P ? j : (j < P + 3 ? j - P : j - P - 3);
          v += H[j] * dcv[(size_t)(row / 3) * BP + (row % 3) * P + p];
        }
        const double h = H[P + 6 + c];
        dv = -v / (h + lam * fmax(h, 1e-12));
      }
      taun[(size_t)k * C + c] = (c == 0) ? 0.0 : fmin(fmax(t + dv, -d.Ts), d.Ts);
      dnt += dv * dv;
      xnt += t * t;
    }
  }
  if (!normt) {
    dn += dnt;
    xn += xnt;
  }
  dn = block_sum(dn, s_red);
  xn = block_sum(xn, s_red);
  if (threadIdx.x == 0 && i < d.nblk) {
    normp[2 * i] = dn;
    normp[2 * i + 1] = xn;
  }
  if (normt) {
    dnt = block_sum(dnt, s_red);
    xnt = block_sum(xnt, s_red);
    if (threadIdx.x == 0 && i < d.nblk) {
      normt[2 * i] = dnt;
      normt[2 * i + 1] = xnt;
    }
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
                                                 int k0, int lo, int hi,
                                                 double* __restrict__ Fm, double* __restrict__ Fq) {
  // block k: measurement of frame k (owned iff lo <= k < hi) and the model stencil ending
  // at row k + 2 (rows k-1..k+2, owned iff lo <= k-1 < hi)
  if (which == 1 && st->status != 0) return;
  const int k = blockIdx.x + k0;
  const bool own_meas = k >= lo && k < hi, own_model = k >= 1 && k - 1 >= lo && k - 1 < hi;
  const int tid = threadIdx.x;
  const int P = d.P, C = d.C, L = d.L;
  const int buf = which == 1 ? (st->cur ^ 1) : st->cur;
  const double* X = Xbuf + (size_t)buf * d.M * P;
  const double* tau = taubuf + (size_t)buf * d.NT + (d.var ? (size_t)k * C : 0);
  __shared__ FkShared fk;
  __shared__ double s_red[64];
  __shared__ double s_dx[3], s_ddx[3];
  const SkelView s = skel_view(I, Rl);  // 64 threads: staging the table in LDS costs more than it saves
  const int f = k + 2;
  if (tid < 3) {
    const double x0 = X[f * P + tid], x1 = X[(f - 1) * P + tid], x2 = X[(f - 2) * P + tid];
    s_dx[tid] = (x0 - x1) / d.Ts;
    s_ddx[tid] = (x0 - 2.0 * x1 + x2) / (d.Ts * d.Ts);
  }
  fk_frame(s, X + f * P, fk, tid, blockDim.x);
  __syncthreads();
  double rho = 0.0;
  for (int o = own_meas ? tid : C * L; o < C * L; o += blockDim.x) {
    const int c = o / L, l = o - (o / L) * L;
    const int node = s.outn[l];
    const double tc = d.Ct ? tau[c] : 0.0;
    double p[3];
    for (int i = 0; i < 3; ++i) {
      p[i] = fk.pos[node][i];
      if (d.im >= 1) p[i] += s_dx[i] * tc;
      if (d.im == 2) p[i] += s_ddx[i] * (tc * tc);
    }
    ProjOut po;
    const size_t mi = ((size_t)k * C + c) * L + l;
    const double wt = wts[mi], mu0 = meas[2 * mi], mv0 = meas[2 * mi + 1];  // one round trip
    fisheye_project<false, true>(cams + c * ACS_CAM_STRIDE, p[0], p[1], p[2], po);
    const double mu = wt != 0.0 ? mu0 : 0.0, mv = wt != 0.0 ? mv0 : 0.0;
    rho += redescending(wt * (po.u - mu), d.la, d.lb, d.lc).f + redescending(wt * (po.v - mv), d.la, d.lb, d.lc).f;
  }
  double q = 0.0;
  if (own_model) {
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
// Every non-init launch ends by writing the LM state into host snapshot slot (launch & 1)
// of `snap` (coherent pinned host memory, acs_pinned) and then the iteration count into the
// word after the two slots, which the host polls: the state goes out as system-scope
// (write-through) stores, and the count only after they have all completed, so a host that
// sees count n reads iteration n's state. No event between iterations: an event record
// between two graph launches cost ~13 us of idle GPU per iteration (a system-scope
// release behind the whole iteration), the poll costs nothing on the device.
__device__ __forceinline__ void fte_snapshot(FteState* st, FteState* snap) {
  if (!snap) return;
  const int slot = st->launch & 1, seq = st->launch + 1;
  st->launch = seq;
  static_assert(sizeof(FteState) % 8 == 0, "FteState is copied in 8-byte words");
  constexpr int NW = (int)(sizeof(FteState) / 8);
  const unsigned long long* src = reinterpret_cast<const unsigned long long*>(st);
  unsigned long long* dst = reinterpret_cast<unsigned long long*>(snap + slot);
  unsigned long long v[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) v[i] = src[i];  // all loads before the first store
#pragma unroll
  for (int i = 0; i < NW; ++i) __hip_atomic_store(dst + i, v[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(reinterpret_cast<int*>(snap + 2), seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one workgroup of FTE_LM_THREADS: the per-frame cost partials and per-block norm partials summed
// in a fixed order (256 threads took 16 us at 10,000 frames: 40 strided terms per thread)
#define FTE_LM_THREADS 1024
__global__ __launch_bounds__(FTE_LM_THREADS) void k_fte_lm(FteDims d, FteState* __restrict__ st, FteOptsDev o, int init,
                                                const double* __restrict__ Fm, const double* __restrict__ Fq,
                                                const double* __restrict__ normp, int spec,
                                                FteState* __restrict__ snap = nullptr) {
  __shared__ double s_red[4 * FTE_LM_THREADS];
  const int tid = threadIdx.x;
  // every load is issued before the LM state is read: both copies of the measurement terms
  // (spec: the trial's are in Floc copy cur ^ 1) and the step / state norm partials
  double acc[3] = {0.0, 0.0, 0.0}, nrm[2] = {0.0, 0.0};
  {
    const double* xs[3] = {Fm, spec ? Fm + d.N : Fm, Fq};
    strided_sums<3>(xs, 1, tid, d.N, blockDim.x, acc);
  }
  if (!init) {
    const double* xs[2] = {normp, normp + 1};
    strided_sums<2>(xs, 2, tid, d.nblk, blockDim.x, nrm);
  }
  const double a = (spec && (st->cur ^ 1)) ? acc[1] : acc[0];
  double sums[4] = {a, acc[2], nrm[0], nrm[1]};
  block_sums<4>(sums, s_red);
  const double fm = sums[0], fq = sums[1], dn = sums[2], xn = sums[3];
  if (init) {
    if (tid == 0) {
      st->F = st->F0 = fm + fq;
      st->Fmeas = fm;
      st->Fmodel = fq;
    }
    return;
  }
  if (st->status != 0) {
    if (tid == 0) fte_snapshot(st, snap);
    return;
  }
  if (tid != 0) return;
  if (st->gmax <= o.gtol) {
    st->status = ACS_STATUS_GTOL;
    fte_snapshot(st, snap);
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
  fte_snapshot(st, snap);
}

// =======================================================================================
// host side
// =======================================================================================
// both copies of X from Xsrc, tau copy 0 from tausrc (zeros if null) and copy 1 zeroed, the
// pivot counter and the tau step zeroed (Xsrc / tausrc may be copy 0 itself)
__global__ __launch_bounds__(256) void k_fte_init_state(double* __restrict__ X, const double* Xsrc, size_t MP,
                                                        double* __restrict__ tau, const double* tausrc, int NT,
                                                        int* __restrict__ bad, double* __restrict__ dtau, int GR,
                                                        int* __restrict__ bk, int nbk,
                                                        unsigned long long* __restrict__ gd, size_t ngd) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < MP) {
    const double v = Xsrc[i];
    X[i] = v;
    X[MP + i] = v;
  }
  if (i < (size_t)NT) {
    const double v = tausrc ? tausrc[i] : 0.0;
    tau[i] = v;
    tau[NT + i] = 0.0;
  }
  if (i < (size_t)GR) dtau[i] = 0.0;
  if (i < (size_t)nbk) bk[i] = 0;
  if (i < ngd) gd[i] = 0ull;
  if (i == 0) *bad = 0;
}

// the LM state of a new solve (acs_fte_dist_create's st0): first round pending, lambda0
__global__ void k_fte_state_reset(FteState* __restrict__ st, double lam0) {
  if (threadIdx.x != 0) return;
  FteState z;
  memset(&z, 0, sizeof(z));
  z.lam = lam0;
  z.relin = 1;
  z.first = 1;
  *st = z;
}

struct FteBuffers {
  int* I;
  double *Rl, *cams, *meas, *w, *qinv, *X, *tau;
  double *Hloc, *gloc, *Floc, *Tc, *Ab, *gb, *Bt, *gmaxp, *Dc, *Ec, *GBc, *Wc, *Tau, *dcv, *dtau, *normp, *Fm, *Fq, *part;
  double* Adiag;
  double *Ec2, *dL, *dR;  // second coupling buffer (levels alternate), pending Schur terms
  // frame-window ranks with per-frame delays: rows' gradients before the delay elimination,
  // per-row max |delay gradient| of the frame the row starts, per-block delay step / state norms
  double *graw, *gmaxt, *normt;
  int* bad;
  int* bk;                    // k_cr_back_all: ticket counter, partials counter
  unsigned long long* gdcv;   // k_cr_back_all: the step rows, then dtau, as {stamp, word} granules
  FteState* st;
};

// k_fte_linearize over frames [k0, k0 + nk) (spec: at the trial state, with the model terms in Fq)
static void fte_launch_lin(const FteDims& d, hipStream_t s, const FteBuffers& b, int force, int k0, int nk, int spec,
                           double* Fq, const double* qinv) {
  const LinKernel kf = lin_kernel(nk);
  const size_t lds = lin_lds_bytes(d);
  hipLaunchKernelGGL(kf, dim3(nk), dim3(256), lds, s, d, b.I, b.Rl, b.cams, b.meas, b.w, b.X, b.tau,
                     b.st, force, k0, b.Hloc, b.gloc, b.Floc, spec, Fq, qinv, b.Tc);
}

struct FteSetup {
  FteState* snap = nullptr;  // pinned host slots the LM kernel writes its state into
  FteDims d;
  FteBuffers b;
};

// Dimensions, device buffers and initial state of one FTE problem. With `owned` == NULL
// the buffers live in the context workspace (acs_fte_solve / acs_fte_eval); otherwise one
// hipMalloc block is allocated for them and returned in *owned (the distributed handles,
// several of which may share a context).
static int fte_setup(acs_ctx* ctx, FteSetup& S, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                     int64_t n_reals, const double* cams, int32_t n_cams, const double* meas, const double* w,
                     int32_t N, int32_t sd, double Ts, const double* qinv, int32_t sd_mode, int32_t intermode,
                     const double* X, const double* tau, double la, double lb, double lc, uint32_t flags,
                     void** owned = nullptr) {
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
  ACS_CHECK(ctx, sd_mode == 0 || sd_mode == 1, "fte: shutter_delay_mode %d (0 const, 1 variable)", sd_mode);
  FteDims& d = S.d;
  d.N = N;
  d.M = N + 2;
  d.P = P;
  d.L = L;
  d.C = n_cams;
  d.var = sd && sd_mode == 1;
  d.Ct = sd ? n_cams : 0;
  d.Cg = sd && !d.var ? n_cams : 0;
  d.NT = d.var ? N * n_cams : n_cams;
  d.nint = (int)n_ints;
  d.nreal = (int)n_reals;
  d.pad_ = 0;
  d.NZ = P + 6 + d.Ct;
  ACS_CHECK(ctx, d.NZ <= FTE_NZP, "fte: P + 6 + C = %d exceeds %d", d.NZ, FTE_NZP);
  d.im = intermode;
  d.Ts = Ts;
  d.la = la;
  d.lb = lb;
  d.lc = lc;
  d.nblk = (d.M + 2) / 3;
  d.BP = ((3 * P + 15) / 16) * 16;
  ACS_CHECK(ctx, d.BP <= CR_MAXBP, "fte: 3P = %d exceeds %d", 3 * P, CR_MAXBP);
  d.GR = ((d.Cg + 1 + 15) / 16) * 16;
  d.nlev = 0;
  for (int s = 1; s < d.nblk; s <<= 1) d.nlev++;
  const int M = d.M, C = d.C, BP = d.BP, GR = d.GR, n = d.nblk;
  FteBuffers& b = S.b;
  size_t off = 0;
  auto take = [&](size_t cnt) {
    size_t o = off;
    off += ((cnt * sizeof(double) + 255) / 256) * 256 / sizeof(double);
    return o;
  };
  const size_t Cg1 = d.Cg ? d.Cg : 1;
  // the per-frame linearisation is double-buffered: the speculative linearisation of the
  // trial state (k_fte_linearize spec = 1) writes copy cur ^ 1 (single-GPU and frame-window)
  const size_t nlin = 2;
  const size_t oX = take((size_t)2 * M * P), oT = take(2 * (size_t)d.NT), oAd = take((size_t)M * P),
               oH = take(nlin * N * FTE_NZP * FTE_NZP), og = take(nlin * N * FTE_NZP), oF = take(nlin * N), oAb = take((size_t)M * 4 * P * P),
               ogb = take((size_t)M * P), oBt = take((size_t)M * P * Cg1), ogm = take(M),
               oD = take((size_t)n * BP * BP), oE = take((size_t)n * BP * BP), oG = take((size_t)n * BP * GR),
               oW = take((size_t)n * BP * (2 * BP + GR)), oTau = take((size_t)n * GR * GR),
               oE2 = take((size_t)n * BP * BP), odL = take((size_t)n * BP * (BP + GR)),
               odR = take((size_t)n * BP * (BP + GR)),
               odc = take((size_t)n * BP), odt = take(GR), opart = take((size_t)CR_NCHUNK * (32 * 32 + 32 + 32 * 32 + 1)),
               onp = take(2 * (size_t)n), oTc = take(nlin * N * std::max(tc_stride(d.Cg), 1)), oFm = take(N), oFq = take(N), ost = take(16), oint = take(8),
               ogr = take((size_t)M * P), ogt = take(M), ont = take(2 * (size_t)n),
               obk = take((size_t)n / 2 + 2), ogd = take((size_t)n * BP * 2 + 64);
  // staged inputs (owned mode only)
  const size_t oI = take((n_ints + 1) / 2 + 1), oR = take(n_reals), oC = take((size_t)ACS_CAM_STRIDE * C),
               oMe = take((size_t)N * C * L * 2), oWt = take((size_t)N * C * L), oQ = take(P);
  double* arena;
  const size_t inputs_from = oI;
  hipStream_t s = ctx->stream;
  const hipMemcpyKind kin = (flags & ACS_DEVICE_PTRS) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  int rc;
  if (owned) {
    void* p = nullptr;
    ACS_HIP(ctx, acs_dev_malloc(&p, off * sizeof(double)));
    *owned = p;
    arena = (double*)p;
    b.I = (int*)(arena + oI);
    b.Rl = arena + oR;
    b.cams = arena + oC;
    b.meas = arena + oMe;
    b.w = arena + oWt;
    b.qinv = arena + oQ;
    ACS_HIP(ctx, hipMemcpyAsync(b.I, skel_ints, sizeof(int32_t) * n_ints, kin, s));
    ACS_HIP(ctx, hipMemcpyAsync(b.Rl, skel_reals, sizeof(double) * n_reals, kin, s));
    ACS_HIP(ctx, hipMemcpyAsync(b.cams, cams, sizeof(double) * ACS_CAM_STRIDE * C, kin, s));
    ACS_HIP(ctx, hipMemcpyAsync(b.meas, meas, sizeof(double) * (size_t)N * C * L * 2, kin, s));
    ACS_HIP(ctx, hipMemcpyAsync(b.w, w, sizeof(double) * (size_t)N * C * L, kin, s));
    ACS_HIP(ctx, hipMemcpyAsync(b.qinv, qinv, sizeof(double) * P, kin, s));
  } else {
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
    arena = (double*)acs_ws(ctx, WS_FTE5, inputs_from * sizeof(double));
    if (!arena) return ACS_E_NOMEM;
  }
  b.X = arena + oX;
  b.tau = arena + oT;
  b.Adiag = arena + oAd;
  b.Hloc = arena + oH;
  b.gloc = arena + og;
  b.Floc = arena + oF;
  b.Tc = arena + oTc;
  b.Ab = arena + oAb;
  b.gb = arena + ogb;
  b.Bt = arena + oBt;
  b.gmaxp = arena + ogm;
  b.Dc = arena + oD;
  b.Ec = arena + oE;
  b.GBc = arena + oG;
  b.Wc = arena + oW;
  b.Tau = arena + oTau;
  b.Ec2 = arena + oE2;
  b.dL = arena + odL;
  b.dR = arena + odR;
  b.dcv = arena + odc;
  b.part = arena + opart;
  b.dtau = arena + odt;
  b.normp = arena + onp;
  b.graw = arena + ogr;
  b.gmaxt = arena + ogt;
  b.normt = arena + ont;
  b.Fm = arena + oFm;
  b.Fq = arena + oFq;
  b.st = (FteState*)(arena + ost);
  b.bad = (int*)(arena + oint);
  b.bk = (int*)(arena + obk);
  b.gdcv = (unsigned long long*)(arena + ogd);
  // state buffers in one launch (was six copies / fills): host inputs are copied into copy 0
  // first and the kernel then works in place
  const double* Xs = X;
  const double* ts = tau;
  if (!(flags & ACS_DEVICE_PTRS)) {
    ACS_HIP(ctx, hipMemcpyAsync(b.X, X, sizeof(double) * M * P, hipMemcpyHostToDevice, s));
    if (tau) ACS_HIP(ctx, hipMemcpyAsync(b.tau, tau, sizeof(double) * d.NT, hipMemcpyHostToDevice, s));
    Xs = b.X;
    ts = tau ? b.tau : nullptr;
  }
  const size_t MP = (size_t)M * P;
  const size_t ngd = (size_t)n * BP * 2 + 64;
  const size_t nI = std::max(std::max(std::max(MP, (size_t)n + 1), ngd), (size_t)std::max(d.NT, GR));
  hipLaunchKernelGGL(k_fte_init_state, dim3(acs_grid((int64_t)nI, 256)), dim3(256), 0, s, b.X, Xs, MP, b.tau, ts,
                     d.NT, b.bad, b.dtau, GR, b.bk, n + 1, b.gdcv, ngd);
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

// workgroups per eliminated block of a k_cr_level launch: enough column waves (16 - NB per
// workgroup), and more of them when few blocks are left (the deep levels are latency-bound):
// the widest split whose grid still fits the 256 CUs in one wave of workgroups (one
// 1024-thread workgroup per CU: the LDS is full), one column-block per workgroup when
// possible, else 6 / 4 / 3 / 2 column-blocks' worth of workgroups per block
static int cr_nsplit(const FteDims& d, int ne, int ns) {
  const int NB = d.BP >> 4, NBB = 2 * NB + d.GR / 16;
  const int need = (NBB + 16 - NB - 1) / (16 - NB);
  int want = 1;
  for (int c : {NBB, 6, 4, 3, 2})
    if (c <= NBB && ne * c + ns <= 256) {
      want = c;
      break;
    }
  int n = std::min(std::max(need, want), NBB);
  // two GB column-blocks (GR = 32) over several workgroups: each workgroup's idle column
  // waves load the GB blocks it does not own (k_cr_level), so keep GRB of them idle
  const int GRB = d.GR / 16;
  while (GRB > 1 && n > 1 && n < NBB && 16 - NB - (NBB + n - 1) / n < GRB) ++n;
  return n;
}

// Pending-term bookkeeping of one cyclic reduction (k_cr_level): the terms of the levels with
// steps lo_s .. (current step)/2 have not been applied to the surviving blocks; bit l of
// symmask: the level of step 2^l stored its D parts as upper tiles.
struct CrPending {
  int lo_s = 1;
  unsigned symmask = 0;
};

// one k_cr_level launch (template on the tile count NB = BP/16). Returns whether this level's
// pending Schur terms are stored as upper tiles (the one-wave-per-column-block path; the deep
// path of k_cr_level writes full tiles).
static int cr_launch_level(const FteDims& d, hipStream_t s, int sl, int a0, int iend, int top, int ne, int ns,
                           int astep, const FteState* st, FteBuffers& b, const double* Ein, double* Eout, int* bad,
                           const CrPending& pend, int l0 = 0, int d_up = 0) {
  if (ne + ns == 0) return 0;
  const int NB = d.BP >> 4, NBB = 2 * NB + d.GR / 16;
  const int nsplit = cr_nsplit(d, ne, ns);
  const int nwg = ne * nsplit + ns;
  const size_t lds = sizeof(double) * cr_level_lds_doubles(d.BP, d.GR);
#define CR_LEVEL_(nb, gb2, dup)                                                                                  \
  hipLaunchKernelGGL((k_cr_level<nb, gb2, dup>), dim3(nwg), dim3(1024), lds, s, d, sl, a0, iend, top, ne, astep,    \
                     nsplit, pend.symmask, pend.lo_s, 0, l0, st, b.Dc, Ein, Eout, b.GBc, b.Wc, b.Tau, b.dL, b.dR, bad, \
                     CrTauSrc{})
#define CR_LEVEL(nb)                \
  if (d.GR > 16)                    \
    CR_LEVEL_(nb, true, false);     \
  else if (d_up)                    \
    CR_LEVEL_(nb, false, true);     \
  else                              \
    CR_LEVEL_(nb, false, false)
  switch (NB) {
    case 1: CR_LEVEL(1); break;
    case 2: CR_LEVEL(2); break;
    case 3: CR_LEVEL(3); break;
    case 4: CR_LEVEL(4); break;
    case 5: CR_LEVEL(5); break;
    default: CR_LEVEL(6); break;
  }
#undef CR_LEVEL
#undef CR_LEVEL_
  // the kernel's deep-path test (full tiles)
  const int BPq = d.BP, BUF = 16 * 17 + 16 * BPq + BPq * 17;
  const bool deep = nsplit >= 3 && ((NBB + nsplit - 1) / nsplit) * BPq * 16 <= 2 * BUF;
  return (ne > 0 && !deep) ? 1 : 0;
}

static bool cr_defer() {
  static const bool v = [] {
    const char* e = std::getenv("ACS_CR_DEFER");
    return e && e[0] == '1';
  }();
  return v;
}
// the single-GPU solve stores D as its upper tiles (k_cr_assemble_build) and levels 0-1 read it
// so (k_cr_level DUP): constant / no delays (the per-frame-delay mode builds through k_cr_build),
// one GB column-block (the GB2 instances have no DUP form), survivors not deferred
// (ACS_D_FULL=1: D stored whole, for A/B timing)
static bool fte_d_upper(const FteDims& d) {
  static const bool full = [] {
    const char* e = std::getenv("ACS_D_FULL");
    return e && e[0] == '1';
  }();
  return !d.var && d.GR <= 16 && !cr_defer() && !full;
}

// Block cyclic reduction of super-blocks [a0, top] (blocks < iend may be eliminated; a
// chain end at iend survives), nlev levels, then (final_apply) every pending Schur term is
// applied to the survivors. Survivor workgroups apply the previous level's terms at every
// level. ACS_CR_DEFER=1 launches them only at a level whose grid then still fits the chip in
// one wave of workgroups, and the blocks subtract the deferred terms when they are next loaded:
// at 10,000 frames that saved 26 us at level 1 and cost 30 us at levels 2-4 (each deferred
// term is one more dependent round of loads, profiles/r05/seq10k_*.log), so it is off.
// Returns the buffer holding the final couplings E; *pend_out: what is still pending (for the
// top block).
static const double* cr_reduce(const FteDims& d, hipStream_t s, const FteState* st, FteBuffers& b, int a0, int iend,
                               int top, int nlev, int* bad, bool final_apply = true, CrPending* pend_out = nullptr,
                               bool e_upper = true, bool d_upper = false) {
  const bool defer = cr_defer();
  const double* Ein = b.Ec;
  double* Eout = b.Ec2;
  CrPending pend;
  int sl = 1;
  for (int lv = 0; lv < nlev; ++lv, sl <<= 1) {
    int ne = 0, ns = 0;
    for (int i = a0 + sl; i < iend; i += 2 * sl) ++ne;
    if (sl > 1)
      for (int j = a0; j <= top; j += 2 * sl) ++ns;
    if (ns && defer && ne * cr_nsplit(d, ne, ns) + ns > 256) ns = 0;  // defer
    // level 0 of a chain built by k_cr_assemble_build / k_cr_build: every E is upper triangular.
    // d_upper (D stored as upper tiles): levels 0 and 1 read D as assembled (the level-1
    // survivors rewrite theirs whole; every block eliminated later is one of them)
    const int sym = cr_launch_level(d, s, sl, a0, iend, top, ne, ns, 2 * sl, st, b, Ein, Eout, bad, pend,
                                    lv == 0 && e_upper ? 1 : 0, d_upper && lv <= 1 ? 1 : 0);
    if (ns) pend.lo_s = sl;  // the survivors now hold every term of the levels below sl
    pend.symmask |= (unsigned)sym << lv;
    double* t = const_cast<double*>(Ein);
    Ein = Eout;
    Eout = t;
  }
  if (nlev > 0 && final_apply) {
    int ns = 0;
    for (int j = a0; j <= top; j += sl) ++ns;
    cr_launch_level(d, s, sl, a0, iend, top, 0, ns, sl, st, b, Ein, Eout, bad, pend, 0, d_upper && nlev <= 1 ? 1 : 0);
    pend.lo_s = sl;
  }
  if (pend_out) *pend_out = pend;
  return Ein;
}

// The single surviving block a0 after nlev levels (step sl = 2^nlev): its pending terms,
// then W_gb = D^-1 GB and Tau = GB^T W_gb on the register-tiled Gauss-Jordan of k_cr_level
// (top_mode); k_cr_top finishes with the tau border.
// with_partials: CR_NCHUNK more workgroups form the tau border partial sums and the frames'
// |g| max (b.part) meanwhile, for k_cr_back_all (the single-GPU chain, a0 = 0)
static void cr_launch_top(const FteDims& d, hipStream_t s, int nlev, int a0, int iend, const FteState* st,
                          FteBuffers& b, int* bad, const CrPending& pend, bool with_partials = false,
                          int d_up = 0) {
  const CrTauSrc ts = with_partials ? CrTauSrc{b.Tc, b.gmaxp, b.part} : CrTauSrc{};
  const int nwg = with_partials ? 1 + CR_NCHUNK : 1;
  const int sl = 1 << nlev, NB = d.BP >> 4;
  const size_t lds = sizeof(double) * cr_level_lds_doubles(d.BP, d.GR);
#define CR_TOP_(nb, gb2, dup)                                                                                        \
  hipLaunchKernelGGL((k_cr_level<nb, gb2, dup>), dim3(nwg), dim3(1024), lds, s, d, sl, a0, iend, a0, 1, sl, 1,      \
                     pend.symmask, pend.lo_s, 1, 0, st, b.Dc, b.Ec, b.Ec2, b.GBc, b.Wc, b.Tau, b.dL, b.dR, bad, ts)
#define CR_TOP(nb)               \
  if (d.GR > 16)                 \
    CR_TOP_(nb, true, false);    \
  else if (d_up)                 \
    CR_TOP_(nb, false, true);    \
  else                           \
    CR_TOP_(nb, false, false)
  switch (NB) {
    case 1: CR_TOP(1); break;
    case 2: CR_TOP(2); break;
    case 3: CR_TOP(3); break;
    case 4: CR_TOP(4); break;
    case 5: CR_TOP(5); break;
    default: CR_TOP(6); break;
  }
#undef CR_TOP
#undef CR_TOP_
}

static void cr_launch_assemble_build(const FteDims& d, hipStream_t s, const FteBuffers& b, int b0 = 0,
                                     int nblk = -1, int lo = 0, int hi = INT_MAX, int end_l = -1, int end_r = -1,
                                     double* rdiag = nullptr, double* graw = nullptr, int d_full = 0) {
  if (nblk < 0) nblk = d.nblk;
  if (nblk <= 0) return;
  static const int n_cu = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    return hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }();
  const bool wide = nblk > 2 * n_cu;  // more than one round of 1024-thread blocks
#define CR_ABUILD_(nb, th)                                                                                  \
  hipLaunchKernelGGL((k_cr_assemble_build<nb, th>), dim3(nblk), dim3(th), asm_build_lds_bytes(d, th < 1024), s, d, b.X, \
                     b.qinv, b.st, b.Hloc, b.gloc, b.Dc, b.Ec, b.GBc, b.gmaxp, b0, lo, hi, end_l, end_r, rdiag, graw, \
                     d_full)
#define CR_ABUILD(nb)         \
  if (wide)                   \
    CR_ABUILD_(nb, 512);      \
  else                        \
    CR_ABUILD_(nb, 1024)
  switch (d.BP >> 4) {
    case 1: CR_ABUILD(1); break;
    case 2: CR_ABUILD(2); break;
    case 3: CR_ABUILD(3); break;
    case 4: CR_ABUILD(4); break;
    case 5: CR_ABUILD(5); break;
    default: CR_ABUILD(6); break;
  }
#undef CR_ABUILD
#undef CR_ABUILD_
}

static void fte_enqueue_linearize(FteSetup& S, hipStream_t s, int force) {
  const FteDims& d = S.d;
  FteBuffers& b = S.b;
  fte_launch_lin(d, s, b, force, 0, d.N, 0, (double*)nullptr, (const double*)nullptr);
  hipLaunchKernelGGL(k_fte_assemble, dim3(d.M), dim3(256), 0, s, d, b.X, b.tau, b.qinv, b.st, force, 0, 0, INT_MAX,
                     b.Hloc, b.gloc, b.Ab, b.gb, b.Bt, b.gmaxp, b.Adiag, 1);
}

// one LM iteration: linearise (if the last step was accepted), cyclic-reduction solve,
// trial state, exact cost, accept/reject — all device-resident, no host round trip
static void fte_enqueue_iteration(FteSetup& S, hipStream_t s, const FteOptsDev& o) {
  const FteDims& d = S.d;
  FteBuffers& b = S.b;
  // the linearisation of X[cur] is already there (initial, or speculative at the last
  // accepted trial): assemble the banded rows and build the damped super-blocks (variable
  // delays: assembled when new or re-eliminated for a new damping, then built)
  if (d.var) {
    hipLaunchKernelGGL(k_fte_assemble, dim3(d.M), dim3(256), 0, s, d, b.X, b.tau, b.qinv, b.st, 0, 0, 0, INT_MAX,
                       b.Hloc, b.gloc, b.Ab, b.gb, b.Bt, b.gmaxp, b.Adiag, 1);
    cr_launch_build(d, s, d.nblk, b.st, b.Ab, b.gb, b.Bt, b.Dc, b.Ec, b.GBc, 0, -1, -1, b.Adiag);
  } else {
    cr_launch_assemble_build(d, s, b, 0, -1, 0, INT_MAX, -1, -1, nullptr, nullptr, fte_d_upper(d) ? 0 : 1);
  }
  const int bend = d.nblk - 1;
  CrPending pend;
  // D stored as upper tiles by k_cr_assemble_build (constant / no delays; the per-frame-delay
  // mode builds through k_cr_build, whole): read as assembled by levels 0-1 and by the top block
  // when no survivor ever rewrote it (nlev <= 1); off with ACS_CR_DEFER (survivors deferred)
  const bool dup = fte_d_upper(d);
  cr_reduce(d, s, b.st, b, 0, d.nblk, d.nblk - 1, d.nlev, b.bad, false, &pend, true, dup);
  cr_launch_top(d, s, d.nlev, 0, d.nblk, b.st, b, b.bad, pend, true, dup && d.nlev <= 1 ? 1 : 0);
  // the top block and every back-substitution level in one launch, chained by
  // per-launch stamps (running the top levels' few blocks one after the other inside one
  // workgroup was tried in r03 and took 30 us: one workgroup streams a block's W at ~2 us, so
  // the W loads of every block have to be in flight at once). Constant / no delays: the
  // trial state is stepped there too; variable delays need the neighbours' rows: k_cr_trial
  double* Xt = d.var ? nullptr : b.X;
  // 8 lanes per row of a block (cr_back_block): 640 threads at BP = 80, so two workgroups
  // share a CU (91 VGPRs, 5 waves per SIMD) and one's W loads overlap the other's wait
  // (template sizes: the columns each lane of a row holds, BP / 8 and GR / 8, no padding)
  const int nth_back = (8 * d.BP + 63) / 64 * 64;
  // blocks of levels >= late_lv wait for their inputs before loading W (ACS_BACK_LATE_LV; 30: never)
  static const int late_lv = [] {
    const char* e = std::getenv("ACS_BACK_LATE_LV");
    const int v = e ? std::atoi(e) : 30;
    return v < 0 ? 0 : (v > 30 ? 30 : v);  // k_cr_back_all shifts 1 << late_lv
  }();
#define CR_BACK_ALL(nb, grb)                                                                                   \
  hipLaunchKernelGGL((k_cr_back_all<nb, grb>), dim3(d.nblk), dim3(nth_back), 0, s, d, bend, b.st,  \
                     (const double*)b.Wc, (const double*)b.Tau, (const double*)b.part, (const double*)b.gmaxp, \
                     b.tau, b.dtau, b.dcv, b.bk, b.gdcv,    \
                     b.bad, Xt, b.normp, late_lv)
#define CR_BACK_ALL_G(nb) \
  if (d.GR <= 16)         \
    CR_BACK_ALL(nb, 1);   \
  else                    \
    CR_BACK_ALL(nb, 2)
  switch (d.BP >> 4) {
    case 1: CR_BACK_ALL_G(1); break;
    case 2: CR_BACK_ALL_G(2); break;
    case 3: CR_BACK_ALL_G(3); break;
    case 4: CR_BACK_ALL_G(4); break;
    case 5: CR_BACK_ALL_G(5); break;
    default: CR_BACK_ALL_G(6); break;
  }
#undef CR_BACK_ALL_G
#undef CR_BACK_ALL
  if (d.var)
    hipLaunchKernelGGL(k_cr_trial, dim3(d.nblk), dim3(256), 0, s, d, b.st, b.dcv, b.dtau, b.Hloc, b.gloc, b.X, b.tau,
                       b.normp, 1, 0, 1);
  // speculative linearisation at the trial state: its measurement terms and the model terms
  // are the trial cost (no separate cost pass)
  fte_launch_lin(d, s, b, 0, 0, d.N, 1, b.Fq, b.qinv);
  hipLaunchKernelGGL(k_fte_lm, dim3(1), dim3(FTE_LM_THREADS), 0, s, d, b.st, o, 0, b.Floc, b.Fq, b.normp, 1, S.snap);
}

// =======================================================================================
// frame-window distributed solve (spec: oracle/fte_dist.py)
//
// Super-blocks are split into R chains [a_r, a_r + 2^k] that share their end blocks
// (a_r = r 2^k; blocks past the sequence are phantoms). A term is owned by the chain
// containing its lowest row, so every term is counted on exactly one rank and the
// chain-end blocks hold partial sums. Per LM iteration:
//   phase 1  linearise owned frames, assemble chain rows, block cyclic reduction of the
//            chain interior down to its two ends (ends undamped), pack the ends' blocks,
//            raw diagonals / gradients, tau partial sums and an interior |g| max into
//            payload 1 (zeros elsewhere)                                 -> all-reduce
//   phase 2  every rank: reduced block-tridiagonal system over the R+1 chain ends + tau
//            (damped with the summed raw diagonals), solved with the same CR kernels;
//            back substitution down its own chain; its rows of delta into payload 2
//                                                                        -> all-reduce
//   phase 3  trial state on every rank (replicated X), cost of the owned terms
//                                                        -> all-reduce (2 doubles)
//   phase 4  the same accept/reject decision on every rank
// =======================================================================================
struct DistLayout {
  size_t oD, oE, oG, oGraw, oRdiag, oTau, oGmax, n1, n2, n3;
};

static DistLayout dist_layout(const FteDims& d, int R) {
  DistLayout L;
  const size_t nb = R + 1, BP = d.BP, GR = d.GR, nE = (size_t)d.Cg * d.Cg + d.Cg + (size_t)GR * GR;
  L.oD = 0;
  L.oE = L.oD + nb * BP * BP;
  L.oG = L.oE + nb * BP * BP;
  L.oGraw = L.oG + nb * BP * GR;
  L.oRdiag = L.oGraw + nb * BP;
  L.oTau = L.oRdiag + nb * BP;
  L.oGmax = L.oTau + nE;
  L.n1 = L.oGmax + R;
  L.n2 = (size_t)d.nblk * BP + (d.var ? (size_t)d.NT : 0);  // solution rows (+ per-frame delays)
  L.n3 = 4;
  return L;
}

// chain ends -> payload slots `rank` (left end a0) and `rank + 1` (right end bend)
__global__ __launch_bounds__(256) void k_dist_pack(FteDims d, const FteState* __restrict__ st, DistLayout Lo,
                                                   int rank, int a0, int bend, const double* __restrict__ Dc,
                                                   const double* __restrict__ Ec, const double* __restrict__ GBc,
                                                   const double* __restrict__ rdiag, const double* __restrict__ gb,
                                                   double* __restrict__ p1) {
  if (st->status != 0) return;
  const int side = blockIdx.y;  // 0 left end, 1 right end
  const int blk = side ? bend : a0, q = rank + side;
  if (blk >= d.nblk) return;
  const int BP = d.BP, GR = d.GR, P = d.P;
  const size_t nBB = (size_t)BP * BP;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < nBB; e += (size_t)gridDim.x * blockDim.x) {
    p1[Lo.oD + q * nBB + e] = Dc[(size_t)blk * nBB + e];
    if (side) p1[Lo.oE + q * nBB + e] = Ec[(size_t)blk * nBB + e];
  }
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < (size_t)BP * GR;
       e += (size_t)gridDim.x * blockDim.x)
    p1[Lo.oG + (size_t)q * BP * GR + e] = GBc[(size_t)blk * BP * GR + e];
  if (blockIdx.x == 0) {
    for (int r = threadIdx.x; r < BP; r += blockDim.x) {
      const int fr = 3 * blk + r / P, pr = r % P;
      const bool in = r < 3 * P && fr < d.M;
      p1[Lo.oGraw + (size_t)q * BP + r] = in ? gb[(size_t)fr * P + pr] : 0.0;
      p1[Lo.oRdiag + (size_t)q * BP + r] = in ? rdiag[(size_t)fr * P + pr] : 0.0;
    }
  }
}

// tau partial sums of the chain (fixed chunk order) and the |g| max of its interior rows
__global__ __launch_bounds__(256) void k_dist_pack_small(FteDims d, const FteState* __restrict__ st, DistLayout Lo,
                                                         int rank, int a0, int bend,
                                                         const double* __restrict__ part,
                                                         const double* __restrict__ gmaxp,
                                                         double* __restrict__ p1,
                                                         const double* __restrict__ gmaxt = nullptr) {
  if (st->status != 0) return;
  __shared__ double s_red[256];
  const int nE = d.Cg * d.Cg + d.Cg + d.GR * d.GR;
  for (int e = threadIdx.x; e < nE; e += blockDim.x) {
    double v = 0.0;
    for (int ch = 0; ch < CR_NCHUNK; ++ch) v += part[(size_t)ch * nE + e];
    p1[Lo.oTau + e] = v;
  }
  const int f0 = 3 * (a0 + 1), f1 = min(3 * min(bend, d.nblk), d.M);
  double mx = 0.0;
  mx = strided_max(gmaxp, f0 + (int)threadIdx.x, f1, blockDim.x, mx);
  // per-frame delays: every owned frame's (rows of the whole chain; other frames give 0)
  if (gmaxt) mx = strided_max(gmaxt, 3 * a0 + (int)threadIdx.x, min(3 * min(bend, d.nblk - 1) + 3, d.M), blockDim.x, mx);
  mx = block_max(mx, s_red);
  if (threadIdx.x == 0) p1[Lo.oGmax + rank] = mx;
}

// reduced system over the chain ends e_q = q 2^k (q = 0..R) from the summed payload
__global__ __launch_bounds__(256) void k_red_build(FteDims d, const FteState* __restrict__ st, DistLayout Lo, int R,
                                                   int span, const double* __restrict__ p1, double* __restrict__ Dr,
                                                   double* __restrict__ Er, double* __restrict__ GBr,
                                                   double* __restrict__ gmaxr) {
  if (st->status != 0) return;
  __shared__ double s_red[256];
  const int q = blockIdx.x, e = q * span;
  const int BP = d.BP, GR = d.GR, P = d.P;
  const size_t nBB = (size_t)BP * BP;
  const double lam = st->lam;
  // rows of block x that are real unknowns (not padding / phantom)
  auto live = [&](int x, int r) { return x >= 0 && x < d.nblk && r < 3 * P && 3 * x + r / P < d.M; };
  for (size_t x = threadIdx.x; x < nBB; x += blockDim.x) {
    const int r = (int)(x / BP), c = (int)(x % BP);
    double v = (r == c) ? 1.0 : 0.0;
    if (live(e, r) && live(e, c)) {
      v = p1[Lo.oD + q * nBB + x];
      if (r == c) v += lam * fmax(p1[Lo.oRdiag + (size_t)q * BP + r], 1e-12);
    }
    Dr[q * nBB + x] = v;
    Er[q * nBB + x] = (q > 0 && live(e, r) && live(e - span, c)) ? p1[Lo.oE + q * nBB + x] : 0.0;
  }
  for (size_t x = threadIdx.x; x < (size_t)BP * GR; x += blockDim.x) {
    const int r = (int)(x / GR);
    GBr[(size_t)q * BP * GR + x] = live(e, r) ? p1[Lo.oG + (size_t)q * BP * GR + x] : 0.0;
  }
  if (q == 0) {
    double mx = 0.0;
    for (int t = threadIdx.x; t < R; t += blockDim.x) mx = fmax(mx, p1[Lo.oGmax + t]);
    for (int t = threadIdx.x; t < (R + 1) * BP; t += blockDim.x) {
      const int qq = t / BP, r = t % BP, ee = qq * span;
      if (ee < d.nblk && r < 3 * P && 3 * ee + r / P < d.M) mx = fmax(mx, fabs(p1[Lo.oGraw + t]));
    }
    mx = block_max(mx, s_red);
    if (threadIdx.x == 0) gmaxr[0] = mx;
  }
}

__global__ void k_red_part(int nE, const DistLayout Lo, const FteState* __restrict__ st,
                           const double* __restrict__ p1, double* __restrict__ partr) {
  if (st->status != 0) return;
  for (int e = threadIdx.x; e < nE; e += blockDim.x) partr[e] += p1[Lo.oTau + e];
}

__global__ void k_dist_scatter(FteDims d, const FteState* __restrict__ st, int rank, int a0, int bend,
                               const double* __restrict__ dcvr, double* __restrict__ dcv) {
  if (st->status != 0) return;
  for (int r = threadIdx.x; r < d.BP; r += blockDim.x) {
    if (a0 < d.nblk) dcv[(size_t)a0 * d.BP + r] = dcvr[(size_t)rank * d.BP + r];
    if (bend < d.nblk) dcv[(size_t)bend * d.BP + r] = dcvr[(size_t)(rank + 1) * d.BP + r];
  }
}

// p3 = (measurement cost, model cost, |step|^2, |X, tau|^2) of this rank's owned terms /
// rows (frames [k0, k1), super-blocks [n0, n1) of the trial's norm partials)
// which = 1: the trial's measurement terms are in Fm's speculative copy (cur ^ 1, N each)
__global__ __launch_bounds__(256) void k_dist_cost_pack(FteState* __restrict__ st, int which, int N, int m0,
                                                        int m1, int q0, int q1, const double* __restrict__ Fm,
                                                        const double* __restrict__ Fq, int n0, int n1,
                                                        const double* __restrict__ normp, double* __restrict__ p3,
                                                        int t0 = 0, int t1 = 0,
                                                        const double* __restrict__ normt = nullptr) {
  if (which == 1 && st->status != 0) return;
  if (which == 1) Fm += (size_t)(st->cur ^ 1) * N;
  __shared__ double s_red[256];
  double a = 0.0, b = 0.0, nrm[2] = {0.0, 0.0};
  {
    const double* xs[1] = {Fm};
    strided_sums<1>(xs, 1, m0 + (int)threadIdx.x, m1, blockDim.x, &a);
  }
  {
    const double* xs[1] = {Fq};
    strided_sums<1>(xs, 1, q0 + (int)threadIdx.x, q1, blockDim.x, &b);
  }
  if (n1 > n0) {
    const double* xs[2] = {normp, normp + 1};
    strided_sums<2>(xs, 2, n0 + (int)threadIdx.x, n1, blockDim.x, nrm);
  }
  if (normt && t1 > t0) {  // per-frame delays of the owned frames, over every block of the chain
    const double* xs[2] = {normt, normt + 1};
    strided_sums<2>(xs, 2, t0 + (int)threadIdx.x, t1, blockDim.x, nrm);
  }
  double dn = nrm[0], xn = nrm[1];
  a = block_sum(a, s_red);
  b = block_sum(b, s_red);
  dn = block_sum(dn, s_red);
  xn = block_sum(xn, s_red);
  if (threadIdx.x == 0) {
    p3[0] = a;
    p3[1] = b;
    p3[2] = dn;
    p3[3] = xn;
    if (which == 1) st->pending = 1;  // this round took a step: its cost travels in p3
  }
}

// X[cur] rows of super-blocks [b_lo, b_hi) in the block layout of the step (BP per block);
// per-frame delays: those of the owned frames [k_lo, k_hi) after the rows
__global__ __launch_bounds__(256) void k_dist_x_out(FteDims d, const FteState* __restrict__ st, int b_lo, int b_hi,
                                                    const double* __restrict__ Xbuf, double* __restrict__ p2,
                                                    const double* __restrict__ taubuf, int k_lo, int k_hi) {
  const double* X = Xbuf + (size_t)st->cur * d.M * d.P;
  const int P = d.P, BP = d.BP;
  for (size_t e = (size_t)b_lo * BP + (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < (size_t)b_hi * BP;
       e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / BP), r = (int)(e % BP), f = 3 * i + r / P;
    if (r < 3 * P && f < d.M) p2[e] = X[(size_t)f * P + r % P];
  }
  if (d.var) {
    const double* tau = taubuf + (size_t)st->cur * d.NT;
    for (size_t e = (size_t)k_lo * d.C + (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < (size_t)k_hi * d.C;
         e += (size_t)gridDim.x * blockDim.x)
      p2[(size_t)d.nblk * BP + e] = tau[e];
  }
}

// every row of X[cur] (and every per-frame delay) from the gathered layout
__global__ __launch_bounds__(256) void k_dist_x_in(FteDims d, const FteState* __restrict__ st,
                                                   const double* __restrict__ p2, double* __restrict__ Xbuf,
                                                   double* __restrict__ taubuf) {
  double* X = Xbuf + (size_t)st->cur * d.M * d.P;
  const int P = d.P, BP = d.BP;
  for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < (size_t)d.nblk * BP;
       e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e / BP), r = (int)(e % BP), f = 3 * i + r / P;
    if (r < 3 * P && f < d.M) X[(size_t)f * P + r % P] = p2[e];
  }
  if (d.var) {
    double* tau = taubuf + (size_t)st->cur * d.NT;
    for (size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x; e < (size_t)d.NT; e += (size_t)gridDim.x * blockDim.x)
      tau[e] = p2[(size_t)d.nblk * BP + e];
  }
}

// Round control (one thread). On the summed payload of the previous round: the first round
// takes the initial cost; otherwise a pending step is accepted or rejected (oracle/fte.py
// solve; every rank takes the same decision). A rejection marks the round SKIP: its solve
// is stale (formed for the trial state) and the round only re-forms the reduced system.
__global__ void k_dist_decide(FteState* __restrict__ st, FteOptsDev o, const double* __restrict__ p3) {
  if (threadIdx.x != 0) return;
  const double fm = p3[0], fq = p3[1];
  if (st->first) {
    st->first = 0;
    st->F = st->F0 = fm + fq;
    st->Fmeas = fm;
    st->Fmodel = fq;
    // max_iters = 0: no step at all, as acs_fte_solve (X0 back, iters 0)
    if (o.max_iters <= 0) st->status = ACS_STATUS_MAXITER;
    return;
  }
  if (st->status != 0 || !st->pending) return;
  st->pending = 0;
  const double Fn = fm + fq, dn = p3[2], xn = p3[3];  // step / state norms summed over the owned rows
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
  if (st->status == 0 && !st->relin) st->status = FTE_STATUS_SKIP;
}

// after the reduced solve of a live round: the gradient test on the summed gradient
__global__ void k_dist_gtol(FteState* __restrict__ st, FteOptsDev o) {
  if (threadIdx.x == 0 && st->status == 0 && st->gmax <= o.gtol) st->status = ACS_STATUS_GTOL;
}

// before / after the round's reduced system: a round that took a step forms it at the trial
// state (copy cur ^ 1, linearised there for the trial cost) with the damping an acceptance
// sets; the LM state is swapped for those kernels and restored after them
__global__ void k_dist_spec(FteState* __restrict__ st, int enter) {
  if (threadIdx.x != 0) return;
  if (enter) {
    if (st->status == FTE_STATUS_SKIP) st->status = 0;
    if (st->status == 0 && st->pending) {
      st->spec_on = 1;
      st->save_cur = st->cur;
      st->save_lam = st->lam;
      st->cur ^= 1;
      st->lam = fmax(st->lam * 0.1, 1e-15);
    }
  } else if (st->spec_on) {
    st->spec_on = 0;
    st->cur = st->save_cur;
    st->lam = st->save_lam;
  }
}

struct acs_fte_dist {
  acs_ctx* ctx;
  FteSetup S;
  void* own = nullptr;
  void* own_red = nullptr;
  FteDims dr;        // reduced system dims (R + 1 blocks)
  FteBuffers r;      // reduced arrays (Dc, Ec, GBc, Wc, Tau, dcv, part, gmaxp)
  DistLayout Lo;
  FteOptsDev o;
  int R, rank, span, a0, bend, klev;
  double lam0;  // the LM's initial damping (acs_fte_dist_reset restarts from it)
  int k_lo, k_hi, f_lo, f_hi, b_hi_build, c_lo, c_hi, own_lo, own_hi, out_lo, out_hi;
  // rounds captured as hipGraphs (one graph launch instead of ~60 kernel launches); key =
  // (input payload, output payload, stream): two graphs for the two payload buffers
  struct Captured {
    hipGraphExec_t exec = nullptr;
    const void* ptr = nullptr;
    const void* ptr2 = nullptr;
    hipStream_t stream = nullptr;
  } g[2];
  // status after each round: pinned ring of ACS_DIST_RING slots with completion events
  int32_t* snap = nullptr;
  hipEvent_t snap_ev[4] = {};
  int64_t rounds = 0;
};
#define ACS_DIST_RING 4

// Run `enqueue` (kernel launches on ctx->stream) through the phase's cached graph,
// capturing it when the key changed; plain launches if capture is unavailable.
template <typename F>
static int dist_run_captured(acs_fte_dist* h, const void* ptr, const void* ptr2, F enqueue) {
  acs_ctx* ctx = h->ctx;
  hipStream_t s = ctx->stream;
  int which = 0;
  for (; which < 2; ++which)
    if (h->g[which].exec && h->g[which].ptr == ptr && h->g[which].ptr2 == ptr2 && h->g[which].stream == s) break;
  if (which == 2) which = (h->g[0].exec && !h->g[1].exec) ? 1 : 0;
  auto& c = h->g[which];
  if (!c.exec || c.ptr != ptr || c.ptr2 != ptr2 || c.stream != s) {
    if (c.exec) (void)hipGraphExecDestroy(c.exec);
    c.exec = nullptr;
    hipGraph_t graph = nullptr;
    if (hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed) == hipSuccess) {
      const int rc = enqueue();
      const hipError_t e = hipStreamEndCapture(s, &graph);
      if (rc) {
        if (graph) (void)hipGraphDestroy(graph);
        return rc;
      }
      if (e == hipSuccess && graph && hipGraphInstantiate(&c.exec, graph, nullptr, nullptr, 0) == hipSuccess) {
        c.ptr = ptr;
        c.ptr2 = ptr2;
        c.stream = s;
      } else {
        c.exec = nullptr;
      }
      if (graph) (void)hipGraphDestroy(graph);
    }
    if (!c.exec) {
      (void)hipGetLastError();
      return enqueue();
    }
  }
  ACS_HIP(ctx, hipGraphLaunch(c.exec, s));
  return ACS_OK;
}

static const double* dist_local_cr(acs_fte_dist* h) {
  const FteDims& d = h->S.d;
  FteBuffers& b = h->S.b;
  const int top = std::min(h->bend, d.nblk - 1);  // last existing block of the chain
  return cr_reduce(d, h->ctx->stream, b.st, b, h->a0, std::min(h->bend, d.nblk), top, h->klev, b.bad);
}

// Wait until the solve loop's iteration count in the pinned word after the two snapshot
// slots (fte_snapshot) reaches `want`. The stream is queried now and then, so a failed or
// drained stream ends the wait with an error instead of a hang.
static int fte_wait_snapshot(acs_ctx* ctx, hipStream_t s, FteState* snap, int want) {
  const int* seqw = reinterpret_cast<const int*>(snap + 2);
  for (unsigned it = 1;; ++it) {
    if (__atomic_load_n(seqw, __ATOMIC_ACQUIRE) >= want) return ACS_OK;
    if ((it & 4095) == 0) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) {  // everything queued has finished: the count is final
        if (__atomic_load_n(seqw, __ATOMIC_ACQUIRE) >= want) return ACS_OK;
        return acs_fail(ctx, ACS_E_HIP, "fte: stream idle at iteration count %d, expected %d",
                        __atomic_load_n(seqw, __ATOMIC_ACQUIRE), want);
      }
      if (q != hipErrorNotReady) return acs_fail(ctx, ACS_E_HIP, "fte: %s", hipGetErrorString(q));
    }
    __builtin_ia32_pause();
  }
}

extern "C" {

void acs_fte_default_opts(acs_fte_opts* o) {
  o->max_iters = 200;
  o->window = 0;
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
  ACS_DEVICE_GUARD(ctx);
  acs_fte_opts op;
  acs_fte_default_opts(&op);
  if (opts) op = *opts;
  ACS_CHECK(ctx, op.max_iters >= 0, "fte: max_iters < 0");
  FteSetup S;
  int rc;
  if ((rc = fte_setup(ctx, S, skel_ints, n_ints, skel_reals, n_reals, cams, n_cams, meas, w, n_frames, shutter_delay,
                      Ts, qinv, sd_mode, intermode, X, tau, op.redesc_a, op.redesc_b, op.redesc_c, flags)))
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
                     b.st, 0, 0, 0, INT_MAX, b.Fm, b.Fq);
  hipLaunchKernelGGL(k_fte_lm, dim3(1), dim3(FTE_LM_THREADS), 0, s, d, b.st, o, 1, b.Fm, b.Fq, b.normp, 0);
  // the linearisation of the initial state (buffer cur = 0); later ones are speculative
  if (op.max_iters > 0)
    fte_launch_lin(d, s, b, 1, 0, d.N, 0, (double*)nullptr, (const double*)nullptr);
  ACS_HIP(ctx, hipGetLastError());
  // enqueue the iterations one ahead of the host: the host reads iteration n's status
  // snapshot (pinned slot n & 1, published with its iteration count, fte_snapshot) while
  // iteration n + 1 runs, so the GPU never waits for the host, and a stop costs one
  // early-exiting iteration. Plain stream launches (~16 per iteration, ~56 us of host time
  // against >= ~100 us of GPU time): a hipGraph replay per iteration left ~9-13 us of idle
  // GPU between replays, 2 % of the 1000-frame solve (profiles/r03/fte_launch_ab.log).
  FteState* snap = nullptr;
  if (op.max_iters > 0) {
    snap = (FteState*)acs_pinned(ctx, 3 * sizeof(FteState));
    if (!snap) return ACS_E_NOMEM;
    std::memset(snap, 0, 3 * sizeof(FteState));
  }
  S.snap = snap;
  FteState hs;
  std::memset(&hs, 0, sizeof(hs));
  if (op.max_iters > 0) {
    // max_iters + 1 launches at most: the kernel sets MAXITER in iteration max_iters
    const int nmax = op.max_iters + 1;
    int last = 0, rc_wait;
    for (int n = 0;; ++n) {
      if (n < nmax) {
        fte_enqueue_iteration(S, s, o);
        ACS_HIP(ctx, hipGetLastError());
        last = n;
      }
      if (n >= 1) {
        // k_fte_lm of iteration n - 1 wrote its state into snap[(n - 1) & 1], then count n
        if ((rc_wait = fte_wait_snapshot(ctx, s, snap, n))) return rc_wait;
        if (snap[(n - 1) & 1].status != 0 || n >= nmax) break;
      }
    }
    // the last queued iteration exits early on a stop status (the state is unchanged)
    if ((rc_wait = fte_wait_snapshot(ctx, s, snap, last + 1))) return rc_wait;
    hs = snap[last & 1];
  } else {
    ACS_HIP(ctx, hipMemcpyAsync(&hs, b.st, sizeof(hs), hipMemcpyDeviceToHost, s));
    ACS_HIP(ctx, hipStreamSynchronize(s));
  }
  const hipMemcpyKind kout = (flags & ACS_DEVICE_PTRS) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  ACS_HIP(ctx, hipMemcpyAsync(X, b.X + (size_t)hs.cur * d.M * d.P, sizeof(double) * d.M * d.P, kout, s));
  if (tau) ACS_HIP(ctx, hipMemcpyAsync(tau, b.tau + (size_t)hs.cur * d.NT, sizeof(double) * d.NT, kout, s));
  int nbad = 0;
  ACS_HIP(ctx, hipMemcpyAsync(&nbad, b.bad, sizeof(int), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipStreamSynchronize(s));
  if (report) {
    report->status = hs.status == 0 ? ACS_STATUS_MAXITER : hs.status;
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
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, !(flags & ACS_DEVICE_PTRS), "acs_fte_eval takes host pointers");
  FteSetup S;
  int rc;
  if ((rc = fte_setup(ctx, S, skel_ints, n_ints, skel_reals, n_reals, cams, n_cams, meas, w, n_frames, shutter_delay,
                      Ts, qinv, sd_mode, intermode, X, tau, 3.0, 10.0, 20.0, 0)))
    return rc;
  const FteDims& d = S.d;
  FteBuffers& b = S.b;
  hipStream_t s = ctx->stream;
  FteState st0;
  std::memset(&st0, 0, sizeof(st0));
  st0.relin = 1;
  ACS_HIP(ctx, hipMemcpyAsync(b.st, &st0, sizeof(st0), hipMemcpyHostToDevice, s));
  fte_enqueue_linearize(S, s, 1);
  hipLaunchKernelGGL(k_fte_cost, dim3(d.N), dim3(64), 0, s, d, b.I, b.Rl, b.cams, b.meas, b.w, b.X, b.tau, b.qinv,
                     b.st, 0, 0, 0, INT_MAX, b.Fm, b.Fq);
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
  const int C = d.C, nv = M * P + (d.var ? N * C : Cg);
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
    if (d.var)
      for (int k = 0; k < N; ++k)
        for (int c = 0; c < C; ++c) grad[M * P + k * C + c] = gl[(size_t)k * FTE_NZP + P + 6 + c];
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
    if (d.var) {
      // frame k's delays couple with its local unknowns: X_{k+2} (all), X_{k+1}, X_k (xyz)
      for (int k = 0; k < N; ++k) {
        const double* Hk = Hl.data() + (size_t)k * FTE_NZP * FTE_NZP;
        for (int c = 0; c < C; ++c) {
          const size_t tc = (size_t)M * P + (size_t)k * C + c;
          for (int j = 0; j < P + 6; ++j) {
            const int row = j < P ? k + 2 : (j < P + 3 ? k + 1 : k);
            const int p = j < P ? j : (j < P + 3 ? j - P : j - P - 3);
            const double v = Hk[j * FTE_NZP + P + 6 + c];
            H[(size_t)(row * P + p) * nv + tc] += v;
            H[tc * nv + row * P + p] += v;
          }
          for (int c2 = 0; c2 < C; ++c2)
            H[tc * nv + M * P + (size_t)k * C + c2] = Hk[(P + 6 + c) * FTE_NZP + P + 6 + c2];
        }
      }
    }
  }
  return ACS_OK;
}

// Test hook (include/acinoset_hip.h): the damped super-blocks D_i of the normal matrix at
// (X, tau), as k_cr_assemble_build forms them, after `levels` cyclic-reduction levels of
// acs_fte_solve's reduction with every pending Schur term applied (levels = 0: as assembled;
// L > 0: blocks j = 2^L m hold the D the next level factors). Constant / no shutter delay.
int acs_fte_debug_blocks(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                         int64_t n_reals, const double* cams, int32_t n_cams, const double* meas, const double* w,
                         int32_t n_frames, int32_t shutter_delay, double Ts, const double* qinv, int32_t sd_mode,
                         int32_t intermode, const double* X, const double* tau, double lam, int32_t levels,
                         double* D_out, int64_t* dims, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, D_out && levels >= 0, "acs_fte_debug_blocks: null D_out or levels < 0");
  ACS_CHECK(ctx, !(shutter_delay && sd_mode == 1), "acs_fte_debug_blocks: constant or no shutter delay only");
  FteSetup S;
  int rc;
  if ((rc = fte_setup(ctx, S, skel_ints, n_ints, skel_reals, n_reals, cams, n_cams, meas, w, n_frames, shutter_delay,
                      Ts, qinv, sd_mode, intermode, X, tau, 3.0, 10.0, 20.0, flags)))
    return rc;
  const FteDims& d = S.d;
  FteBuffers& b = S.b;
  hipStream_t s = ctx->stream;
  FteState st0;
  std::memset(&st0, 0, sizeof(st0));
  st0.lam = lam;
  st0.relin = 1;
  ACS_HIP(ctx, hipMemcpyAsync(b.st, &st0, sizeof(st0), hipMemcpyHostToDevice, s));
  fte_launch_lin(d, s, b, 1, 0, d.N, 0, (double*)nullptr, (const double*)nullptr);
  const int L = std::min((int)levels, d.nlev);
  // as the solve stores it (upper tiles) unless the assembled D itself is asked for
  cr_launch_assemble_build(d, s, b, 0, -1, 0, INT_MAX, -1, -1, nullptr, nullptr, L == 0 || !fte_d_upper(d) ? 1 : 0);
  if (L > 0) cr_reduce(d, s, b.st, b, 0, d.nblk, d.nblk - 1, L, b.bad, true, nullptr, true, fte_d_upper(d));
  ACS_HIP(ctx, hipGetLastError());
  const size_t bytes = sizeof(double) * (size_t)d.nblk * d.BP * d.BP;
  ACS_HIP(ctx, hipMemcpyAsync(D_out, b.Dc, bytes, (flags & ACS_DEVICE_PTRS) ? hipMemcpyDeviceToDevice
                                                                            : hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipStreamSynchronize(s));
  if (dims) {
    dims[0] = d.nblk;
    dims[1] = d.BP;
    dims[2] = L;
  }
  return ACS_OK;
}

#ifdef FTE_PROFILE
void acs_fte_prof_read(unsigned long long* out) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fte_prof), sizeof(g_fte_prof));
}
void acs_fte_back_trace_read(unsigned long long* out) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_back_trace), sizeof(g_back_trace));
}
#endif
}  // extern "C"

// ---------------------------------------------------------------------------------------
// distributed handle API (include/acinoset_hip.h, §8(e)); payloads are device pointers
// ---------------------------------------------------------------------------------------
extern "C" {

int acs_fte_dist_create(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals,
                        int64_t n_reals, const double* cams, int32_t n_cams, const double* meas, const double* w,
                        int32_t n_frames, int32_t shutter_delay, double Ts, const double* qinv, int32_t sd_mode,
                        int32_t intermode, const double* X, const double* tau, const acs_fte_opts* opts, int32_t rank,
                        int32_t world, acs_fte_dist** out, int64_t* payload_sizes, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  acs_fte_opts op;
  acs_fte_default_opts(&op);
  if (opts) op = *opts;
  ACS_CHECK(ctx, op.max_iters >= 0, "fte: max_iters < 0");
  ACS_CHECK(ctx, world >= 1 && world <= 1024 && rank >= 0 && rank < world, "fte_dist: rank %d / world %d", rank,
            world);
  acs_fte_dist* h = new acs_fte_dist();
  h->ctx = ctx;
  int rc = fte_setup(ctx, h->S, skel_ints, n_ints, skel_reals, n_reals, cams, n_cams, meas, w, n_frames,
                     shutter_delay, Ts, qinv, sd_mode, intermode, X, tau, op.redesc_a, op.redesc_b, op.redesc_c, flags, &h->own);
  if (rc) {
    if (h->own) (void)acs_dev_free(h->own);
    delete h;
    return rc;
  }
  const FteDims& d = h->S.d;
  h->R = world;
  h->rank = rank;
  h->lam0 = op.lambda0;
  h->o = FteOptsDev{op.max_iters, op.ftol, op.xtol, op.gtol};
  // chain length 2^k: smallest k >= 1 with R 2^k >= nblk - 1
  h->klev = 1;
  while ((int64_t)world * (1 << h->klev) < d.nblk - 1) h->klev++;
  h->span = 1 << h->klev;
  h->a0 = rank * h->span;
  h->bend = h->a0 + h->span;
  const int N = d.N, M = d.M;
  auto clampi = [](int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); };
  h->own_lo = 3 * h->a0;                    // owned terms: lowest row in [own_lo, own_hi)
  h->own_hi = rank == world - 1 ? INT_MAX / 2 : 3 * h->bend;  // the last rank owns the tail
  h->k_lo = clampi(h->own_lo, 0, N);        // frames to linearise
  h->k_hi = clampi(h->own_hi, 0, N);
  h->f_lo = clampi(3 * h->a0, 0, M);        // rows to assemble (chain incl. its right end)
  h->f_hi = clampi(3 * h->bend + 3, 0, M);
  h->c_lo = clampi(h->own_lo, 0, N);        // cost blocks: frames [lo, hi) and stencils up to hi
  h->c_hi = clampi(h->own_hi + 1, 0, N);
  h->out_lo = clampi(h->a0, 0, d.nblk);     // step rows this rank publishes
  h->out_hi = clampi(rank == world - 1 ? h->bend + 1 : h->bend, 0, d.nblk);
  h->Lo = dist_layout(d, world);
  // reduced system arrays
  FteDims& dr = h->dr;
  dr = d;
  dr.nblk = world + 1;
  dr.M = 1;
  dr.N = 0;
  dr.nlev = 0;
  for (int s = 1; s < dr.nblk; s <<= 1) dr.nlev++;
  const size_t nb = dr.nblk, BP = d.BP, GR = d.GR;
  size_t off = 0;
  auto take = [&](size_t cnt) {
    size_t o = off;
    off += ((cnt * sizeof(double) + 255) / 256) * 256 / sizeof(double);
    return o;
  };
  const size_t oD = take(nb * BP * BP), oE = take(nb * BP * BP), oG = take(nb * BP * GR),
               oW = take(nb * BP * (2 * BP + GR)), oT = take(nb * GR * GR), odc = take(nb * BP),
               oE2 = take(nb * BP * BP), odL = take(nb * BP * (BP + GR)), odR = take(nb * BP * (BP + GR)),
               op_ = take((size_t)CR_NCHUNK * (16 * 16 + 16 + 32 * 32)), ogm = take(4);
  void* p = nullptr;
  if (acs_dev_malloc(&p, off * sizeof(double)) != hipSuccess) {
    (void)acs_dev_free(h->own);
    delete h;
    return acs_fail(ctx, ACS_E_NOMEM, "fte_dist: reduced-system allocation failed");
  }
  h->own_red = p;
  double* a = (double*)p;
  h->r = h->S.b;
  h->r.Dc = a + oD;
  h->r.Ec = a + oE;
  h->r.GBc = a + oG;
  h->r.Wc = a + oW;
  h->r.Tau = a + oT;
  h->r.Ec2 = a + oE2;
  h->r.dL = a + odL;
  h->r.dR = a + odR;
  h->r.dcv = a + odc;
  h->r.part = a + op_;
  h->r.gmaxp = a + ogm;
  FteState st0;
  std::memset(&st0, 0, sizeof(st0));
  st0.lam = op.lambda0;
  st0.relin = 1;
  st0.first = 1;
  ACS_HIP(ctx, hipMemcpyAsync(h->S.b.st, &st0, sizeof(st0), hipMemcpyHostToDevice, ctx->stream));
  ACS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  bool snap_ok = acs_host_malloc((void**)&h->snap, sizeof(int32_t) * ACS_DIST_RING, hipHostMallocDefault) == hipSuccess;
  for (auto& e : h->snap_ev)
    if (snap_ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      e = nullptr;
      snap_ok = false;
    }
  if (!snap_ok) {
    acs_fte_dist_destroy(h);
    return acs_fail(ctx, ACS_E_HIP, "fte_dist: pinned status ring allocation failed");
  }
  if (payload_sizes) {
    payload_sizes[0] = (int64_t)(h->Lo.n1 + h->Lo.n3);
    payload_sizes[1] = (int64_t)h->Lo.n2;
    payload_sizes[2] = (int64_t)h->Lo.n3;
  }
  *out = h;
  return ACS_OK;
}

// A solve restarted on the same handle: X / tau from the caller (host or, with
// ACS_DEVICE_PTRS, device pointers; tau NULL = zeros), the LM state of acs_fte_dist_create
// (first round pending, lambda0), the back-substitution tickets and granules zeroed. The
// arena, the reduced-system arrays, the status ring and the captured round graphs are kept:
// no allocation, so a timed multi-GPU solve can reuse one handle per rank.
int acs_fte_dist_reset(acs_fte_dist* h, const double* X, const double* tau, uint32_t flags) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  ACS_CHECK(h ? h->ctx : nullptr, h && X, "fte_dist_reset: null handle or X");
  acs_ctx* ctx = h->ctx;
  const FteDims& d = h->S.d;
  FteBuffers& b = h->S.b;
  hipStream_t s = ctx->stream;
  // rounds of the previous solve still queued finish first (their snapshots are then stale)
  ACS_HIP(ctx, hipStreamSynchronize(s));
  const double* Xs = X;
  const double* ts = tau;
  if (!(flags & ACS_DEVICE_PTRS)) {
    ACS_HIP(ctx, hipMemcpyAsync(b.X, X, sizeof(double) * d.M * d.P, hipMemcpyHostToDevice, s));
    if (tau) ACS_HIP(ctx, hipMemcpyAsync(b.tau, tau, sizeof(double) * d.NT, hipMemcpyHostToDevice, s));
    Xs = b.X;
    ts = tau ? b.tau : nullptr;
  }
  const int n = d.nblk, BP = d.BP, GR = d.GR;
  const size_t MP = (size_t)d.M * d.P;
  const size_t ngd = (size_t)n * BP * 2 + 64;
  const size_t nI = std::max(std::max(std::max(MP, (size_t)n + 1), ngd), (size_t)std::max(d.NT, GR));
  hipLaunchKernelGGL(k_fte_init_state, dim3(acs_grid((int64_t)nI, 256)), dim3(256), 0, s, b.X, Xs, MP, b.tau, ts,
                     d.NT, b.bad, b.dtau, GR, b.bk, n + 1, b.gdcv, ngd);
  hipLaunchKernelGGL(k_fte_state_reset, dim3(1), dim3(64), 0, s, b.st, h->lam0);
  ACS_HIP(ctx, hipGetLastError());
  h->rounds = 0;
  return ACS_OK;
}

int acs_fte_dist_destroy(acs_fte_dist* h) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  if (!h) return ACS_OK;
  (void)hipStreamSynchronize(h->ctx->stream);
  for (auto& c : h->g)
    if (c.exec) (void)hipGraphExecDestroy(c.exec);
  for (auto& e : h->snap_ev)
    if (e) (void)hipEventDestroy(e);
  if (h->snap) (void)acs_host_free(h->snap);
  if (h->own) (void)acs_dev_free(h->own);
  if (h->own_red) (void)acs_dev_free(h->own_red);
  delete h;
  return ACS_OK;
}

static int dist_phase1_body(acs_fte_dist* h, double* p1);

// payload of the starting state: the reduced system at X0 and the owned terms' cost
int acs_fte_dist_init(acs_fte_dist* h, double* payload) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  acs_ctx* ctx = h->ctx;
  const FteDims& d = h->S.d;
  FteBuffers& b = h->S.b;
  hipStream_t s = ctx->stream;
  double* p3 = payload + h->Lo.n1;
  if (h->c_hi > h->c_lo)
    hipLaunchKernelGGL(k_fte_cost, dim3(h->c_hi - h->c_lo), dim3(64), 0, s, d, b.I, b.Rl, b.cams, b.meas, b.w, b.X,
                       b.tau, b.qinv, b.st, 0, h->c_lo, h->own_lo, h->own_hi, b.Fm, b.Fq);
  hipLaunchKernelGGL(k_dist_cost_pack, dim3(1), dim3(256), 0, s, b.st, 0, d.N, h->c_lo, h->c_hi, h->c_lo, h->c_hi,
                     (const double*)b.Fm, (const double*)b.Fq, 0, 0, (const double*)nullptr, p3);
  // the linearisation of the starting state (copy 0); later ones are speculative (phase 3)
  if (h->a0 < d.nblk && h->k_hi > h->k_lo)
    fte_launch_lin(d, s, b, 1, h->k_lo, h->k_hi - h->k_lo, 0, (double*)nullptr, (const double*)nullptr);
  ACS_HIP(ctx, hipGetLastError());
  return dist_phase1_body(h, payload);
}

static int dist_phase1_body(acs_fte_dist* h, double* p1) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  acs_ctx* ctx = h->ctx;
  const FteDims& d = h->S.d;
  FteBuffers& b = h->S.b;
  hipStream_t s = ctx->stream;
  ACS_HIP(ctx, hipMemsetAsync(p1, 0, sizeof(double) * h->Lo.n1, s));
  if (h->a0 < d.nblk) {
    // the linearisation of X[cur] is there already (init, or the speculative one of phase 3)
    // the chain's rows assembled in LDS and its super-blocks built in one pass (the banded
    // rows never reach HBM), as the single-GPU solve; the ends' raw diagonals / gradients
    // go to Adiag / gb (row layout) for the payload
    const int top = std::min(h->bend, d.nblk - 1);
    if (d.var) {
      // per-frame delays: eliminated per frame in the row assembly (damped with the LM
      // lambda), the rows' gradients before that kept for the payload, then the build
      hipLaunchKernelGGL(k_fte_assemble, dim3(h->f_hi - h->f_lo), dim3(256), 0, s, d, b.X, b.tau, b.qinv, b.st, 0,
                         h->f_lo, h->own_lo, h->own_hi, b.Hloc, b.gloc, b.Ab, b.gb, b.Bt, b.gmaxp, b.Adiag, 1, b.graw,
                         b.gmaxt);
      cr_launch_build(d, s, top - h->a0 + 1, b.st, b.Ab, b.gb, b.Bt, b.Dc, b.Ec, b.GBc, h->a0, h->a0, h->bend, b.Adiag);
    } else {
      cr_launch_assemble_build(d, s, b, h->a0, top - h->a0 + 1, h->own_lo, h->own_hi, h->a0, h->bend, b.Adiag, b.graw);
    }
    const double* Efin = dist_local_cr(h);
    hipLaunchKernelGGL(k_cr_tau_partial, dim3(CR_NCHUNK), dim3(512), 0, s, d, b.st, b.Hloc, b.gloc, b.Tau, b.part,
                       h->k_lo, h->k_hi, h->a0 + 1, std::min(h->bend, d.nblk), 1,
                       (const double*)b.Tc);
    hipLaunchKernelGGL(k_dist_pack, dim3(32, 2), dim3(256), 0, s, d, b.st, h->Lo, h->rank, h->a0, h->bend, b.Dc, Efin,
                       b.GBc, b.Adiag, b.graw, p1);
    hipLaunchKernelGGL(k_dist_pack_small, dim3(1), dim3(256), 0, s, d, b.st, h->Lo, h->rank, h->a0, h->bend, b.part,
                       b.gmaxp, p1, d.var ? (const double*)b.gmaxt : (const double*)nullptr);
  }
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

// ACS_DIST_BACK_LEVELS=1: the rank chain's back substitution as one k_cr_back launch per level
// plus k_cr_trial (the round-5 form, kept for A/B timing); default: k_cr_back_chain
static bool dist_back_levels() {
  static const bool v = [] {
    const char* e = std::getenv("ACS_DIST_BACK_LEVELS");
    return e && e[0] == '1';
  }();
  return v;
}

static int dist_phase2_body(acs_fte_dist* h, const double* p1) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  acs_ctx* ctx = h->ctx;
  const FteDims& d = h->S.d;
  const FteDims& dr = h->dr;
  FteBuffers& b = h->S.b;
  FteBuffers& r = h->r;
  hipStream_t s = ctx->stream;
  // reduced system (identical on every rank)
  hipLaunchKernelGGL(k_red_build, dim3(dr.nblk), dim3(256), 0, s, d, b.st, h->Lo, h->R, h->span, p1, r.Dc, r.Ec,
                     r.GBc, r.gmaxp);
  const int rb = dr.nblk - 1;
  CrPending pend;
  cr_reduce(dr, s, b.st, r, 0, dr.nblk, rb, dr.nlev, b.bad, false, &pend, false);
  cr_launch_top(dr, s, dr.nlev, 0, dr.nblk, b.st, r, b.bad, pend);
  hipLaunchKernelGGL(k_cr_tau_partial, dim3(CR_NCHUNK), dim3(512), 0, s, dr, b.st, r.Hloc, r.gloc, r.Tau, r.part, 0,
                     0, 0, dr.nblk, 0, (const double*)nullptr);
  const int nE = d.Cg * d.Cg + d.Cg + d.GR * d.GR;
  hipLaunchKernelGGL(k_red_part, dim3(1), dim3(256), 0, s, nE, h->Lo, b.st, p1, r.part);
  hipLaunchKernelGGL(k_cr_top, dim3(1), dim3(1024), 0, s, dr, b.st, (const double*)r.Wc, r.part, r.gmaxp, b.tau, r.dcv,
                     b.dtau, b.bad);
  hipLaunchKernelGGL(k_dist_gtol, dim3(1), dim3(64), 0, s, b.st, h->o);
  for (int lv = dr.nlev - 1; lv >= 0; --lv) {
    const int st = 1 << lv;
    const int ne = (dr.nblk - st + 2 * st - 1) / (2 * st);
    hipLaunchKernelGGL(k_cr_back, dim3(ne), dim3(1024), 0, s, dr, st, 0, rb, b.st, r.Wc, b.dtau, r.dcv);
  }
  // this chain: ends from the reduced solve, interior by back substitution, then the trial
  // rows of the whole chain (its end blocks are shared: both neighbours step them alike) and
  // the replicated delays; the norm partials of the owned blocks go to phase 3's payload
  if (h->a0 < d.nblk && !d.var && !dist_back_levels()) {
    hipLaunchKernelGGL(k_dist_scatter, dim3(1), dim3(128), 0, s, d, b.st, h->rank, h->a0, h->bend, r.dcv, b.dcv);
    // the chain's back substitution and trial rows in one launch (k_cr_back_chain)
    const int iend = std::min(h->bend, d.nblk);
    int nint = 0;
    for (int lv = h->klev - 1; lv >= 0; --lv) {
      const int sv = 1 << lv;
      nint += std::max(0, (iend - h->a0 - sv + 2 * sv - 1) / (2 * sv));
    }
    const int nwork = (h->bend < d.nblk ? 2 : 1) + nint;
    const int nth_back = (8 * d.BP + 63) / 64 * 64;
#define CR_BACK_CHAIN(nb, grb)                                                                                  \
  hipLaunchKernelGGL((k_cr_back_chain<nb, grb>), dim3(nwork), dim3(nth_back), 0, s, d, h->a0, h->bend, h->klev,  \
                     h->rank == 0 ? 1 : 0, (const FteState*)b.st, (const double*)b.Wc, (const double*)b.dtau, b.dcv, \
                     b.bk, b.gdcv, b.bad, b.X, b.tau, b.normp)
#define CR_BACK_CHAIN_G(nb) \
  if (d.GR <= 16)           \
    CR_BACK_CHAIN(nb, 1);   \
  else                      \
    CR_BACK_CHAIN(nb, 2)
    switch (d.BP >> 4) {
      case 1: CR_BACK_CHAIN_G(1); break;
      case 2: CR_BACK_CHAIN_G(2); break;
      case 3: CR_BACK_CHAIN_G(3); break;
      case 4: CR_BACK_CHAIN_G(4); break;
      case 5: CR_BACK_CHAIN_G(5); break;
      default: CR_BACK_CHAIN_G(6); break;
    }
#undef CR_BACK_CHAIN_G
#undef CR_BACK_CHAIN
  } else if (h->a0 < d.nblk) {
    hipLaunchKernelGGL(k_dist_scatter, dim3(1), dim3(128), 0, s, d, b.st, h->rank, h->a0, h->bend, r.dcv, b.dcv);
    for (int lv = h->klev - 1; lv >= 0; --lv) {
      const int st = 1 << lv;
      int ne = 0;
      for (int i = h->a0 + st; i < std::min(h->bend, d.nblk); i += 2 * st) ++ne;
      if (ne)
        hipLaunchKernelGGL(k_cr_back, dim3(ne), dim3(1024), 0, s, d, st, h->a0, h->bend, b.st, b.Wc, b.dtau, b.dcv);
    }
    const int top = std::min(h->bend, d.nblk - 1);
    hipLaunchKernelGGL(k_cr_trial, dim3(top - h->a0 + 1), dim3(256), 0, s, d, b.st, (const double*)b.dcv, b.dtau,
                       b.Hloc, b.gloc, b.X, b.tau, b.normp, 1, h->a0, h->rank == 0 ? 1 : 0, h->k_lo, h->k_hi,
                       b.normt);
  } else {
    // a rank past the last block still steps the replicated delays
    hipLaunchKernelGGL(k_cr_trial, dim3(1), dim3(256), 0, s, d, b.st, (const double*)b.dcv, b.dtau, b.Hloc, b.gloc,
                       b.X, b.tau, b.normp, 0, d.nblk, h->rank == 0 ? 1 : 0);
  }
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

static int dist_phase3_body(acs_fte_dist* h, double* p3) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  acs_ctx* ctx = h->ctx;
  const FteDims& d = h->S.d;
  FteBuffers& b = h->S.b;
  hipStream_t s = ctx->stream;
  // speculative linearisation of the trial rows: its measurement terms (owned frames
  // [k_lo, k_hi)) and model stencils (owned: k - 1 in [own_lo, own_hi), so frames up to k_hi
  // inclusive; the one extra frame's own terms are not counted) are the trial cost, and an
  // accepted step needs no new linearisation in phase 1
  const int l_hi = std::min(h->k_hi + 1, d.N);
  if (h->a0 < d.nblk && l_hi > h->k_lo)
    fte_launch_lin(d, s, b, 0, h->k_lo, l_hi - h->k_lo, 1, b.Fq, b.qinv);
  const int q0 = std::max(h->k_lo + 1, 1), q1 = l_hi;
  const int t_hi = std::min(h->bend, d.nblk - 1) + 1;
  hipLaunchKernelGGL(k_dist_cost_pack, dim3(1), dim3(256), 0, s, b.st, 1, d.N, h->k_lo, h->k_hi, q0,
                     std::max(q0, q1), (const double*)b.Floc, (const double*)b.Fq, h->out_lo, h->out_hi, b.normp, p3,
                     d.var ? h->a0 : 0, d.var ? t_hi : 0, (const double*)b.normt);
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

// one LM step: decide on the pending step (summed cost in `in`), solve the summed reduced
// system of `in`, step the chain, the new trial cost -> `out`, then the reduced system at the
// trial state (or, after a rejection, at the unchanged state) -> `out`
int acs_fte_dist_round(acs_fte_dist* h, const double* in, double* out) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  ACS_CHECK(h ? h->ctx : nullptr, h && in && out && in != out, "fte_dist_round: two distinct payload buffers");
  acs_ctx* ctx = h->ctx;
  FteBuffers& b = h->S.b;
  hipStream_t s = ctx->stream;
  const size_t n1 = h->Lo.n1;
  int rc = dist_run_captured(h, in, out, [&] {
    hipLaunchKernelGGL(k_dist_decide, dim3(1), dim3(64), 0, s, b.st, h->o, in + n1);
    int r2 = dist_phase2_body(h, in);
    if (r2) return r2;
    if ((r2 = dist_phase3_body(h, out + n1))) return r2;
    hipLaunchKernelGGL(k_dist_spec, dim3(1), dim3(64), 0, s, b.st, 1);
    if ((r2 = dist_phase1_body(h, out))) return r2;
    hipLaunchKernelGGL(k_dist_spec, dim3(1), dim3(64), 0, s, b.st, 0);
    ACS_HIP(ctx, hipGetLastError());
    return ACS_OK;
  });
  if (rc) return rc;
  const int slot = (int)(h->rounds % ACS_DIST_RING);
  ACS_HIP(ctx, hipMemcpyAsync(h->snap + slot, &b.st->status, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipEventRecord(h->snap_ev[slot], s));
  h->rounds++;
  return ACS_OK;
}

// LM status after round r (waits for that round only)
int acs_fte_dist_poll(acs_fte_dist* h, int64_t round, int32_t* status) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  ACS_CHECK(h ? h->ctx : nullptr, h && status && round >= 0 && round < h->rounds && round >= h->rounds - ACS_DIST_RING,
            "fte_dist_poll: round %lld not among the last %d enqueued", (long long)round, ACS_DIST_RING);
  const int slot = (int)(round % ACS_DIST_RING);
  ACS_HIP(h->ctx, hipEventSynchronize(h->snap_ev[slot]));
  *status = h->snap[slot];
  return ACS_OK;
}

int acs_fte_dist_gather(acs_fte_dist* h, double* p2) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  acs_ctx* ctx = h->ctx;
  const FteDims& d = h->S.d;
  FteBuffers& b = h->S.b;
  hipStream_t s = ctx->stream;
  ACS_HIP(ctx, hipMemsetAsync(p2, 0, sizeof(double) * h->Lo.n2, s));
  if (h->out_hi > h->out_lo)
    hipLaunchKernelGGL(k_dist_x_out, dim3(64), dim3(256), 0, s, d, b.st, h->out_lo, h->out_hi, (const double*)b.X, p2,
                       (const double*)b.tau, h->k_lo, h->k_hi);
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

int acs_fte_dist_scatter(acs_fte_dist* h, const double* p2) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  acs_ctx* ctx = h->ctx;
  const FteDims& d = h->S.d;
  FteBuffers& b = h->S.b;
  hipLaunchKernelGGL(k_dist_x_in, dim3(64), dim3(256), 0, ctx->stream, d, b.st, p2, b.X, b.tau);
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

int acs_fte_dist_result(acs_fte_dist* h, double* X, double* tau, acs_fte_report* report, uint32_t flags) {
  ACS_DEVICE_GUARD(h ? h->ctx : nullptr);
  acs_ctx* ctx = h->ctx;
  const FteDims& d = h->S.d;
  FteBuffers& b = h->S.b;
  hipStream_t s = ctx->stream;
  FteState hs;
  ACS_HIP(ctx, hipMemcpyAsync(&hs, b.st, sizeof(hs), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipStreamSynchronize(s));
  const hipMemcpyKind kout = (flags & ACS_DEVICE_PTRS) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  if (X) ACS_HIP(ctx, hipMemcpyAsync(X, b.X + (size_t)hs.cur * d.M * d.P, sizeof(double) * d.M * d.P, kout, s));
  if (tau) ACS_HIP(ctx, hipMemcpyAsync(tau, b.tau + (size_t)hs.cur * d.NT, sizeof(double) * d.NT, kout, s));
  int nbad = 0;
  ACS_HIP(ctx, hipMemcpyAsync(&nbad, b.bad, sizeof(int), hipMemcpyDeviceToHost, s));
  ACS_HIP(ctx, hipStreamSynchronize(s));
  if (report) {
    report->status = hs.status == 0 ? ACS_STATUS_MAXITER : hs.status;
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

}  // extern "C"
