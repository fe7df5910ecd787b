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
//      evaluated together, every thread on independent (pose, joint) / (pose, marker) items
//      (ekf_fk_batch), then the fisheye projection of (P+1) x C x L markers
//   3. Kalman update in information form on the pose block: with H = [H_x 0 0] and R
//      diagonal, K r = P[:,x] (I + A P_xx)^-1 b and (I - K H) P = P - P[:,x] (I + A P_xx)^-1
//      A P[x,:], A = H_x^T R^-1 H_x, b = H_x^T R^-1 r (Woodbury, instead of inverting the
//      2CL x 2CL S of :267). (I + A P_xx)^-1 = W^-1 P_xx with W = P_xx + P_xx A P_xx
//      symmetric positive definite: one P x P Gauss-Jordan with the pivots on the diagonal
//      (no pivot search). Analytic H: A, b and the outlier diagonal in marker space (3 L
//      rows, not 2 C L).
//   4. the reference's 3-sigma outlier count from diag(S) = diag(H_x P_xx H_x^T) + diag R
// With F32 (the reference numerics) the predicted state is rounded to float32 (:79), the
// FK trig runs in float32, and the Jacobian perturbation is x + 1e-3 in float32.
//
// RTS backward pass (:292-296): the gains A_i = P_est[i] F^T P_pred[i+1]^-1 do not depend
// on the smoothed states, so k_ekf_gain computes them for every (sequence, frame) pair in
// parallel (blocked Gauss-Jordan on f64 MFMA tiles), and k_ekf_smooth_x runs the state
// recursion per sequence; k_ekf_smooth (sequential) when the smoothed covariances are asked.
#include "fk.hpp"
#include "mfma64.hpp"

#define EKF_WAVES 8

struct EkfDims {
  int N, C, L, P, J, n, npad, Ppad, m, mpad, S, n_ints, n_reals;
  double sT, thresh, maxpix, eps;
};

// doubles of an FkShared (the analytic-H FK); its FkDeriv follows it
__host__ __device__ constexpr size_t ekf_fk_shared_doubles() { return (sizeof(FkShared) + 7) / 8; }
__host__ __device__ constexpr size_t ekf_fk_ah_doubles() {
  return ekf_fk_shared_doubles() + (sizeof(FkDeriv) + 7) / 8;
}

// LDS doubles of the batched FK of the P+1 Jacobian poses (ekf_fk_batch)
__host__ __device__ inline size_t ekf_fk_lds(int P, int J, int L) {
  return (size_t)FK_MAXJ * 9 + (size_t)(FK_MAXP + 1) * 9 + (size_t)(P + 1) * (9 * J + 3 * L + 6) + 4 * FK_MAXP;
}

// LDS doubles of the measurement model's FK region: the batched FK of the forward
// differences, or the analytic H's FkShared + FkDeriv, whichever is larger
__host__ __device__ inline size_t ekf_w1_fk_doubles(int P, int J, int L) {
  const size_t a = ekf_fk_lds(P, J, L), b = ekf_fk_ah_doubles();
  return a > b ? a : b;
}

// Analytic H in marker space (k_ekf_filter<*, true>): rows of the per-marker operands
// (3 L padded to a multiple of 16), and the LDS doubles of FkShared + FkDeriv followed by
// D = d pos / d x, T = M D, S = D P_xx (R3 x (Ppad + 1) each), g (R3), N (9 L), M (6 L)
__host__ __device__ inline int ekf_ah_rows(int L) { return (3 * L + 15) & ~15; }
__host__ __device__ inline size_t ekf_ah_base() { return (ekf_fk_ah_doubles() + 3) & ~(size_t)3; }
__host__ __device__ inline size_t ekf_ah_alg_doubles(int L, int Ppad) {
  const size_t R3 = ekf_ah_rows(L);
  return ekf_ah_base() + 3 * R3 * (Ppad + 1) + R3 + 15 * (size_t)L;
}
// the 8-wave filter's algebra region: P[:, x] (npad x (Ppad + 1); before it, C and A C of the
// update's solve, 2 Ppad rows), aug (Ppad x AW) and A (Ppad x (Ppad + 1)); the odd row stride
// keeps the MFMA A-operand reads (16 rows, one column) on distinct LDS banks
__host__ __device__ inline int ekf_wg_px_rows(int npad, int Ppad) { return npad > 2 * Ppad ? npad : 2 * Ppad; }
__host__ __device__ inline size_t ekf_wg_la_doubles(int npad, int Ppad) {
  return (size_t)ekf_wg_px_rows(npad, Ppad) * (Ppad + 1) + (size_t)Ppad * (Ppad + npad + 1) +
         (size_t)Ppad * (Ppad + 1);
}
// the forward-difference A / b phase streams H through LDS in chunks of EKF_FD_RCH rows: the
// KS = 4 partial-tile tree buffer, then the chunk (stride Ppad + 1) and its weights / residuals
#define EKF_FD_RCH 128
__host__ __device__ inline size_t ekf_fd_chunk_doubles(int Ppad) {
  return 2 * 5 * 256 + (size_t)EKF_FD_RCH * (Ppad + 1) + 2 * EKF_FD_RCH;
}
// the 8-wave filter's measurement-model region: batched FK (forward differences) or the
// analytic H's FK and marker-space operands, whichever is larger
__host__ __device__ inline size_t ekf_wg_fk_doubles(int P, int J, int L, int Ppad) {
  const size_t a = ekf_w1_fk_doubles(P, J, L), b = ekf_ah_alg_doubles(L, Ppad), c = ekf_fd_chunk_doubles(Ppad);
  return a > b ? (a > c ? a : c) : (b > c ? b : c);
}

// Parameter p of Jacobian pose q (q = 0: the predicted state; q > 0: parameter q-1 moved by
// eps, in float32 with the reference numerics, src/core/ekf.py:81-96).
template <bool F32>
__device__ __forceinline__ double ekf_xq(const double* s, int q, int p, double eps) {
  const double v = s[p];
  if (q > 0 && p == q - 1) return F32 ? (double)((float)v + (float)eps) : v + eps;
  return v;
}

// ekf_fk_batch's phase 0: sin / cos of every parameter as given (sc rows 0, 1) and as moved by
// eps (rows 2, 3; FK_MAXP per row), and the root / world translation of every Jacobian pose
// (rw: 6 per pose). The caller synchronises.
template <bool F32>
__device__ void ekf_fk_trig_trans(const SkelView& sk, const double* ss, double eps, double* sc, double* rw, int tid,
                                  int nth) {
  const int P = sk.P, NQ = P + 1;
  const int* pk = sk.pk;
  for (int e = tid; e < 2 * P + 2 * NQ; e += nth) {
    if (e < 2 * P) {
      const int p = e % P, mv = e / P;
      const double v = ekf_xq<F32>(ss, mv ? p + 1 : 0, p, eps);
      double sn, cs;
      if (F32) {
        float sf, cf;
        sincosf((float)v, &sf, &cf);
        sn = sf;
        cs = cf;
      } else {
        sincos(v, &sn, &cs);
      }
      sc[(2 * mv) * FK_MAXP + p] = sn;
      sc[(2 * mv + 1) * FK_MAXP + p] = cs;
    } else {
      const int q = (e - 2 * P) >> 1, kind = ((e - 2 * P) & 1) ? PK_WORLD : PK_TRANS;
      double t[3] = {0.0, 0.0, 0.0};
      for (int p = 0; p < P; ++p)
        if (pk[4 * p] == kind) {
          const int a = pk[4 * p + 1];
          const double x = ekf_xq<F32>(ss, q, p, eps);
          t[0] += a == 0 ? x : 0.0;
          t[1] += a == 1 ? x : 0.0;
          t[2] += a == 2 ? x : 0.0;
        }
      double* dst = rw + q * 6 + (kind == PK_WORLD ? 3 : 0);
      dst[0] = t[0];
      dst[1] = t[1];
      dst[2] = t[2];
    }
  }
}

// Marker positions of all P+1 poses of the forward-difference Jacobian at once, every
// thread of the workgroup on independent (pose, joint) / (pose, marker) items. Same
// arithmetic as fk_frame (fk.hpp), so bit-identical positions: G_j = A_{n-1}..A_0 per
// joint, M_j = G_root .. G_parent G_j by 3x3 products walking to the root, node = sum of
// M_frame offsets walking to the root. A pose differs from pose 0 in one parameter, so
// only one G per pose is recomputed (that of the parameter's joint, if a rotation).
// Output: pos (P+1) x L x 3 in LDS (after the final barrier).
template <bool F32>
__device__ void ekf_fk_batch(const SkelView& sk, const double* ss, double eps, double* fk, int tid, int nth) {
  const int P = sk.P, J = sk.J, L = sk.L, NQ = P + 1;
  double* Gb = fk;                        // FK_MAXJ x 9: G of pose 0
  double* Gq = Gb + FK_MAXJ * 9;          // (FK_MAXP + 1) x 9: G of the moved joint of pose q
  double* M = Gq + (FK_MAXP + 1) * 9;     // NQ x J x 9
  double* pos = M + (size_t)NQ * J * 9;   // NQ x L x 3
  double* rw = pos + (size_t)NQ * L * 3;  // NQ x 6: root, world translation
  double* sc = rw + (size_t)NQ * 6;       // sin, cos of pose 0; sin, cos of the moved parameter
  const int* pk = sk.pk;
  // 0. trig of every parameter (as given and as moved), per-pose translations
  ekf_fk_trig_trans<F32>(sk, ss, eps, sc, rw, tid, nth);
  __syncthreads();
  // 1. G of every joint at pose 0, and of the moved joint of each pose q > 0
  for (int e = tid; e < J + P; e += nth) {
    int j, moved;
    double* out;
    if (e < J) {
      j = e;
      moved = -1;
      out = Gb + 9 * j;
    } else {
      moved = e - J;  // pose q = moved + 1
      if (pk[4 * moved] != PK_ROT) continue;
      j = pk[4 * moved + 1];
      out = Gq + 9 * (moved + 1);
    }
    const int* jt = sk.joints + 8 * j;
    const int nrot = jt[1];
#pragma unroll
    for (int col = 0; col < 3; ++col) {
      double v[3] = {col == 0 ? 1.0 : 0.0, col == 1 ? 1.0 : 0.0, col == 2 ? 1.0 : 0.0};
      for (int r = 0; r < nrot; ++r) {
        double w[3];
        const int p = jt[5 + r];
        const int mv = p == moved ? 2 : 0;
        act_rot_vec(jt[2 + r], sc[mv * FK_MAXP + p], sc[(mv + 1) * FK_MAXP + p], v, w);
        v[0] = w[0];
        v[1] = w[1];
        v[2] = w[2];
      }
      out[col] = v[0];
      out[3 + col] = v[1];
      out[6 + col] = v[2];
    }
  }
  __syncthreads();
  // 2. M_j of every pose
  for (int e = tid; e < NQ * J; e += nth) {
    const int q = e / J, j = e - q * J;
    const int mj = (q > 0 && pk[4 * (q - 1)] == PK_ROT) ? pk[4 * (q - 1) + 1] : -1;
    auto G = [&](int k) -> const double* { return k == mj ? Gq + 9 * q : Gb + 9 * k; };
    double Mm[9], T[9];
    const double* g0 = G(j);
#pragma unroll
    for (int i = 0; i < 9; ++i) Mm[i] = g0[i];
    int k = sk.joints[8 * j];
    while (k >= 0) {
      mat3_mul(G(k), Mm, T);
#pragma unroll
      for (int i = 0; i < 9; ++i) Mm[i] = T[i];
      k = sk.joints[8 * k];
    }
    double* o = M + (size_t)e * 9;
#pragma unroll
    for (int i = 0; i < 9; ++i) o[i] = Mm[i];
  }
  __syncthreads();
  // 3. marker positions
  for (int e = tid; e < NQ * L; e += nth) {
    const int q = e / L, l = e - q * L;
    const double* Mq = M + (size_t)q * J * 9;
    double p0 = 0.0, p1 = 0.0, p2 = 0.0;
    int node = sk.outn[l];
    while (true) {
      const int* nd = sk.nodes + 4 * node;
      const int base = nd[0];
      if (base == -2 || base == -1) {
        const double* t = rw + q * 6 + (base == -2 ? 3 : 0);
        p0 += t[0];
        p1 += t[1];
        p2 += t[2];
        break;
      }
      const double* Mf = Mq + 9 * nd[1];
      double o0 = sk.off[3 * node], o1 = sk.off[3 * node + 1], o2 = sk.off[3 * node + 2];
      if (nd[2] >= 0) o0 = ekf_xq<F32>(ss, q, nd[2], eps);
      p0 += Mf[0] * o0 + Mf[1] * o1 + Mf[2] * o2;
      p1 += Mf[3] * o0 + Mf[4] * o1 + Mf[5] * o2;
      p2 += Mf[6] * o0 + Mf[7] * o1 + Mf[8] * o2;
      node = base;
    }
    double* o = pos + (size_t)e * 3;
    o[0] = p0;
    o[1] = p1;
    o[2] = p2;
  }
  __syncthreads();
}

// Marker l's position at Jacobian pose q in one thread, from ekf_fk_trig_trans's tables:
// ekf_fk_batch's phases 1-3 (the same G, M and node sums in the same order, so the same
// bits) without their shared tables and barriers. For skeletons of one joint (the head
// model), where recomputing a joint's rotation per (pose, marker) item is cheaper than the
// batch's three dependent workgroup phases.
template <bool F32>
__device__ void ekf_fk_point(const SkelView& sk, const double* ss, double eps, const double* sc, const double* rw, int q,
                             int l, double* out) {
  const int moved = q - 1;  // the parameter moved in pose q (none for q = 0)
  auto G_of = [&](int j, double* G) {
    const int* jt = sk.joints + 8 * j;
    const int nrot = jt[1];
#pragma unroll
    for (int col = 0; col < 3; ++col) {
      double v[3] = {col == 0 ? 1.0 : 0.0, col == 1 ? 1.0 : 0.0, col == 2 ? 1.0 : 0.0};
      for (int r = 0; r < nrot; ++r) {
        double w[3];
        const int p = jt[5 + r];
        const int mv = p == moved ? 2 : 0;
        act_rot_vec(jt[2 + r], sc[mv * FK_MAXP + p], sc[(mv + 1) * FK_MAXP + p], v, w);
        v[0] = w[0];
        v[1] = w[1];
        v[2] = w[2];
      }
      G[col] = v[0];
      G[3 + col] = v[1];
      G[6 + col] = v[2];
    }
  };
  double p0 = 0.0, p1 = 0.0, p2 = 0.0;
  int node = sk.outn[l];
  while (true) {
    const int* nd = sk.nodes + 4 * node;
    const int base = nd[0];
    if (base == -2 || base == -1) {  // the root (or world) translation of pose q
      const double* t = rw + q * 6 + (base == -2 ? 3 : 0);
      p0 += t[0];
      p1 += t[1];
      p2 += t[2];
      break;
    }
    double Mm[9], G[9], T[9];  // M of the node's frame: G_root .. G_parent G_frame
    G_of(nd[1], Mm);
    for (int k = sk.joints[8 * nd[1]]; k >= 0; k = sk.joints[8 * k]) {
      G_of(k, G);
      mat3_mul(G, Mm, T);
#pragma unroll
      for (int i = 0; i < 9; ++i) Mm[i] = T[i];
    }
    double o0 = sk.off[3 * node], o1 = sk.off[3 * node + 1], o2 = sk.off[3 * node + 2];
    if (nd[2] >= 0) o0 = ekf_xq<F32>(ss, q, nd[2], eps);
    p0 += Mm[0] * o0 + Mm[1] * o1 + Mm[2] * o2;
    p1 += Mm[3] * o0 + Mm[4] * o1 + Mm[5] * o2;
    p2 += Mm[6] * o0 + Mm[7] * o1 + Mm[8] * o2;
    node = base;
  }
  out[0] = p0;
  out[1] = p1;
  out[2] = p2;
}

// ekf_fk_point's table walk for one (pose q, marker l) item of a one-joint skeleton, resolved
// once per kernel: the joint's rotations (axis, row of its sine in ekf_fk_trig_trans's table
// for pose q) and the node chain's offsets, in walk order. ekf_point_eval then repeats
// ekf_fk_point's arithmetic in the same order from registers, with every table read of a frame
// issued at once (the walk was a chain of dependent LDS loads per frame). Same bits.
// ok = false: the chain is longer than EKF_PLAN_D or leaves joint 0, and the caller walks the
// table as before. (Tried, r06l: each item forming its own sines / cosines and translation,
// which drops the trig table's phase and barrier: the FK/proj phase went 2.8 -> 2.5 us, but
// the extra live state slowed the later phases by 1.1 us per frame.)
#define EKF_PLAN_D 2
struct EkfPointPlan {
  bool ok;
  int nrot, nstep, tr;       // tr: rw offset of the pose's root / world translation
  int ax[3], sci[3];
  int op[EKF_PLAN_D];        // offset parameter of each step (-1: the table offset)
  double off[EKF_PLAN_D][3];
};

__device__ inline EkfPointPlan ekf_point_plan(const SkelView& sk, int q, int l) {
  EkfPointPlan pl;
  const int* jt = sk.joints;
  const int moved = q - 1;
  pl.nrot = jt[1] < 3 ? jt[1] : 3;
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int p = r < pl.nrot ? jt[5 + r] : 0;
    pl.ax[r] = r < pl.nrot ? jt[2 + r] : 0;
    pl.sci[r] = (p == moved ? 2 : 0) * FK_MAXP + p;
  }
  // the node chain in walk order, with compile-time indices only (a runtime index would put
  // the plan in scratch memory)
  bool live = sk.J == 1 && jt[0] < 0 && jt[1] <= 3, done = false;
  int node = sk.outn[l], base = -1;
  pl.nstep = 0;
#pragma unroll
  for (int s = 0; s <= EKF_PLAN_D; ++s) {
    int b = -1, fr = 0, op = -1;
    double o0 = 0.0, o1 = 0.0, o2 = 0.0;
    if (live && !done) {
      const int* nd = sk.nodes + 4 * node;
      b = nd[0];
      fr = nd[1];
      op = nd[2];
      o0 = sk.off[3 * node];
      o1 = sk.off[3 * node + 1];
      o2 = sk.off[3 * node + 2];
      if (b == -2 || b == -1) {
        done = true;
        base = b;
      } else if (s == EKF_PLAN_D || fr != 0) {
        live = false;
      } else {
        pl.nstep = s + 1;
        node = b;
      }
    }
    if (s < EKF_PLAN_D) {
      pl.op[s] = live && !done ? op : -1;  // a chain step (not its end)
      pl.off[s][0] = o0;
      pl.off[s][1] = o1;
      pl.off[s][2] = o2;
    }
  }
  pl.ok = live && done;
  pl.tr = q * 6 + (base == -2 ? 3 : 0);
  return pl;
}

template <bool F32>
__device__ __forceinline__ void ekf_point_eval(const EkfPointPlan& pl, const double* ss, double eps, const double* sc,
                                               const double* rw, int q, double* out) {
  // every table value of the frame first: the joint's sines / cosines, the offset
  // parameters, the translation
  double sn[3], cs[3], xo[EKF_PLAN_D], t[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    sn[r] = sc[pl.sci[r]];
    cs[r] = sc[pl.sci[r] + FK_MAXP];
  }
#pragma unroll
  for (int s = 0; s < EKF_PLAN_D; ++s) xo[s] = pl.op[s] >= 0 ? ekf_xq<F32>(ss, q, pl.op[s], eps) : 0.0;
#pragma unroll
  for (int i = 0; i < 3; ++i) t[i] = rw[pl.tr + i];
  double Mm[9];  // G of joint 0 (ekf_fk_point's G_of; no parent)
#pragma unroll
  for (int col = 0; col < 3; ++col) {
    double v[3] = {col == 0 ? 1.0 : 0.0, col == 1 ? 1.0 : 0.0, col == 2 ? 1.0 : 0.0};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      if (r >= pl.nrot) break;
      double w[3];
      act_rot_vec(pl.ax[r], sn[r], cs[r], v, w);
      v[0] = w[0];
      v[1] = w[1];
      v[2] = w[2];
    }
    Mm[col] = v[0];
    Mm[3 + col] = v[1];
    Mm[6 + col] = v[2];
  }
  double p0 = 0.0, p1 = 0.0, p2 = 0.0;
#pragma unroll
  for (int s = 0; s < EKF_PLAN_D; ++s) {
    if (s >= pl.nstep) break;
    const double o0 = pl.op[s] >= 0 ? xo[s] : pl.off[s][0], o1 = pl.off[s][1], o2 = pl.off[s][2];
    p0 += Mm[0] * o0 + Mm[1] * o1 + Mm[2] * o2;
    p1 += Mm[3] * o0 + Mm[4] * o1 + Mm[5] * o2;
    p2 += Mm[6] * o0 + Mm[7] * o1 + Mm[8] * o2;
  }
  out[0] = p0 + t[0];
  out[1] = p1 + t[1];
  out[2] = p2 + t[2];
}

// Row / column of the flat index e = tid, tid + nth, ... over rows of nc columns, stepped
// without an integer division per element (nth / nc and nth % nc once per loop).
struct Walk2 {
  int e, r, c, de, dr, dc, nc;
  __device__ Walk2(int tid, int nth, int nc_) : e(tid), de(nth), nc(nc_) {
    r = tid / nc;
    c = tid - r * nc;
    dr = nth / nc;
    dc = nth - dr * nc;
  }
  __device__ void next() {
    e += de;
    r += dr;
    c += dc;
    if (c >= nc) {
      c -= nc;
      ++r;
    }
  }
};

// k_ekf_filter's update solve for a W that is not positive definite: [I + A C | I] (A and C
// zero outside P x P), then Gauss-Jordan with partial pivoting, register-resident like the
// diagonal solve; pivoting is implicit (rows stay in place, a row is "used" once it has been a
// pivot): step k takes the unused row with the largest |a[r][k]| (ties: lowest row), and at
// the end row pv_k over its pivot is row k of V, written to sC. Called by every thread (not
// inlined: the common path keeps its registers).
__device__ __noinline__ void ekf_update_pivoted(double* aug, int AW, const double* sA, double* sC, int LPx,
                                                double* colb, int P, int Pp, int* s_sing) {
  constexpr int NCG = 4;
  const int tid = threadIdx.x, nth = blockDim.x;
  const int gr = tid & 31, cg = tid >> 5, half = cg & 1;
  double av[NCG];
  // [I + A C | I] (A and C are zero outside P x P), then Gauss-Jordan with partial
  // pivoting, register-resident as above; pivoting is implicit (rows stay in place, a
  // row is "used" once it has been a pivot): step k takes the unused row with the
  // largest |a[r][k]| (ties: lowest row), and at the end row pv_k over its pivot is row k
  // of V
  for (int e = tid; e < Pp * Pp; e += nth) {
    const int r = e / Pp, c = e - r * Pp;
    aug[r * AW + c] = r == c ? 1.0 : 0.0;
    aug[r * AW + Pp + c] = r == c ? 1.0 : 0.0;
  }
  __syncthreads();
  wg_mgemm<false, false>(aug, AW, sA, LPx, sC, LPx, Pp, Pp, Pp, 1.0, 1.0);  // I + A C
#pragma unroll
  for (int j = 0; j < NCG; ++j) {
    const int c = cg + 16 * j;
    av[j] = (c < 2 * Pp && gr < Pp) ? aug[gr * AW + c] : 0.0;
  }
  int* pvb = reinterpret_cast<int*>(colb + 64);  // 2 ints
  bool used = gr >= P;
  int myk = -1;
  double myp = 1.0;
  int nsing = 0;
  for (int k = 0; k < P; ++k) {
    const int buf = k & 1;
    if (cg == (k & 15)) {
      const double colv = (k >> 4) ? av[1] : av[0];
      // arg max over the 32 lanes: DPP inside each 16-lane row, then the row pair
      double best = used ? -1.0 : fabs(colv);
      int bi = gr;
      auto take = [&](double ob, int oi) {
        const bool t = (ob > best) | ((ob == best) & (oi < bi));
        best = t ? ob : best;
        bi = t ? oi : bi;
      };
      take(dpp_f64<0xB1>(best), __builtin_amdgcn_mov_dpp(bi, 0xB1, 0xF, 0xF, false));
      take(dpp_f64<0x4E>(best), __builtin_amdgcn_mov_dpp(bi, 0x4E, 0xF, 0xF, false));
      take(dpp_f64<0x141>(best), __builtin_amdgcn_mov_dpp(bi, 0x141, 0xF, 0xF, false));
      take(dpp_f64<0x140>(best), __builtin_amdgcn_mov_dpp(bi, 0x140, 0xF, 0xF, false));
      {
        const auto bh = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(best),
                                                         (unsigned)__double2hiint(best), false, false);
        const auto bl = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(best),
                                                         (unsigned)__double2loint(best), false, false);
        const auto bx = __builtin_amdgcn_permlane16_swap((unsigned)bi, (unsigned)bi, false, false);
        const double b0 = __hiloint2double((int)bh[0], (int)bl[0]), b1 = __hiloint2double((int)bh[1], (int)bl[1]);
        best = b0;
        bi = (int)bx[0];
        take(b1, (int)bx[1]);
      }
      const double p = read_lane_f64(colv, bi + 32 * half);
      colb[buf * 32 + gr] = gr == bi ? p : colv * (1.0 / p);
      if (gr == 0) pvb[buf] = bi;
    }
    __syncthreads();
    const int pv = pvb[buf];
    const double f = colb[buf * 32 + gr];
    const bool piv = gr == pv;
    if (piv) {
      used = true;
      myk = k;
      myp = f;
      nsing += f == 0.0 ? 1 : 0;
    }
    const bool upd = !piv && gr < P;
    const int src = (pv + 32 * half) << 2;  // the pivot row's lane of this half-wave
    double prow[NCG];
#pragma unroll
    for (int j = 0; j < NCG; ++j)
      prow[j] = __hiloint2double(__builtin_amdgcn_ds_bpermute(src, __double2hiint(av[j])),
                                 __builtin_amdgcn_ds_bpermute(src, __double2loint(av[j])));
#pragma unroll
    for (int j = 0; j < NCG; ++j) {
      const double nv = fma(-f, prow[j], av[j]);
      av[j] = (upd && (cg + 16 * j > k)) ? nv : av[j];
    }
  }
  if (myk >= 0) {  // sC was last read by the product above
    const double ip = 1.0 / myp;
#pragma unroll
    for (int j = 0; j < NCG; ++j) {
      const int c = cg + 16 * j;
      if (c >= Pp && c < Pp + P) sC[myk * LPx + c - Pp] = av[j] * ip;
    }
  }
  if (nsing && cg == 0) atomicAdd(s_sing, nsing);  // singular I + A C (counted, not hidden)
}

template <bool F32, bool AH>
__global__ __launch_bounds__(512) void k_ekf_filter(EkfDims d, const int* __restrict__ I,
                                                    const double* __restrict__ Rl, const double* __restrict__ cams,
                                                    const double* __restrict__ meas, const double* __restrict__ lik,
                                                    const double* __restrict__ rbase, const double* __restrict__ Q,
                                                    const double* __restrict__ P0, const double* __restrict__ s0,
                                                    double* __restrict__ xpred, double* __restrict__ xest,
                                                    double* __restrict__ Ppred, double* __restrict__ Pest,
                                                    double* __restrict__ scratch, long long* __restrict__ outliers,
                                                    int* __restrict__ bad, [[maybe_unused]] unsigned long long* ekf_prof) {
  const int seq = blockIdx.x;
  const int tid = threadIdx.x, nth = blockDim.x, lane = tid & 63, wave = tid >> 6;
  const int n = d.n, P = d.P, m = d.m, LDP = d.npad + 1, Pp = d.Ppad;
  const int AW = Pp + d.npad + 1;  // [M | G | b]
  extern __shared__ double lds[];
  double* sP = lds;                                   // npad x LDP: covariance
  double* U = sP + (size_t)d.npad * LDP;              // union: FK phase / algebra phase
  double* fkb = U;                                    // batched FK of the P+1 poses
  const int LPx = Pp + 1;                             // row stride of sPx and sA
  double* sPx = U;                                    // npad x LPx: P[:, x] before the update
  double* aug = sPx + (size_t)ekf_wg_px_rows(d.npad, Pp) * LPx;  // Pp x AW
  double* sA = aug + (size_t)Pp * AW;                 // Pp x LPx
  // the FK and algebra phases share U; what follows must start past the larger of the two
  const size_t u_fk = ekf_wg_fk_doubles(P, d.J, d.L, Pp);  // batched FK, or the analytic H's region
  const size_t u_la = ekf_wg_la_doubles(d.npad, Pp);
  double* ss = U + (u_fk > u_la ? u_fk : u_la);      // n: state
  double* sCam = ss + d.npad;                         // camera records (every projection reads them)
  double* sRl = sCam + (size_t)d.C * ACS_CAM_STRIDE;  // skeleton table (reals, then ints)
  int* sI = reinterpret_cast<int*>(sRl + d.n_reals);
#ifdef EKF_PROFILE  // per-phase cycle counts (tools/prof_ekf_phases.py)
  __shared__ unsigned long long s_prof[8];
  unsigned long long t_last = 0;
  if (tid < 8) s_prof[tid] = 0;
#define EKF_TICK(k)                                                   \
  do {                                                                \
    __syncthreads();                                                  \
    const unsigned long long t_now = clock64();                       \
    if (tid == 0 && t_last) s_prof[(k + 7) % 8] += t_now - t_last;    \
    t_last = t_now;                                                   \
  } while (0)
#else
#define EKF_TICK(k) \
  do {              \
  } while (0)
#endif
  __shared__ unsigned long long s_out;
  __shared__ int s_piv, s_sing;  // pivoted update solve from now on (sticky); singular solves
  for (int e = tid; e < d.n_ints; e += nth) sI[e] = I[e];  // the FK walks the table: keep it in LDS
  for (int e = tid; e < d.n_reals; e += nth) sRl[e] = Rl[e];
  for (int e = tid; e < d.C * ACS_CAM_STRIDE; e += nth) sCam[e] = cams[e];
  __syncthreads();  // skel_view reads the header right away
  const SkelView sk = skel_view(sI, sRl);
  const double sT = d.sT, h2 = 0.5 * sT * sT;
  // per-sequence scratch: hpose (P+1) x m (analytic H: h, then 6 CL projection Jacobians);
  // H, W H (mpad x Pp, forward differences); res, w (mpad)
  const int mp = d.mpad;
  double* hpose = scratch + (size_t)seq * ((size_t)(P + 1) * m + 2 * (size_t)mp * Pp + 2 * mp);
  double* H = hpose + (size_t)(P + 1) * m;
  double* HW = H + (size_t)mp * Pp;
  double* res = HW + (size_t)mp * Pp;
  double* wr = res + mp;
  const size_t fstride = (size_t)d.C * d.L;  // measurements per frame
  for (int e = tid; e < d.npad * LDP; e += nth) {
    const int r = e / LDP, c = e % LDP;
    sP[e] = (r < n && c < n) ? P0[r * n + c] : 0.0;
  }
  for (int r = tid; r < d.npad; r += nth) ss[r] = r < n ? s0[(size_t)seq * n + r] : 0.0;
  if (tid == 0) {
    s_out = 0;
    s_piv = 0;
    s_sing = 0;
  }
  __syncthreads();

  for (int i = 0; i < d.N; ++i) {
    const size_t fo = ((size_t)seq * d.N + i);
    EKF_TICK(0);
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
    // F X: row block 0 += sT block 1 + sT^2/2 block 2, then block 1 += sT block 2 (each pass
    // reads only rows not yet updated); then the same on the columns for (F X) F^T
    for (Walk2 w(tid, nth, n); w.e < P * n; w.next()) {
      const int r = w.r, c = w.c;
      sP[r * LDP + c] += sT * sP[(r + P) * LDP + c] + h2 * sP[(r + 2 * P) * LDP + c];
    }
    __syncthreads();
    for (Walk2 w(tid, nth, n); w.e < P * n; w.next()) {
      const int r = P + w.r, c = w.c;
      sP[r * LDP + c] += sT * sP[(r + P) * LDP + c];
    }
    __syncthreads();
    for (Walk2 w(tid, nth, P); w.e < P * n; w.next()) {
      const int r = w.r, c = w.c;
      sP[r * LDP + c] += sT * sP[r * LDP + c + P] + h2 * sP[r * LDP + c + 2 * P];
    }
    __syncthreads();
    for (Walk2 w(tid, nth, P); w.e < P * n; w.next()) {
      const int r = w.r, c = P + w.c;
      sP[r * LDP + c] += sT * sP[r * LDP + c + P];
    }
    __syncthreads();
    for (Walk2 w(tid, nth, n); w.e < n * n; w.next()) {  // + Q, stored as P_pred (own elements)
      const double v = sP[w.r * LDP + w.c] + Q[w.e];
      sP[w.r * LDP + w.c] = v;
      Ppred[fo * n * n + w.e] = v;
    }

    EKF_TICK(1);
    const int CL = d.C * d.L;
    if constexpr (AH) {
      // ---- 2'. analytic H: one FK with its Jacobian (fk.hpp) and the
      // projection with its 2x3 world Jacobian; H row r = J_proj(obs) . d pos / d x_q.
      // hpose[0, m): h(x); hpose[m + 6 o ..]: the projection Jacobian of observation o
      FkShared& fsh = *reinterpret_cast<FkShared*>(fkb);
      fk_frame<false>(sk, ss, fsh, tid, nth);
      __syncthreads();
      // per-parameter derivative data resolved once (fk_deriv_prep: no table walk per entry)
      if (tid < P) fk_deriv_prep(sk, fsh, *reinterpret_cast<FkDeriv*>(fkb + ekf_fk_shared_doubles()), tid);
      for (int o = tid; o < CL; o += nth) {
        const int c = o / d.L, l = o - c * d.L;
        const double* x = fsh.pos[sk.outn[l]];
        ProjOut po;
        fisheye_project<true>(sCam + c * ACS_CAM_STRIDE, x[0], x[1], x[2], po);
        hpose[2 * o] = po.u;
        hpose[2 * o + 1] = po.v;
        double* jo = hpose + m + 6 * (size_t)o;
#pragma unroll
        for (int k = 0; k < 6; ++k) jo[k] = po.J[k];
      }
      __syncthreads();
    } else {
    // ---- 2. poses of the forward-difference Jacobian --------------------------------
    {
#ifdef EKF_PROFILE
      const unsigned long long tf0 = clock64();
#endif
      ekf_fk_batch<F32>(sk, ss, d.eps, fkb, tid, nth);
#ifdef EKF_PROFILE
      if (tid == 0) s_prof[7] += clock64() - tf0;  // FK share of the FK/proj phase
#endif
      const double* pos = fkb + FK_MAXJ * 9 + (FK_MAXP + 1) * 9 + (size_t)(P + 1) * d.J * 9;
      for (int e = tid; e < (P + 1) * CL; e += nth) {
        const int q = e / CL, o = e - q * CL;
        const int c = o / d.L, l = o - c * d.L;
        const double* x = pos + ((size_t)q * d.L + l) * 3;
        ProjOut po;
        fisheye_project<false>(sCam + c * ACS_CAM_STRIDE, x[0], x[1], x[2], po);
        hpose[(size_t)q * m + 2 * o] = po.u;
        hpose[(size_t)q * m + 2 * o + 1] = po.v;
      }
      __syncthreads();
    }
    }
    EKF_TICK(2);
    // residual and R^-1 per row (row r = 2 (c L + l) + d, the reference's ordering; rows
    // past m are zero padding for the MFMA products), then (forward differences) H and W H
    // element-parallel (coalesced stores)
    for (int r = tid; r < mp; r += nth) {
      double e = 0.0, w = 0.0;
      if (r < m) {
        const int o = r >> 1, c = o / d.L;
        e = meas[fo * fstride * 2 + r] - hpose[r];
        if (!isfinite(e)) e = (e != e) ? 0.0 : (e > 0 ? 1.7976931348623157e308 : -1.7976931348623157e308);
        const double lk = lik[fo * fstride + o];
        const double sd = (lk < d.thresh) ? d.maxpix : rbase[c];
        w = 1.0 / (sd * sd);
      }
      res[r] = e;
      wr[r] = w;
    }
    __syncthreads();
    // operands of the A / b products below: A = opW^T opH, b = opW^T opr over nks k-steps of
    // 4 rows (forward differences: H rows of every observation; analytic: per-marker rows)
    const double* opW = HW;
    const double* opH = H;
    const double* opr = res;
    int nks = mp >> 2, ldo = Pp;
    if constexpr (AH) {
      // Marker space. Row r of H is j_r D_l (j_r: a row of the observation's 2x3 projection
      // Jacobian, D_l = d pos_l / d x: 3 x P, the same for every camera), so
      //   A = sum_l D_l^T M_l D_l,  M_l = sum_c J^T W J (3x3),
      //   b = sum_l D_l^T g_l,      g_l = sum_c J^T W r,
      //   diag(H P_xx H^T)_r = j_r N_l j_r^T,  N_l = D_l P_xx D_l^T (3x3):
      // the products run over 3 L rows instead of 2 C L (the same sums in another order)
      const FkShared& fsh = *reinterpret_cast<const FkShared*>(fkb);
      const FkDeriv& fkd = *reinterpret_cast<const FkDeriv*>(fkb + ekf_fk_shared_doubles());
      const int L = d.L, R3 = ekf_ah_rows(L), LD = Pp + 1;  // odd row stride: MFMA A reads
      double* sD = fkb + ekf_ah_base();
      double* sTm = sD + (size_t)R3 * LD;
      double* sS = sTm + (size_t)R3 * LD;
      double* sg = sS + (size_t)R3 * LD;
      double* sN = sg + R3;
      double* sM = sN + 9 * L;
      for (int e = tid; e < L * Pp; e += nth) {  // D rows 3 l + k (zero padding columns)
        const int l = e / Pp, q = e - l * Pp;
        double dp[3] = {0.0, 0.0, 0.0};
        if (q < P) fk_dpos_fast(sk, fsh, fkd, sk.outn[l], q, dp);
#pragma unroll
        for (int k = 0; k < 3; ++k) sD[(3 * l + k) * LD + q] = dp[k];
      }
      for (int e = tid; e < (R3 - 3 * L) * Pp; e += nth) {  // padding rows
        const int r = e / Pp;
        sD[(3 * L + r) * LD + e - r * Pp] = 0.0;
      }
      for (int e = tid; e < 9 * L; e += nth) {  // M_l (6 entries of the symmetric 3x3), g_l (3)
        const int l = e / 9, k = e - 9 * l;
        const int a = k < 3 ? 0 : (k < 5 ? 1 : (k < 6 ? 2 : k - 6));
        const int b = k < 3 ? k : (k < 5 ? k - 2 : 2);
        double v = 0.0;
        for (int c = 0; c < d.C; ++c) {
          const int o = c * L + l;
          const double* J = hpose + m + 6 * (size_t)o;
          const double wu = wr[2 * o], wv = wr[2 * o + 1];
          if (k < 6)
            v += wu * J[a] * J[b] + wv * J[3 + a] * J[3 + b];
          else
            v += wu * J[a] * res[2 * o] + wv * J[3 + a] * res[2 * o + 1];
        }
        if (k < 6)
          sM[6 * l + k] = v;
        else
          sg[3 * l + a] = v;
      }
      for (int r = 3 * L + tid; r < R3; r += nth) sg[r] = 0.0;
      __syncthreads();
      for (int e = tid; e < R3 * Pp; e += nth) {  // T = M D
        const int row = e / Pp, q = e - row * Pp;
        double t = 0.0;
        if (row < 3 * L) {
          const int l = row / 3, k = row - 3 * l;
          const double* Ml = sM + 6 * l;
          const double m0 = k == 0 ? Ml[0] : (k == 1 ? Ml[1] : Ml[2]);
          const double m1 = k == 0 ? Ml[1] : (k == 1 ? Ml[3] : Ml[4]);
          const double m2 = k == 0 ? Ml[2] : (k == 1 ? Ml[4] : Ml[5]);
          t = m0 * sD[(3 * l) * LD + q] + m1 * sD[(3 * l + 1) * LD + q] + m2 * sD[(3 * l + 2) * LD + q];
        }
        sTm[row * LD + q] = t;
      }
      // S = D P[0:Pp, 0:Pp] on MFMA (D is zero past column P; S is read only below column P)
      wg_mgemm<false, false>(sS, LD, sD, LD, sP, LDP, R3, Pp, Pp, 1.0, 0.0);
      for (int e = tid; e < 9 * L; e += nth) {  // N_l = S_l D_l^T
        const int l = e / 9, k = e - 9 * l, a = k / 3, b = k - 3 * a;
        double v = 0.0;
        for (int q = 0; q < P; ++q) v = fma(sS[(3 * l + a) * LD + q], sD[(3 * l + b) * LD + q], v);
        sN[e] = v;
      }
      __syncthreads();
      // 3-sigma outlier count (:259-264), an observation if either of its rows fails
      unsigned long long cnt = 0;
      for (int o = tid; o < CL; o += nth) {
        const double* J = hpose + m + 6 * (size_t)o;
        const double* N = sN + 9 * (o % L);
        bool outl = false;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
          const double* j = J + 3 * side;
          const double q = j[0] * (N[0] * j[0] + N[1] * j[1] + N[2] * j[2]) +
                           j[1] * (N[3] * j[0] + N[4] * j[1] + N[5] * j[2]) +
                           j[2] * (N[6] * j[0] + N[7] * j[1] + N[8] * j[2]);
          const int r = 2 * o + side;
          const double Srr = q + 1.0 / wr[r];
          outl = outl || fabs(res[r]) > 3.0 * sqrt(Srr);
        }
        if (outl) ++cnt;
      }
      if (cnt) atomicAdd(&s_out, cnt);
      opW = sD;
      opH = sTm;
      opr = sg;
      nks = R3 >> 2;
      ldo = LD;
    }  // forward differences: H is formed chunk by chunk in LDS in the products below
    __syncthreads();
    EKF_TICK(3);
    // ---- 3. information-form update -------------------------------------------------
    {
      // A = H^T R^-1 H (upper tiles) and b = H^T R^-1 r (a 16-column tile whose column 0 is
      // r) on MFMA, the k-steps (4 rows of H each) dealt round-robin to KS waves, 4 k-steps
      // of operands loaded before their MFMAs; the KS partial tiles are summed in a fixed
      // tree through LDS (sPx / aug are free until the products below)
      const int li = lane & 15, lk = lane >> 4;
      const int NTt = Pp >> 4, nAt = NTt * (NTt + 1) / 2, nt = nAt + NTt;
      const size_t avail = (size_t)d.npad * Pp + (size_t)Pp * AW;
      int KS = AH ? EKF_WAVES : 4;  // forward differences: waves 4-7 count the outliers
      while (KS > 1 && (size_t)(KS / 2) * nt * 256 > avail) KS >>= 1;
      double* red = sPx;
      constexpr int NTMAX = 5;  // 3 upper A tiles + 2 b tiles at Ppad = 32
      dbl4 acc[NTMAX];
#pragma unroll
      for (int t = 0; t < NTMAX; ++t) acc[t] = dbl4{0.0, 0.0, 0.0, 0.0};
      auto tile_ij = [&](int t, int& i0, int& j0) {  // t < nAt: upper A tiles; then b tiles
        if (t < nAt) {
          i0 = (NTt == 2 && t == 2) ? 16 : 0;
          j0 = (NTt == 2 && t >= 1) ? 16 : 0;
        } else {
          i0 = (t - nAt) * 16;
          j0 = -1;
        }
      };
      unsigned long long cnt_fd = 0;
      if constexpr (!AH) {
        // Forward differences: H (:81-96) in chunks of EKF_FD_RCH rows, formed from the pixel
        // table into LDS with their weights and residuals (one global round trip per chunk);
        // waves 0-3 add the chunk's k-steps to A and b on MFMA while waves 4-7 run the 3-sigma
        // test of its rows (diag S = rows of H_x P_xx . H_x, + R, row tiles on MFMA)
        const int LDc = Pp + 1;
        double* sHc = sPx + 2 * 5 * 256;  // after the KS = 4 tree buffer
        double* sWc = sHc + (size_t)EKF_FD_RCH * LDc;
        double* sRc = sWc + EKF_FD_RCH;
        for (int r0 = 0; r0 < mp; r0 += EKF_FD_RCH) {
          const int rows = min(EKF_FD_RCH, mp - r0);  // a multiple of 16
          for (int e = tid; e < rows * Pp; e += nth) {  // rows fastest: coalesced pixel loads
            const int q = e / rows, rr = e - q * rows, r = r0 + rr;
            double hq = 0.0;
            if (r < m && q < P) hq = (hpose[(size_t)(q + 1) * m + r] - hpose[r]) / d.eps;
            sHc[rr * LDc + q] = hq;
          }
          for (int rr = tid; rr < rows; rr += nth) {
            sWc[rr] = wr[r0 + rr];
            sRc[rr] = res[r0 + rr];
          }
          __syncthreads();
          if (wave < KS) {
            for (int st = wave; st < (rows >> 2); st += KS) {
              const int kl = 4 * st + lk;
              const double wk = sWc[kl];
              double av[2], bv[2];
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                bv[h] = h < NTt ? sHc[kl * LDc + 16 * h + li] : 0.0;
                av[h] = wk * bv[h];  // (W H)[k][q]
              }
              const double rv = li == 0 ? sRc[kl] : 0.0;
#pragma unroll
              for (int t = 0; t < NTMAX; ++t) {
                if (t >= nt) break;
                int i0, j0;
                tile_ij(t, i0, j0);
                const double aop = i0 ? av[1] : av[0];
                const double bop = j0 < 0 ? rv : (j0 ? bv[1] : bv[0]);
                acc[t] = mfma64(aop, bop, acc[t]);
              }
            }
          } else {
            for (int rt = wave - KS; rt < (rows >> 4); rt += EKF_WAVES - KS) {
              const int i0 = rt << 4;
              double ha[8];
#pragma unroll
              for (int s8 = 0; s8 < 8; ++s8) ha[s8] = (4 * s8 < Pp) ? sHc[(i0 + li) * LDc + 4 * s8 + lk] : 0.0;
              double hr[2][4];
#pragma unroll
              for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int q = 0; q < 4; ++q) hr[h][q] = h < NTt ? sHc[(i0 + lk + 4 * q) * LDc + 16 * h + li] : 0.0;
              double dq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
              for (int h = 0; h < 2; ++h) {
                if (h >= NTt) break;
                dbl4 g = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int s8 = 0; s8 < 8; ++s8)
                  if (4 * s8 < Pp) g = mfma64(ha[s8], sP[(4 * s8 + lk) * LDP + 16 * h + li], g);
#pragma unroll
                for (int q = 0; q < 4; ++q) dq[q] += g[q] * hr[h][q];
              }
              // the 16-lane sums are all-reduced (every lane holds them, bit-identical); lane
              // li = q < 4 tests row i0 + lk + 4 q, so the 4 rows' divisions and square roots
              // run side by side instead of one after another
#pragma unroll
              for (int q = 0; q < 4; ++q) dq[q] = group_sum<16>(dq[q]);
              const double dsel = li == 1 ? dq[1] : li == 2 ? dq[2] : li == 3 ? dq[3] : dq[0];
              const int rl = i0 + lk + 4 * (li & 3), r = r0 + rl;
              bool outl = false;
              if (li < 4 && r < m) {
                const double Srr = dsel + 1.0 / sWc[rl];
                outl = fabs(sRc[rl]) > 3.0 * sqrt(Srr);
              }
              // rows 2 pt (lk even) and 2 pt + 1 (lane + 16)
              const int other = __shfl_xor((int)outl, 16);
              if (li < 4 && !(lk & 1) && r < m && (outl || other)) ++cnt_fd;
            }
          }
          __syncthreads();
        }
      }
      if (AH && wave < KS) {
        constexpr int UB = 2;  // k-steps per batch of loads
        for (int s0 = wave; s0 < nks; s0 += UB * KS) {
          double av[UB][2], bv[UB][2], rv[UB];
#pragma unroll
          for (int u = 0; u < UB; ++u) {
            const int k = 4 * (s0 + u * KS) + lk;
            const bool ok = s0 + u * KS < nks;
            const double wk = (!AH && ok) ? wr[k] : 0.0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              bv[u][h] = (ok && h < NTt) ? opH[(size_t)k * ldo + 16 * h + li] : 0.0;
              if constexpr (AH)
                av[u][h] = (ok && h < NTt) ? opW[(size_t)k * ldo + 16 * h + li] : 0.0;
              else
                av[u][h] = wk * bv[u][h];  // (W H)[k][q], the product the scratch copy held
            }
            rv[u] = (ok && li == 0) ? opr[k] : 0.0;
          }
#pragma unroll
          for (int u = 0; u < UB; ++u)
#pragma unroll
            for (int t = 0; t < NTMAX; ++t) {
              if (t >= nt) break;
              int i0, j0;
              tile_ij(t, i0, j0);
              const double aop = i0 ? av[u][1] : av[u][0];  // selects: no dynamic register index
              const double bop = j0 < 0 ? rv[u] : (j0 ? bv[u][1] : bv[u][0]);
              acc[t] = mfma64(aop, bop, acc[t]);
            }
        }
      }
      // fixed-order tree over the KS partials
      if constexpr (AH) __syncthreads();  // the tree's buffer overlaps the marker-space operands
      for (int h = KS >> 1; h >= 1; h >>= 1) {
        if (wave >= h && wave < 2 * h)
#pragma unroll
          for (int t = 0; t < NTMAX; ++t)
            if (t < nt)
#pragma unroll
              for (int q = 0; q < 4; ++q) red[((size_t)(wave - h) * nt + t) * 256 + q * 64 + lane] = acc[t][q];
        __syncthreads();
        if (wave < h)
#pragma unroll
          for (int t = 0; t < NTMAX; ++t)
            if (t < nt)
#pragma unroll
              for (int q = 0; q < 4; ++q) acc[t][q] += red[((size_t)wave * nt + t) * 256 + q * 64 + lane];
        __syncthreads();
      }
      if (wave == 0) {
#pragma unroll
        for (int t = 0; t < NTMAX; ++t) {
          if (t >= nt) break;
          int i0, j0;
          tile_ij(t, i0, j0);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int row = i0 + lk + 4 * q;
            if (j0 >= 0) {
              sA[row * LPx + j0 + li] = acc[t][q];
              sA[(j0 + li) * LPx + row] = acc[t][q];  // lower triangle (symmetric)
            } else if (li == 0) {
              aug[row * AW + Pp + d.npad] = row < P ? acc[t][q] : 0.0;
            }
          }
        }
      }
      // 3-sigma outlier count (:259-264): diag S = rows of H_x P_xx . H_x, + R. Row tiles of
      // H P_xx on MFMA (operands loaded first), each row's dot with its own H row summed
      // across the 16 column lanes (DPP) and the column tiles
      unsigned long long cnt = cnt_fd;  // forward differences: counted in the chunks above
      if (cnt) atomicAdd(&s_out, cnt);
      __syncthreads();
    }
    EKF_TICK(4);
    // The update needs (I + A C)^-1 [A P[x, :] | b], C = P_xx. With W = C + C A C = C (I + A C)
    // (symmetric), (I + A C)^-1 = W^-1 C: a Gauss-Jordan on [W | C] with the pivots on the
    // diagonal (no pivot search; the pivot row of step k is row k) gives V = (I + A C)^-1, then
    // Z_G = (V A) P[x, :] and Z_b = V b on MFMA / per thread.
    // W is positive definite exactly when C is (A is PSD), and then diagonal pivots are stable.
    // The reference's default P0 is not (src/core/ekf.py:155, neck length -0.28), so every
    // pivot is checked: all positive certifies W > 0 (Sylvester); the first that is not ends
    // the diagonal solve, and V comes from a partially pivoted Gauss-Jordan on [I + A C | I]
    // instead, for this frame and (sticky, s_piv) every later frame of the sequence.
    // Scratch: C, then V, in sPx's first Ppad x LPx; A C, then V A, in the next; [W | C] in
    // aug's first 2 Ppad columns (P[:, x] is copied into sPx once they are consumed).
    double* sC = sPx;
    double* sAC = sPx + (size_t)Pp * LPx;
    for (int e = tid; e < Pp * Pp; e += nth) {
      const int r = e / Pp, c = e - r * Pp;
      const double v = (r < P && c < P) ? sP[r * LDP + c] : 0.0;
      sC[r * LPx + c] = v;
      aug[r * AW + c] = v;
      aug[r * AW + Pp + c] = v;
    }
    __syncthreads();
    wg_mgemm<false, false>(sAC, LPx, sA, LPx, sC, LPx, Pp, Pp, Pp, 1.0, 0.0);  // A C
    wg_mgemm<false, false>(aug, AW, sC, LPx, sAC, LPx, Pp, Pp, Pp, 1.0, 1.0);  // W = C + C (A C)
    EKF_TICK(5);
    // Gauss-Jordan on [W | C], register-resident, one barrier per pivot. Thread (row
    // gr = tid & 31, column group cg = tid >> 5) holds aug[gr][cg + 16 j]. Step k: the 32
    // lanes owning column k publish the row factors a[r][k] / a[k][k] (slot k carries the
    // pivot); after the barrier every other row subtracts its factor times row k (read from
    // the owning lane of the same wave by ds_bpermute). At the end row k over its pivot is
    // row k of V.
    {
      constexpr int NCG = 4;  // 2 Ppad <= 64 columns
      const int gr = tid & 31, cg = tid >> 5, half = cg & 1;
      double av[NCG];
      double* colb = sAC;                           // 2 x 32 doubles (A C is consumed)
      bool diag = s_piv == 0;                       // uniform
      if (diag) {
#pragma unroll
        for (int j = 0; j < NCG; ++j) {
          const int c = cg + 16 * j;
          av[j] = (c < 2 * Pp && gr < Pp) ? aug[gr * AW + c] : 0.0;
        }
        double myp = 1.0;
        __syncthreads();  // sAC free
        for (int k = 0; k < P; ++k) {
          const int buf = k & 1;
          if (cg == (k & 15)) {
            const double colv = (k >> 4) ? av[1] : av[0];  // k < P <= FK_MAXP = 32 (checked on entry)
            const double p = read_lane_f64(colv, k + 32 * half);
            colb[buf * 32 + gr] = gr == k ? p : colv * rcp_nr(p);  // one reciprocal (rcp + Newton), uniform
          }
          __syncthreads();
          const double f = colb[buf * 32 + gr];
          if (!(colb[buf * 32 + k] > 0.0)) {  // W not positive definite: the pivoted solve below
            diag = false;
            break;
          }
          if (gr == k) myp = f;
          const bool upd = gr != k && gr < P;
          const int src = (k + 32 * half) << 2;  // row k's lane of this half-wave
          double prow[NCG];
#pragma unroll
          for (int j = 0; j < NCG; ++j)
            prow[j] = __hiloint2double(__builtin_amdgcn_ds_bpermute(src, __double2hiint(av[j])),
                                       __builtin_amdgcn_ds_bpermute(src, __double2loint(av[j])));
#pragma unroll
          for (int j = 0; j < NCG; ++j) {
            const double nv = fma(-f, prow[j], av[j]);
            av[j] = (upd && (cg + 16 * j > k)) ? nv : av[j];
          }
        }
        if (diag && gr < P) {  // V rows into sC (every thread read sC into aug above)
          const double ip = rcp_nr(myp);
#pragma unroll
          for (int j = 0; j < NCG; ++j) {
            const int c = cg + 16 * j;
            if (c >= Pp && c < Pp + P) sC[gr * LPx + c - Pp] = av[j] * ip;
          }
        }
      }
      if (!diag) {
        __syncthreads();  // every thread past the diagonal solve's LDS reads
        if (tid == 0) s_piv = 1;
        ekf_update_pivoted(aug, AW, sA, sC, LPx, colb, P, Pp, &s_sing);
      }
      __syncthreads();
    }
    wg_mgemm<false, false>(sAC, LPx, sC, LPx, sA, LPx, Pp, Pp, Pp, 1.0, 0.0);  // Y = V A
    if (tid < P) {  // Z_b = V b -> sA (A is consumed)
      double v = 0.0;
      for (int k = 0; k < P; ++k) v = fma(sC[tid * LPx + k], aug[k * AW + Pp + d.npad], v);
      sA[tid] = v;
    }
    wg_mgemm<false, false>(aug + Pp, AW, sAC, LPx, sP, LDP, Pp, d.npad, Pp, 1.0, 0.0);  // Z_G = Y P[0:Pp, :]
    for (int e = tid; e < d.npad * Pp; e += nth) {  // P[:, x] (V and Y are consumed)
      const int r = e / Pp, c = e % Pp;
      sPx[r * LPx + c] = (r < n && c < P) ? sP[r * LDP + c] : 0.0;
    }
    for (int e = tid; e < Pp * d.npad; e += nth) {  // Z_G columns >= n must be zero
      const int r = e / d.npad, c = e % d.npad;
      if (c >= n) aug[r * AW + Pp + c] = 0.0;
    }
    __syncthreads();
    EKF_TICK(6);
    // s += P[:, x] Z_b ;  P -= P[:, x] Z_G  (MFMA; sPx / Z are zero outside the live block)
    if (tid < n) {
      double v = 0.0;
      for (int k = 0; k < P; ++k) v += sPx[tid * LPx + k] * sA[k];
      ss[tid] += v;
    }
    wg_mgemm<false, false>(sP, LDP, sPx, LPx, aug + Pp, AW, d.npad, d.npad, Pp, -1.0, 1.0);
    EKF_TICK(7);
    if (tid < n) xest[fo * n + tid] = ss[tid];
    for (Walk2 w(tid, nth, n); w.e < n * n; w.next()) Pest[fo * n * n + w.e] = sP[w.r * LDP + w.c];
    __syncthreads();
  }
#ifdef EKF_PROFILE
  if (tid == 0 && ekf_prof)
    for (int k = 0; k < 8; ++k) ekf_prof[seq * 8 + k] = s_prof[k];
#endif
  if (tid == 0) {
    outliers[seq] = (long long)s_out;
    if (s_sing) atomicAdd(bad, s_sing);
  }
}

// ---------------------------------------------------------------------------------------
// Small-state filter: the head model (P = EKF_W1_P = 6 parameters, n = 18), the parameter
// count a compile-time constant, NW = 4 waves per sequence (1 for A/B: ACS_EKF_W1_WAVES=1). At
// 6 parameters the per-frame algebra is a few thousand flops, and the 8-wave workgroup of
// k_ekf_filter spent its frame on barriers, LDS round trips and MFMA tiles that are mostly
// padding (24 us per 12-camera frame, profiles/r03/ekf_phases_head12.log). Here:
//   * prediction and the measurement model as k_ekf_filter (same device code: the P F P^T
//     passes, ekf_fk_batch / fk_frame, the fisheye projection), all scratch in LDS;
//   * A = H^T R^-1 H and b = H^T R^-1 r one entry per lane of wave 0 (rows split over its
//     half-waves, one shuffle); the 3-sigma test one observation per lane with P_xx in
//     registers, compared squared (r^2 > 9 S_rr: no square root, no division);
//   * [W | P_xx], W = P_xx + P_xx A P_xx, column-per-lane of wave 0 (2 P = 12 columns) and
//     Gauss-Jordan with the pivots on the diagonal in its registers (W is symmetric positive
//     definite: no pivot search), the column-k entries by readlane, one reciprocal per step:
//     V = (I + A P_xx)^-1 with no LDS round trip or barrier; meanwhile wave 1 forms
//     [A P[x,:] | b], and [Z_G | Z_b] = V [A P[x,:] | b] column per thread;
//   * the state / covariance update from the solution rows in LDS.
// Same algebra as k_ekf_filter; the sums are in another order, so results agree to rounding
// (tests/test_gpu_ekf.py; tools/ekf_drift.py: the same drift against the oracle as the
// 8-wave kernel over 250 frames).
#define EKF_W1_P 6
// A / B switch (tools/gpu_r06m.sh): 0 = Q, the measurements and the likelihoods read from
// global memory inside each frame, as before round 6
#ifndef EKF_W1_PREFETCH
#define EKF_W1_PREFETCH 1
#endif
// A / B switch (tools/gpu_r06n.sh): 0 = the one-joint FK's trig tables formed at the start of
// the FK / projection phase, behind their own barrier
#ifndef EKF_W1_TRIG_EARLY
#define EKF_W1_TRIG_EARLY 1
#endif

// LDS doubles of k_ekf_filter_w1
__host__ __device__ inline size_t ekf_w1_lds(const EkfDims& d) {
  const size_t n = d.n, P = d.P, m = d.m;
  return n * (n + 1) + d.npad + (P + 1) * m + m * P + 3 * m + n * P + P * (n + 1) + 2 * P * P + P +
         ekf_w1_fk_doubles(d.P, d.J, d.L) + (size_t)d.C * ACS_CAM_STRIDE + d.n_reals + (d.n_ints + 1) / 2 + 1;
}

// k_ekf_filter_w1's update solve for a W that is not positive definite: column c of
// [I + A C | I] on lane c of wave 0, Gauss-Jordan with partial pivoting in its registers (the
// pivot column's lane finds the pivot row in its own registers: largest |a|, lowest row on
// ties); row pv_k over its pivot ends as row k of V (not inlined: the common path keeps its
// registers).
template <int P>
__device__ __noinline__ void ekf_w1_pivoted(const double* sA, const double* sP, int LDP, double* sV, int tid,
                                            int* __restrict__ bad) {
  double a[P];
  const int c = tid;
  if (c < P) {  // column c of I + A C
#pragma unroll
    for (int r = 0; r < P; ++r) {
      double v = r == c ? 1.0 : 0.0;
#pragma unroll
      for (int k = 0; k < P; ++k) v = fma(sA[r * P + k], sP[k * LDP + c], v);
      a[r] = v;
    }
  } else {
#pragma unroll
    for (int r = 0; r < P; ++r) a[r] = r == c - P ? 1.0 : 0.0;
  }
  // the pivot column's lane finds the pivot row in its own registers (largest |a|,
  // lowest row on ties); row pv_k over its pivot ends as row k of V
  unsigned used = 0;
  int pvk[P];
  double pk[P];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    double best = -1.0;
    int bi = 0;
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const bool cand = !((used >> r) & 1u) && fabs(a[r]) > best;
      best = cand ? fabs(a[r]) : best;
      bi = cand ? r : bi;
    }
    const int pv = __builtin_amdgcn_readlane(bi, k);
    double colv[P];
#pragma unroll
    for (int r = 0; r < P; ++r) colv[r] = read_lane_f64(a[r], k);
    double pp = 0.0, prow = 0.0;
#pragma unroll
    for (int r = 0; r < P; ++r) {
      pp = r == pv ? colv[r] : pp;
      prow = r == pv ? a[r] : prow;
    }
    const double ip = 1.0 / pp;
#pragma unroll
    for (int r = 0; r < P; ++r) {
      const double nv = fma(-(colv[r] * ip), prow, a[r]);
      a[r] = (r != pv && tid > k) ? nv : a[r];
    }
    used |= 1u << pv;
    pvk[k] = pv;
    pk[k] = pp;
  }
  if (tid >= P && tid < 2 * P) {
#pragma unroll
    for (int k = 0; k < P; ++k) {
      double v = 0.0;
#pragma unroll
      for (int r = 0; r < P; ++r) v = r == pvk[k] ? a[r] : v;
      sV[k * P + tid - P] = v / pk[k];
    }
  }
  if (tid == 0) {
    int ns = 0;
#pragma unroll
    for (int k = 0; k < P; ++k) ns += pk[k] == 0.0 ? 1 : 0;
    if (ns) atomicAdd(bad, ns);  // singular I + A C (counted, not hidden)
  }
}

template <bool F32, bool AH, int PM, int NW>
__global__ __launch_bounds__(64 * NW) void k_ekf_filter_w1(EkfDims d, const int* __restrict__ I,
                                                      const double* __restrict__ Rl, const double* __restrict__ cams,
                                                      const double* __restrict__ meas, const double* __restrict__ lik,
                                                      const double* __restrict__ rbase, const double* __restrict__ Q,
                                                      const double* __restrict__ P0, const double* __restrict__ s0,
                                                      double* __restrict__ xpred, double* __restrict__ xest,
                                                      double* __restrict__ Ppred, double* __restrict__ Pest,
                                                      long long* __restrict__ outliers, int* __restrict__ bad,
                                                      [[maybe_unused]] unsigned long long* ekf_prof) {
  constexpr int P = PM, n = 3 * PM, LDP = n + 1, NZ1 = n + 1;
  static_assert(n + 1 <= 64 && 2 * P <= 64, "one column per lane");
  const int seq = blockIdx.x;
  const int tid = threadIdx.x, nth = 64 * NW;
  const int m = d.m, CL = d.C * d.L;
  __shared__ long long s_nout;
  if (tid == 0) s_nout = 0;
  extern __shared__ double lds[];
  double* sP = lds;                                     // n x LDP: covariance
  double* ss = sP + (size_t)n * LDP;                    // npad: state
  double* hp = ss + d.npad;                             // (P+1) x m: FD poses' pixels | AH: h + 6 CL Jacobians
  double* sH = hp + (size_t)(P + 1) * m;                // m x P
  double* sr = sH + (size_t)m * P;                      // m: residuals
  double* sw = sr + m;                                  // m: 1 / sd^2
  double* sd2 = sw + m;                                 // m: sd^2
  double* sPx = sd2 + m;                                // n x P: P[:, x] before the update
  double* sZ = sPx + (size_t)n * P;                     // P x (n + 1): [Z_G | Z_b]
  double* sA = sZ + (size_t)P * NZ1;                    // P x P, then b (P)
  double* sV = sA + P * P + P;                          // P x P: (I + A P_xx)^-1
  double* fkb = sV + P * P;                             // FK scratch
  double* sCam = fkb + ekf_w1_fk_doubles(P, d.J, d.L);  // camera records (read by every projection)
  double* sRl = sCam + (size_t)d.C * ACS_CAM_STRIDE;     // skeleton table (reals, then ints)
  int* sI = reinterpret_cast<int*>(sRl + d.n_reals);
#ifdef EKF_PROFILE
  unsigned long long s_prof[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_last = 0, s_sub = 0;
#define EKF_TICK1(k)                                                              \
  do {                                                                            \
    __syncthreads();                                                              \
    const unsigned long long t_now = clock64();                                   \
    if (t_last) s_prof[(k + 7) % 8] += t_now - t_last;                            \
    t_last = t_now;                                                               \
  } while (0)
#else
#define EKF_TICK1(k) \
  do {               \
  } while (0)
#endif
  for (int e = tid; e < d.n_ints; e += nth) sI[e] = I[e];
  for (int e = tid; e < d.n_reals; e += nth) sRl[e] = Rl[e];
  for (int e = tid; e < d.C * ACS_CAM_STRIDE; e += nth) sCam[e] = cams[e];
  for (int e = tid; e < n * LDP; e += nth) {
    const int r = e / LDP, c = e - r * LDP;
    sP[e] = c < n ? P0[r * n + c] : 0.0;
  }
  for (int r = tid; r < d.npad; r += nth) ss[r] = r < n ? s0[(size_t)seq * n + r] : 0.0;
  __syncthreads();
  const SkelView sk = skel_view(sI, sRl);
  const double sT = d.sT, h2 = 0.5 * sT * sT;
  const size_t fstride = (size_t)CL;
  long long nout = 0;
  constexpr int nA = P * (P + 1) / 2, nAb = nA + P;
  static_assert(nAb <= 32, "one A / b entry per lane of a half-wave");
  // this lane's A / b entry: (ea, eb), ea <= eb, row-major upper triangle, then b_ea (eb < 0)
  int ea = 0, eb = -1;
  {
    const int t = tid & 31;
    if (t < nA) {
      int tt = t;
      while (tt >= P - ea) {
        tt -= P - ea;
        ++ea;
      }
      eb = ea + tt;
    } else if (t < nAb) {
      ea = t - nA;
    }
  }
  // one-joint skeletons with one (pose, observation) item per thread: the item's table walk
  // resolved once (ekf_point_plan); otherwise ekf_fk_point walks it every frame
  EkfPointPlan pl;
  pl.ok = false;
  if constexpr (!AH) {
    if (sk.J == 1 && (P + 1) * CL <= nth && tid < (P + 1) * CL) pl = ekf_point_plan(sk, tid / CL, (tid % CL) % d.L);
  }
  // no global load on a frame's chain: Q in registers (the predict phase's elements of this
  // thread), this thread's measurement row loaded one frame ahead, its camera's weights formed
  // once (the same expressions, so the same bits)
  constexpr int QR = (n * n + 64 * NW - 1) / (64 * NW);
  double qreg[QR];
#pragma unroll
  for (int k = 0; k < QR; ++k) qreg[k] = tid + k * nth < n * n ? Q[tid + k * nth] : 0.0;
  const bool pf = EKF_W1_PREFETCH && m <= nth;
  // the trig tables formed inside the prediction when the second covariance pass (P n threads,
  // rounded up to a wave) leaves enough threads idle for their 2 P + 2 (P + 1) items
  const int trig_t0 = ((P * n + 63) / 64) * 64;
  const bool trig_early = EKF_W1_TRIG_EARLY && !AH && sk.J == 1 && trig_t0 + 4 * P + 2 <= nth;
  double m_nx = 0.0, l_nx = 0.0, w_rb = 0.0, s2_rb = 0.0;
  const double w_mx = 1.0 / (d.maxpix * d.maxpix), s2_mx = d.maxpix * d.maxpix;
  if (pf && tid < m) {
    const double rb = rbase[(tid >> 1) / d.L];
    w_rb = 1.0 / (rb * rb);
    s2_rb = rb * rb;
    const size_t f0 = (size_t)seq * d.N;
    m_nx = meas[f0 * fstride * 2 + tid];
    l_nx = lik[f0 * fstride + (tid >> 1)];
  }
  for (int i = 0; i < d.N; ++i) {
    const size_t fo = (size_t)seq * d.N + i;
    const double m_cur = m_nx, l_cur = l_nx;
    if (pf && tid < m && i + 1 < d.N) {
      m_nx = meas[(fo + 1) * fstride * 2 + tid];
      l_nx = lik[(fo + 1) * fstride + (tid >> 1)];
    }
    EKF_TICK1(0);
    // ---- 1. prediction (k_ekf_filter's arithmetic) ------------------------------------
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
    for (Walk2 w(tid, nth, n); w.e < P * n; w.next())
      sP[w.r * LDP + w.c] += sT * sP[(w.r + P) * LDP + w.c] + h2 * sP[(w.r + 2 * P) * LDP + w.c];
    __syncthreads();
    // the one-joint FK's trig / translation tables from the predicted state (visible from here)
    // by threads the covariance passes leave idle (visible to the FK items after the next
    // barriers)
    if (trig_early && tid >= trig_t0)
      ekf_fk_trig_trans<F32>(sk, ss, d.eps, fkb, fkb + 4 * FK_MAXP, tid - trig_t0, nth - trig_t0);
    for (Walk2 w(tid, nth, n); w.e < P * n; w.next()) sP[(P + w.r) * LDP + w.c] += sT * sP[(w.r + 2 * P) * LDP + w.c];
    __syncthreads();
    for (Walk2 w(tid, nth, P); w.e < P * n; w.next())
      sP[w.r * LDP + w.c] += sT * sP[w.r * LDP + w.c + P] + h2 * sP[w.r * LDP + w.c + 2 * P];
    __syncthreads();
    for (Walk2 w(tid, nth, P); w.e < P * n; w.next()) sP[w.r * LDP + P + w.c] += sT * sP[w.r * LDP + w.c + 2 * P];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < QR; ++k) {
      const int e = tid + k * nth;
      if (e < n * n) {
        const int r = e / n, c = e - r * n;
        const double v = sP[r * LDP + c] + (EKF_W1_PREFETCH ? qreg[k] : Q[e]);
        sP[r * LDP + c] = v;
        Ppred[fo * n * n + e] = v;
      }
    }
    EKF_TICK1(1);
    // ---- 2. measurement model ---------------------------------------------------------
    if constexpr (AH) {
      FkShared& fsh = *reinterpret_cast<FkShared*>(fkb);
      fk_frame<false>(sk, ss, fsh, tid, nth);
      __syncthreads();
      if (tid < P) fk_deriv_prep(sk, fsh, *reinterpret_cast<FkDeriv*>(fkb + ekf_fk_shared_doubles()), tid);
      for (int o = tid; o < CL; o += nth) {
        const int c = o / d.L, l = o - c * d.L;
        const double* x = fsh.pos[sk.outn[l]];
        ProjOut po;
        fisheye_project<true>(sCam + c * ACS_CAM_STRIDE, x[0], x[1], x[2], po);
        hp[2 * o] = po.u;
        hp[2 * o + 1] = po.v;
#pragma unroll
        for (int k = 0; k < 6; ++k) hp[m + 6 * o + k] = po.J[k];
      }
    } else if (sk.J == 1) {
      // one joint: the trig and translation tables of every Jacobian pose, then every (pose,
      // observation) item computes its marker from them and projects it
      double* sc = fkb;                      // 4 x FK_MAXP
      double* rw = sc + 4 * FK_MAXP;         // (P+1) x 6
      if (!trig_early) {
        ekf_fk_trig_trans<F32>(sk, ss, d.eps, sc, rw, tid, nth);
        __syncthreads();
      }
#ifdef EKF_PROFILE
      s_sub += clock64() - t_last;  // the trig / translation tables' share of the FK/proj phase
#endif
      for (int e = tid; e < (P + 1) * CL; e += nth) {
        const int q = e / CL, o = e - q * CL;
        const int c = o / d.L, l = o - c * d.L;
        double x[3];
        if (pl.ok)
          ekf_point_eval<F32>(pl, ss, d.eps, sc, rw, q, x);
        else
          ekf_fk_point<F32>(sk, ss, d.eps, sc, rw, q, l, x);
        ProjOut po;
        fisheye_project<false>(sCam + c * ACS_CAM_STRIDE, x[0], x[1], x[2], po);
        hp[(size_t)q * m + 2 * o] = po.u;
        hp[(size_t)q * m + 2 * o + 1] = po.v;
      }
    } else {
      ekf_fk_batch<F32>(sk, ss, d.eps, fkb, tid, nth);
      const double* pos = fkb + FK_MAXJ * 9 + (FK_MAXP + 1) * 9 + (size_t)(P + 1) * d.J * 9;
      for (int e = tid; e < (P + 1) * CL; e += nth) {
        const int q = e / CL, o = e - q * CL;
        const int c = o / d.L, l = o - c * d.L;
        const double* x = pos + ((size_t)q * d.L + l) * 3;
        ProjOut po;
        fisheye_project<false>(sCam + c * ACS_CAM_STRIDE, x[0], x[1], x[2], po);
        hp[(size_t)q * m + 2 * o] = po.u;
        hp[(size_t)q * m + 2 * o + 1] = po.v;
      }
    }
    __syncthreads();
    EKF_TICK1(2);
    for (int r = tid; r < m; r += nth) {
      const int o = r >> 1, c = o / d.L;
      double e = (pf ? m_cur : meas[fo * fstride * 2 + r]) - hp[r];
      if (!isfinite(e)) e = (e != e) ? 0.0 : (e > 0 ? 1.7976931348623157e308 : -1.7976931348623157e308);
      const double lk = pf ? l_cur : lik[fo * fstride + o];
      const bool mx = lk < d.thresh;
      sr[r] = e;
      if (pf) {
        sw[r] = mx ? w_mx : w_rb;
        sd2[r] = mx ? s2_mx : s2_rb;
      } else {
        const double sd = mx ? d.maxpix : rbase[c];
        sw[r] = 1.0 / (sd * sd);
        sd2[r] = sd * sd;
      }
    }
    // H rows (P entries in registers, stored together); analytic: both rows of an
    // observation from one d pos / d x_q
    if constexpr (AH) {
      const FkShared& fsh = *reinterpret_cast<const FkShared*>(fkb);
      const FkDeriv& fkd = *reinterpret_cast<const FkDeriv*>(fkb + ekf_fk_shared_doubles());
      for (int o = tid; o < CL; o += nth) {
        const double* jr = hp + m + 6 * (size_t)o;
        const int node = sk.outn[o % d.L];
#pragma unroll
        for (int q = 0; q < P; ++q) {
          double dp[3];
          fk_dpos_fast(sk, fsh, fkd, node, q, dp);
          sH[2 * o * P + q] = jr[0] * dp[0] + jr[1] * dp[1] + jr[2] * dp[2];
          sH[(2 * o + 1) * P + q] = jr[3] * dp[0] + jr[4] * dp[1] + jr[5] * dp[2];
        }
      }
    } else {
      for (int r = tid; r < m; r += nth) {
        double hr[P];
        const double h0 = hp[r];
#pragma unroll
        for (int q = 0; q < P; ++q) hr[q] = (hp[(size_t)(q + 1) * m + r] - h0) / d.eps;
#pragma unroll
        for (int q = 0; q < P; ++q) sH[r * P + q] = hr[q];
      }
    }
    __syncthreads();
    EKF_TICK1(3);
    // ---- 3. A = H^T R^-1 H, b = H^T R^-1 r (entry per lane), 3-sigma outliers ----------
    if (tid < 64) {  // wave 0
      const int t = tid & 31, part = tid >> 5, mh = (m + 1) >> 1;
      const int r0 = part ? mh : 0, r1 = part ? m : mh;
      double v = 0.0;
      if (t < nAb) {
        // rows 8 at a time, their loads issued before the FMAs (same summation order)
        const double* ca = sH + ea;
        const double* cb = eb >= 0 ? sH + eb : sr;
        const int sb = eb >= 0 ? P : 1;
        int r = r0;
        for (; r + 8 <= r1; r += 8) {
          double wa[8], bb[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            wa[u] = sw[r + u] * ca[(r + u) * P];
            bb[u] = cb[(r + u) * sb];
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) v = fma(wa[u], bb[u], v);
        }
        for (; r < r1; ++r) v = fma(sw[r] * ca[r * P], cb[r * sb], v);
      }
      v += __shfl_xor(v, 32);
      if (part == 0 && t < nAb) {
        if (eb >= 0) {
          sA[ea * P + eb] = v;
          sA[eb * P + ea] = v;
        } else {
          sA[P * P + ea] = v;
        }
      }
    }
    {
      // outliers: q_r = h_r P_xx h_r^T + sd_r^2 per row, an observation if either row fails;
      // P_xx (uniform) in registers
      double pxx[P][P];
#pragma unroll
      for (int a = 0; a < P; ++a)
#pragma unroll
        for (int b = 0; b < P; ++b) pxx[a][b] = sP[a * LDP + b];
      // the observations go to waves 1.. first (wave 0 forms A and b meanwhile)
      for (int o = NW > 1 ? (tid + nth - 64) % nth : tid; o < CL; o += nth) {
        bool out = false;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
          const int r = 2 * o + side;
          double h[P];
#pragma unroll
          for (int a = 0; a < P; ++a) h[a] = sH[r * P + a];
          double q = 0.0;
#pragma unroll
          for (int a = 0; a < P; ++a) {
            double tv = 0.0;
#pragma unroll
            for (int b = 0; b < P; ++b) tv = fma(pxx[a][b], h[b], tv);
            q = fma(h[a], tv, q);
          }
          // |r| > 3 sqrt(S_rr), S_rr = q + sd^2, compared squared (no sqrt, no division); a
          // negative S_rr (P_xx not positive definite) is no outlier, as the reference's
          // comparison with sqrt(S_rr) = NaN is false (src/core/ekf.py:272-275)
          const double Srr = q + sd2[r];
          out = out || (Srr >= 0.0 && sr[r] * sr[r] > 9.0 * Srr);
        }
        const unsigned long long bal = __ballot(out);
        if ((tid & 63) == 0) nout += __popcll(bal);
      }
    }
    for (int e = tid; e < n * P; e += nth) {
      const int r = e / P, c = e - r * P;
      sPx[e] = sP[r * LDP + c];
    }
    __syncthreads();
    EKF_TICK1(4);
    // ---- 4. [W | C], W = C + C A C (C = P_xx), column c on lane c of wave 0 ----------
    // (I + A C)^-1 = W^-1 C with W = C (I + A C) symmetric positive definite, so the solve
    // needs no pivot search: Gauss-Jordan on the diagonal, every pivot row known in advance
    double a[P];
    if (tid < 64) {
      const int c = tid;
      if (c < P) {
        double ac[P];  // (A C)[:, c]
#pragma unroll
        for (int r = 0; r < P; ++r) {
          double v = 0.0;
#pragma unroll
          for (int k = 0; k < P; ++k) v = fma(sA[r * P + k], sP[k * LDP + c], v);
          ac[r] = v;
        }
#pragma unroll
        for (int r = 0; r < P; ++r) {
          double v = sP[r * LDP + c];
#pragma unroll
          for (int k = 0; k < P; ++k) v = fma(sP[r * LDP + k], ac[k], v);
          a[r] = v;
        }
      } else {
        const int j = c < 2 * P ? c - P : 0;
#pragma unroll
        for (int r = 0; r < P; ++r) a[r] = c < 2 * P ? sP[r * LDP + j] : 0.0;
      }
    }
    // G = [A P[x, :] | b] into sZ, column c per thread: on wave 1 while wave 0 solves (one
    // wave: before its solve)
    auto g_column = [&](int c) {
#pragma unroll
      for (int r = 0; r < P; ++r) {
        double v = 0.0;
        if (c < n) {
#pragma unroll
          for (int k = 0; k < P; ++k) v = fma(sA[r * P + k], sP[k * LDP + c], v);
        } else {
          v = sA[P * P + r];
        }
        sZ[r * NZ1 + c] = v;
      }
    };
    if constexpr (NW > 1) {
      if (tid >= 64 && tid < 64 + n + 1) g_column(tid - 64);
    } else {
      if (tid < n + 1) g_column(tid);
    }
    EKF_TICK1(5);
    // ---- 5. Gauss-Jordan without pivot search, in wave 0's registers -----------------
    // step k: row k over its pivot, then a[r][k] times it off every other row (the
    // column-k entries by readlane); at the end the right-hand block is V = (I + A C)^-1.
    // Every pivot positive certifies W > 0 (Sylvester), where diagonal pivots are stable; a
    // P0 that is not positive definite makes W indefinite, and then V comes from a partially
    // pivoted Gauss-Jordan on [I + A C | I] in the same registers.
    if (tid < 64) {
      bool spd = true;  // uniform (the pivots come by readlane)
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const double p = read_lane_f64(a[k], k);
        spd = spd && p > 0.0;
        const double ip = rcp_nr(p);
        const double pr = tid > k ? a[k] * ip : a[k];
        a[k] = pr;
#pragma unroll
        for (int r = 0; r < P; ++r) {
          if (r == k) continue;
          const double nv = fma(-read_lane_f64(a[r], k), pr, a[r]);
          a[r] = tid > k ? nv : a[r];
        }
      }
      if (spd) {
        if (tid >= P && tid < 2 * P) {
#pragma unroll
          for (int k = 0; k < P; ++k) sV[k * P + tid - P] = a[k];
        }
      } else {
        ekf_w1_pivoted<P>(sA, sP, LDP, sV, tid, bad);
      }
    }
    __syncthreads();
    // [Z_G | Z_b] = V G, column c in place by thread c
    if (tid < n + 1) {
      const int c = tid;
      double g[P];
#pragma unroll
      for (int k = 0; k < P; ++k) g[k] = sZ[k * NZ1 + c];
#pragma unroll
      for (int r = 0; r < P; ++r) {
        double v = 0.0;
#pragma unroll
        for (int k = 0; k < P; ++k) v = fma(sV[r * P + k], g[k], v);
        sZ[r * NZ1 + c] = v;
      }
    }
    __syncthreads();
    EKF_TICK1(6);
    // ---- 6. s += P[:, x] Z_b ; P -= P[:, x] Z_G ---------------------------------------
    // (the outputs stored by the threads that form them: no store phase and no second barrier;
    // 8.35 -> 8.19 us per frame, profiles/r06/bench_ekf_*_r06s.log)
    if (tid < n) {
      double v = 0.0;
#pragma unroll
      for (int k = 0; k < P; ++k) v += sPx[tid * P + k] * sZ[k * NZ1 + n];
      const double x = ss[tid] + v;
      ss[tid] = x;
      xest[fo * n + tid] = x;
    }
    for (Walk2 w(tid, nth, n); w.e < n * n; w.next()) {
      double v = 0.0;
#pragma unroll
      for (int k = 0; k < P; ++k) v = fma(sPx[w.r * P + k], sZ[k * NZ1 + w.c], v);
      const double x = sP[w.r * LDP + w.c] - v;
      sP[w.r * LDP + w.c] = x;
      Pest[fo * n * n + w.e] = x;
    }
    __syncthreads();
    EKF_TICK1(7);
  }
#ifdef EKF_PROFILE
  if (tid == 0 && ekf_prof) {
    for (int k = 0; k < 8; ++k) ekf_prof[seq * 8 + k] = s_prof[k];
    if (seq == 0) ekf_prof[8] = s_sub;  // the profiling tool's ninth slot (one sequence)
  }
#endif
#undef EKF_TICK1
  if ((tid & 63) == 0 && nout) atomicAdd(reinterpret_cast<unsigned long long*>(&s_nout), (unsigned long long)nout);
  __syncthreads();
  if (tid == 0) outliers[seq] = s_nout;
}

// RTS smoother with the smoothed covariances (src/core/ekf.py:292-296), one workgroup per
// sequence walking back through the frames (k_ekf_gain + k_ekf_smooth_x when the
// covariances are not wanted).
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
    for (int e = tid; e < (keep_P ? (int)nn : 0); e += nth) {  // T = P_est F^T ; D = Ps[i+1] - Ppred[i+1]
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
    for (int r = tid; r < np_; r += nth)
      sv[r] = r < n ? xs[(base + i + 1) * n + r] - xpred[(base + i + 1) * n + r] : 0.0;
    __syncthreads();
    wg_mgemm<false, false>(A, np_, T, np_, sInv, LD, np_, np_, np_, 1.0, 0.0);  // A = T Pp^-1
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
    for (int e = tid; e < (int)nn0; e += nth) Ps[(base + i) * nn0 + e] = Pn[(size_t)(e / n) * np_ + e % n];
    __syncthreads();
  }
}

// RTS gains without the smoothed covariances (the reference never outputs them): the gain
// A_i = P_est[i] F^T P_pred[i+1]^-1 (src/core/ekf.py:294) does not depend on the smoothed
// states, so every (sequence, frame) pair is an independent workgroup here, and only the
// state recursion below is sequential. A_i overwrites P_pred[i+1] (read first, by this
// workgroup only). Product order as the reference: (P_est F^T) P_pred^-1, with P_est F^T
// formed on the fly as the MFMA A operand.
__global__ __launch_bounds__(256) void k_ekf_gain(EkfDims d, const double* __restrict__ Pest, double* Ppred,
                                                  int* __restrict__ bad) {
  const int N1 = d.N - 1;
  const int seq = blockIdx.x / N1, i = blockIdx.x - seq * N1;
  const int tid = threadIdx.x, nth = blockDim.x, lane = tid & 63, wave = tid >> 6;
  const int n = d.n, P = d.P, np_ = d.npad, LD = np_ + 1, nb = np_ >> 4;
  const double sT = d.sT, h2 = 0.5 * sT * sT;
  extern __shared__ double lds[];
  double* sInv = lds;                      // np x LD
  double* tmp = sInv + (size_t)np_ * LD;   // 512
  const size_t nn0 = (size_t)n * n, base = (size_t)seq * d.N;
  const double* Pe = Pest + (base + i) * nn0;
  double* Pp1 = Ppred + (base + i + 1) * nn0;
  for (int e = tid; e < np_ * LD; e += nth) {
    const int r = e / LD, c = e - r * LD;
    sInv[e] = (r < n && c < n) ? Pp1[r * n + c] : (r == c ? 1.0 : 0.0);
  }
  __syncthreads();
  wg_gj_inverse<false>(sInv, LD, nb, tmp, bad);
  const int li = lane & 15, lk = lane >> 4;
  for (int t = wave; t < nb * nb; t += nth >> 6) {
    const int i0 = (t / nb) << 4, j0 = (t % nb) << 4;
    const int r = i0 + li;
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < np_; k0 += 4) {
      const int k = k0 + lk;
      double a = 0.0;  // (P_est F^T)[r][k]
      if (r < n && k < n) {
        a = Pe[r * n + k];
        if (k < 2 * P) a += sT * Pe[r * n + k + P];
        if (k < P) a += h2 * Pe[r * n + k + 2 * P];
      }
      acc = mfma64(a, sInv[k * LD + j0 + li], acc);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rr = i0 + lk + 4 * q, cc = j0 + li;
      if (rr < n && cc < n) Pp1[rr * n + cc] = acc[q];
    }
  }
}

// k_ekf_gain_w's path for a P_pred that is not positive definite (not inlined: the kernel's
// common path keeps its registers)
template <int NN>
__device__ __noinline__ void ekf_gain_pivoted(const double* __restrict__ Pe, double* Pp1, int P, double sT, double h2,
                                              int lane, int* __restrict__ bad) {
  double a[NN];
  // P_pred is not positive definite (a P0 that is not, or rounding): Gauss-Jordan with partial
  // pivoting on the same columns, reloaded. Step k: the pivot column's lane picks the unused
  // row with the largest |a| (lowest on ties; the index is uniform, so it stays scalar), the
  // pivot row is normalised and column k eliminated from every other row; row pv_k ends as
  // row k of the solution.
  if (lane < NN) {
#pragma unroll
    for (int r = 0; r < NN; ++r) a[r] = Pp1[r * NN + lane];
  } else if (lane < 2 * NN) {
    const int c = lane - NN;
#pragma unroll
    for (int k = 0; k < NN; ++k) {
      double v = Pe[c * NN + k];
      if (k < 2 * P) v += sT * Pe[c * NN + k + P];
      if (k < P) v += h2 * Pe[c * NN + k + 2 * P];
      a[k] = v;
    }
  }
  // (a rare path: rolled loops, pv_k kept in lane k, so it adds few registers to the kernel)
  unsigned used = 0;
  int mypv = 0, nsing = 0;
#pragma unroll 1
  for (int k = 0; k < NN; ++k) {
    double best = -1.0;
    int bi = 0;
#pragma unroll
    for (int r = 0; r < NN; ++r) {
      const bool cand = !((used >> r) & 1u) && fabs(a[r]) > best;
      best = cand ? fabs(a[r]) : best;
      bi = cand ? r : bi;
    }
    const int pv = __builtin_amdgcn_readlane(bi, k);
    double prow = 0.0;
#pragma unroll
    for (int r = 0; r < NN; ++r) prow = r == pv ? a[r] : prow;
    const double pp = read_lane_f64(prow, k);
    nsing += pp == 0.0 ? 1 : 0;
    const double pn = lane > k ? prow * (1.0 / pp) : prow;
#pragma unroll
    for (int r = 0; r < NN; ++r) {
      const double nv = fma(-read_lane_f64(a[r], k), pn, a[r]);
      a[r] = lane > k ? (r == pv ? pn : nv) : a[r];
    }
    used |= 1u << pv;
    mypv = lane == k ? pv : mypv;
  }
  if (nsing && lane == 0) atomicAdd(bad, nsing);  // singular P_pred (counted, reported by the host)
#pragma unroll 1
  for (int k = 0; k < NN; ++k) {
    const int pv = __builtin_amdgcn_readlane(mypv, k);
    double v = 0.0;
#pragma unroll
    for (int r = 0; r < NN; ++r) v = r == pv ? a[r] : v;
    if (lane >= NN && lane < 2 * NN) Pp1[(lane - NN) * NN + k] = v;
  }
}

// The same gains for small states (n = NN <= 32, the head model), one wave per (sequence,
// frame), GW waves per workgroup. A_i^T = P_pred^-1 (P_est F^T)^T comes from a Gauss-Jordan
// on [P_pred | (P_est F^T)^T] with the pivots on the diagonal (no pivot search) when P_pred is
// positive definite (every pivot positive), else with partial pivoting: column c on lane c,
// rows in registers, the column-k entries by readlane. Lane NN + c ends with column c of
// A_i^T, i.e. row c of A_i.
template <int NN, int GW>
__global__ __launch_bounds__(64 * GW) void k_ekf_gain_w(EkfDims d, const double* __restrict__ Pest, double* Ppred,
                                                        int* __restrict__ bad) {
  static_assert(2 * NN <= 64, "one column per lane");
  const int N1 = d.N - 1, lane = threadIdx.x & 63;
  const long long g = (long long)blockIdx.x * GW + (threadIdx.x >> 6);
  if (g >= (long long)d.S * N1) return;  // whole wave
  const int seq = (int)(g / N1), i = (int)(g - (long long)seq * N1);
  const int P = d.P;
  const double sT = d.sT, h2 = 0.5 * sT * sT;
  constexpr size_t nn0 = (size_t)NN * NN;
  const size_t base = (size_t)seq * d.N;
  const double* Pe = Pest + (base + i) * nn0;
  double* Pp1 = Ppred + (base + i + 1) * nn0;
  double a[NN];
  if (lane < NN) {
#pragma unroll
    for (int r = 0; r < NN; ++r) a[r] = Pp1[r * NN + lane];
  } else if (lane < 2 * NN) {
    const int c = lane - NN;  // row c of P_est F^T, as column c of its transpose
#pragma unroll
    for (int k = 0; k < NN; ++k) {
      double v = Pe[c * NN + k];
      if (k < 2 * P) v += sT * Pe[c * NN + k + P];
      if (k < P) v += h2 * Pe[c * NN + k + 2 * P];
      a[k] = v;
    }
  } else {
#pragma unroll
    for (int r = 0; r < NN; ++r) a[r] = 0.0;
  }
  bool spd = true;  // every pivot positive certifies P_pred > 0 (uniform: pivots by readlane)
#pragma unroll
  for (int k = 0; k < NN; ++k) {
    const double p = read_lane_f64(a[k], k);
    spd = spd && p > 0.0;
    const double ip = rcp_nr(p);
    const double pr = lane > k ? a[k] * ip : a[k];
    a[k] = pr;
#pragma unroll
    for (int r = 0; r < NN; ++r) {
      if (r == k) continue;
      const double nv = fma(-read_lane_f64(a[r], k), pr, a[r]);
      a[r] = lane > k ? nv : a[r];
    }
  }
  if (spd) {
    if (lane >= NN && lane < 2 * NN) {  // P_pred[i+1] was read by this wave only: A_i in its place
      const int c = lane - NN;
#pragma unroll
      for (int k = 0; k < NN; ++k) Pp1[c * NN + k] = a[k];
    }
    return;
  }
  ekf_gain_pivoted<NN>(Pe, Pp1, P, sT, h2, lane, bad);
}

#define EKF_GAIN_W 4

// The gains of the larger states (n = 33..96: the default model's 87), one workgroup of NB
// waves per (sequence, frame), NB = n padded to 16 / 16: A_i = (P_est F^T) P_pred^-1 with the
// explicit inverse, as the reference (src/core/ekf.py:294; on these covariances, cond ~1e12,
// a solve instead of the inverse moves the smoothed states by 1e-5 relative, while any
// explicit inverse then product agrees with numpy's to 1e-9). k_ekf_gain's arithmetic (the
// blocked Gauss-Jordan of wg_gj_inverse, then the product in the same k order), so the same
// bits, organised for throughput:
//  * P_pred's 16 x 16 tiles in LDS (72 KB, two workgroups per CU; k_ekf_gain's padded copy
//    plus scratch held one), in a swizzled layout: element (r, c) of a tile at
//    r * 16 + (c ^ 4 ((r >> 1) & 3)), so every fragment read is 2-way, the minimum;
//  * wave I owns row block I. Step k: wave k inverts the diagonal tile in registers
//    (tile16_gj_inverse) and forms its row panel W A_kJ; after one barrier every other wave
//    updates its whole row, A_IJ -= A_Ik A_kJ, then A_Ik <- -A_Ik W (it is the only reader of
//    its A_Ik): two barriers per step instead of four;
//  * the product's A operand, row block I of P_est F^T, is loaded into registers at entry
//    (its loads in flight during the inverse); k_ekf_gain read it from global memory inside
//    the MFMA loop.
// Every scalar pivot positive certifies P_pred > 0 (Sylvester); otherwise the workgroup writes
// nothing and flags the gain for k_ekf_gain_piv (partial pivoting). k_ekf_gain took 9.6 ms for
// the bench's 64 x 499 gains of the default model.
__device__ __forceinline__ int gt_idx(int r, int c) { return r * 16 + (c ^ (((r >> 1) & 3) << 2)); }

#ifdef EKF_PROFILE
// k_ekf_gain_t per-workgroup phase times (wall clock, 100 MHz): load, Gauss-Jordan, product,
// count, first entry, last exit (tools/prof_ekf_gain.py)
__device__ unsigned long long g_gain_prof[8];
__device__ unsigned long long g_gain_trace[2 * 32768];  // per workgroup: entry, exit (last launch)
#define GAIN_TICK(slot, t_prev)                                                   \
  do {                                                                          \
    __syncthreads();                                                            \
    const unsigned long long t_now_ = wall_clock64();                           \
    if (threadIdx.x == 0) atomicAdd(&g_gain_prof[slot], t_now_ - t_prev);       \
    t_prev = t_now_;                                                            \
  } while (0)
#else
#define GAIN_TICK(slot, t_prev)
#endif

// __launch_bounds__(1024), not 64 NB GP: a 384-thread bound made workgroups of >= 54 KB of LDS
// run one per CU (tools/probe/lds_occ_probe.hip, profiles/r05/lds_occ_probe_c.log)
template <int NB, int GP>
__global__ __launch_bounds__(1024) void k_ekf_gain_t(EkfDims d, const double* __restrict__ Pest,
                                                             double* Ppred, int* __restrict__ flag, int ng) {
#ifdef EKF_PROFILE
  unsigned long long t_g = wall_clock64();
  if (threadIdx.x == 0) atomicMin(&g_gain_prof[4], t_g);
  if (threadIdx.x == 0 && blockIdx.x < 32768) g_gain_trace[2 * blockIdx.x] = t_g;
#endif
  // GP gains per workgroup, NB waves each (their own LDS matrices; the barriers are shared)
  __shared__ double sAll[GP * NB * NB * 256];
  __shared__ int s_bads[GP];
  const int sub = (int)threadIdx.x / (64 * NB);
  const int g = (int)blockIdx.x * GP + sub;
  const bool live = g < ng;  // a missing last gain's waves only keep the barriers
  double* sA = sAll + sub * NB * NB * 256;
  int& s_bad = s_bads[sub];
  const int N1 = d.N - 1;
  const int seq = (live ? g : 0) / N1, i = (live ? g : 0) - seq * N1;
  const int tid = (int)threadIdx.x - sub * 64 * NB, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lk = lane >> 4;
  const int n = d.n, P = d.P;
  const double sT = d.sT, h2 = 0.5 * sT * sT;
  const size_t nn0 = (size_t)n * n, base = (size_t)seq * d.N;
  const double* Pe = Pest + (base + i) * nn0;
  double* Pp1 = Ppred + (base + i + 1) * nn0;
  auto tile = [&](int I, int J) { return sA + (I * NB + J) * 256; };
  if (tid == 0) s_bad = 0;
  // P_pred (identity on the padding): every load in flight before the first LDS store (a
  // loop waiting for each round of loads made the kernel 5x slower)
  {
    constexpr int NL = NB * 4;  // NB * NB * 256 elements / (64 NB threads)
    double pv[NL];
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      const int e = tid + 64 * NB * q;
      const int t = e >> 8, r = (e >> 4) & 15, c = e & 15, I = t / NB, J = t - I * NB;
      const int R = 16 * I + r, C = 16 * J + c;
      pv[q] = (live && R < n && C < n) ? Pp1[(size_t)R * n + C] : (R == C ? 1.0 : 0.0);
    }
#pragma unroll
    for (int q = 0; q < NL; ++q) {
      const int e = tid + 64 * NB * q;
      sA[(e >> 8) * 256 + gt_idx((e >> 4) & 15, e & 15)] = pv[q];
    }
  }
  __syncthreads();
  GAIN_TICK(0, t_g);
  int nbad = 0;
  auto inv_tile = [&](double* T, double* v) {  // the pivot tile, inverted in registers
    tile16_gj_steps<true>(v, lane, nbad, std::make_integer_sequence<int, 16>{});
#pragma unroll
    for (int q = 0; q < 4; ++q) T[gt_idx(lk + 4 * q, li)] = v[q];
  };
  if (wave == 0) {
    double v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = sA[gt_idx(lk + 4 * q, li)];
    inv_tile(sA, v);
  }
  __syncthreads();
#pragma unroll 1
  for (int k = 0; k < NB; ++k) {
    double* W = tile(k, k);
    // row panel A_kJ <- W_k A_kJ, tile J by wave J (J != k)
    if (wave != k) {
      double* AkJ = tile(k, wave);
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = mfma64(W[gt_idx(li, 4 * q + lk)], AkJ[gt_idx(4 * q + lk, li)], acc);
#pragma unroll
      for (int q = 0; q < 4; ++q) AkJ[gt_idx(lk + 4 * q, li)] = acc[q];
    }
    __syncthreads();
    if (wave != k) {
      // row block I = wave: A_IJ -= A_Ik A_kJ (J != k), then A_Ik <- -A_Ik W_k. Wave k + 1
      // updates its diagonal tile first and inverts it at once: the next step's pivot
      double* AIk = tile(wave, k);
      double aik[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) aik[q] = AIk[gt_idx(li, 4 * q + lk)];
      const int J0 = wave == k + 1 ? wave : 0;
#pragma unroll 1
      for (int jj = 0; jj < NB; ++jj) {
        const int J = jj == 0 ? J0 : (jj <= J0 ? jj - 1 : jj);  // J0 first, then the others in order
        if (J == k) continue;
        double* AIJ = tile(wave, J);
        const double* AkJ = tile(k, J);
        dbl4 acc;
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = AIJ[gt_idx(lk + 4 * q, li)];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc = mfma64(-aik[q], AkJ[gt_idx(4 * q + lk, li)], acc);
        if (J == k + 1 && wave == k + 1) {
          double v[4] = {acc[0], acc[1], acc[2], acc[3]};
          inv_tile(AIJ, v);
        } else {
#pragma unroll
          for (int q = 0; q < 4; ++q) AIJ[gt_idx(lk + 4 * q, li)] = acc[q];
        }
      }
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = mfma64(-aik[q], W[gt_idx(4 * q + lk, li)], acc);
#pragma unroll
      for (int q = 0; q < 4; ++q) AIk[gt_idx(lk + 4 * q, li)] = acc[q];
    }
    __syncthreads();
  }
  // A operand of the product, row block `wave` of P_est F^T: ba[K][s] = (P_est F^T)[r][16K + 4s + lk],
  // loaded after the inverse: held through it, its 48 VGPRs made the kernel 129 VGPRs, 3 waves
  // per SIMD, and the two workgroups per CU the LDS allows never shared one (253 in flight)
  double ba[NB][4];
  {
    const int r = 16 * wave + li;
    const double* pr = Pe + (size_t)(r < n ? r : 0) * n;
#pragma unroll
    for (int K = 0; K < NB; ++K)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = 16 * K + 4 * q + lk;
        double a = 0.0;
        if (live && r < n && k < n) {
          a = pr[k];
          if (k < 2 * P) a += sT * pr[k + P];
          if (k < P) a += h2 * pr[k + 2 * P];
        }
        ba[K][q] = a;
      }
  }
  if (nbad && lane == 0) s_bad = 1;
  __syncthreads();
  GAIN_TICK(1, t_g);
  if (!live) return;
  if (s_bad) {  // not positive definite: P_pred left as it is, k_ekf_gain_piv takes the gain
    if (tid == 0) flag[g] = 1;
    return;
  }
  if (tid == 0) flag[g] = 0;
  // A_i row block `wave` = (P_est F^T) P_pred^-1, k in order (k_ekf_gain's sums); P_pred[i+1]
  // was read by this workgroup only
#pragma unroll 1
  for (int J = 0; J < NB; ++J) {
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int K = 0; K < NB; ++K) {
      const double* X = tile(K, J);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc = mfma64(ba[K][q], X[gt_idx(4 * q + lk, li)], acc);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int rr = 16 * wave + lk + 4 * q, cc = 16 * J + li;
      if (rr < n && cc < n) Pp1[(size_t)rr * n + cc] = acc[q];
    }
  }
#ifdef EKF_PROFILE
  GAIN_TICK(2, t_g);
  if (threadIdx.x == 0) {
    atomicAdd(&g_gain_prof[3], 1ull);
    const unsigned long long t_e = wall_clock64();
    atomicMax(&g_gain_prof[5], t_e);
    if (blockIdx.x < 32768) g_gain_trace[2 * blockIdx.x + 1] = t_e;
  }
#endif
}

// The gains k_ekf_gain_t flagged (P_pred not positive definite): the inverse by Gauss-Jordan
// with partial pivoting on [P_pred | I] in LDS (the reference inverts by LAPACK's pivoted LU,
// src/core/ekf.py:294), then (P_est F^T) P_pred^-1. Step k: wave 0 picks the unused row with
// the largest |a_rk| (lowest on ties), the pivot row is normalised and column k eliminated
// from every other row; row pv_k of the right half ends as row k of the inverse. A rare path
// (an indefinite P_pred), one workgroup per gain, every other workgroup returns at once.
__global__ __launch_bounds__(256) void k_ekf_gain_piv(EkfDims d, const double* __restrict__ Pest, double* Ppred,
                                                      const int* __restrict__ flag, int* __restrict__ bad) {
  if (!flag[blockIdx.x]) return;
  const int N1 = d.N - 1;
  const int seq = blockIdx.x / N1, i = blockIdx.x - seq * N1;
  const int tid = threadIdx.x, nth = blockDim.x, n = d.n, P = d.P, LDM = 2 * n + 1;
  const double sT = d.sT, h2 = 0.5 * sT * sT;
  const size_t nn0 = (size_t)n * n, base = (size_t)seq * d.N;
  const double* Pe = Pest + (base + i) * nn0;
  double* Pp1 = Ppred + (base + i + 1) * nn0;
  extern __shared__ double lds[];
  double* M = lds;                         // n x LDM
  double* fcol = M + (size_t)n * LDM;      // n: column k before the step
  int* s_pv = (int*)(fcol + n);            // n: pivot row of step k
  __shared__ unsigned long long s_used[2];
  __shared__ int s_sing, s_skip[2];
  for (int e = tid; e < n * 2 * n; e += nth) {
    const int r = e / (2 * n), c = e - r * 2 * n;
    M[(size_t)r * LDM + c] = c < n ? Pp1[(size_t)r * n + c] : (c - n == r ? 1.0 : 0.0);
  }
  if (tid == 0) {
    s_used[0] = s_used[1] = 0ull;
    s_sing = 0;
  }
  __syncthreads();
  for (int k = 0; k < n; ++k) {
    if (tid < 64) {
      double best = -1.0;
      int bi = n;
      for (int r = tid; r < n; r += 64) {
        const bool used = (s_used[r >> 6] >> (r & 63)) & 1ull;
        const double a = fabs(M[(size_t)r * LDM + k]);
        if (!used && a > best) {
          best = a;
          bi = r;
        }
      }
#pragma unroll
      for (int h = 32; h > 0; h >>= 1) {
        const double ob = __shfl_xor(best, h, 64);
        const int oi = __shfl_xor(bi, h, 64);
        if (ob > best || (ob == best && oi < bi)) {
          best = ob;
          bi = oi;
        }
      }
      if (tid == 0) {
        // no usable pivot (every unused entry of column k zero or NaN): take the first unused
        // row so that the pivot stays inside the matrix, count the step as singular and skip its
        // elimination (the host raises the error; the gain's values are then meaningless)
        const bool sing = !(best > 0.0);
        if (bi >= n) {
          bi = 0;
          while (bi < n - 1 && ((s_used[bi >> 6] >> (bi & 63)) & 1ull)) ++bi;
        }
        s_pv[k] = bi;
        s_used[bi >> 6] |= 1ull << (bi & 63);
        s_skip[k & 1] = sing ? 1 : 0;
        if (sing) s_sing += 1;
      }
    }
    __syncthreads();
    if (s_skip[k & 1]) continue;  // uniform; double-buffered against step k + 1's write
    const int pv = s_pv[k];
    const double p = M[(size_t)pv * LDM + k];
    const double ip = p != 0.0 ? 1.0 / p : 0.0;
    for (int r = tid; r < n; r += nth) fcol[r] = M[(size_t)r * LDM + k];
    __syncthreads();
    for (int c = tid; c < 2 * n; c += nth) M[(size_t)pv * LDM + c] *= ip;
    __syncthreads();
    for (int e = tid; e < n * 2 * n; e += nth) {
      const int r = e / (2 * n), c = e - r * 2 * n;
      if (r != pv) M[(size_t)r * LDM + c] = fma(-fcol[r], M[(size_t)pv * LDM + c], M[(size_t)r * LDM + c]);
    }
    __syncthreads();
  }
  if (tid == 0 && s_sing) atomicAdd(bad, s_sing);
  // A_i[r][c] = sum_k (P_est F^T)[r][k] inv[k][c], inv[k] = row pv_k of the right half
  for (int e = tid; e < n * n; e += nth) {
    const int r = e / n, c = e - r * n;
    const double* pr = Pe + (size_t)r * n;
    double v = 0.0;
    for (int k = 0; k < n; ++k) {
      double a = pr[k];
      if (k < 2 * P) a += sT * pr[k + P];
      if (k < P) a += h2 * pr[k + 2 * P];
      v = fma(a, M[(size_t)s_pv[k] * LDM + n + c], v);
    }
    Pp1[(size_t)r * n + c] = v;
  }
}

// Smoothed states x_s[i] = x_est[i] + A_i (x_s[i+1] - x_pred[i+1]) (src/core/ekf.py:295), one
// workgroup per sequence: a row per aligned group of 8 lanes (3 passes cover n <= 96), the
// gain of the next frame loaded while this frame's products are summed.
#define EKF_SX_NQ 12
__global__ __launch_bounds__(256) void k_ekf_smooth_x(EkfDims d, const double* __restrict__ xpred,
                                                      const double* __restrict__ xest, const double* __restrict__ Ag,
                                                      double* __restrict__ xs) {
  const int seq = blockIdx.x, tid = threadIdx.x;
  const int n = d.n;
  const size_t nn0 = (size_t)n * n, base = (size_t)seq * d.N;
  __shared__ double sv[2][96];
  const int j = tid & 7, g = tid >> 3;  // 32 groups of 8 lanes
  for (int r = tid; r < n; r += blockDim.x) {
    const double v = xest[(base + d.N - 1) * n + r];
    xs[(base + d.N - 1) * n + r] = v;
    sv[(d.N - 1) & 1][r] = v - xpred[(base + d.N - 1) * n + r];
  }
  double a[3][EKF_SX_NQ], xe[3], xp[3];
  auto load = [&](int i) {  // A_i = the gain stored in P_pred[i+1]'s slot; x_est[i], x_pred[i]
    const double* A = Ag + (base + i + 1) * nn0;
#pragma unroll
    for (int ps = 0; ps < 3; ++ps) {
      const int r = ps * 32 + g;
#pragma unroll
      for (int q = 0; q < EKF_SX_NQ; ++q) {
        const int c = j + 8 * q;
        a[ps][q] = (r < n && c < n) ? A[r * n + c] : 0.0;
      }
      xe[ps] = (j == 0 && r < n) ? xest[(base + i) * n + r] : 0.0;
      xp[ps] = (j == 0 && r < n) ? xpred[(base + i) * n + r] : 0.0;
    }
  };
  if (d.N >= 2) load(d.N - 2);
  for (int i = d.N - 2; i >= 0; --i) {
    __syncthreads();
    const double* v = sv[(i + 1) & 1];
    double acc[3], xe_i[3], xp_i[3];
#pragma unroll
    for (int ps = 0; ps < 3; ++ps) {
      xe_i[ps] = xe[ps];
      xp_i[ps] = xp[ps];
      double s = 0.0;
#pragma unroll
      for (int q = 0; q < EKF_SX_NQ; ++q) {
        const int c = j + 8 * q;
        if (c < n) s = fma(a[ps][q], v[c], s);
      }
      acc[ps] = s;
    }
    if (i > 0) load(i - 1);
#pragma unroll
    for (int ps = 0; ps < 3; ++ps) {
      const double s = group_sum<8>(acc[ps]);
      const int r = ps * 32 + g;
      if (j == 0 && r < n) {
        const double x = xe_i[ps] + s;
        xs[(base + i) * n + r] = x;
        sv[i & 1][r] = x - xp_i[ps];
      }
    }
  }
}

// The same recursion for the models' state sizes (n = NN: 18, 87): a row per group of 8 lanes,
// QN = ceil(NN / 8) columns per lane, and the gains of the next D frames already in registers
// (a ring of D register sets, the frame loop unrolled by D so every index is static). A step
// is then one LDS read, QN FMAs, a 3-step DPP sum and a barrier; the gain loads of frame i
// are issued D steps before they are used, which hides their latency (one frame ahead
// left ~1.7 us of it per frame, profiles/r04).
template <int NN, int D>
__global__ __launch_bounds__(((8 * NN + 63) / 64) * 64) void k_ekf_smooth_xs(EkfDims d, const double* __restrict__ xpred,
                                                                             const double* __restrict__ xest,
                                                                             const double* __restrict__ Ag,
                                                                             double* __restrict__ xs) {
  constexpr int QN = (NN + 7) / 8;
  constexpr size_t nn0 = (size_t)NN * NN;
  const int seq = blockIdx.x, tid = threadIdx.x;
  const size_t base = (size_t)seq * d.N;
  __shared__ double sv[2][NN];
  const int j = tid & 7, r = tid >> 3;
  const bool live = r < NN;
  if (tid < NN) {
    const double v = xest[(base + d.N - 1) * NN + tid];
    xs[(base + d.N - 1) * NN + tid] = v;
    sv[(d.N - 1) & 1][tid] = v - xpred[(base + d.N - 1) * NN + tid];
  }
  double a[D][QN], xe[D], xp[D];
  auto load = [&](int u, int i) {  // slot u <- A_i (in P_pred[i+1]'s slot), x_est[i], x_pred[i]
    const double* A = Ag + (base + i + 1) * nn0;
#pragma unroll
    for (int q = 0; q < QN; ++q) {
      const int c = j + 8 * q;
      a[u][q] = (live && c < NN && i >= 0) ? A[r * NN + c] : 0.0;
    }
    xe[u] = (live && j == 0 && i >= 0) ? xest[(base + i) * NN + r] : 0.0;
    xp[u] = (live && j == 0 && i >= 0) ? xpred[(base + i) * NN + r] : 0.0;
  };
#pragma unroll
  for (int u = 0; u < D; ++u) load(u, d.N - 2 - u);
  for (int i0 = d.N - 2; i0 >= 0; i0 -= D) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      const int i = i0 - u;
      if (i < 0) break;  // uniform
      __syncthreads();
      const double* v = sv[(i + 1) & 1];
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < QN; ++q) {
        const int c = j + 8 * q;
        if (c < NN) acc = fma(a[u][q], v[c], acc);
      }
      const double xe_i = xe[u], xp_i = xp[u];
      load(u, i - D);
      acc = group_sum<8>(acc);
      if (live && j == 0) {
        const double x = xe_i + acc;
        xs[(base + i) * NN + r] = x;
        sv[i & 1][r] = x - xp_i;
      }
    }
  }
}
#define EKF_SX_D 8
// deep register ring for small states, 2 frames ahead for the 29-parameter model (11
// waves: the VGPR budget of 3 waves per SIMD)
#define EKF_SMOOTH_XS(NN_, D_)                                                                                  \
  hipLaunchKernelGGL((k_ekf_smooth_xs<NN_, D_>), dim3(n_seq), dim3(((8 * NN_ + 63) / 64) * 64), 0, s, d,      \
                     (const double*)dxp, (const double*)dxe, (const double*)dPp, dxs)

unsigned long long* g_ekf_prof = nullptr;

// Filter + smoother on device buffers (common.hpp). hdr = the skeleton table header. x_pred
// may be null (workspace then), P_est null = workspace, P_smooth null = no covariance
// smoother (gains in parallel, then the state recursion). Sets io.outliers (device,
// n_seq long longs) and io.x_pred / io.P_est to the buffers used.
int acs_ekf_enqueue(acs_ctx* ctx, int n_ints, int n_reals, const int* hdr, int n_cams, int n_seq, int n_frames,
                    double fps, double thresh, double max_pixel_err, double eps, int ref_numerics, EkfIo& io) {
  const int Jn = hdr[0], K = hdr[1], P = hdr[2], L = hdr[3];
  ACS_CHECK(ctx, Jn > 0 && Jn <= FK_MAXJ && K <= FK_MAXN && P >= 3 && P <= FK_MAXP && L >= 1 && L <= K,
            "ekf: skeleton table out of range");
  ACS_CHECK(ctx, n_ints == FK_HDR + 9 * Jn + 4 * K + L + 4 * P + K * P && n_reals == 3 * K, "ekf: blob sizes");
  ACS_CHECK(ctx, n_seq >= 1 && n_frames >= 1 && n_cams >= 1 && n_cams <= 64 && fps > 0 && eps > 0,
            "ekf: n_seq=%d n_frames=%d n_cams=%d", n_seq, n_frames, n_cams);
  EkfDims d;
  d.N = n_frames;
  d.C = n_cams;
  d.L = L;
  d.P = P;
  d.J = Jn;
  d.n = 3 * P;
  d.npad = ((d.n + 15) / 16) * 16;
  d.Ppad = ((P + 15) / 16) * 16;
  d.m = 2 * n_cams * L;
  d.mpad = ((d.m + 15) / 16) * 16;
  d.n_ints = n_ints;
  d.n_reals = n_reals;
  d.S = n_seq;
  d.sT = 1.0 / fps;
  d.thresh = thresh;
  d.maxpix = max_pixel_err;
  d.eps = eps;
  const int n = d.n;
  const size_t NF = (size_t)n_seq * n_frames;
  hipStream_t s = ctx->stream;
  if (!io.x_pred) io.x_pred = (double*)acs_ws(ctx, WS_FTE10, sizeof(double) * NF * n);
  // covariance histories: always needed by the smoother; the caller's buffer when given
  if (!io.P_est) io.P_est = (double*)acs_ws(ctx, WS_FTE13, sizeof(double) * NF * n * n);
  double* dPp = (double*)acs_ws(ctx, WS_FTE14, sizeof(double) * NF * n * n);
  const size_t scr_f = (size_t)n_seq * ((size_t)(P + 1) * d.m + 2 * (size_t)d.mpad * d.Ppad + 2 * d.mpad);
  const size_t scr_s = (size_t)n_seq * 5 * d.npad * d.npad;
  // tail: outlier counts (n_seq), the singular-solve counter, then k_ekf_gain_t's per-gain flags
  double* scr = (double*)acs_ws(ctx, WS_FTE6, sizeof(double) * std::max(scr_f, scr_s) + 64 * (size_t)n_seq * 8 +
                                                  sizeof(int) * (size_t)n_seq * n_frames + 64);
  if (!io.x_pred || !io.P_est || !dPp || !scr) return ACS_E_NOMEM;
  double *dxp = io.x_pred, *dxe = io.x_est, *dxs = io.x_smooth, *dPe = io.P_est, *dPs = io.P_smooth;
  long long* dout = (long long*)(scr + std::max(scr_f, scr_s));
  io.outliers = dout;
  // the singular-solve counter lives in its own context allocation (acs_ekf_singular_count
  // reads it after a device-pointer call); the scratch word after the outlier counts stays
  // reserved so the per-gain flags keep their place
  if (!ctx->ekf_bad) {
    void* p = nullptr;
    ACS_HIP(ctx, acs_dev_malloc(&p, 256));
    ctx->ekf_bad = (int*)p;
  }
  int* dbad = ctx->ekf_bad;
  io.bad = dbad;
  ACS_HIP(ctx, hipMemsetAsync(dbad, 0, sizeof(int), s));
  const size_t U = std::max(ekf_wg_fk_doubles(P, Jn, L, d.Ppad), ekf_wg_la_doubles(d.npad, d.Ppad));
  const size_t lds_f = sizeof(double) * ((size_t)d.npad * (d.npad + 1) + U + d.npad +
                                          (size_t)n_cams * ACS_CAM_STRIDE + n_reals + (n_ints + 1) / 2 + 1);
  const size_t lds_w1 = sizeof(double) * ekf_w1_lds(d);
  // ACS_EKF_WG=1 keeps the 8-wave kernel for every model (A/B measurements, tools/ekf_drift.py)
  static const bool force_wg = [] {
    const char* e = std::getenv("ACS_EKF_WG");
    return e && e[0] == '1';
  }();
  const bool w1 = P == EKF_W1_P && lds_w1 <= 64 * 1024 && !force_wg;
  // ACS_EKF_W1_WAVES: waves per sequence of the small-state filter (4 by default; 1 for A/B)
  static const int w1_waves = [] {
    const char* e = std::getenv("ACS_EKF_W1_WAVES");
    return e && e[0] == '1' ? 1 : 4;
  }();
  ACS_CHECK(ctx, w1 || lds_f <= 160 * 1024, "ekf: P = %d needs %zu bytes of LDS", P, lds_f);
  ACS_CHECK(ctx, ref_numerics >= 0 && ref_numerics <= ACS_EKF_ANALYTIC_H, "ekf: numerics mode %d", ref_numerics);
  // analytic H: the FkShared of one FK lives in the batched-FK region of the LDS union
  // small states (the head model): k_ekf_filter_w1
#define EKF_W1_NW(f32, ah, nw)                                                                                     \
  hipLaunchKernelGGL((k_ekf_filter_w1<f32, ah, EKF_W1_P, nw>), dim3(n_seq), dim3(64 * nw), lds_w1, s, d, io.I, \
                     io.R, io.cams, io.meas, io.lik, io.rstd, io.Q, io.P0, io.s0, dxp, dxe, dPp, dPe, dout, dbad,         \
                     g_ekf_prof)
#define EKF_W1(f32, ah)          \
  if (w1_waves == 4)             \
    EKF_W1_NW(f32, ah, 4);       \
  else                           \
    EKF_W1_NW(f32, ah, 1)
#define EKF_FILTER(f32, ah)                                                                                         \
  if (w1)                                                                                                           \
    EKF_W1(f32, ah);                                                                                                \
  else                                                                                                              \
    hipLaunchKernelGGL((k_ekf_filter<f32, ah>), dim3(n_seq), dim3(512), lds_f, s, d, io.I, io.R, io.cams, io.meas, \
                       io.lik, io.rstd, io.Q, io.P0, io.s0, dxp, dxe, dPp, dPe, scr, dout, dbad, g_ekf_prof)
  if (ref_numerics == ACS_EKF_ANALYTIC_H)
    EKF_FILTER(false, true);
  else if (ref_numerics)
    EKF_FILTER(true, false);
  else
    EKF_FILTER(false, false);
#undef EKF_FILTER
  ACS_HIP(ctx, hipGetLastError());
  const size_t lds_s = sizeof(double) * ((size_t)d.npad * (d.npad + 1) + 512 + d.npad);
  if (dPs) {
    hipLaunchKernelGGL(k_ekf_smooth, dim3(n_seq), dim3(256), lds_s, s, d, dxp, dxe, dPp, dPe, dxs, dPs, scr, dbad, 1);
  } else {
    // gains in parallel over (sequence, frame), then the state recursion per sequence
    ACS_CHECK(ctx, d.npad <= 96, "ekf: n = %d", d.n);
    if (n_frames >= 2 && n == 3 * EKF_W1_P) {  // small states: one wave per gain
      const size_t ng = (size_t)n_seq * (n_frames - 1);
      hipLaunchKernelGGL((k_ekf_gain_w<3 * EKF_W1_P, EKF_GAIN_W>), dim3((unsigned)((ng + EKF_GAIN_W - 1) / EKF_GAIN_W)),
                         dim3(64 * EKF_GAIN_W), 0, s, d, (const double*)dPe, dPp, dbad);
    } else if (n_frames >= 2 && d.npad >= 48) {
      // tiled gains, then the pivoted path for any P_pred that is not positive definite
      const unsigned ng = (unsigned)((size_t)n_seq * (n_frames - 1));
      int* dflag = (int*)(scr + std::max(scr_f, scr_s)) + 16 * (size_t)n_seq + 16;
  // two gains per workgroup: one 144 KB workgroup per CU (a workgroup of >= 54 KB of LDS never
  // shares a CU, tools/probe/lds_occ_probe.hip: the 72 KB one-gain form ran one gain per CU)
  // one gain per workgroup, two workgroups per CU: 4.09 ms for the bench's 64 x 499 gains;
  // two gains per 768-thread workgroup (lockstep barriers) 4.31 ms (ACS_EKF_GAIN_GP=2, A/B)
  static const int gp = [] {
    const char* e = std::getenv("ACS_EKF_GAIN_GP");
    return e && std::atoi(e) == 2 ? 2 : 1;
  }();
#define EKF_GAIN_T(NB)                                                                                          \
  if (gp == 1)                                                                                                  \
    hipLaunchKernelGGL((k_ekf_gain_t<NB, 1>), dim3(ng), dim3(64 * NB), 0, s, d, (const double*)dPe, dPp, dflag, \
                       (int)ng);                                                                                \
  else                                                                                                          \
    hipLaunchKernelGGL((k_ekf_gain_t<NB, 2>), dim3((ng + 1) / 2), dim3(128 * NB), 0, s, d, (const double*)dPe,  \
                       dPp, dflag, (int)ng)
      switch (d.npad >> 4) {
        case 3: EKF_GAIN_T(3); break;
        case 4: EKF_GAIN_T(4); break;
        case 5: EKF_GAIN_T(5); break;
        default: EKF_GAIN_T(6); break;
      }
#undef EKF_GAIN_T
      const size_t lds_p = sizeof(double) * ((size_t)n * (2 * n + 1) + n) + sizeof(int) * n;
      hipLaunchKernelGGL(k_ekf_gain_piv, dim3(ng), dim3(256), lds_p, s, d, (const double*)dPe, dPp,
                         (const int*)dflag, dbad);
      ACS_HIP(ctx, hipGetLastError());
    } else if (n_frames >= 2) {
      const size_t lds_g = sizeof(double) * ((size_t)d.npad * (d.npad + 1) + 512);
      hipLaunchKernelGGL(k_ekf_gain, dim3((unsigned)((size_t)n_seq * (n_frames - 1))), dim3(256), lds_g, s, d,
                         (const double*)dPe, dPp, dbad);
      ACS_HIP(ctx, hipGetLastError());
    }
    if (n == 3 * EKF_W1_P)
      EKF_SMOOTH_XS(3 * EKF_W1_P, EKF_SX_D);
    else if (n == 87)  // default
      EKF_SMOOTH_XS(87, 2);
    else
      hipLaunchKernelGGL(k_ekf_smooth_x, dim3(n_seq), dim3(256), 0, s, d, (const double*)dxp, (const double*)dxe,
                         (const double*)dPp, dxs);
  }
  ACS_HIP(ctx, hipGetLastError());
  return ACS_OK;
}

extern "C" {
void acs_ekf_prof(unsigned long long* p) { g_ekf_prof = p; }
#ifdef EKF_PROFILE
void acs_ekf_gain_prof(unsigned long long* out, int reset) {
  if (reset) {
    unsigned long long z[8] = {0, 0, 0, 0, ~0ull, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_gain_prof), z, sizeof(z));
  } else {
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gain_prof), sizeof(g_gain_prof));
  }
}
void acs_ekf_gain_trace(unsigned long long* out) {
  (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gain_trace), sizeof(g_gain_trace));
}
#endif

int acs_ekf_run(acs_ctx* ctx, const int32_t* skel_ints, int64_t n_ints, const double* skel_reals, int64_t n_reals,
                const double* cams, int32_t n_cams, const double* meas, const double* likelihood, int32_t n_seq,
                int32_t n_frames, double fps, double thresh, double max_pixel_err, const double* r_std_base,
                const double* Q, const double* P0, const double* s0, int32_t ref_numerics, double eps,
                double* x_pred, double* x_est, double* x_smooth, double* P_est, double* P_smooth,
                int64_t* outliers, uint32_t flags) {
  ACS_DEVICE_GUARD(ctx);
  int hdr[FK_HDR];
  if (flags & ACS_DEVICE_PTRS)
    ACS_HIP(ctx, hipMemcpy(hdr, skel_ints, sizeof(hdr), hipMemcpyDeviceToHost));
  else
    std::memcpy(hdr, skel_ints, sizeof(hdr));
  ACS_CHECK(ctx, x_est && x_smooth, "ekf: x_est and x_smooth are required");
  const int P = hdr[2], L = hdr[3], n = 3 * P;
  ACS_CHECK(ctx, P >= 3 && P <= FK_MAXP && L >= 1 && n_seq >= 1 && n_frames >= 1 && n_cams >= 1 && n_cams <= 64,
            "ekf: P=%d L=%d n_seq=%d n_frames=%d n_cams=%d", P, L, n_seq, n_frames, n_cams);
  const size_t NF = (size_t)n_seq * n_frames;
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
  EkfIo io;
  io.I = (const int*)dI;
  io.R = (const double*)dR;
  io.cams = (const double*)dC;
  io.meas = (const double*)dM;
  io.lik = (const double*)dL;
  io.rstd = (const double*)dRb;
  io.Q = (const double*)dQ;
  io.P0 = (const double*)dP0;
  io.s0 = (const double*)dS0;
  io.x_pred = x_pred ? (double*)acs_out_buf(ctx, WS_FTE10, x_pred, sizeof(double) * NF * n, flags) : nullptr;
  io.x_est = (double*)acs_out_buf(ctx, WS_FTE11, x_est, sizeof(double) * NF * n, flags);
  io.x_smooth = (double*)acs_out_buf(ctx, WS_FTE12, x_smooth, sizeof(double) * NF * n, flags);
  io.P_est = (flags & ACS_DEVICE_PTRS) ? P_est : nullptr;
  io.P_smooth = P_smooth ? ((flags & ACS_DEVICE_PTRS) ? P_smooth
                                                      : (double*)acs_ws(ctx, WS_FTE15, sizeof(double) * NF * n * n))
                         : nullptr;
  if ((x_pred && !io.x_pred) || !io.x_est || !io.x_smooth || (P_smooth && !io.P_smooth)) return ACS_E_NOMEM;
  if ((rc = acs_ekf_enqueue(ctx, (int)n_ints, (int)n_reals, hdr, n_cams, n_seq, n_frames, fps, thresh, max_pixel_err,
                            eps, ref_numerics, io)))
    return rc;
  hipStream_t s = ctx->stream;
  if (x_pred && (rc = acs_stage_out(ctx, x_pred, io.x_pred, sizeof(double) * NF * n, flags))) return rc;
  if ((rc = acs_stage_out(ctx, x_est, io.x_est, sizeof(double) * NF * n, flags))) return rc;
  if ((rc = acs_stage_out(ctx, x_smooth, io.x_smooth, sizeof(double) * NF * n, flags))) return rc;
  if (P_est && !(flags & ACS_DEVICE_PTRS) &&
      (rc = acs_stage_out(ctx, P_est, io.P_est, sizeof(double) * NF * n * n, flags)))
    return rc;
  if (P_smooth && !(flags & ACS_DEVICE_PTRS) &&
      (rc = acs_stage_out(ctx, P_smooth, io.P_smooth, sizeof(double) * NF * n * n, flags)))
    return rc;
  if (outliers || !(flags & ACS_DEVICE_PTRS)) {
    // a call that synchronises anyway also reports singular solves (numpy's inv raises on
    // them, src/core/ekf.py:267,294); a device-pointer call without outliers stays asynchronous
    std::vector<long long> ho(n_seq);
    int hbad = 0;
    if (outliers)
      ACS_HIP(ctx, hipMemcpyAsync(ho.data(), io.outliers, sizeof(long long) * n_seq, hipMemcpyDeviceToHost, s));
    ACS_HIP(ctx, hipMemcpyAsync(&hbad, io.bad, sizeof(int), hipMemcpyDeviceToHost, s));
    ACS_HIP(ctx, hipStreamSynchronize(s));
    if (outliers)
      for (int q = 0; q < n_seq; ++q) outliers[q] = ho[q];
    ACS_CHECK(ctx, hbad == 0, "ekf: %d singular solve(s) (I + A P_xx in the update or P_pred in a gain)", hbad);
  }
  return ACS_OK;
}

// Singular solves of the last EKF enqueue on this context (acs_ekf_run or the pipeline):
// waits for the stream. A device-pointer call without an outlier report stays asynchronous and
// does not check the counter itself; this reads it afterwards.
int acs_ekf_singular_count(acs_ctx* ctx, int32_t* count) {
  ACS_DEVICE_GUARD(ctx);
  ACS_CHECK(ctx, count != nullptr, "acs_ekf_singular_count: null count");
  *count = 0;
  if (!ctx->ekf_bad) return ACS_OK;
  int h = 0;
  ACS_HIP(ctx, hipMemcpyAsync(&h, ctx->ekf_bad, sizeof(int), hipMemcpyDeviceToHost, ctx->stream));
  ACS_HIP(ctx, hipStreamSynchronize(ctx->stream));
  *count = h;
  return ACS_OK;
}

}  // extern "C"
