// mfma64.hpp — workgroup-level f64 dense kernels on v_mfma_f64_16x16x4f64 (gfx950).
//
// Fragment maps (cdna_hip_programming.md §3): for D(16x16) = A(16x4) B(4x16) + C, lane l
// supplies A[l & 15][l >> 4] and B[l >> 4][l & 15] (one f64 each); the accumulator holds
// 4 f64 per lane, element r at row (l >> 4) + 4 r, column l & 15.
// All matrices are row-major with explicit leading dimensions; M, N are multiples of 16 and
// K of 4. Every routine is called by all threads of the workgroup (blockDim = 256, 4 waves)
// and ends with a __syncthreads().
#pragma once
#include <type_traits>
#include <utility>

#include "common.hpp"

typedef double dbl4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ dbl4 mfma64(double a, double b, dbl4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// C = beta*C + alpha * op(A) op(B)    (op = transpose when TA / TB)
template <bool TA, bool TB>
__device__ void wg_mgemm(double* C, int ldc, const double* A, int lda, const double* B, int ldb, int M, int N, int K,
                         double alpha, double beta) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int tn = N >> 4, nt = (M >> 4) * tn;
  const int li = lane & 15, lk = lane >> 4;
  for (int t = wave; t < nt; t += nw) {
    const int i0 = (t / tn) << 4, j0 = (t % tn) << 4;
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int k0 = 0; k0 < K; k0 += 4) {
      const int k = k0 + lk;
      const double a = TA ? A[k * lda + i0 + li] : A[(i0 + li) * lda + k];
      const double b = TB ? B[(j0 + li) * ldb + k] : B[k * ldb + j0 + li];
      acc = mfma64(a, b, acc);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double* c = C + (size_t)(i0 + lk + 4 * r) * ldc + j0 + li;
      *c = (beta == 0.0 ? 0.0 : beta * *c) + alpha * acc[r];
    }
  }
  __syncthreads();
}

// Cross-lane moves for a 16x16 f64 tile in accumulator layout (lane l: column l & 15 of
// rows (l >> 4) + 4q), all on the VALU (no LDS round trip):
//   tile_row_bcast<R>(x): every lane gets x from lane 16 R + (l & 15) — the row-of-16 R copied
//                         to all four (gfx950 v_permlane32_swap + v_permlane16_swap);
//   tile_col_bcast<S>(x): every lane gets x from lane 16 (l >> 4) + S — DPP row_newbcast:S.
template <int R>
__device__ __forceinline__ unsigned tile_row_bcast_u32(unsigned x) {
  const auto h = __builtin_amdgcn_permlane32_swap(x, x, false, false);  // [lo|lo], [hi|hi]
  const unsigned y = R < 2 ? h[0] : h[1];
  const auto q = __builtin_amdgcn_permlane16_swap(y, y, false, false);  // even rows, odd rows
  return (R & 1) ? q[1] : q[0];
}
template <int R>
__device__ __forceinline__ double tile_row_bcast(double x) {
  return __hiloint2double((int)tile_row_bcast_u32<R>((unsigned)__double2hiint(x)),
                          (int)tile_row_bcast_u32<R>((unsigned)__double2loint(x)));
}
template <int S>
__device__ __forceinline__ double tile_col_bcast(double x) {
  return __hiloint2double(__builtin_amdgcn_mov_dpp(__double2hiint(x), 0x150 + S, 0xf, 0xf, true),
                          __builtin_amdgcn_mov_dpp(__double2loint(x), 0x150 + S, 0xf, 0xf, true));
}
__device__ __forceinline__ double read_lane_f64(double x, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                          __builtin_amdgcn_readlane(__double2loint(x), l));
}
// x from lane 16 (l >> 4) + S as one 64-bit DPP move (gfx950 DPP64 row_newbcast; the
// 32-bit form, tile_col_bcast, needs two)
template <int S>
__device__ __forceinline__ double tile_col_bcast64(double x) {
  const long long b = __double_as_longlong(x);
  return __longlong_as_double(__builtin_amdgcn_update_dpp(b, b, 0x150 + S, 0xf, 0xf, true));
}

// One Gauss-Jordan step (pivot S) of tile16_gj_inverse; nbad counts failed pivots (uniform).
// With aip_c = a_Sc / p off column S and 1 / p on it, every element off the pivot row is
// a_ic [c != S] - a_iS aip_c  (c = S: -a_iS / p; else a_ic - a_iS a_Sc / p) and the pivot row
// is aip: per register a multiply by the column mask, one 64-bit DPP broadcast of the pivot
// column and one FMA. The roundings are the select form's (tile16_gj_step_v1): 3,723 instead
// of 4,386 clock ticks per 16x16 inverse, bit-identical results (tools/probe/tile_inv_probe.hip,
// profiles/r03/tile_inv_dpp2.log). Tried: the broadcast folded into v_fmac_f64_dpp by
// inline asm (3,887 ticks in the probe, but the asm operands made k_cr_level spill), the
// pivot row through ds_bpermute (4,338: its latency sits on the step's chain) and the
// positivity count on the SALU from the pivot's bits (4,597).
// `mhi`: high word of the column mask (1.0 off column S, 0.0 on it), rotated one lane per
// step (DPP row_ror:1) rather than formed per step: sixteen lane-constant masks would be
// hoisted to the kernel entry and cost 32 VGPRs in the callers.
__device__ __forceinline__ unsigned tile16_colmask_init(int lane) { return (lane & 15) == 0 ? 0u : 0x3FF00000u; }
template <int S, bool SPD>
__device__ __forceinline__ void tile16_gj_step(double* v, int lane, int& nbad, unsigned& mhi) {
  constexpr int QS = S >> 2, RS = S & 3;
  const bool rowS = (lane >> 4) == RS, colS = (lane & 15) == S;
  double p = read_lane_f64(v[QS], RS * 16 + S);  // A[S][S] (uniform)
  const double asc = tile_row_bcast<RS>(v[QS]);  // A[S][c]
  const bool ok = SPD ? p > 0.0 : fabs(p) > 1e-300;
  nbad += ok ? 0 : 1;
  p = ok ? p : 1e-300;
  const double ip = rcp_nr(p);
  const double aip = colS ? ip : asc * ip;
  const double m = __hiloint2double((int)mhi, 0);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const double t = fma(-tile_col_bcast64<S>(v[q]), aip, v[q] * m);
    v[q] = (q == QS && rowS) ? aip : t;
  }
  if (S < 15) mhi = (unsigned)__builtin_amdgcn_mov_dpp((int)mhi, 0x121, 0xf, 0xf, false);  // row_ror:1
}
template <int S, bool SPD>
__device__ __forceinline__ void tile16_gj_step_v1(double* v, int lane, int& nbad) {
  constexpr int QS = S >> 2, RS = S & 3;
  const bool rowS = (lane >> 4) == RS, colS = (lane & 15) == S;
  double p = read_lane_f64(v[QS], RS * 16 + S);  // A[S][S] (uniform)
  const double asc = tile_row_bcast<RS>(v[QS]);  // A[S][c]
  double ais[4];                                 // A[i][S], i = (lane >> 4) + 4q
#pragma unroll
  for (int q = 0; q < 4; ++q) ais[q] = tile_col_bcast<S>(v[q]);
  const bool ok = SPD ? p > 0.0 : fabs(p) > 1e-300;
  nbad += ok ? 0 : 1;
  p = ok ? p : 1e-300;
  const double ip = rcp_nr(p);
  const double aip = asc * ip;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    // a_ic - a_iS a_Sc / p off the pivot row / column, -a_iS / p on the column
    const double t = colS ? -ais[q] * ip : fma(-ais[q], aip, v[q]);
    // pivot row (only register QS holds it): a_Sc / p, and 1 / p on the diagonal
    v[q] = (q == QS && rowS) ? (colS ? ip : aip) : t;
  }
}
template <bool SPD, int... S>
__device__ __forceinline__ void tile16_gj_steps(double* v, int lane, int& nbad, std::integer_sequence<int, S...>) {
  unsigned mhi = tile16_colmask_init(lane);
  (tile16_gj_step<S, SPD>(v, lane, nbad, mhi), ...);
}

// The same 16 steps with hook(std::integral_constant<int, s>) called after step s: lets
// a caller slot independent MFMA work (the matrix core runs it asynchronously) into the
// VALU-bound pivot chain.
template <bool SPD, typename Hook, int... S>
__device__ __forceinline__ void tile16_gj_steps_hook(double* v, int lane, int& nbad, Hook& hook,
                                                     std::integer_sequence<int, S...>) {
  unsigned mhi = tile16_colmask_init(lane);
  ((tile16_gj_step<S, SPD>(v, lane, nbad, mhi), hook(std::integral_constant<int, S>{})), ...);
}
template <bool SPD, typename Hook>
__device__ __forceinline__ void tile16_gj_inverse_hook(double* v, int lane, int* bad, Hook&& hook) {
  int nbad = 0;
  tile16_gj_steps_hook<SPD>(v, lane, nbad, hook, std::make_integer_sequence<int, 16>{});
  if (nbad && bad && lane == 0) atomicAdd(bad, nbad);
}

// the select form of the step (round 1-2), kept for tools/probe/tile_inv_probe.hip
template <bool SPD, int... S>
__device__ __forceinline__ void tile16_gj_steps_v1(double* v, int lane, int& nbad, std::integer_sequence<int, S...>) {
  (tile16_gj_step_v1<S, SPD>(v, lane, nbad), ...);
}
template <bool SPD>
__device__ __forceinline__ void tile16_gj_inverse_v1(double* v, int lane, int* bad) {
  int nbad = 0;
  tile16_gj_steps_v1<SPD>(v, lane, nbad, std::make_integer_sequence<int, 16>{});
  if (nbad && bad && lane == 0) atomicAdd(bad, nbad);
}

// Block Gauss-Jordan form of the 16x16 tile inverse: four steps of a 4x4 pivot block
// (rows / columns 4k..4k+3, register k of every lane) instead of sixteen scalar steps. Per
// step: the pivot block P made uniform (readlanes), its LU without pivoting solved by every
// lane for column lk of P^-1 (uniform operands, no cross-lane traffic on the chain), then two
// f64 MFMAs: B' = P^-1 [M_K with identity on columns K] (A operand = P^-1 rows replicated,
// so every accumulator register holds B' in B layout) and M <- M~ - M_{:,K} B' (rows K set
// to B', columns K of the other rows to -M_{:,K} P^-1). The column panel M_{:,K} reaches the
// A layout by ds_bpermute, off the chain. The LU pivots are the scalar form's pivots, so the
// SPD check and the 1e-300 replacement keep their meaning.
// Measured and not adopted (kept for tools/probe/tile_inv_probe.hip): 3,830 ticks per
// inverse against the scalar DPP64 form's 3,721, and the FTE iteration 331 -> 342 us with it
// in k_cr_level (profiles/r03/tile_inv_block4.log, fte_breakdown_r03y_blockinv_tried.log):
// the four LU pivots' reciprocals and the two MFMA round trips per step cost as much as the
// sixteen scalar steps' chain.
template <int K, bool SPD>
__device__ __forceinline__ void tile16_bgj_step(double* v, int lane, int& nbad) {
  const int li = lane & 15, lk = lane >> 4;
  // A layout of the column panel: lane (li, lk) <- M[li][4K + lk] = v[li >> 2] of lane
  // 16 (li & 3) + 4K + lk
  const int src = (16 * (li & 3) + 4 * K + lk) << 2;
  double g[4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
    g[q] = __hiloint2double(__builtin_amdgcn_ds_bpermute(src, __double2hiint(v[q])),
                            __builtin_amdgcn_ds_bpermute(src, __double2loint(v[q])));
  double p[4][4];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < 4; ++c) p[r][c] = read_lane_f64(v[K], 16 * r + 4 * K + c);
  auto piv = [&](double u) {
    const bool ok = SPD ? u > 0.0 : fabs(u) > 1e-300;
    nbad += ok ? 0 : 1;
    return rcp_nr(ok ? u : 1e-300);
  };
  // LU (Doolittle, no pivoting) of the uniform 4x4 pivot block
  const double i0 = piv(p[0][0]);
  const double l10 = p[1][0] * i0, l20 = p[2][0] * i0, l30 = p[3][0] * i0;
  const double a11 = fma(-l10, p[0][1], p[1][1]), a12 = fma(-l10, p[0][2], p[1][2]), a13 = fma(-l10, p[0][3], p[1][3]);
  const double a21 = fma(-l20, p[0][1], p[2][1]), a22 = fma(-l20, p[0][2], p[2][2]), a23 = fma(-l20, p[0][3], p[2][3]);
  const double a31 = fma(-l30, p[0][1], p[3][1]), a32 = fma(-l30, p[0][2], p[3][2]), a33 = fma(-l30, p[0][3], p[3][3]);
  const double i1 = piv(a11);
  const double l21 = a21 * i1, l31 = a31 * i1;
  const double b22 = fma(-l21, a12, a22), b23 = fma(-l21, a13, a23);
  const double b32 = fma(-l31, a12, a32), b33 = fma(-l31, a13, a33);
  const double i2 = piv(b22);
  const double l32 = b32 * i2;
  const double c33 = fma(-l32, b23, b33);
  const double i3 = piv(c33);
  // column lk of P^-1: L y = e_lk, U x = y
  const double y0 = lk == 0 ? 1.0 : 0.0;
  const double y1 = fma(-l10, y0, lk == 1 ? 1.0 : 0.0);
  const double y2 = fma(-l21, y1, fma(-l20, y0, lk == 2 ? 1.0 : 0.0));
  const double y3 = fma(-l32, y2, fma(-l31, y1, fma(-l30, y0, lk == 3 ? 1.0 : 0.0)));
  const double x3 = y3 * i3;
  const double x2 = fma(-b23, x3, y2) * i2;
  const double x1 = fma(-a12, x2, fma(-a13, x3, y1)) * i1;
  const double x0 = fma(-p[0][1], x1, fma(-p[0][2], x2, fma(-p[0][3], x3, y0))) * i0;
  const int rr = li & 3;
  const double pinv = rr == 0 ? x0 : (rr == 1 ? x1 : (rr == 2 ? x2 : x3));  // P^-1[li & 3][lk]
  const bool colK = (li >> 2) == K;
  const double bk = colK ? ((li & 3) == lk ? 1.0 : 0.0) : v[K];
  const dbl4 z = {0.0, 0.0, 0.0, 0.0};
  const double bp = mfma64(pinv, bk, z)[0];  // B'[lk][li]
  const double gq = li < 4 ? g[0] : (li < 8 ? g[1] : (li < 12 ? g[2] : g[3]));
  const double a2 = colK ? 0.0 : -gq;
  dbl4 c;
#pragma unroll
  for (int q = 0; q < 4; ++q) c[q] = q == K ? bp : (colK ? 0.0 : v[q]);
  c = mfma64(a2, bp, c);
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = c[q];
}
template <bool SPD, typename Hook, int... K>
__device__ __forceinline__ void tile16_bgj_steps_hook(double* v, int lane, int& nbad, Hook& hook,
                                                      std::integer_sequence<int, K...>) {
  ((tile16_bgj_step<K, SPD>(v, lane, nbad), hook(std::integral_constant<int, 4 * K>{}),
    hook(std::integral_constant<int, 4 * K + 1>{}), hook(std::integral_constant<int, 4 * K + 2>{}),
    hook(std::integral_constant<int, 4 * K + 3>{})),
   ...);
}
template <bool SPD, typename Hook>
__device__ __forceinline__ void tile16_bgj_inverse_hook(double* v, int lane, int* bad, Hook&& hook) {
  int nbad = 0;
  tile16_bgj_steps_hook<SPD>(v, lane, nbad, hook, std::make_integer_sequence<int, 4>{});
  if (nbad && bad && lane == 0) atomicAdd(bad, nbad);
}
template <bool SPD>
__device__ __forceinline__ void tile16_bgj_inverse(double* v, int lane, int* bad) {
  tile16_bgj_inverse_hook<SPD>(v, lane, bad, [](auto) {});
}

// In-register Gauss-Jordan inverse of one 16x16 tile held by a wave in accumulator layout
// (lane l: column l & 15 of rows (l >> 4) + 4q). The pivot (v_readlane), pivot row
// (permlane swaps) and pivot column (DPP row_newbcast) of each of the 16 steps move on the
// VALU: no barrier, no LDS. SPD: pivots must be positive; otherwise |p| > 1e-300. A failed
// pivot is replaced by 1e-300 and counted in *bad.
template <bool SPD>
__device__ __forceinline__ void tile16_gj_inverse(double* v, int lane, int* bad) {
  int nbad = 0;
  tile16_gj_steps<SPD>(v, lane, nbad, std::make_integer_sequence<int, 16>{});
  if (nbad && bad && lane == 0) atomicAdd(bad, nbad);
}

// In-place inverse of an SPD matrix (n = 16*nb, LDS or global, ld) by blocked
// Gauss-Jordan without pivoting (SPD + LM damping: every pivot block is SPD).
// tmp: 512 doubles of LDS. Non-positive pivots are counted in *bad.
template <bool SPD = true>
__device__ void wg_gj_inverse(double* A, int lda, int nb, double* tmp, int* bad);

__device__ void wg_spd_inverse(double* A, int lda, int nb, double* tmp, int* bad) {
  wg_gj_inverse<true>(A, lda, nb, tmp, bad);
}

// Blocked Gauss-Jordan inverse without pivoting. SPD: pivots must be positive; otherwise
// (symmetric indefinite, e.g. the reference EKF's covariances) any pivot with |p| > 1e-300.
// wg_gj_inverse_body: the same, inlined into the caller (whose register budget then holds
// for it: a called function's VGPRs count against the kernel's occupancy unconstrained)
template <bool SPD>
__device__ __forceinline__ void wg_gj_inverse_body(double* A, int lda, int nb, double* tmp, int* bad);
template <bool SPD>
__device__ void wg_gj_inverse(double* A, int lda, int nb, double* tmp, int* bad) {
  wg_gj_inverse_body<SPD>(A, lda, nb, tmp, bad);
}
template <bool SPD>
__device__ __forceinline__ void wg_gj_inverse_body(double* A, int lda, int nb, double* tmp, int* bad) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = blockDim.x >> 6;
  const int li = lane & 15, lk = lane >> 4;
  for (int k = 0; k < nb; ++k) {
    double* Akk = A + (size_t)(k << 4) * lda + (k << 4);
    // 1. 16x16 diagonal block: unblocked Gauss-Jordan by wave 0 in registers (lane l holds
    //    column l & 15 of rows (l >> 4) + 4q); pivot row / column travel by shuffles, so the
    //    16 steps need no workgroup barrier. Same arithmetic as an entry-per-thread version.
    if (wave == 0) {
      const int r0 = lane >> 4, c = lane & 15;
      double v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = Akk[(r0 + 4 * q) * lda + c];
      tile16_gj_inverse<SPD>(v, lane, bad);
#pragma unroll
      for (int q = 0; q < 4; ++q) Akk[(r0 + 4 * q) * lda + c] = v[q];
    }
    (void)tmp;
    __syncthreads();
    // 2. row panel A_kJ <- Akk^-1 A_kJ (J != k); each tile read and written by one wave
    for (int J = wave; J < nb; J += nw) {
      if (J == k) continue;
      double* AkJ = A + (size_t)(k << 4) * lda + (J << 4);
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k0 = 0; k0 < 16; k0 += 4) acc = mfma64(Akk[li * lda + k0 + lk], AkJ[(k0 + lk) * lda + li], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) AkJ[(lk + 4 * r) * lda + li] = acc[r];
    }
    __syncthreads();
    // 3. trailing A_IJ -= A_Ik A_kJ (I, J != k)
    const int nt = nb * nb;
    for (int t = wave; t < nt; t += nw) {
      const int I = t / nb, J = t % nb;
      if (I == k || J == k) continue;
      double* AIJ = A + (size_t)(I << 4) * lda + (J << 4);
      const double* AIk = A + (size_t)(I << 4) * lda + (k << 4);
      const double* AkJ = A + (size_t)(k << 4) * lda + (J << 4);
      dbl4 acc;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] = AIJ[(lk + 4 * r) * lda + li];
#pragma unroll
      for (int k0 = 0; k0 < 16; k0 += 4) acc = mfma64(-AIk[li * lda + k0 + lk], AkJ[(k0 + lk) * lda + li], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) AIJ[(lk + 4 * r) * lda + li] = acc[r];
    }
    __syncthreads();
    // 4. column panel A_Ik <- -A_Ik Akk^-1 (I != k)
    for (int I = wave; I < nb; I += nw) {
      if (I == k) continue;
      double* AIk = A + (size_t)(I << 4) * lda + (k << 4);
      dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k0 = 0; k0 < 16; k0 += 4) acc = mfma64(-AIk[li * lda + k0 + lk], Akk[(k0 + lk) * lda + li], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) AIk[(lk + 4 * r) * lda + li] = acc[r];
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------
// LDS-staged variants. Operands are copied into LDS with an odd leading dimension
// (ld = cols + 1 doubles) so that the 16 rows a fragment touches land on distinct banks;
// the MFMA loop then reads only LDS. `consume(i0, j0, acc)` receives each finished
// 16x16 tile (lane layout: element r at row i0 + (lane>>4) + 4r, column j0 + (lane&15)).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int lds_ld(int cols) { return cols + 1; }

// dst (rows x cols, ld = cols+1) <- src (row-major, ld_src) or its transpose
template <bool TRANS>
__device__ void lds_stage(double* dst, const double* __restrict__ src, int ld_src, int rows, int cols) {
  const int ld = lds_ld(cols);
  for (int e = threadIdx.x; e < rows * cols; e += blockDim.x) {
    if (TRANS) {
      const int c = e / rows, r = e % rows;  // coalesced along the source rows
      dst[r * ld + c] = src[(size_t)c * ld_src + r];
    } else {
      const int r = e / cols, c = e % cols;
      dst[r * ld + c] = src[(size_t)r * ld_src + c];
    }
  }
}

template <typename F>
__device__ void lds_gemm(const double* A, int lda, const double* B, int ldb, int M, int N, int K, F&& consume) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int tn = N >> 4, nt = (M >> 4) * tn;
  const int li = lane & 15, lk = lane >> 4;
  for (int t = wave; t < nt; t += nw) {
    const int i0 = (t / tn) << 4, j0 = (t % tn) << 4;
    dbl4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll 4
    for (int k0 = 0; k0 < K; k0 += 4)
      acc = mfma64(A[(i0 + li) * lda + k0 + lk], B[(k0 + lk) * ldb + j0 + li], acc);
    consume(i0, j0, acc);
  }
}
