// wgla.hpp — workgroup-cooperative dense f64 linear algebra on small blocks
// (P x P frame blocks, 3P x 3P separator blocks). Row-major, explicit leading
// dimensions; every routine is called by all threads of the workgroup and ends with a
// __syncthreads(). Operands may live in LDS or global memory (the workgroup's own
// writes are visible to it after the barrier).
#pragma once
#include "common.hpp"

// C(m x n) += alpha * op(A)(m x k) * op(B)(k x n)
template <bool TA, bool TB>
__device__ void wg_gemm(double* __restrict__ C, int ldc, const double* __restrict__ A, int lda,
                        const double* __restrict__ B, int ldb, int m, int n, int k, double alpha) {
  const int tid = threadIdx.x, nth = blockDim.x;
  for (int idx = tid; idx < m * n; idx += nth) {
    const int i = idx / n, j = idx - (idx / n) * n;
    double s = 0.0;
    for (int t = 0; t < k; ++t) {
      const double a = TA ? A[t * lda + i] : A[i * lda + t];
      const double b = TB ? B[j * ldb + t] : B[t * ldb + j];
      s = fma(a, b, s);
    }
    C[i * ldc + j] += alpha * s;
  }
  __syncthreads();
}

// In-place lower Cholesky of the n x n matrix C (upper triangle left untouched).
// Non-positive pivots are replaced by sqrt(tiny) and counted in *bad (if non-null).
__device__ void wg_chol(double* __restrict__ C, int ld, int n, int* bad) {
  const int tid = threadIdx.x, nth = blockDim.x;
  __shared__ double s_piv;
  for (int k = 0; k < n; ++k) {
    if (tid == 0) {
      double d = C[k * ld + k];
      if (!(d > 0.0)) {
        if (bad) atomicAdd(bad, 1);
        d = 1e-300;
      }
      d = sqrt(d);
      C[k * ld + k] = d;
      s_piv = 1.0 / d;
    }
    __syncthreads();
    const double ip = s_piv;
    for (int i = k + 1 + tid; i < n; i += nth) C[i * ld + k] *= ip;
    __syncthreads();
    const int r = n - k - 1;
    for (int idx = tid; idx < r * r; idx += nth) {
      const int i = k + 1 + idx / r, j = k + 1 + idx % r;
      if (j <= i) C[i * ld + j] -= C[i * ld + k] * C[j * ld + k];
    }
    __syncthreads();
  }
}

// B(m x n) <- B * L^{-T}  (L n x n lower): row-parallel forward substitution.
__device__ void wg_trsm_rlt(double* __restrict__ B, int ldb, const double* __restrict__ Lm, int ldl, int m, int n) {
  const int tid = threadIdx.x, nth = blockDim.x;
  for (int i = tid; i < m; i += nth) {
    double* row = B + i * ldb;
    for (int j = 0; j < n; ++j) {
      double s = row[j];
      for (int t = 0; t < j; ++t) s -= row[t] * Lm[j * ldl + t];
      row[j] = s / Lm[j * ldl + j];
    }
  }
  __syncthreads();
}

// Y(n x m) <- L^{-1} Y  (L n x n lower): column-parallel forward substitution.
__device__ void wg_trsm_lln(double* __restrict__ Y, int ldy, const double* __restrict__ Lm, int ldl, int n, int m) {
  const int tid = threadIdx.x, nth = blockDim.x;
  for (int c = tid; c < m; c += nth) {
    for (int i = 0; i < n; ++i) {
      double s = Y[i * ldy + c];
      for (int t = 0; t < i; ++t) s -= Lm[i * ldl + t] * Y[t * ldy + c];
      Y[i * ldy + c] = s / Lm[i * ldl + i];
    }
  }
  __syncthreads();
}

// Y(n x m) <- L^{-T} Y  (L n x n lower): column-parallel backward substitution.
__device__ void wg_trsm_llt(double* __restrict__ Y, int ldy, const double* __restrict__ Lm, int ldl, int n, int m) {
  const int tid = threadIdx.x, nth = blockDim.x;
  for (int c = tid; c < m; c += nth) {
    for (int i = n - 1; i >= 0; --i) {
      double s = Y[i * ldy + c];
      for (int t = i + 1; t < n; ++t) s -= Lm[t * ldl + i] * Y[t * ldy + c];
      Y[i * ldy + c] = s / Lm[i * ldl + i];
    }
  }
  __syncthreads();
}

__device__ void wg_copy(double* __restrict__ D, int ldd, const double* __restrict__ S, int lds, int m, int n) {
  const int tid = threadIdx.x, nth = blockDim.x;
  for (int idx = tid; idx < m * n; idx += nth) {
    const int i = idx / n, j = idx % n;
    D[i * ldd + j] = S[i * lds + j];
  }
  __syncthreads();
}

__device__ void wg_zero(double* __restrict__ D, int ldd, int m, int n) {
  const int tid = threadIdx.x, nth = blockDim.x;
  for (int idx = tid; idx < m * n; idx += nth) D[(idx / n) * ldd + idx % n] = 0.0;
  __syncthreads();
}
