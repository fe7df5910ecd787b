// Check + time tile16_gj_inverse (VALU cross-lane moves) against the LDS-shuffle version
// and a host Gauss-Jordan, on random SPD 16x16 tiles.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include tools/probe/tile_inv_probe.hip -o tools/probe/tile_inv_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include "../../acinoset_amd/csrc/mfma64.hpp"

__device__ void inv_shfl(double* v, int lane) {
  const int r0 = lane >> 4, c = lane & 15;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const int qs = s >> 2, rs = s & 3;
    double p = __shfl(v[qs], rs * 16 + s);
    const double asc = __shfl(v[qs], rs * 16 + c);
    double ais[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) ais[q] = __shfl(v[q], r0 * 16 + s);
    const double ip = 1.0 / p;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = r0 + 4 * q;
      if (i == s && c == s) v[q] = ip;
      else if (i == s) v[q] = asc * ip;
      else if (c == s) v[q] = -ais[q] * ip;
      else v[q] = v[q] - ais[q] * asc * ip;
    }
  }
}
template <int MODE>
__global__ void k_inv(const double* A, double* out, long long* cyc, int* bad, int reps) {
  const int lane = threadIdx.x, r0 = lane >> 4, c = lane & 15;
  const double* a = A + blockIdx.x * 256;
  double v[4];
  for (int q = 0; q < 4; ++q) v[q] = a[(r0 + 4 * q) * 16 + c];
  long long t0 = clock64();
  for (int r = 0; r < reps; ++r) {
    if (MODE == 0) inv_shfl(v, lane);
    else if (MODE == 1) tile16_gj_inverse_v1<true>(v, lane, bad);
    else if (MODE == 2) tile16_gj_inverse<true>(v, lane, bad);
    else tile16_bgj_inverse<true>(v, lane, bad);
  }
  long long t1 = clock64();
  for (int q = 0; q < 4; ++q) out[blockIdx.x * 256 + (r0 + 4 * q) * 16 + c] = v[q];
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}
static void host_inv(const double* a, double* x) {
  double m[16][32];
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 32; ++j) m[i][j] = j < 16 ? a[i * 16 + j] : (j - 16 == i);
  for (int k = 0; k < 16; ++k) {
    double p = m[k][k];
    for (int j = 0; j < 32; ++j) m[k][j] /= p;
    for (int i = 0; i < 16; ++i) if (i != k) { double f = m[i][k]; for (int j = 0; j < 32; ++j) m[i][j] -= f * m[k][j]; }
  }
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) x[i * 16 + j] = m[i][16 + j];
}
int main() {
  const int NT = 64;
  double* hA = (double*)malloc(NT * 256 * 8);
  double* ref = (double*)malloc(NT * 256 * 8);
  double* o0 = (double*)malloc(NT * 256 * 8);
  double* o1 = (double*)malloc(NT * 256 * 8);
  double* o2 = (double*)malloc(NT * 256 * 8);
  double* o3 = (double*)malloc(NT * 256 * 8);
  srand(1);
  for (int t = 0; t < NT; ++t) {
    double B[256];
    for (int e = 0; e < 256; ++e) B[e] = (rand() / (double)RAND_MAX - 0.5) * pow(10.0, (e % 7) - 3);
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
      double s = (i == j) ? 1e-3 * (t + 1) : 0.0;
      for (int k = 0; k < 16; ++k) s += B[i * 16 + k] * B[j * 16 + k];
      hA[t * 256 + i * 16 + j] = s;
    }
    host_inv(hA + t * 256, ref + t * 256);
  }
  double *dA, *dO; long long* dc; int* db;
  hipMalloc(&dA, NT * 256 * 8); hipMalloc(&dO, NT * 256 * 8); hipMalloc(&dc, NT * 8); hipMalloc(&db, 4);
  hipMemcpy(dA, hA, NT * 256 * 8, hipMemcpyHostToDevice); hipMemset(db, 0, 4);
  long long cyc[NT];
  const char* names[4] = {"shfl", "valu-select", "valu-dpp64", "block4-mfma"};
  double* outs[4] = {o0, o1, o2, o3};
  for (int mode = 0; mode < 4; ++mode) {
    for (int reps : {1, 1, 9}) {
      if (mode == 0) hipLaunchKernelGGL(k_inv<0>, dim3(NT), dim3(64), 0, 0, dA, dO, dc, db, reps);
      else if (mode == 1) hipLaunchKernelGGL(k_inv<1>, dim3(NT), dim3(64), 0, 0, dA, dO, dc, db, reps);
      else if (mode == 2) hipLaunchKernelGGL(k_inv<2>, dim3(NT), dim3(64), 0, 0, dA, dO, dc, db, reps);
      else hipLaunchKernelGGL(k_inv<3>, dim3(NT), dim3(64), 0, 0, dA, dO, dc, db, reps);
      hipDeviceSynchronize();
      hipMemcpy(cyc, dc, NT * 8, hipMemcpyDeviceToHost);
      if (reps == 1) hipMemcpy(outs[mode], dO, NT * 256 * 8, hipMemcpyDeviceToHost);
      double mc = 0; for (int t = 0; t < NT; ++t) mc += cyc[t];
      printf("mode %s reps %d: %.0f clock64 ticks per inverse\n", names[mode], reps, mc / NT / reps);
    }
  }
  long long ndiff = 0;
  for (int e = 0; e < NT * 256; ++e) ndiff += (o1[e] != o2[e]);
  printf("dpp64 vs select: %lld of %d elements differ\n", ndiff, NT * 256);
  double e0 = 0, e1 = 0, e01 = 0, e3 = 0;
  for (int t = 0; t < NT; ++t) {
    double mx = 0; for (int e = 0; e < 256; ++e) mx = fmax(mx, fabs(ref[t * 256 + e]));
    for (int e = 0; e < 256; ++e) {
      e0 = fmax(e0, fabs(o0[t * 256 + e] - ref[t * 256 + e]) / mx);
      e1 = fmax(e1, fabs(o1[t * 256 + e] - ref[t * 256 + e]) / mx);
      e01 = fmax(e01, fabs(o1[t * 256 + e] - o0[t * 256 + e]) / mx);
      e3 = fmax(e3, fabs(o3[t * 256 + e] - ref[t * 256 + e]) / mx);
    }
  }
  int hb; hipMemcpy(&hb, db, 4, hipMemcpyDeviceToHost);
  printf("max rel err: shfl vs host %.3e, valu vs host %.3e, valu vs shfl %.3e, block4 vs host %.3e, bad %d\n", e0, e1, e01, e3, hb);
  return (e1 < 1e-8 && e3 < 1e-8 && hb == 0) ? 0 : 1;
}
