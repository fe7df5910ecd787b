// Cycle cost of v_mfma_f64_16x16x4f64 on gfx950: one chain, four independent chains, and
// several waves per SIMD. Build: hipcc -O3 --offload-arch=gfx950 tools/probe/mfma_f64_probe.hip -o tools/probe/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));
template <int CH>
__global__ void k_probe(double* out, long long* cyc, int n) {
  const int lane = threadIdx.x & 63;
  double a = 1.0 + 1e-9 * lane, b = 1.0 - 1e-9 * lane;
  dbl4 acc[CH];
  for (int c = 0; c < CH; ++c) acc[c] = dbl4{0.0, 0.0, 0.0, 0.0};
  __syncthreads();
  const long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
  }
  double s = 0;
  for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
  const long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}
template <int CH>
void run(int waves, int n) {
  double* o; long long* c;
  hipMalloc(&o, 64 * waves * sizeof(double));
  hipMalloc(&c, waves * sizeof(long long));
  hipLaunchKernelGGL(k_probe<CH>, dim3(1), dim3(64 * waves), 0, 0, o, c, n);
  hipLaunchKernelGGL(k_probe<CH>, dim3(1), dim3(64 * waves), 0, 0, o, c, n);
  long long h[64];
  hipMemcpy(h, c, waves * sizeof(long long), hipMemcpyDeviceToHost);
  long long mx = 0;
  for (int w = 0; w < waves; ++w) mx = h[w] > mx ? h[w] : mx;
  printf("chains %d waves/WG %2d: %.1f clock64 ticks per MFMA per wave (max over waves)\n", CH, waves,
         (double)mx / (n * CH));
  hipFree(o); hipFree(c);
}
int main() {
  const int n = 4096;
  run<1>(1, n); run<2>(1, n); run<4>(1, n); run<8>(1, n);
  run<1>(4, n); run<4>(4, n); run<1>(8, n); run<4>(8, n); run<1>(16, n); run<4>(16, n);
  // clock64 rate vs wall clock
  return 0;
}
