// Issue cost of f64 VALU work in one wave as a function of the active lanes: 8 independent
// FMA chains (throughput, not latency) with 64 / 32 / 16 / 8 lanes active. If a partially
// active wave64 issued in fewer passes, packing fewer lane groups per wave would shorten
// the SBA LM chain. Build: hipcc -O3 --offload-arch=gfx950 tools/probe/exec_mask_probe.hip -o tools/probe/exec_mask_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(double* out, long long* cyc, int n, int active) {
  const int lane = threadIdx.x;
  double a[8];
  for (int u = 0; u < 8; ++u) a[u] = 1.0 + 1e-3 * (lane + u);
  const double y = 1.0000001;
  __syncthreads();
  const long long t0 = clock64();
  if (lane < active) {
    for (int i = 0; i < n; ++i) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = fma(a[u], y, 1e-9);
    }
  }
  __syncthreads();
  const long long t1 = clock64();
  double s = 0;
  for (int u = 0; u < 8; ++u) s += a[u];
  out[lane] = s;
  if (lane == 0) cyc[0] = t1 - t0;
}

int main() {
  double* o;
  long long* c;
  hipMalloc(&o, 64 * 8);
  hipMalloc(&c, 8);
  const int n = 1024;
  for (int active : {64, 48, 32, 16, 8, 1}) {
    long long h = 0;
    for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, c, n, active);
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("active lanes %2d: %.2f ticks per f64 FMA instruction (8 independent chains)\n", active,
           (double)h / (n * 8));
  }
  return 0;
}
