// FETCH_SIZE calibration for the access widths the FTE kernels use (MI355X_MICROARCH.md: on
// gfx950 FETCH_SIZE counts half the bytes of 16-B-per-lane streams; other widths are
// uncalibrated). Streams a 1 GiB buffer (past the 256 MiB last-level cache) once per kernel
// with 8-B (double) and with 16-B (double2) coalesced loads. Under `rocprofv3 --pmc FETCH_SIZE`
// each dispatch's FETCH_SIZE x 1024 divided by the bytes printed here is the counter's factor
// for that width.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/fetch_calib.hip -o tools/probe/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_read8(const double* __restrict__ a, size_t n, double* __restrict__ out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 12345.678) out[0] = s;  // keeps the loads
}

__global__ void k_read16(const double2* __restrict__ a, size_t n2, double* __restrict__ out) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;
}

int main() {
  const size_t bytes = (size_t)1 << 30, n = bytes / 8;
  double *a, *out;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  hipMemset(a, 0, bytes);
  hipDeviceSynchronize();
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_read8, dim3(4096), dim3(256), 0, 0, a, n, out);
    hipLaunchKernelGGL(k_read16, dim3(4096), dim3(256), 0, 0, (const double2*)a, n / 2, out);
  }
  hipDeviceSynchronize();
  printf("bytes per dispatch: %zu (k_read8: 8 B per lane, k_read16: 16 B per lane)\n", bytes);
  hipFree(a);
  hipFree(out);
  return 0;
}
