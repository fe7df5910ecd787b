// Dependent-chain latency (clock64 ticks per op, one wave) of the f64 / cross-lane VALU
// operations the latency-bound kernels are built from.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/probe/valu_lat_probe.hip -o tools/probe/valu_lat_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../acinoset_amd/csrc/mfma64.hpp"
template <int OP>
__global__ void k(double* out, long long* cyc, int n, double seed) {
  const int lane = threadIdx.x;
  double x = seed + 1e-3 * lane, y = 1.0000001;
  long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (OP == 0) x = fma(x, y, 1e-9);
      if (OP == 1) x = __builtin_amdgcn_rcp(x);
      if (OP == 2) x = tile_col_bcast<3>(x) * y;
      if (OP == 3) x = tile_row_bcast<2>(x) * y;
      if (OP == 4) x = read_lane_f64(x, 5) * y;
      if (OP == 5) x = __shfl(x, (lane + 5) & 63) * y;
      if (OP == 6) x = 1.0 / x;
      if (OP == 7) x = x * y;
      if (OP == 8) x = rcp_nr(x);
      if (OP == 9) x = sqrt(x);
      if (OP == 10) x = (float)x * 1.0000001f;
      if (OP == 11) x = atan(x) + 0.5;
      if (OP == 12) x = log1p(x);
      if (OP == 13) x = exp(-x);
      if (OP == 14) { double r = __builtin_amdgcn_rsq(x); r = r * fma(-0.5 * x * r, r, 1.5); x = r * fma(-0.5 * x * r, r, 1.5) + 0.1; }
    }
  }
  long long t1 = clock64();
  out[threadIdx.x] = x;
  if (lane == 0) cyc[0] = t1 - t0;
}
template <int OP>
void run(const char* name) {
  double* o; long long* c; long long h;
  hipMalloc(&o, 64 * 8); hipMalloc(&c, 8);
  const int n = 256;
  for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(k<OP>, dim3(1), dim3(64), 0, 0, o, c, n, 1.5);
  hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
  printf("%-28s %7.1f ticks/op\n", name, (double)h / (n * 8));
  hipFree(o); hipFree(c);
}
int main() {
  run<0>("fma f64");
  run<7>("mul f64");
  run<1>("v_rcp_f64");
  run<8>("rcp + 2 Newton");
  run<6>("1.0/x (IEEE)");
  run<9>("sqrt f64");
  run<2>("dpp row_newbcast x2 + mul");
  run<3>("permlane swap x4 + mul");
  run<4>("readlane x2 + mul");
  run<5>("__shfl f64 + mul");
  run<10>("cvt f32 mul cvt");
  run<11>("atan f64 (+add)");
  run<12>("log1p f64");
  run<13>("exp f64");
  run<14>("rsq + 2 Newton (+add)");
  return 0;
}
