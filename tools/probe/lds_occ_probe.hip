// Workgroups per CU that co-reside at a given static LDS size: each workgroup (384 threads)
// spins ~20 us on the wall clock and records its entry / exit; the host reports the mean
// number in flight. Build: hipcc --offload-arch=gfx950 -O2 tools/probe/lds_occ_probe.hip -o
// tools/probe/lds_occ_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int KB, int LB>
__global__ __launch_bounds__(LB) void k_probe(unsigned long long* tr, double* sink) {
  __shared__ double buf[KB * 128];
  const unsigned long long t0 = wall_clock64();
  for (int i = threadIdx.x; i < KB * 128; i += blockDim.x) buf[i] = i;
  __syncthreads();
  double acc = 0.0;
  while (wall_clock64() - t0 < 2000) acc += buf[(threadIdx.x * 7) % (KB * 128)];  // ~20 us
  if (acc == -1.0) sink[0] = acc;
  if (threadIdx.x == 0) {
    tr[2 * blockIdx.x] = t0;
    tr[2 * blockIdx.x + 1] = wall_clock64();
  }
}

template <int KB, int LB = 1024>
void run(unsigned long long* d, double* s, int nwg, int nth = 384) {
  hipLaunchKernelGGL((k_probe<KB, LB>), dim3(nwg), dim3(nth), 0, 0, d, s);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(2 * nwg);
  (void)hipMemcpy(h.data(), d, 16 * nwg, hipMemcpyDeviceToHost);
  unsigned long long lo = ~0ull, hi = 0;
  double life = 0;
  for (int i = 0; i < nwg; ++i) {
    lo = std::min(lo, h[2 * i]);
    hi = std::max(hi, h[2 * i + 1]);
    life += (double)(h[2 * i + 1] - h[2 * i]);
  }
  printf("%4d threads (launch bound %4d), LDS %3d KB per workgroup: mean in flight %.0f (span %.0f us)\n", nth, LB, KB, life / (double)(hi - lo),
         (hi - lo) * 1e-2);
  (void)nth;
}

int main(int argc, char**) {
  const int nwg = 4096;
  unsigned long long* d;
  double* s;
  (void)hipMalloc(&d, 16 * nwg);
  (void)hipMalloc(&s, 8);
  if (argc > 1) {  // 256-thread workgroups between 24 and 32 KB, launch bound 256 vs 1024
    run<24, 256>(d, s, nwg, 256);
    run<24, 1024>(d, s, nwg, 256);
    run<26, 256>(d, s, nwg, 256);
    run<26, 1024>(d, s, nwg, 256);
    run<27, 256>(d, s, nwg, 256);
    run<27, 1024>(d, s, nwg, 256);
    run<28, 256>(d, s, nwg, 256);
    run<28, 1024>(d, s, nwg, 256);
    run<30, 256>(d, s, nwg, 256);
    run<30, 1024>(d, s, nwg, 256);
    run<32, 1024>(d, s, nwg, 256);
    return 0;
  }
  run<40, 384>(d, s, nwg);
  run<40, 1024>(d, s, nwg);
  run<54, 384>(d, s, nwg);
  run<54, 1024>(d, s, nwg);
  run<72, 384>(d, s, nwg);
  run<72, 1024>(d, s, nwg);
  run<80, 384>(d, s, nwg);
  run<80, 1024>(d, s, nwg);
  run<30, 256>(d, s, nwg, 256);
  run<36, 256>(d, s, nwg, 256);
  run<40, 768>(d, s, nwg, 768);
  run<40, 1024>(d, s, nwg, 768);
  run<54, 768>(d, s, nwg, 768);
  run<54, 1024>(d, s, nwg, 768);
  return 0;
}
