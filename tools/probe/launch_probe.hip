// Per-kernel cost of a chain of dependent launches on gfx950: plain stream launches vs one
// hipGraph, empty kernels vs a kernel that reads a flag and returns, 1 vs 1000 workgroups.
// Build: hipcc -O3 --offload-arch=gfx950 tools/probe/launch_probe.hip -o tools/probe/launch_probe
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int* flag) {}
__global__ void k_flag(const int* flag, double* out) {
  if (*flag != 0) return;
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] += 1.0;
}

static float time_chain(bool graph, int nk, int grid, bool flagk, int* flag, double* out, hipStream_t s) {
  auto enqueue = [&]() {
    for (int i = 0; i < nk; ++i) {
      if (flagk)
        hipLaunchKernelGGL(k_flag, dim3(grid), dim3(256), 0, s, flag, out);
      else
        hipLaunchKernelGGL(k_empty, dim3(grid), dim3(256), 0, s, flag);
    }
  };
  hipGraphExec_t exec = nullptr;
  hipGraph_t g = nullptr;
  if (graph) {
    hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
    enqueue();
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
  }
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    hipEventRecord(a, s);
    if (graph)
      hipGraphLaunch(exec, s);
    else
      enqueue();
    hipEventRecord(b, s);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  if (exec) hipGraphExecDestroy(exec);
  if (g) hipGraphDestroy(g);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return best * 1e3f / nk;
}

int main() {
  hipStream_t s;
  hipStreamCreate(&s);
  int* flag;
  double* out;
  hipMalloc(&flag, sizeof(int));
  hipMalloc(&out, sizeof(double));
  hipMemset(flag, 0, sizeof(int));
  hipMemset(out, 0, sizeof(double));
  const int nk = 200;
  for (int graph = 0; graph < 2; ++graph)
    for (int grid : {1, 64, 1000, 4000})
      for (int fk = 0; fk < 2; ++fk)
        printf("%-7s grid %5d %-6s: %.2f us per kernel (chain of %d)\n", graph ? "graph" : "stream", grid,
               fk ? "flag" : "empty", time_chain(graph, nk, grid, fk, flag, out, s), nk);
  // one-kernel graph launched repeatedly (a cached graph per API call)
  for (int grid : {1, 64}) {
    hipGraph_t g1;
    hipGraphExec_t e1;
    hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed);
    hipLaunchKernelGGL(k_flag, dim3(grid), dim3(256), 0, s, flag, out);
    hipStreamEndCapture(s, &g1);
    hipGraphInstantiate(&e1, g1, nullptr, nullptr, 0);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a, s);
      for (int i = 0; i < nk; ++i) hipGraphLaunch(e1, s);
      hipEventRecord(b, s);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("graph1  grid %5d flag  : %.2f us per launch of a one-kernel graph (%d launches)\n", grid,
           best * 1e3f / nk, nk);
  }
  hipMemset(flag, 1, sizeof(int));
  for (int grid : {1, 1000})
    printf("graph   grid %5d early-exit (flag set): %.2f us per kernel\n", grid,
           time_chain(true, nk, grid, true, flag, out, s));
  return 0;
}
