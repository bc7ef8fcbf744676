// Grid-wide barrier latency on MI355X: could a persistent single-launch LeNet step (phases separated
// by grid barriers instead of hipGraph kernel boundaries, ~1.2 us each) be faster?
// Each of G co-resident blocks (one per CU) runs N barrier rounds: block-level sync, one agent-scope
// atomic arrival per block on a monotonically increasing counter, spin (relaxed loads + s_sleep)
// until the counter reaches round * G, one acquire fence.  Every spin has a wall-clock timeout, so a
// missing block cannot hang the GPU (the kernel records the failure and exits).
//   hipcc --offload-arch=gfx950 -O3 tools/native/grid_barrier_bench.hip -o /tmp/gbb && /tmp/gbb
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ __launch_bounds__(256) void k_barriers(unsigned* ctr, int rounds, int* fail, int sleep) {
  const unsigned G = gridDim.x;
  for (int r = 1; r <= rounds; ++r) {
    __syncthreads();
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)r * G;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        if (sleep) __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {   // 1 s at 100 MHz
          atomicAdd(fail, 1);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }
}

__global__ void k_empty() {}

int main() {
  unsigned* ctr;
  int* fail;
  hipMalloc(&ctr, 4);
  hipMalloc(&fail, 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int G : {128, 256}) {
    for (int sleep : {0, 1}) {
      const int rounds = 1000;
      float best = 1e30f;
      for (int rep = 0; rep < 5; ++rep) {
        hipMemset(ctr, 0, 4);
        hipMemset(fail, 0, 4);
        hipEventRecord(a);
        hipLaunchKernelGGL(k_barriers, dim3(G), dim3(256), 0, 0, ctr, rounds, fail, sleep);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      int f = 0;
      hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost);
      printf("{\"blocks\": %d, \"sleep\": %d, \"us_per_barrier\": %.3f, \"failures\": %d}\n", G, sleep,
             best * 1000.f / rounds, f);
    }
  }
  // reference: back-to-back empty kernels (stream order) and the same through a graph
  {
    const int n = 1000;
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a);
      for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, 0);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("{\"empty_kernel_stream_us\": %.3f}\n", best * 1000.f / n);
    hipStream_t s;
    hipStreamCreate(&s);
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, s);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
    best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      hipEventRecord(a, s);
      for (int i = 0; i < 10; ++i) hipGraphLaunch(ge, s);
      hipEventRecord(b, s);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      if (ms < best) best = ms;
    }
    printf("{\"empty_kernel_graph_us\": %.3f}\n", best * 1000.f / 1000);
  }
  return 0;
}
