// Micro-benchmark: per-kernel cost of dependent back-to-back launches on one
// stream, eager vs captured in a hipGraph (how much does a kernel boundary cost?).
// hipcc --offload-arch=gfx950 -O3 tools/launch_rate.hip -o tools/launch_rate
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int *p) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1;
}
__global__ void k_touch(float *p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] * 0.5f + 1.0f;
}

int main() {
  int *d; float *f;
  hipMalloc(&d, 64); hipMemset(d, 0, 64);
  const int n = 1 << 20;
  hipMalloc(&f, n * 4); hipMemset(f, 0, n * 4);
  hipStream_t s; hipStreamCreate(&s);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const int N = 2000;
  float ms;
  for (int rep = 0; rep < 2; ++rep) {
    for (int blocks : {1, 256, 4096}) {
      hipEventRecord(a, s);
      for (int i = 0; i < N; ++i) {
        if (blocks == 1) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d);
        else hipLaunchKernelGGL(k_touch, dim3(blocks), dim3(256), 0, s, f, blocks * 256);
      }
      hipEventRecord(b, s); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
      printf("eager  %5d blocks: %.2f us per kernel\n", blocks, ms * 1000 / N);
      hipGraph_t g; hipGraphExec_t ge;
      hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
      for (int i = 0; i < N; ++i) {
        if (blocks == 1) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d);
        else hipLaunchKernelGGL(k_touch, dim3(blocks), dim3(256), 0, s, f, blocks * 256);
      }
      hipStreamEndCapture(s, &g);
      hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      hipGraphLaunch(ge, s); hipStreamSynchronize(s);
      hipEventRecord(a, s);
      hipGraphLaunch(ge, s);
      hipEventRecord(b, s); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
      printf("graph  %5d blocks: %.2f us per kernel\n", blocks, ms * 1000 / N);
      hipGraphExecDestroy(ge); hipGraphDestroy(g);
    }
  }
  return 0;
}
