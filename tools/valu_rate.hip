// Micro-benchmark: cycles per VALU instruction for one wave per SIMD, dependent
// vs independent chains (answers "does a single wave issue a dependent VALU op
// every 4 cycles on gfx950?").  hipcc --offload-arch=gfx950 -O3 tools/valu_rate.hip -o /tmp/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <int ILP>
__global__ __launch_bounds__(512) void k_chain(float *out, long long *cyc, int iters) {
  float a[ILP];
#pragma unroll
  for (int k = 0; k < ILP; ++k) a[k] = threadIdx.x * 1e-3f + k;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u)
#pragma unroll
      for (int k = 0; k < ILP; ++k) a[k] = a[k] * 0.999f + 0.5f;   // v_fma chain per k
  }
  const long long t1 = clock64();
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < ILP; ++k) s += a[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ __launch_bounds__(256) void k_min3(unsigned *out, long long *cyc, int iters) {
  unsigned a = threadIdx.x, b = threadIdx.x * 3u, c = threadIdx.x * 7u, d = 5u;
  const long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      a = min(min(a, b + 1u), c + 2u);     // add, add, min3: dependent through a
      b = max(a, b) ^ d;
    }
  }
  const long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a + b + c;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float *out; unsigned *outu; long long *cyc;
  hipMalloc(&out, 256 * 256 * 4); hipMalloc(&outu, 256 * 256 * 4); hipMalloc(&cyc, 256 * 8);
  long long h[256];
  const int iters = 1000;
  auto rep = [&](const char *name, double instr) {
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double m = 0; for (int i = 0; i < 256; ++i) m += h[i]; m /= 256;
    printf("%-28s %8.2f cycles per instruction\n", name, m / instr);
  };
  for (int rep_i = 0; rep_i < 2; ++rep_i) {
    k_chain<1><<<256, 256>>>(out, cyc, iters); hipDeviceSynchronize(); rep("fma dependent (ILP 1)", 16.0 * iters);
    k_chain<2><<<256, 256>>>(out, cyc, iters); hipDeviceSynchronize(); rep("fma ILP 2", 32.0 * iters);
    k_chain<4><<<256, 256>>>(out, cyc, iters); hipDeviceSynchronize(); rep("fma ILP 4", 64.0 * iters);
    k_chain<8><<<256, 256>>>(out, cyc, iters); hipDeviceSynchronize(); rep("fma ILP 8", 128.0 * iters);
    k_chain<1><<<256, 512>>>(out, cyc, iters); hipDeviceSynchronize(); rep("fma dep, 2 waves/SIMD", 16.0 * iters);
    k_min3<<<256, 256>>>(outu, cyc, iters); hipDeviceSynchronize(); rep("add/min3/max/xor mix", 16.0 * 6 * iters);
  }
  return 0;
}
