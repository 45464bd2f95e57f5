// Memory-shape probe of the env-step kernel (k_env_step): does giving each env TWO lanes (4 waves per SIMD at
// 131,072 envs instead of 2) shorten a kernel with the step's traffic and structure?  Synthetic stand-in, not the
// step: one thread (LPE = 1) or a lane pair (LPE = 2) per env loads R SoA rows up front (the lane pair splits them
// and exchanges a partial sum with one shuffle), runs a dependent chain of K fmas (the integrator / reward
// math), then a second dependent round trip of 4 texel loads inside an env-private 90 KB region (the potential
// sample), and stores W SoA rows (split over the pair).  R = 96, W = 67 and the texels give ~110 MB per launch at
// 131,072 envs, close to k_env_step's 118 MB (PMC).  Timed with HIP events, median of 20 launches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/envstep_mem_probe.hip -o /tmp/envstep_mem_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int kField = 22528;   // floats per env of the field region (USV_FIELD_STRIDE)

template <int LPE, int R, int W, int K>
__global__ __launch_bounds__(256) void k_probe(const float *__restrict__ in, const float *__restrict__ field,
                                               float *__restrict__ out, int n) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  const int e = g / LPE, half = g % LPE;
  if (e >= n) return;
  constexpr int RL = R / LPE, WL = W / LPE;
  float v[RL];
#pragma unroll
  for (int r = 0; r < RL; ++r) v[r] = in[(size_t)(half * RL + r) * n + e];
#pragma unroll
  for (int w = RL / 2; w >= 1; w >>= 1)
#pragma unroll
    for (int r = 0; r < w; ++r) v[r] += v[r + w];
  float x = v[0];
  if (LPE == 2) x += __shfl_xor(x, 1, 64);
#pragma unroll 8
  for (int k = 0; k < K; ++k) x = fmaf(x, 0.9999f, 1e-3f);
  // the potential sample: 4 texels (2 x 2 block, two rows) at a data-dependent cell of the env's region
  const unsigned cell = (__float_as_uint(x) * 2654435761u) % (unsigned)(kField - 160);
  const float *f = field + (size_t)e * kField + cell;
  float t = 0.f;
  if (LPE == 1 || half == 0) t = (f[0] + f[1]) + (f[150] + f[151]);
  if (LPE == 2) t = __shfl(t, (threadIdx.x & 63) & ~1, 64);
  const float y = x + t;
#pragma unroll
  for (int w = 0; w < WL; ++w) out[(size_t)(half * WL + w) * n + e] = y + (float)w;
}

// two envs per thread (n / 2 threads: one wave per SIMD at 131,072 envs), software-pipelined: both envs' loads
// first, then env A's chain and texel loads, env B's chain and texel loads, A's stores, B's stores -- A's store
// burst and B's dependent math overlap instead of every wave being in the same phase
template <int R, int W, int K>
__global__ __launch_bounds__(256) void k_probe_pipe(const float *__restrict__ in, const float *__restrict__ field,
                                                    float *__restrict__ out, int n) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int h = n / 2;
  if (t >= h) return;
  const int eA = t, eB = t + h;
  float a[R], b[R];
#pragma unroll
  for (int r = 0; r < R; ++r) a[r] = in[(size_t)r * n + eA];
#pragma unroll
  for (int r = 0; r < R; ++r) b[r] = in[(size_t)r * n + eB];
#pragma unroll
  for (int w = R / 2; w >= 1; w >>= 1)
#pragma unroll
    for (int r = 0; r < w; ++r) a[r] += a[r + w];
  float xa = a[0];
#pragma unroll 8
  for (int k = 0; k < K; ++k) xa = fmaf(xa, 0.9999f, 1e-3f);
  const unsigned ca = (__float_as_uint(xa) * 2654435761u) % (unsigned)(kField - 160);
  const float *fa = field + (size_t)eA * kField + ca;
  const float ta0 = fa[0], ta1 = fa[1], ta2 = fa[150], ta3 = fa[151];
#pragma unroll
  for (int w = R / 2; w >= 1; w >>= 1)
#pragma unroll
    for (int r = 0; r < w; ++r) b[r] += b[r + w];
  float xb = b[0];
#pragma unroll 8
  for (int k = 0; k < K; ++k) xb = fmaf(xb, 0.9999f, 1e-3f);
  const unsigned cb = (__float_as_uint(xb) * 2654435761u) % (unsigned)(kField - 160);
  const float *fb = field + (size_t)eB * kField + cb;
  const float tb0 = fb[0], tb1 = fb[1], tb2 = fb[150], tb3 = fb[151];
  const float ya = xa + ((ta0 + ta1) + (ta2 + ta3));
#pragma unroll
  for (int w = 0; w < W; ++w) out[(size_t)w * n + eA] = ya + (float)w;
  const float yb = xb + ((tb0 + tb1) + (tb2 + tb3));
#pragma unroll
  for (int w = 0; w < W; ++w) out[(size_t)w * n + eB] = yb + (float)w;
}

template <int R, int W, int K>
static float run_pipe(const float *in, const float *field, float *out, int n) {
  const int blocks = (n / 2 + 255) / 256;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<float> ms;
  for (int it = 0; it < 25; ++it) {
    hipEventRecord(a, 0);
    hipLaunchKernelGGL((k_probe_pipe<R, W, K>), dim3(blocks), dim3(256), 0, 0, in, field, out, n);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float t;
    hipEventElapsedTime(&t, a, b);
    if (it >= 5) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  return ms[ms.size() / 2] * 1e3f;
}

template <int LPE, int R, int W, int K>
static float run(const float *in, const float *field, float *out, int n) {
  const int threads = n * LPE, blocks = (threads + 255) / 256;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<float> ms;
  for (int it = 0; it < 25; ++it) {
    hipEventRecord(a, 0);
    hipLaunchKernelGGL((k_probe<LPE, R, W, K>), dim3(blocks), dim3(256), 0, 0, in, field, out, n);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float t;
    hipEventElapsedTime(&t, a, b);
    if (it >= 5) ms.push_back(t);
  }
  std::sort(ms.begin(), ms.end());
  return ms[ms.size() / 2] * 1e3f;
}

int main() {
  const int n = 131072;
  float *in, *field, *out;
  hipMalloc(&in, (size_t)96 * n * 4);
  hipMalloc(&field, (size_t)kField * n * 4);
  hipMalloc(&out, (size_t)67 * n * 4);
  hipMemset(in, 0, (size_t)96 * n * 4);
  hipMemset(field, 0, (size_t)kField * n * 4);
  const double mb = ((96.0 + 67.0) * 4 * n + 2 * 128.0 * n) / 1e6;
  printf("{\"envs\": %d, \"approx_mb\": %.1f}\n", n, mb);
  printf("{\"lpe\": 1, \"K\": 0, \"us\": %.2f}\n", run<1, 96, 67, 0>(in, field, out, n));
  printf("{\"lpe\": 2, \"K\": 0, \"us\": %.2f}\n", run<2, 96, 67, 0>(in, field, out, n));
  printf("{\"lpe\": 1, \"K\": 1500, \"us\": %.2f}\n", run<1, 96, 67, 1500>(in, field, out, n));
  printf("{\"lpe\": 2, \"K\": 1500, \"us\": %.2f}\n", run<2, 96, 67, 1500>(in, field, out, n));
  printf("{\"lpe\": 1, \"K\": 3000, \"us\": %.2f}\n", run<1, 96, 67, 3000>(in, field, out, n));
  printf("{\"lpe\": 2, \"K\": 3000, \"us\": %.2f}\n", run<2, 96, 67, 3000>(in, field, out, n));
  printf("{\"pipe\": 2, \"K\": 0, \"us\": %.2f}\n", run_pipe<96, 67, 0>(in, field, out, n));
  printf("{\"pipe\": 2, \"K\": 1500, \"us\": %.2f}\n", run_pipe<96, 67, 1500>(in, field, out, n));
  printf("{\"pipe\": 2, \"K\": 3000, \"us\": %.2f}\n", run_pipe<96, 67, 3000>(in, field, out, n));
  printf("{\"lpe\": 1, \"K\": 1500, \"repeat\": true, \"us\": %.2f}\n", run<1, 96, 67, 1500>(in, field, out, n));
  printf("{\"lpe\": 2, \"K\": 1500, \"R_only\": true, \"us\": %.2f}\n", run<2, 96, 2, 1500>(in, field, out, n));
  printf("{\"lpe\": 1, \"K\": 1500, \"R_only\": true, \"us\": %.2f}\n", run<1, 96, 2, 1500>(in, field, out, n));
  hipFree(in);
  hipFree(field);
  hipFree(out);
  return 0;
}
