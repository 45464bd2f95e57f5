// rl_games PPO hot path (a2c_continuous, actor_critic_mlp_dict 33-128-128-{2,1},
// continuous_a2c_logstd) for MI355X (gfx950), fp32 end to end.
//
// Replaces (rl_games/rl_games/...):
//   common/a2c_common.py:385-430,670-774   get_action_values/get_values, play_steps
//   common/a2c_common.py:525-540,1257-1332 discount_values (GAE), prepare_dataset
//   algos_torch/a2c_continuous.py:78-217    calc_gradients, bound_loss
//   common/common_losses.py:6-48            actor_loss, critic_loss
//   common/a2c_common.py:308-330,1200-1235  trancate_gradients_and_step, adaptive LR
//   algos_torch/running_mean_std.py:44-139  RunningMeanStd (fp64 stats)
//   algos_torch/torch_ext.py:27-36          policy_kl
//   common/datasets.py:25-29                update_mu_sigma
//
// Block forward/backward (RB = 32 rows per 256-thread workgroup, 4 waves):
// every 32x128 / 128x128 product runs on the f32 matrix cores
// (v_mfma_f32_32x32x2_f32, an exact k-ordered fmaf chain, so the layer
// outputs equal a sequential fmaf loop over k).  The weights are staged once
// per workgroup into LDS (W2 with a 130-float row stride: conflict-free
// operand reads for both the W2 and W2^T access patterns the forward and the
// backward need), activations never leave LDS, and each workgroup writes one
// deterministic partial gradient (param layout) that k_reduce_partials sums
// in a fixed order.  clip + Adam + the adaptive LR run in k_apply.
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "usv_device.h"

USV_PROBE_DEFINE(ppo)
USV_PROBE_DEFINE(pol)
USV_PROBE_DEFINE(red)

namespace {

constexpr int NIN = PPO_NIN, NH = PPO_NH, NA = PPO_NA;
constexpr int RB = 32;          // rows per block
constexpr int TB = 256;         // threads per block (4 waves; wave w owns output columns 32w..32w+31)
constexpr int XS = 35;          // row stride of x / W1 in LDS (k 33, 34 zero; odd: the layer-1 operand
                                // reads x[i][k] / W1[i][k] of 32 lanes i hit 32 different banks)
constexpr int HS = 129;         // row stride of h1 / h2 / W2 in LDS (odd: the matrix-core operand reads of
                                // a column, 32 lanes = 32 rows, hit 32 different banks)
constexpr int NPART = PPO_NPARAM + 8;   // partial row: params + loss sums
constexpr int NPART_PAD = (NPART + 3) & ~3;   // partial row stride (16-B aligned rows)
constexpr int P_LOSS = PPO_NPARAM;      // a, c, entropy, b, kl sums
constexpr float kLog2Pi = 1.8378770664093453f;  // 0.5*log(2*pi)*2 (models.py:400)

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// bf16 GEMM mode (ppo_cfg_t.bf16_gemm, BASELINE configs[2]): the three 128 x 128 products (layer 2,
// dW2, dh1) take bf16 operands (round to nearest even from the fp32 values in LDS) on
// v_mfma_f32_32x32x16_bf16 with fp32 accumulation: lane l supplies row / column l & 31 and the 8
// consecutive k of group l >> 5.  Everything else stays fp32.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 ld8(const float *p) {          // 8 consecutive floats
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (__bf16)p[j];
  return v;
}
__device__ __forceinline__ bf16x8 ld8s(const float *p, int stride) {   // 8 floats, stride apart
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (__bf16)p[j * stride];
  return v;
}
// C/D layout of a 32x32 tile: lane l holds column l&31, rows (r&3) + 8(r>>2) + 4(l>>5), r = 0..15
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ float rms_norm(float x, double mean, double var, float eps) {
  // RunningMeanStd.forward (running_mean_std.py:113-118): fp32 math on fp64 stats
  const float y = (x - (float)mean) / sqrtf((float)var + eps);
  return clampt(y, -5.0f, 5.0f);
}

constexpr int TAIL = PPO_NPARAM - PPO_OFF_B2;     // b2, Wv, bv, Wmu, bmu (contiguous)
constexpr int T_B2 = 0, T_WV = NH, T_BV = 2 * NH, T_WMU = 2 * NH + 1, T_BMU = 4 * NH + 1;

struct MlpSmem {
  float w2[NH * HS];      // W2[j][k]
  float w1[NH * XS];      // W1[j][k], k 33, 34 = 0
  float x[RB * XS];       // normalised obs (later unchanged: dW1 operand)
  float h1[RB * HS];      // tanh layer 1 (later dz1)
  float h2[RB * HS];      // tanh layer 2 (later dz2)
  float out[RB * 4];      // mu0, mu1, value
  float g[RB * 4];        // dmu0, dmu1, dv, dnlp per row
  float hg[2][4][NH];     // head-gradient / bias half sums
  float b1[NH];
  float tail[TAIL + 1];   // params from b2 on (T_* offsets)
  float om[NIN], od[NIN]; // policy step: (float)mean, sqrtf((float)var + eps) of the obs statistics
  float zz[2][RB * 2];    // policy step: the N(0,1) draws of a tile's rows, one tile ahead
};

// Weight staging in two halves: every global load is issued up front into
// registers (compile-time trip counts); W1 / biases / heads go to LDS before
// layer 1, W2 is committed after layer 1's matrix-core loop so its loads
// overlap the first layer.
constexpr int NW2 = NH * NH / TB, NW1 = (NH * XS + TB - 1) / TB, NTL = (TAIL + TB - 1) / TB;
static_assert(NH * NH % TB == 0, "staging trip counts");
struct StagedW {
  float w2r[NW2];   // W2 element tid + u TB: a wave's LDS writes are 64 consecutive words of one row
  float w1r[NW1], tlr[NTL], b1r;
};

__device__ __forceinline__ void stage_load(const float *__restrict__ P, StagedW &r) {
  const int tid = threadIdx.x;
  // branch-free: clamped indices, masked after every load is issued
#pragma unroll
  for (int u = 0; u < NW1; ++u) {
    const int i = min(tid + u * TB, NH * XS - 1), j = i / XS, k = i % XS;
    r.w1r[u] = P[PPO_OFF_W1 + j * NIN + min(k, NIN - 1)];
  }
#pragma unroll
  for (int u = 0; u < NTL; ++u) r.tlr[u] = P[PPO_OFF_B2 + min(tid + u * TB, TAIL - 1)];
  r.b1r = P[PPO_OFF_B1 + (tid & (NH - 1))];
#pragma unroll
  for (int u = 0; u < NW2; ++u) r.w2r[u] = P[PPO_OFF_W2 + tid + u * TB];
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int u = 0; u < NW1; ++u)
    if ((tid + u * TB) % XS >= NIN) r.w1r[u] = 0.f;
}

__device__ __forceinline__ void stage_store_small(const StagedW &r, MlpSmem &s) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < NW1; ++u)
    if (tid + u * TB < NH * XS) s.w1[tid + u * TB] = r.w1r[u];
#pragma unroll
  for (int u = 0; u < NTL; ++u)
    if (tid + u * TB < TAIL) s.tail[tid + u * TB] = r.tlr[u];
  if (tid < NH) s.b1[tid] = r.b1r;
}

__device__ __forceinline__ void stage_store_w2(const StagedW &r, MlpSmem &s) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < NW2; ++u) {
    const int e = tid + u * TB;
    s.w2[(e / NH) * HS + e % NH] = r.w2r[u];
  }
}

// tanh(x) = 1 - 2 / (exp(2x) + 1) from one exp2 and one reciprocal (v_exp_f32 / v_rcp_f32) and an fma: |error| <
// 2e-7 absolute against float64 tanh over the whole range (exp2 overflows to +inf and gives 1, underflows to 0 and
// gives -1; parity tolerances are 1e-5).  Round 5 used the odd form (1 - e) / (1 + e) of |x| with a 3-term series
// below 2^-7 for relative accuracy at tiny arguments: ~8 more VALU operations per activation, on the forward's
// critical path in the gradient and policy kernels, for an accuracy no consumer needs.
#ifndef USV_TANH_ODD
#define USV_TANH_ODD 0
#endif
__device__ __forceinline__ float fast_tanh(float x) {
  if constexpr (USV_TANH_ODD != 0) {
    const float ax = fabsf(x);
    const float e = __builtin_amdgcn_exp2f(ax * -2.8853900817779268f);   // exp(-2|x|)
    const float big = (1.0f - e) * __builtin_amdgcn_rcpf(1.0f + e);
    const float x2 = ax * ax;
    const float small = ax * (1.0f - x2 * (0.33333334f - 0.13333334f * x2));
    return copysignf(ax < 0.0078125f ? small : big, x);
  }
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);        // exp(2x)
  return fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
}

// The persistent forward kernels' obs path: a thread's slots q = tid + u TB of a tile's RB x XS
// block sit in the same columns for every tile, so the running statistics are loaded once per
// launch; the next tile's rows are loaded (clamped, unconditionally) while the current one runs.
// The rollout's experience-buffer stores are non-temporal: the 16 steps' 350 MB at 131072 envs exceed the
// Infinity Cache and the update reads them only after the rollout, so cached they would only evict the env
// state the next env step reads (same-box A/B: env step 26.7 -> 24.8 us, rollout and update unchanged)
#ifndef USV_EXP_NT
#define USV_EXP_NT 1
#endif
template <class T>
__device__ __forceinline__ void exp_st(T *p, T v) {
  if constexpr (USV_EXP_NT != 0) __builtin_nontemporal_store(v, p);
  else *p = v;
}
constexpr int NUO = (RB * XS + TB - 1) / TB;
struct ObsCols {
  double mu[NUO], var[NUO];
};
__device__ __forceinline__ void load_obs_cols(const double *__restrict__ obs_rms, ObsCols &oc) {
#pragma unroll
  for (int u = 0; u < NUO; ++u) {
    const int kc = min(((int)threadIdx.x + u * TB) % XS, NIN - 1);
    oc.mu[u] = obs_rms[kc];
    oc.var[u] = obs_rms[NIN + kc];
  }
}
__device__ __forceinline__ void load_obs_tile(const float *__restrict__ obs, int n, int tile, float (&x)[NUO]) {
  const int row0 = tile * RB, nrows = min(RB, n - row0);
#pragma unroll
  for (int u = 0; u < NUO; ++u) {
    const int q = min((int)threadIdx.x + u * TB, RB * XS - 1);
    const int r = min(q / XS, nrows - 1), kc = min(q % XS, NIN - 1);
    x[u] = obs[(size_t)(row0 + r) * NIN + kc];
  }
}
// normalised rows into s.x; with exp_obs, the raw rows also to the experience buffer (row
// env * H + t, swap_and_flatten01 layout)
template <class S>
__device__ __forceinline__ void put_obs_tile(const float (&x)[NUO], const ObsCols &oc, int row0, int nrows,
                                             bool normalize, float eps, S &s, float *exp_obs, int H, int t) {
#pragma unroll
  for (int u = 0; u < NUO; ++u) {
    const int q = threadIdx.x + u * TB;
    if (q >= RB * XS) continue;
    const int r = q / XS, k = q % XS;
    float v = 0.f;
    if (r < nrows && k < NIN) {
      v = x[u];
      if (exp_obs) exp_obs[((size_t)(row0 + r) * H + t) * NIN + k] = v;
      if (normalize) v = rms_norm(v, oc.mu[u], oc.var[u], eps);
    }
    s.x[q] = v;
  }
}

// The policy step's obs path runs on waves 1-3 (OT threads, tt = tid - 64) while wave 0 samples
// the previous tile's actions and draws the next tile's normals; the statistics' per-column float
// mean and denominator come from LDS (rms_norm's operations, so the same bits).
constexpr int OT = TB - 64;
constexpr int NUO3 = (RB * XS + OT - 1) / OT;
__device__ __forceinline__ void load_obs_tile3(const float *__restrict__ obs, int n, int tile, int tt,
                                               float (&x)[NUO3]) {
  const int row0 = tile * RB, nrows = min(RB, n - row0);
#pragma unroll
  for (int u = 0; u < NUO3; ++u) {
    const int q = min(tt + u * OT, RB * XS - 1);
    const int r = min(q / XS, nrows - 1), kc = min(q % XS, NIN - 1);
    x[u] = obs[(size_t)(row0 + r) * NIN + kc];
  }
}
template <class S>
__device__ __forceinline__ void put_obs_tile3(const float (&x)[NUO3], int tt, int row0, int nrows, bool normalize,
                                              float eps, S &s, float *exp_obs, int H, int t) {
#pragma unroll
  for (int u = 0; u < NUO3; ++u) {
    const int q = tt + u * OT;
    if (q >= RB * XS) continue;
    const int r = q / XS, k = q % XS;
    float v = 0.f;
    if (r < nrows && k < NIN) {
      v = x[u];
      exp_st(&exp_obs[((size_t)(row0 + r) * H + t) * NIN + k], v);
      if (normalize) v = clampt((v - s.om[k]) / s.od[k], -5.0f, 5.0f);   // = rms_norm
    }
    s.x[q] = v;
  }
}

template <class S>
__device__ __forceinline__ void block_heads(S &s);

// Forward of the RB rows staged in s.x (W1, biases, heads staged; W2 still in
// registers on a launch's first tile, committed after layer 1); leaves h1, h2, out.
// fp32 always: the reference's mixed_precision autocast covers calc_gradients only
// (a2c_continuous.py:121); get_action_values / get_values run in fp32 under no_grad.
__device__ void block_forward(const StagedW &wr, MlpSmem &s, bool first_tile) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 31, h = lane >> 5, n0 = 32 * w;
  // ---- layer 1: h1 = tanh(x W1^T + b1), K = 34 (k = 33 is zero) ----
  {
    f32x16 acc = {};
#pragma unroll
    for (int st = 0; st < 17; ++st) {
      const int k = 2 * st + h;
      acc = mfma32(s.x[i * XS + k], s.w1[(n0 + i) * XS + k], acc);
    }
    const float bj = s.b1[n0 + i];
#pragma unroll
    for (int r = 0; r < 16; ++r) s.h1[crow(r, h) * HS + n0 + i] = fast_tanh(acc[r] + bj);
  }
  if (first_tile) stage_store_w2(wr, s);   // nothing else writes s.w2: later tiles reuse it
  __syncthreads();
  // ---- layer 2: h2 = tanh(h1 W2^T + b2) ----
  {
    f32x16 acc = {};
#pragma unroll 16
    for (int st = 0; st < NH / 2; ++st) {
      const int k = 2 * st + h;
      acc = mfma32(s.h1[i * HS + k], s.w2[(n0 + i) * HS + k], acc);
    }
    const float bj = s.tail[T_B2 + n0 + i];
#pragma unroll
    for (int r = 0; r < 16; ++r) s.h2[crow(r, h) * HS + n0 + i] = fast_tanh(acc[r] + bj);
  }
  __syncthreads();
  block_heads(s);
}

// heads: mu = Wmu h2 + bmu, value = Wv h2 + bv (8 threads per row, k = part + 8 kk: the 8 threads of a row read 8
// consecutive words, not 8 words 16 apart -- no 4-way bank conflicts)
template <class S>
__device__ __forceinline__ void block_heads(S &s) {
  const int tid = threadIdx.x;
  {
    const int r = tid / 8, part = tid % 8;
    float a0 = 0.f, a1 = 0.f, av = 0.f;
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      const int k = part + 8 * kk;
      const float hv = s.h2[r * HS + k];
      a0 = fmaf(s.tail[T_WMU + k], hv, a0);
      a1 = fmaf(s.tail[T_WMU + NH + k], hv, a1);
      av = fmaf(s.tail[T_WV + k], hv, av);
    }
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) {
      a0 += __shfl_xor(a0, m, 64);
      a1 += __shfl_xor(a1, m, 64);
      av += __shfl_xor(av, m, 64);
    }
    if (part == 0) {
      s.out[r * 4 + 0] = a0 + s.tail[T_BMU];
      s.out[r * 4 + 1] = a1 + s.tail[T_BMU + 1];
      s.out[r * 4 + 2] = av + s.tail[T_BV];
    }
  }
  __syncthreads();
}

// The policy step with its weights in registers: wave w keeps rows 32w..32w+31 of W1 and W2 as the B operands of
// its matrix-core steps (lane (i, h) of step st holds W[32w + i][2 st + h]: 17 + 64 VGPRs) and the two biases, so
// the workgroup needs 41 KB of LDS instead of 129 KB and two of them share a CU (2 waves per SIMD instead of
// one; USV_POL_WPC).  The products see the same operands in the same order as block_forward's: the same bits.
#ifndef USV_POL_WPC
#define USV_POL_WPC 2
#endif
constexpr int POL_WPC = USV_POL_WPC;
#ifndef USV_POL_L2B
#define USV_POL_L2B 1   // layer 2 of the register-weight form: a scheduling fence every 16 steps
#endif
struct PolSmem {
  float x[RB * XS];       // normalised obs
  float h1[RB * HS];
  float h2[RB * HS];
  float out[RB * 4];      // mu0, mu1, value
  float tail[TAIL + 1];   // params from b2 on (T_* offsets)
  float om[NIN], od[NIN]; // (float)mean, sqrtf((float)var + eps) of the obs statistics
  float zz[2][RB * 2];    // the N(0,1) draws of a tile's rows, one tile ahead
};
struct RegW {
  float w1[17], w2[NH / 2], b1, b2, tlr[NTL];
  float hm0[NH / 8], hm1[NH / 8], hv[NH / 8];   // the heads' weights at k = tid % 8 + 8 kk (block_heads' k)
};
__device__ __forceinline__ void regw_load(const float *__restrict__ P, RegW &r) {
  const int tid = threadIdx.x, lane = tid & 63, i = lane & 31, h = lane >> 5, n = 32 * (tid >> 6) + i;
#pragma unroll
  for (int st = 0; st < 17; ++st) r.w1[st] = P[PPO_OFF_W1 + n * NIN + min(2 * st + h, NIN - 1)];
  r.b1 = P[PPO_OFF_B1 + n];
  r.b2 = P[PPO_OFF_B2 + n];
#pragma unroll
  for (int kk = 0; kk < NH / 8; ++kk) {
    const int k = (tid & 7) + 8 * kk;
    r.hm0[kk] = P[PPO_OFF_WMU + k];
    r.hm1[kk] = P[PPO_OFF_WMU + NH + k];
    r.hv[kk] = P[PPO_OFF_WV + k];
  }
#pragma unroll
  for (int u = 0; u < NTL; ++u) r.tlr[u] = P[PPO_OFF_B2 + min(tid + u * TB, TAIL - 1)];
#pragma unroll
  for (int st = 0; st < NH / 2; ++st) r.w2[st] = P[PPO_OFF_W2 + n * NH + 2 * st + h];
  __builtin_amdgcn_sched_barrier(0);
  static_assert(2 * 16 + 1 == NIN, "k = 33 is layer 1's only zero column");
  if (h) r.w1[16] = 0.f;
}
__device__ __forceinline__ void regw_store_tail(const RegW &r, PolSmem &s) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int u = 0; u < NTL; ++u)
    if (tid + u * TB < TAIL) s.tail[tid + u * TB] = r.tlr[u];
}
// probe build: per-phase wall-clock sums over a workgroup's tiles (wave 0's view), slots 5.. of g_probe_pol
#ifdef USV_PHASE_PROBE
struct PolAcc {
  unsigned long long t, d[6];
  __device__ void mark(int k) {
    const unsigned long long q = wall_clock64();
    d[k] += q - t;
    t = q;
  }
};
#else
struct PolAcc {
  __device__ void mark(int) {}
};
#endif
__device__ __forceinline__ void block_forward_rw(const RegW &wr, PolSmem &s, PolAcc &pa) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 31, h = lane >> 5, n0 = 32 * w;
  {
    f32x16 acc = {};
#pragma unroll
    for (int st = 0; st < 17; ++st) acc = mfma32(s.x[i * XS + 2 * st + h], wr.w1[st], acc);
#pragma unroll
    for (int r = 0; r < 16; ++r) s.h1[crow(r, h) * HS + n0 + i] = fast_tanh(acc[r] + wr.b1);
  }
  __syncthreads();
  pa.mark(1);
  {
    f32x16 acc = {};
#pragma unroll
    for (int st = 0; st < NH / 2; ++st) {
      acc = mfma32(s.h1[i * HS + 2 * st + h], wr.w2[st], acc);
      // at most 16 operand reads in flight (a fully hoisted loop would hold 64 of them in registers)
      if (USV_POL_L2B && st % 16 == 15) __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) s.h2[crow(r, h) * HS + n0 + i] = fast_tanh(acc[r] + wr.b2);
  }
  __syncthreads();
  pa.mark(2);
  {   // block_heads with the head weights from registers (the same fmaf chains)
    const int r = tid / 8, part = tid % 8;
    float a0 = 0.f, a1 = 0.f, av = 0.f;
#pragma unroll
    for (int kk = 0; kk < NH / 8; ++kk) {
      const float hv = s.h2[r * HS + part + 8 * kk];
      a0 = fmaf(wr.hm0[kk], hv, a0);
      a1 = fmaf(wr.hm1[kk], hv, a1);
      av = fmaf(wr.hv[kk], hv, av);
    }
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) {
      a0 += __shfl_xor(a0, m, 64);
      a1 += __shfl_xor(a1, m, 64);
      av += __shfl_xor(av, m, 64);
    }
    if (part == 0) {
      s.out[r * 4 + 0] = a0 + s.tail[T_BMU];
      s.out[r * 4 + 1] = a1 + s.tail[T_BMU + 1];
      s.out[r * 4 + 2] = av + s.tail[T_BV];
    }
  }
  __syncthreads();
  pa.mark(3);
}

// ------------------------------------------------------------------ rollout
// workgroups of the persistent forward kernels: one 32-row tile each up to 256
// (one per CU at this LDS size), then tiles loop
__host__ __device__ constexpr int policy_grid(int n) {
  return (n + RB - 1) / RB < 256 ? (n + RB - 1) / RB : 256;
}
// kRW: the register-weight form (PolSmem / RegW above), grid up to 256 x POL_WPC workgroups; else the weights
// staged in LDS once per workgroup, one workgroup per CU
template <bool kRW>
__global__ __launch_bounds__(TB, kRW ? POL_WPC : 1) void k_policy_step(ppo_cfg_t c, const float *__restrict__ P,
                                                    const double *__restrict__ obs_rms,
                                                    const double *__restrict__ val_rms, const float *__restrict__ obs,
                                                    int t, float *exp_obs, float *exp_act, float *exp_nlp,
                                                    float *exp_val, float *exp_mu, float *exp_sigma, uint8_t *exp_done,
                                                    const int64_t *__restrict__ dones_prev, float *actions_out,
                                                    uint64_t seed, uint64_t step, const uint64_t *step_dev,
                                                    const float *eps_inject) {
  __shared__ std::conditional_t<kRW, PolSmem, MlpSmem> s;
  USV_PHASE(pol, 0);
  const int n = c.n_envs, H = c.horizon;
  if (step_dev) step = *step_dev + (uint64_t)t;   // the rollout's first step + slot
  // persistent over 32-row tiles: the weights are staged once per workgroup, not once per tile.
  // Per tile: the forward on all four waves; then wave 0 samples the tile's actions, stores its
  // experience rows and draws the next tile's normals while waves 1-3 stage the next tile's obs
  // (loaded during the forward) -- one barrier per tile outside the forward
  std::conditional_t<kRW, RegW, StagedW> wr;
  if constexpr (kRW) regw_load(P, wr);
  else stage_load(P, wr);
  const int ntiles = (n + RB - 1) / RB;
  const int w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int tt = (int)threadIdx.x - 64;
  const bool normalize = c.normalize_input != 0;
  if ((int)blockIdx.x >= ntiles) return;   // (the grid is at most ntiles; uniform)
  // N(0,1) draws of tile `tl`'s rows (wave 0, lane = row) into s.zz[buf]
  // (lane 32 j + r of wave 0: row r's component j -- the two components' transcendentals in parallel)
  auto draw = [&](int tl, int buf) {
    if (w == 0) {
      const int r = lane & (RB - 1), j = lane >> 5;
      const int e = min(tl * RB + r, n - 1);
      float zj;
      if (eps_inject) {
        zj = eps_inject[2 * e + j];
      } else {  // Normal.sample via Box-Muller on Philox(site 0x200): z_j from (u[2 j], u[2 j + 1])
        float u[4];
        philox_u4(seed, (uint32_t)e, step, 0x200u, u);
        const float ua = j ? u[2] : u[0], ub = j ? u[3] : u[1];
        const float rr = sqrtf(-2.0f * logf(1.0f - ua));
        zj = rr * cosf(USV_2PI_F * ub);
      }
      s.zz[buf][2 * r + j] = zj;
    }
  };
  if (threadIdx.x < NIN) {
    s.om[threadIdx.x] = (float)obs_rms[threadIdx.x];
    s.od[threadIdx.x] = sqrtf((float)obs_rms[NIN + threadIdx.x] + c.rms_eps);
  }
  float xo[NUO3];
  if (w > 0) load_obs_tile3(obs, n, blockIdx.x, tt, xo);
  __syncthreads();
  if (w > 0) {
    const int row0 = blockIdx.x * RB;
    put_obs_tile3(xo, tt, row0, min(RB, n - row0), normalize, c.rms_eps, s, exp_obs, H, t);
  }
  draw(blockIdx.x, 0);
  if constexpr (kRW) regw_store_tail(wr, s);
  else stage_store_small(wr, s);
  __syncthreads();
  int buf = 0;
  PolAcc pa{};
#ifdef USV_PHASE_PROBE
  pa.t = wall_clock64();
#endif
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const int row0 = tile * RB;
  const int nrows = min(RB, n - row0);
  const int nt = tile + (int)gridDim.x;
  float xn[NUO3];   // the next tile's rows, in flight during the forward
  // the obs path's slot indices recomputed per tile (opaque to the optimiser): hoisted out of the loop they held
  // ~50 VGPRs through the forward, which the register-weight form cannot spare
  int ttv = tt;
  if constexpr (kRW) __asm__ volatile("" : "+v"(ttv));
  if (w > 0 && nt < ntiles) load_obs_tile3(obs, n, nt, ttv, xn);
  USV_PHASE(pol, 1);   // (probe slots 1-4: the launch's last tile)
  USV_PHASE(pol, 2);
  pa.mark(0);
  if constexpr (kRW) block_forward_rw(wr, s, pa);
  else block_forward(wr, s, tile == (int)blockIdx.x);
  USV_PHASE(pol, 3);
  if (w == 0) {
    // lane 32 j + r: row r's action component j; the neglogp's two terms meet by one cross-half exchange
    const int r = lane & (RB - 1), j = lane >> 5;
    const bool rowok = r < nrows;
    const int e = row0 + (rowok ? r : 0);
    const size_t slot = (size_t)e * H + t;
    const float muj = s.out[r * 4 + j];
    const float lsj = muj * 0.f + P[PPO_OFF_SIGMA + j];
    const float sgj = expf(lsj);
    const float aj = muj + sgj * s.zz[buf][2 * r + j];
    const float qj = (aj - muj) / sgj;
    const float qo = __shfl_xor(qj, 32, 64), lso = __shfl_xor(lsj, 32, 64);
    const float q0 = j ? qo : qj, q1 = j ? qj : qo, ls0 = j ? lso : lsj, ls1 = j ? lsj : lso;
    if (rowok) {
      exp_st(&exp_act[slot * 2 + j], aj);
      exp_st(&exp_mu[slot * 2 + j], muj);
      exp_st(&exp_sigma[slot * 2 + j], sgj);
      // preprocess_actions: clamp(-1,1) then rescale to [low, high] = identity (a2c_common.py:1134-1144)
      actions_out[2 * e + j] = clampt(aj, -1.0f, 1.0f);
      if (j == 0) {
        const float nlp = 0.5f * (q0 * q0 + q1 * q1) + kLog2Pi + (ls0 + ls1);
        float vd = s.out[r * 4 + 2];
        if (c.normalize_value) {  // denorm_value (running_mean_std.py:113-115)
          vd = clampt(vd, -5.0f, 5.0f);
          vd = sqrtf((float)val_rms[1] + c.rms_eps) * vd + (float)val_rms[0];
        }
        exp_st(&exp_nlp[slot], nlp);
        exp_st(&exp_val[slot], vd);
        exp_st(&exp_done[slot], (uint8_t)(dones_prev[e] != 0));
      }
    }
    if (c.nan_probe && c.nan_flag) {   // wave 0, uniform
      const bool bad = lane < nrows && (nonfinite(s.out[lane * 4]) | nonfinite(s.out[lane * 4 + 1]) |
                                        nonfinite(s.out[lane * 4 + 2]));
      nan_report(c.nan_flag, bad ? USV_NAN_POLICY : 0u);
    }
    if (nt < ntiles) draw(nt, buf ^ 1);
  } else if (nt < ntiles) {   // s.x was last read by the forward's layer 1 (before its first barrier)
    put_obs_tile3(xn, ttv, nt * RB, min(RB, n - nt * RB), normalize, c.rms_eps, s, exp_obs, H, t);
  }
  __syncthreads();   // s.out / s.zz[buf] read above before the next tile's forward and draws rewrite them
  USV_PHASE(pol, 4);
  pa.mark(4);
  buf ^= 1;
  }
#ifdef USV_PHASE_PROBE
  if (threadIdx.x == 0 && blockIdx.x < 4096)
    for (int k = 0; k < 5; ++k) g_probe_pol[blockIdx.x][5 + k] = pa.d[k];
#endif
}

// kRW: the register-weight form of the policy step (RegW / PolSmem), up to 256 x POL_WPC workgroups
template <bool kRW>
__global__ __launch_bounds__(TB, kRW ? POL_WPC : 1) void k_value(ppo_cfg_t c, const float *__restrict__ P,
                                                                 const double *obs_rms, const double *val_rms,
                                                                 const float *__restrict__ obs, float *values) {
  __shared__ std::conditional_t<kRW, PolSmem, MlpSmem> s;
  const int n = c.n_envs;
  std::conditional_t<kRW, RegW, StagedW> wr;
  if constexpr (kRW) regw_load(P, wr);
  else stage_load(P, wr);
  PolAcc pa{};
  const int ntiles = (n + RB - 1) / RB;
  ObsCols oc;
  load_obs_cols(obs_rms, oc);
  float xo[NUO];
  load_obs_tile(obs, n, min((int)blockIdx.x, ntiles - 1), xo);
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {   // persistent, as k_policy_step
    const int row0 = tile * RB;
    const int nrows = min(RB, n - row0);
    float xn[NUO];
    load_obs_tile(obs, n, min(tile + (int)gridDim.x, ntiles - 1), xn);
    put_obs_tile(xo, oc, row0, nrows, c.normalize_input != 0, c.rms_eps, s, nullptr, 0, 0);
    if (tile == (int)blockIdx.x) {
      if constexpr (kRW) regw_store_tail(wr, s);
      else stage_store_small(wr, s);
    }
    __syncthreads();
    if constexpr (kRW) block_forward_rw(wr, s, pa);
    else block_forward(wr, s, tile == (int)blockIdx.x);
    const int r = threadIdx.x;
    if (r < nrows) {
      float vd = s.out[r * 4 + 2];
      if (c.normalize_value) {
        vd = clampt(vd, -5.0f, 5.0f);
        vd = sqrtf((float)val_rms[1] + c.rms_eps) * vd + (float)val_rms[0];
      }
      values[row0 + r] = vd;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NUO; ++u) xo[u] = xn[u];
  }
}

// rewards_shaper + episode meters (a2c_common.py:721-759, tr_helpers.py:33-43).
// meter = [H][4] per-slot sums (reward of done envs, shaped reward, length, count),
// then [H][nblk][4] per-workgroup partials: every workgroup stores its sums (no
// float atomics), k_meter_fold adds them in workgroup order after the last slot,
// so the meters are bit-identical run to run (graph replay == eager).
constexpr int kStoreTB = 256;
__global__ __launch_bounds__(kStoreTB) void k_store_reward(ppo_cfg_t c, const float *__restrict__ rew, const int64_t *__restrict__ dones, int t,
                               float *exp_rew, float *cur_rew, float *cur_shaped, float *cur_len, float *meter,
                               uint64_t *step_dev) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  // the rollout's Philox step advances by the horizon after its last slot (the policy kernel of slot t
  // reads step_dev + t, so no policy launch depends on this kernel within a rollout)
  if (step_dev && e == 0 && t == c.horizon - 1) *step_dev += (uint64_t)c.horizon;
  const int n = c.n_envs;
  float s_rew = 0.f, s_shaped = 0.f, s_len = 0.f, s_cnt = 0.f;
  if (e < n) {
    const float r = rew[e];
    const float shaped = (r + c.reward_shift) * c.reward_scale;
    exp_rew[(size_t)e * c.horizon + t] = shaped;
    const float cr = cur_rew[e] + r, cs = cur_shaped[e] + shaped, cl = cur_len[e] + 1.0f;
    const bool d = dones[e] != 0;
    if (d) { s_rew = cr; s_shaped = cs; s_len = cl; s_cnt = 1.f; }
    const float nd = 1.0f - (float)d;
    cur_rew[e] = cr * nd;
    cur_shaped[e] = cs * nd;
    cur_len[e] = cl * nd;
  }
  s_rew = wave_sum(s_rew); s_shaped = wave_sum(s_shaped); s_len = wave_sum(s_len); s_cnt = wave_sum(s_cnt);
  __shared__ float red[kStoreTB / 64][4];
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[wv][0] = s_rew; red[wv][1] = s_shaped; red[wv][2] = s_len; red[wv][3] = s_cnt; }
  __syncthreads();
  if (threadIdx.x < 4) {
    float a = red[0][threadIdx.x];
#pragma unroll
    for (int w = 1; w < kStoreTB / 64; ++w) a += red[w][threadIdx.x];
    meter[c.horizon * 4 + ((size_t)t * gridDim.x + blockIdx.x) * 4 + threadIdx.x] = a;
  }
}

// meter[t][q] = sum over workgroups (in order) of the slot's partials; 64 threads = 16 slots x 4
__global__ void k_meter_fold(ppo_cfg_t c, float *meter, int nblk) {
  const int tq = blockIdx.x * blockDim.x + threadIdx.x;
  if (tq >= c.horizon * 4) return;
  const int t = tq >> 2, q = tq & 3;
  const float *part = meter + c.horizon * 4 + (size_t)t * nblk * 4 + q;
  float a = 0.f;
  constexpr int U = 16;   // loads in flight, added in workgroup order
  for (int b0 = 0; b0 < nblk; b0 += U) {
    float x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = part[(size_t)min(b0 + u, nblk - 1) * 4];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b0 + u < nblk) a += x[u];
  }
  meter[tq] = a;
}

// ---------------------------------------------------------- GAE + stats ---
// work (doubles): [0..5] sums (v, v^2, ret, ret^2, adv, adv^2) accumulated
// per block into work[8 + 8*blk ...]; finalize in k_prepare_finalize.
// kH > 0: the horizon as a compile-time constant (16, the packaged configs): an env's kH rows of val / rew / done
// are loaded up front as 16-byte vectors and ret / adv stored the same way (the runtime-H loop issued one dependent
// round of scattered 4-byte loads per slot: 63 us per epoch at 131072 envs); the same operations in the same order
template <int kH>
__global__ __launch_bounds__(TB) void k_gae(ppo_cfg_t c, const float *__restrict__ last_val,
                                            const int64_t *__restrict__ last_dones, const uint8_t *__restrict__ done,
                                            const float *__restrict__ val, const float *__restrict__ rew, float *ret,
                                            float *adv, double *work) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int H = kH > 0 ? kH : c.horizon;
  double sv = 0, sv2 = 0, sr = 0, sr2 = 0, sa = 0, sa2 = 0;
  if (e < c.n_envs) {
    const size_t base = (size_t)e * H;
    float lastgaelam = 0.f;
    if constexpr (kH > 0) {
      static_assert(kH % 16 == 0, "16-byte row vectors");
      float v[kH], rw[kH], R[kH], A[kH];
      uint8_t d[kH];
#pragma unroll
      for (int q = 0; q < kH / 4; ++q) {
        const float4 a = reinterpret_cast<const float4 *>(val + base)[q];
        const float4 b = reinterpret_cast<const float4 *>(rew + base)[q];
        v[4 * q] = a.x; v[4 * q + 1] = a.y; v[4 * q + 2] = a.z; v[4 * q + 3] = a.w;
        rw[4 * q] = b.x; rw[4 * q + 1] = b.y; rw[4 * q + 2] = b.z; rw[4 * q + 3] = b.w;
      }
#pragma unroll
      for (int q = 0; q < kH / 16; ++q) {
        const uint4 dd = reinterpret_cast<const uint4 *>(done + base)[q];
        const uint32_t w4[4] = {dd.x, dd.y, dd.z, dd.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) d[16 * q + j] = (uint8_t)(w4[j >> 2] >> (8 * (j & 3)));
      }
      const float nnt_last = 1.0f - (float)(last_dones[e] != 0), nv_last = last_val[e];
#pragma unroll
      for (int t = kH - 1; t >= 0; --t) {
        const float nnt = t == kH - 1 ? nnt_last : 1.0f - (float)d[t + 1];
        const float nv = t == kH - 1 ? nv_last : v[t + 1];
        const float delta = rw[t] + c.gamma * nv * nnt - v[t];
        lastgaelam = delta + c.gamma * c.tau * nnt * lastgaelam;
        R[t] = lastgaelam + v[t];
        A[t] = R[t] - v[t];
        sv += v[t]; sv2 += (double)v[t] * v[t]; sr += R[t]; sr2 += (double)R[t] * R[t];
        sa += A[t]; sa2 += (double)A[t] * A[t];
      }
#pragma unroll
      for (int q = 0; q < kH / 4; ++q) {
        reinterpret_cast<float4 *>(ret + base)[q] = make_float4(R[4 * q], R[4 * q + 1], R[4 * q + 2], R[4 * q + 3]);
        reinterpret_cast<float4 *>(adv + base)[q] = make_float4(A[4 * q], A[4 * q + 1], A[4 * q + 2], A[4 * q + 3]);
      }
    } else {
      for (int t = H - 1; t >= 0; --t) {
        float nnt, nv;
        if (t == H - 1) {
          nnt = 1.0f - (float)(last_dones[e] != 0);
          nv = last_val[e];
        } else {
          nnt = 1.0f - (float)done[base + t + 1];
          nv = val[base + t + 1];
        }
        const float v = val[base + t];
        const float delta = rew[base + t] + c.gamma * nv * nnt - v;
        lastgaelam = delta + c.gamma * c.tau * nnt * lastgaelam;
        const float R = lastgaelam + v;          // returns = advs + values (:763)
        const float A = R - v;                   // prepare_dataset :1269
        ret[base + t] = R;
        adv[base + t] = A;
        sv += v; sv2 += (double)v * v; sr += R; sr2 += (double)R * R; sa += A; sa2 += (double)A * A;
      }
    }
  }
  __shared__ double red[6][TB / 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double vals[6] = {sv, sv2, sr, sr2, sa, sa2};
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    double x = vals[q];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    if (lane == 0) red[q][wid] = x;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    double x = 0;
    for (int w = 0; w < TB / 64; ++w) x += red[threadIdx.x][w];
    work[8 + (size_t)blockIdx.x * 8 + threadIdx.x] = x;
  }
}

__device__ __forceinline__ void rms_merge(double *rm, int len, const double *bmean, const double *bvar, double bcount) {
  // _update_mean_var_count_from_moments (running_mean_std.py:29-39); count at rm[2*len]
  const double count = rm[2 * len];
  const double tot = count + bcount;
  for (int k = 0; k < len; ++k) {
    const double delta = bmean[k] - rm[k];
    const double new_mean = rm[k] + delta * bcount / tot;
    const double m_a = rm[len + k] * count;
    const double m_b = bvar[k] * bcount;
    const double M2 = m_a + m_b + delta * delta * count * bcount / tot;
    rm[k] = new_mean;
    rm[len + k] = M2 / tot;
  }
  rm[2 * len] = tot;
}

// One 256-thread workgroup: thread t folds the block partials t, t + 256, ... in order, then a
// fixed LDS tree (deterministic, independent of timing) -- the serial fold of 512 partials by one
// thread was 116 us per epoch at 131072 envs
constexpr int FIN_TB = 256;
__global__ __launch_bounds__(FIN_TB) void k_prepare_finalize(ppo_cfg_t c, double *val_rms, double *work, int nblk) {
  __shared__ double red[6][FIN_TB];
  const int tid = threadIdx.x;
  {
    double a[6] = {0, 0, 0, 0, 0, 0};
    constexpr int U = 4;   // partial rows in flight per thread
    for (int b0 = tid; b0 < nblk; b0 += U * FIN_TB) {
      double x[U][6];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int b = min(b0 + u * FIN_TB, nblk - 1);
#pragma unroll
        for (int q = 0; q < 6; ++q) x[u][q] = work[8 + (size_t)b * 8 + q];
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (b0 + u * FIN_TB < nblk) {
#pragma unroll
          for (int q = 0; q < 6; ++q) a[q] += x[u][q];
        }
    }
#pragma unroll
    for (int q = 0; q < 6; ++q) red[q][tid] = a[q];
  }
  __syncthreads();
  for (int wdt = FIN_TB / 2; wdt > 0; wdt >>= 1) {
    if (tid < wdt) {
#pragma unroll
      for (int q = 0; q < 6; ++q) red[q][tid] += red[q][tid + wdt];
    }
    __syncthreads();
  }
  if (tid != 0) return;
  double s[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) s[q] = red[q][0];
  const double B = (double)c.n_envs * c.horizon;
  const double mv = s[0] / B, vv = (s[1] - B * mv * mv) / (B - 1.0);
  const double mr = s[2] / B, vr = (s[3] - B * mr * mr) / (B - 1.0);
  const double ma = s[4] / B, va = (s[5] - B * ma * ma) / (B - 1.0);
  // value_mean_std.train(); values = vms(values); returns = vms(returns) (:1271-1275)
  double stats_v[2] = {0.0, 1.0}, stats_r[2] = {0.0, 1.0};
  if (c.normalize_value) {
    rms_merge(val_rms, 1, &mv, &vv, B);
    stats_v[0] = val_rms[0]; stats_v[1] = val_rms[1];
    rms_merge(val_rms, 1, &mr, &vr, B);
    stats_r[0] = val_rms[0]; stats_r[1] = val_rms[1];
  }
  work[0] = stats_v[0]; work[1] = stats_v[1];
  work[2] = stats_r[0]; work[3] = stats_r[1];
  work[4] = ma;
  work[5] = sqrt(va > 0 ? va : 0.0);
}

__global__ void k_prepare_apply(ppo_cfg_t c, const double *work, float *val, float *ret, float *adv) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t B = (size_t)c.n_envs * c.horizon;
  if (i >= B) return;
  if (c.normalize_value) {
    val[i] = rms_norm(val[i], work[0], work[1], c.rms_eps);
    ret[i] = rms_norm(ret[i], work[2], work[3], c.rms_eps);
  }
  if (c.normalize_advantage) {
    // (adv - adv.mean()) / (adv.std() + 1e-8)  (:1287)
    adv[i] = (adv[i] - (float)work[4]) / ((float)work[5] + 1e-8f);
  }
}

// ------------------------------------------------------- obs RMS (mb) -----
// RunningMeanStd.train on the minibatch obs (running_mean_std.py:29-39, 84-111):
// each workgroup sums a chunk of rows for all 33 columns (fp64) into
// part[blk][66]; the last workgroup to finish (counter *cnt) folds the
// partials in block order and merges them into the running statistics.
__global__ __launch_bounds__(TB) void k_obs_stats(ppo_cfg_t c, const float *__restrict__ obs, int row0, int rows,
                                                  double *part, double *obs_rms, unsigned *cnt) {
  __shared__ double acc[2][NIN][TB / NIN + 1];
  __shared__ bool last;
  const int tid = threadIdx.x;
  const int col = tid % NIN, lane_r = tid / NIN;   // 7 row-lanes x 33 cols
  const int nl = TB / NIN;
  double s = 0, s2 = 0;
  if (lane_r < nl) {
    const int chunk = (rows + gridDim.x - 1) / gridDim.x;
    const int a = blockIdx.x * chunk, bnd = min(rows, a + chunk);
    // rows a + lane_r, + nl, ... in that order; 8 loads in flight per batch
    for (int r0 = a + lane_r; r0 < bnd; r0 += 8 * nl) {
      float xv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) xv[u] = obs[(size_t)(row0 + min(r0 + u * nl, bnd - 1)) * NIN + col];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (r0 + u * nl < bnd) {
          const double x = xv[u];
          s += x; s2 += x * x;
        }
    }
    acc[0][col][lane_r] = s;
    acc[1][col][lane_r] = s2;
  }
  __syncthreads();
  if (tid < NIN) {
    double t = 0, t2 = 0;
    for (int l = 0; l < nl; ++l) { t += acc[0][tid][l]; t2 += acc[1][tid][l]; }
    part[(size_t)blockIdx.x * 2 * NIN + tid] = t;
    part[(size_t)blockIdx.x * 2 * NIN + NIN + tid] = t2;
  }
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    last = atomicAdd(cnt, 1u) == gridDim.x - 1;
    __threadfence();
  }
  __syncthreads();
  if (!last) return;
  const double count = obs_rms[2 * NIN];
  if (tid < NIN) {
    const int k = tid;
    double sa = 0, sb = 0;
#pragma unroll 8
    for (int bb = 0; bb < (int)gridDim.x; ++bb) {
      sa += part[(size_t)bb * 2 * NIN + k];
      sb += part[(size_t)bb * 2 * NIN + NIN + k];
    }
    const double bmean = sa / rows;
    const double bvar = (sb - rows * bmean * bmean) / (rows - 1.0);
    const double tot = count + (double)rows;
    const double delta = bmean - obs_rms[k];
    const double M2 = obs_rms[NIN + k] * count + bvar * rows + delta * delta * count * rows / tot;
    obs_rms[k] = obs_rms[k] + delta * rows / tot;
    obs_rms[NIN + k] = M2 / tot;
  }
  __syncthreads();
  if (tid == 0) {
    obs_rms[2 * NIN] = count + (double)rows;
    *cnt = 0u;
  }
}

// ---------------------------------------------- obs RMS over one epoch ----
// RunningMeanStd.train in mini-epoch 0 (a2c_common.py:1243-1244, running_mean_std.py:44-111)
// depends only on the rollout's observations, so the whole sequence of running statistics is
// formed once per epoch: k_obs_moments sums each minibatch's columns (fp64, OM_CH row chunks per
// minibatch), k_obs_rms_seq merges them in minibatch order (Chan's formula as k_obs_stats) and
// writes the statistics after merge k to seq[k] -- what minibatch k normalises with -- and the
// final state to obs_rms.  Two launches per epoch instead of one per minibatch.
constexpr int OM_CH = 8;
__global__ __launch_bounds__(TB) void k_obs_moments(ppo_cfg_t c, const float *__restrict__ obs, double *part) {
  __shared__ double acc[2][NIN][TB / NIN + 1];
  const int tid = threadIdx.x, mb = blockIdx.x, ch = blockIdx.y;
  const int col = tid % NIN, lane_r = tid / NIN, nl = TB / NIN;
  const int M = c.minibatch, chunk = (M + OM_CH - 1) / OM_CH;
  const int a = mb * M + ch * chunk, bnd = mb * M + min(M, (ch + 1) * chunk);
  double s = 0, s2 = 0;
  if (lane_r < nl) {
    for (int r0 = a + lane_r; r0 < bnd; r0 += 8 * nl) {
      float xv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) xv[u] = obs[(size_t)min(r0 + u * nl, bnd - 1) * NIN + col];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (r0 + u * nl < bnd) {
          const double x = xv[u];
          s += x; s2 += x * x;
        }
    }
    acc[0][col][lane_r] = s;
    acc[1][col][lane_r] = s2;
  }
  __syncthreads();
  if (tid < NIN) {
    double t = 0, t2 = 0;
    for (int l = 0; l < nl; ++l) { t += acc[0][tid][l]; t2 += acc[1][tid][l]; }
    double *o = part + ((size_t)mb * OM_CH + ch) * 2 * NIN;
    o[tid] = t;
    o[NIN + tid] = t2;
  }
}

// One 256-thread workgroup.  Phase 1 (all threads, parallel over (minibatch, column)): each
// minibatch's moments (bmean, unbiased bvar), staged in seq[mb] itself.  Phase 2 (thread k < 33):
// Chan's merge in minibatch order -- the only serial part -- reading 8 minibatches' moments ahead
// of the dependent fp64 chain, writing the running (mean, var) over them.
constexpr int RS_TB = 256, RS_U = 8;
__global__ __launch_bounds__(RS_TB) void k_obs_rms_seq(ppo_cfg_t c, const double *__restrict__ part, int nmb,
                                                       double *obs_rms, double *seq) {
  const double rows = (double)c.minibatch;
  for (int q = threadIdx.x; q < nmb * NIN; q += RS_TB) {
    const int mb = q / NIN, k = q % NIN;
    double sa = 0, sb = 0;
#pragma unroll
    for (int ch = 0; ch < OM_CH; ++ch) {
      const double *o = part + ((size_t)mb * OM_CH + ch) * 2 * NIN;
      sa += o[k];
      sb += o[NIN + k];
    }
    const double bmean = sa / rows;
    seq[(size_t)mb * 2 * NIN + k] = bmean;
    seq[(size_t)mb * 2 * NIN + NIN + k] = (sb - rows * bmean * bmean) / (rows - 1.0);
  }
  __syncthreads();   // (workgroup-scope release / acquire of the staged moments)
  const int k = threadIdx.x;
  if (k < NIN) {
    double mean = obs_rms[k], var = obs_rms[NIN + k], count = obs_rms[2 * NIN];
    for (int mb0 = 0; mb0 < nmb; mb0 += RS_U) {
      double bm[RS_U], bv[RS_U];
#pragma unroll
      for (int u = 0; u < RS_U; ++u) {
        const int mb = min(mb0 + u, nmb - 1);
        bm[u] = seq[(size_t)mb * 2 * NIN + k];
        bv[u] = seq[(size_t)mb * 2 * NIN + NIN + k];
      }
#pragma unroll
      for (int u = 0; u < RS_U; ++u) {
        if (mb0 + u >= nmb) break;
        const double tot = count + rows;
        const double delta = bm[u] - mean;
        const double M2 = var * count + bv[u] * rows + delta * delta * count * rows / tot;
        mean = mean + delta * rows / tot;
        var = M2 / tot;
        count = tot;
        seq[(size_t)(mb0 + u) * 2 * NIN + k] = mean;
        seq[(size_t)(mb0 + u) * 2 * NIN + NIN + k] = var;
      }
    }
    obs_rms[k] = mean;
    obs_rms[NIN + k] = var;
    if (k == 0) obs_rms[2 * NIN] = count;   // (every thread's count is the same)
  }
}

// ------------------------------------------------------ minibatch grad ----
// One 512-thread workgroup (8 waves, two per SIMD) per 32 minibatch rows, 256
// workgroups for a 8192-row minibatch (every CU).  The second wave of each SIMD
// takes the upper half of K of the long matrix-core chains (layer 2 and dh1:
// K = 128) and the halves meet in LDS in a fixed order (lower + upper); the
// 16 dW2 tiles go two per wave; the row inputs of the losses are loaded with the
// weights, so nothing in the loss phase waits on memory.
constexpr int GTB = 512;          // threads per workgroup
#ifndef USV_BWD_SYNC
#define USV_BWD_SYNC 0   // 1: dh1 alone on the matrix core, then dW2 beside dz1 -> dW1: measured +1.1 us per minibatch
                         // (dW2's 64 KB of partial stores then leave in 1.7 us and meet the write bandwidth)
#endif
#ifndef USV_BWD_PRIO
#define USV_BWD_PRIO 0   // s_setprio of the dh1 -> dz1 -> dW1 waves in the two-group backward (1: measured the same)
#endif

// k_reduce_partials geometry (RED_BLOCKS chunk squares follow the gradient in grad[])
#ifndef USV_RD_P
#define USV_RD_P 128
#endif
#ifndef USV_RD_NT
#define USV_RD_NT 1   // non-temporal loads of the partial rows (A/B builds override it)
#endif
typedef float f32x4v __attribute__((ext_vector_type(4)));
constexpr int RD_TB = 512, RD_P = USV_RD_P;            // threads, slots per workgroup
constexpr int RD_L = RD_P / 4;                          // lanes per row segment (float4 each)
constexpr int RD_G = (RD_TB / RD_L);                    // row groups
constexpr int RD_KB = 16;                               // loads in flight per lane
constexpr int RED_BLOCKS = (PPO_NPARAM + 5 + RD_P - 1) / RD_P;
static_assert(RD_P % 4 == 0 && 64 % RD_L == 0 && RD_P <= RD_TB, "reduce geometry");
static_assert(RED_BLOCKS <= 256, "chunk squares: one per thread of waves 0-3");

// ---- Adam (torch.optim.Adam, amsgrad off), shared by k_apply, the speculative step of
// k_reduce_partials and the redo of a clipped step in the chained gradient kernel ----
struct AdamBanks {                 // state before ([0]) and after ([1]) one step
  const float *P0, *m0, *v0;
  float *P1, *m1, *v1;
};
struct AdamK {
  float step_size, bc2s;
};
__device__ __forceinline__ AdamK adam_consts(const ppo_cfg_t &c, float lr, float step) {
  // torch.optim.Adam forms the bias corrections in Python doubles
  const double bc1 = 1.0 - pow((double)c.adam_b1, (double)step);
  const double bc2 = 1.0 - pow((double)c.adam_b2, (double)step);
  return {(float)((double)lr / bc1), (float)sqrt(bc2)};
}
__device__ __forceinline__ void adam_one(const ppo_cfg_t &c, const AdamK &k, float g, float p_old, float m_old,
                                         float v_old, float &pn, float &mn, float &vn) {
  if (c.weight_decay != 0.f) g = g + c.weight_decay * p_old;
  mn = m_old + (1.0f - c.adam_b1) * (g - m_old);          // exp_avg.lerp_(grad, 1 - beta1)
  vn = v_old * c.adam_b2 + (1.0f - c.adam_b2) * g * g;    // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
  const float denom = sqrtf(vn) / k.bc2s + c.adam_eps;
  pn = p_old - k.step_size * (mn / denom);
}
// clip_grad_norm_'s coefficient (1 without truncate_grads)
__device__ __forceinline__ float clip_coef(const ppo_cfg_t &c, float total_norm) {
  float coef = 1.0f;
  if (c.truncate_grads) {
    coef = c.grad_norm / (total_norm + 1e-6f);
    coef = fminf(coef, 1.0f);
  }
  return coef;
}
// The next step's bias-corrected constants travel in opt[4..7] = (step_size, bc2s, for step,
// for lr), written by opt_store: a step whose (lr, step) match the tags takes them instead of
// evaluating the two double pow() again (identical inputs, identical values); anything else --
// zero-initialised scalars, a learning rate or step count set by the host -- recomputes.
__device__ __forceinline__ AdamK adam_consts_tagged(const ppo_cfg_t &c, float lr, float step, float t_ss,
                                                    float t_bc, float t_step, float t_lr) {
  if (t_step == step && t_lr == lr) return {t_ss, t_bc};
  return adam_consts(c, lr, step);
}
// AdaptiveScheduler.update on a minibatch's KL (schedulers.py:26-32) and the optimiser
// scalars after its step: opt_in -> opt_out = (lr, step, kl, norm, next step's constants).
// opt_next needs only opt_in and the KL, so a launch can evaluate it (two double pow) in the
// shadow of its loads; opt_store then writes it with the clip norm.
struct OptNext {
  float nl, kl_keep, step;
  AdamK nk;
};
template <class OptIn>
__device__ __forceinline__ OptNext opt_next(const ppo_cfg_t &c, const OptIn &opt_in, float kl) {
  const float lr = opt_in[0];
  float nl = lr, kl_keep = opt_in[2];
  if (c.lr_adaptive) {
    if (kl > 2.0f * c.kl_threshold) nl = fmaxf(lr / 1.5f, c.lr_min);
    if (kl < 0.5f * c.kl_threshold) nl = fminf(lr * 1.5f, c.lr_max);
    kl_keep = kl;
  }
  const float step = opt_in[1] + 1.0f;
  return {nl, kl_keep, step, adam_consts(c, nl, step + 1.0f)};
}
__device__ __forceinline__ void opt_store(const ppo_cfg_t &c, const OptNext &x, float *opt_out, float total_norm,
                                          float kl, float *kl_out) {
  if (c.lr_adaptive && kl_out) *kl_out = kl;
  opt_out[0] = x.nl;
  opt_out[1] = x.step;
  opt_out[2] = x.kl_keep;
  opt_out[3] = total_norm;
  opt_out[4] = x.nk.step_size;
  opt_out[5] = x.nk.bc2s;
  opt_out[6] = x.step + 1.0f;
  opt_out[7] = x.nl;
}

// The chained single-GPU update (ppo_minibatch_fused): minibatch k's gradient kernel stages
// the parameters minibatch k-1's reduce kernel stepped speculatively (bank cur), checks that
// step's clip norm and, when clipping was due, redoes it from bank prev (and writes the redone
// state over bank cur); workgroup 0 advances the optimiser scalars of minibatch k-1.
struct ChainIn {
  const float *P_prev, *m_prev, *v_prev;   // state before minibatch k-1's step
  float *P_cur, *m_cur, *v_cur;            // its speculative result (the kernel's P)
  const float *grad;                       // minibatch k-1: gradient, KL, chunk squares
  const float *opt_prev;                   // optimiser scalars read by minibatch k-1's step
  float *opt_cur;                          // ... and the ones after it (read by minibatch k's)
  float *kl_out;                           // minibatch k-1's KL (log)
  uint32_t *dp_clock;                      // several ranks: the minibatch counter the next reduction keys its
                                           // exchange on (advanced here, by workgroup 0; nullable)
  int fold_skip;                           // group fold: arrive but fold nothing (tests: the reduction's raw-row path)
  float gscale;                            // collective chain (kColl): 1 / world, the all-reduced gradient's scale
};

// x rows of the gradient kernel padded to whole staging passes: every thread stores its slots
// unconditionally (see the obs staging in mb_grad8w)
constexpr int XG = XS;          // row stride of x / W1 in the gradient kernel's LDS
constexpr int GX = ((RB * XG + GTB - 1) / GTB) * GTB;
struct GradSmem {
  float w2[NH * HS];              // W2[j][k]
  float w1[NH * XG];              // W1[j][k], k 33, 34 = 0
  float x[GX];                    // normalised obs (dW1 operand); [RB * XG, GX) staging overflow slots
  float h1[RB * HS];              // tanh layer 1, later dz1
  float h2[RB * HS];              // tanh layer 2, later dz2
  float xch[4][16][64];           // upper-K partial accumulators of layer 2 / dh1 (per wave, register, lane)
  float out[RB * 4];              // mu0, mu1, value
  float g[RB * 4];                // dmu0, dmu1, dv, dnlp per row
  float hg[4][4][NH];             // head-gradient / b2 quarter sums
  float b1[NH];
  float tail[TAIL + 1];
  float nrm[4];                   // chained update: wave sums of the chunk squares
  int fold[2];                    // group fold: all members arrived, this launch's generation
};

// Partial-gradient slot layout (a permutation of the parameters, then the loss sums): the
// matrix-core accumulators of dW2 and dW1[:, :32] are stored in their register order, so each
// lane writes 4 consecutive values of one tile with one 16-byte store ([tile][a][lane][4],
// value r = 4a + r4 of the lane's 16); the remaining parameters follow in parameter order
// (sigma, b1, b2..bmu, the last W1 column).  k_reduce_partials maps slots back to parameters.
constexpr int S_W2 = 0, S_W1 = NH * NH, S_SIG = S_W1 + NH * 32, S_B1 = S_SIG + 2, S_TAIL = S_B1 + NH,
              S_W1C = S_TAIL + TAIL, S_END = S_W1C + NH;
static_assert(S_END == PPO_NPARAM && S_W1 % 4 == 0 && NIN == 33, "partial slot layout");
__device__ __forceinline__ int tail_slot(int param) { return S_TAIL + param - PPO_OFF_B2; }
// tile t of a 32x32 accumulator: slot of the lane's values 4a..4a+3
__device__ __forceinline__ int acc_slot(int base, int tile, int a, int lane) { return base + ((tile * 4 + a) * 64 + lane) * 4; }
// parameter index of a partial slot (-1: a loss sum)
__device__ __forceinline__ int param_of_slot(int s) {
  if (s < S_W1) {             // W2 tiles: tile = 4 cb + k block
    const int tile = s >> 10, a = (s >> 8) & 3, lane = (s >> 2) & 63, q = 4 * a + (s & 3);
    const int n = 32 * (tile >> 2) + crow(q, lane >> 5), k = 32 * (tile & 3) + (lane & 31);
    return PPO_OFF_W2 + n * NH + k;
  }
  if (s < S_SIG) {            // W1[:, :32] tiles: tile = cb
    const int t = s - S_W1, tile = t >> 10, a = (t >> 8) & 3, lane = (t >> 2) & 63, q = 4 * a + (t & 3);
    const int n = 32 * tile + crow(q, lane >> 5), k = lane & 31;
    return PPO_OFF_W1 + n * NIN + k;
  }
  if (s < S_B1) return PPO_OFF_SIGMA + (s - S_SIG);
  if (s < S_TAIL) return PPO_OFF_B1 + (s - S_B1);
  if (s < S_W1C) return PPO_OFF_B2 + (s - S_TAIL);
  if (s < S_END) return PPO_OFF_W1 + (s - S_W1C) * NIN + (NIN - 1);
  return -1;
}

// USV_ROW_NT: the gradient kernel's row inputs (experience rows, read once per mini-epoch) as non-temporal loads
#ifndef USV_ROW_NT
#define USV_ROW_NT 0
#endif
__device__ __forceinline__ float row_ld(const float *p) {
  if constexpr (USV_ROW_NT != 0) return __builtin_nontemporal_load(p);
  else return *p;
}
// per-row inputs of the losses (wave 0: lane = row), loaded with the weights
struct RowIn {
  float act0, act1, nlp, val, ret, adv, mu0, mu1, sg0, sg1;
};

// Partial-gradient stores are non-temporal (nt) and k_reduce_partials reads them with non-temporal
// loads: the 21.8 MB per minibatch stream through without the reduction leaving their lines in the
// caches, where the next minibatch's stores to the same rows met them (same-box A/B at 131072 envs,
// rocprof means of gradient + reduction: sc1 write-through + plain loads 21.08 + 6.31 us, nt + nt loads
// 18.01 + 6.96; sc1 + nt loads 19.94 + 6.86; nt stores with plain loads, round 2: 21.08 + 7.27)
#ifndef USV_PART_AUX
#define USV_PART_AUX 2   // cache-policy bits of the partial stores: nt (A/B builds override it)
#endif
// Partial layout.  Row-major (kCM false; the group fold's): row b = [NPART_PAD] at b NPART_PAD.  Chunk-major
// (USV_PART_CM, the default otherwise): the reduction's chunks of RD_P slots are the outer index, [chunk][nblk][RD_P],
// so each reduction workgroup reads one contiguous nblk x RD_P block (128 KB at 8192 rows) instead of 256
// segments 85 KB apart; a gradient workgroup writes its row as RED_BLOCKS segments of 512 B.
template <int kAux, bool kCM>
struct PartOutT {
  __amdgpu_buffer_rsrc_t r;
  uint32_t cs;   // chunk-major: bytes from one chunk of a row to the next (nblk RD_P 4)
  __device__ __forceinline__ uint32_t off(int idx) const {
    if constexpr (kCM) return (uint32_t)(idx / RD_P) * cs + (uint32_t)(idx % RD_P) * 4u;
    else return (uint32_t)idx * 4u;
  }
  __device__ __forceinline__ void operator()(int idx, float v) const {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off(idx), 0, kAux);
  }
  __device__ __forceinline__ void x4(int idx, float a, float b, float c, float d) const {
    const u32x4_t v = {__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, c),
                       __builtin_bit_cast(uint32_t, d)};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off(idx), 0, kAux);   // idx % 4 == 0: inside one chunk
  }
};
#ifndef USV_PART_CM
#define USV_PART_CM 1
#endif
constexpr int AUX_SC1 = 16;   // sc1: write-through (the in-launch group fold reads the rows from another CU)

// ---- The XCD-group fold of the partial rows (kFold launches of k_mb_grad; k_reduce_partials(fold = 1)) ----
// The 256 per-workgroup partial rows of an 8192-row minibatch (21.8 MB) were written by the gradient kernel and
// read back whole by the reduction.  With the fold, workgroups b = g + 8 m (group g = b % 8, member m: the blocks
// the dispatcher deals to one XCD, speed only -- correctness holds at any placement) meet at a per-group arrival
// counter after storing their rows write-through (sc1, every wave drained); member m then sums the M = nblk / 8
// rows of its group over slice m of the row (sc1 loads) and writes the group row's slice, so the reduction reads
// 8 group rows per slot instead of nblk rows.  Summation order (the same bits in every path):
//   group(g) = half0 + half1,  half0 = 0 + p[g] + p[g + 8] + ... (m < H0),  half1 = 0 + ... (H0 <= m < M),
//   H0 = (M + 1) / 2;  gradient = 0 + group(0) + ... + group(7).
// A member that does not see its whole group arrive within FOLD_WAIT_TICKS (another kernel or process holding
// CUs: the group's rows cannot all be resident) folds nothing; the reduction then forms that group's sum from
// the raw rows in the same order, so the result does not depend on whether a group folded.
// Buffer (ppo_partials_floats): [nblk][NPART_PAD] rows | [8][NPART_PAD] group rows | fold control: per group
// one 128-B line holding the arrival counter (monotonic: a member's arrival value tells its launch generation)
// and 32 slice words (the generation whose fold wrote slice m).
constexpr int FOLD_G = 8;
static_assert(RD_G >= FOLD_G, "k_reduce_partials(fold = 1) reads one group row per row group");
constexpr int FOLD_MAX_M = 32;                      // nblk <= 256: the grid is resident at one workgroup per CU
constexpr int FOLD_CTL_STRIDE = 64;                 // u32 words per group: [0] counter, [32 + m] slice gens
constexpr uint64_t FOLD_WAIT_TICKS = 10000;         // 100 us at the 100 MHz wall clock
// floats in front of the fold control words: the larger of the chunk-major rows (RED_BLOCKS x RD_P per row, 112
// floats more than a row-major row) and the row-major rows + the group rows, so every minibatch size has a layout
__host__ __device__ constexpr size_t part_body_floats(int nblk) {
  return (size_t)nblk * RED_BLOCKS * RD_P > (size_t)(nblk + FOLD_G) * NPART_PAD ? (size_t)nblk * RED_BLOCKS * RD_P
                                                                                 : (size_t)(nblk + FOLD_G) * NPART_PAD;
}
__device__ __forceinline__ uint32_t *fold_ctl(float *partials, int nblk) {
  return reinterpret_cast<uint32_t *>(partials + part_body_floats(nblk));
}
__device__ __forceinline__ const uint32_t *fold_ctl(const float *partials, int nblk) {
  return reinterpret_cast<const uint32_t *>(partials + part_body_floats(nblk));
}
__device__ __forceinline__ f32x4v ld4_sc1(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
  return __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, AUX_SC1));
}

// chained update, clipping due: minibatch k-1's step redone from bank prev with the clip
// coefficient, straight into this workgroup's LDS weights (and sigma into ls0 / ls1);
// workgroup (q / GTB) % grid writes parameter chunk q / GTB of the redone state over bank cur
// (no workgroup of this launch reads bank cur after its first barrier)
// (scale: 1 on one rank; the collective chain's 1 / world -- k_apply's g * grad_scale * coef)
__device__ __forceinline__ void redo_step(const ppo_cfg_t &c, const ChainIn &ch, const float (&op)[8], float coef,
                                          float scale, GradSmem &s, float &ls0, float &ls1) {
  const AdamK ak = adam_consts_tagged(c, op[0], op[1] + 1.0f, op[4], op[5], op[6], op[7]);
  for (int q = threadIdx.x; q < PPO_NPARAM; q += GTB) {
    float pn, mn, vn;
    adam_one(c, ak, ch.grad[q] * scale * coef, ch.P_prev[q], ch.m_prev[q], ch.v_prev[q], pn, mn, vn);
    if ((q / GTB) % gridDim.x == blockIdx.x) {
      ch.P_cur[q] = pn; ch.m_cur[q] = mn; ch.v_cur[q] = vn;
    }
    if (q >= PPO_OFF_B2) {
      s.tail[q - PPO_OFF_B2] = pn;
    } else if (q >= PPO_OFF_W2) {
      const int e = q - PPO_OFF_W2;
      s.w2[(e / NH) * HS + e % NH] = pn;
    } else if (q >= PPO_OFF_B1) {
      s.b1[q - PPO_OFF_B1] = pn;
    } else if (q >= PPO_OFF_W1) {
      const int e = q - PPO_OFF_W1;
      s.w1[(e / NIN) * XG + e % NIN] = pn;
    }
  }
  float pn, mn, vn;
  adam_one(c, ak, ch.grad[PPO_OFF_SIGMA] * scale * coef, ch.P_prev[PPO_OFF_SIGMA], ch.m_prev[PPO_OFF_SIGMA],
           ch.v_prev[PPO_OFF_SIGMA], pn, mn, vn);
  ls0 = pn;
  adam_one(c, ak, ch.grad[PPO_OFF_SIGMA + 1] * scale * coef, ch.P_prev[PPO_OFF_SIGMA + 1],
           ch.m_prev[PPO_OFF_SIGMA + 1], ch.v_prev[PPO_OFF_SIGMA + 1], pn, mn, vn);
  ls1 = pn;
}

// The norm of the all-reduced, scaled gradient as k_apply<false, ..> forms it (the same 256 threads, float4
// order, fma chain, wave sums and wave order), so the collective chain's step is the split path's bit for bit
constexpr int APN_TB = 256;
__device__ __forceinline__ float apply_norm_part(const float *__restrict__ grad_in, float grad_scale, int tid) {
  constexpr int N4 = PPO_NPARAM / 4, U = (N4 + APN_TB - 1) / APN_TB;
  const float4 *g4 = reinterpret_cast<const float4 *>(grad_in);
  float4 gv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) gv[u] = g4[min(tid + u * APN_TB, N4 - 1)];
  float ss = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (tid + u * APN_TB >= N4) continue;
    const float x = gv[u].x * grad_scale, y = gv[u].y * grad_scale;
    const float z = gv[u].z * grad_scale, w = gv[u].w * grad_scale;
    ss = fmaf(x, x, ss); ss = fmaf(y, y, ss); ss = fmaf(z, z, ss); ss = fmaf(w, w, ss);
  }
  for (int r = 4 * N4 + tid; r < PPO_NPARAM; r += APN_TB) {
    const float g = grad_in[r] * grad_scale;
    ss = fmaf(g, g, ss);
  }
  return ss;
}

// kColl (several ranks without the peer exchange: ppo_minibatch_coll): ch.grad holds minibatch k-1's gradient and
// KL after the host's in-stream SUM all-reduce; nothing was stepped speculatively, so every workgroup takes that
// step itself (redo_step from bank prev with coefficient and scale, k_apply's norm of the scaled gradient).
template <bool kBf, bool kChain, bool kFold, bool kColl = false>
__device__ __forceinline__ void mb_grad8w(const ppo_cfg_t &c, const ChainIn &ch, const float *__restrict__ P,
                                          const double *__restrict__ obs_rms, int row0,
                                          const float *__restrict__ e_obs, const float *__restrict__ e_act,
                                          const float *__restrict__ e_nlp, const float *__restrict__ e_val,
                                          const float *__restrict__ e_ret, const float *__restrict__ e_adv,
                                          float *e_mu, float *e_sigma, float *partials, GradSmem &s) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int kh = w >> 2, cb = w & 3, n0 = 32 * cb;      // K half, column block
#ifdef USV_DIAG_HOT_ROWS
  const int rb0 = blockIdx.x * RB;   // DIAGNOSTIC build only (wrong rows): every minibatch reads the first one's rows
#else
  const int rb0 = row0 + blockIdx.x * RB;               // first row of this workgroup
#endif
  const float invB = 1.0f / (float)c.minibatch;
  USV_PHASE(ppo, 0);
  // several ranks: this minibatch's exchange key (the previous reduction has finished: stream order)
  if (ch.dp_clock && blockIdx.x == 0 && tid == 0) *ch.dp_clock += 1u;
  // ---- every global load issued up front (compile-time trip counts) ----
  // W2 element tid + u GTB per thread (4-byte loads): each wave's LDS commit is 64 consecutive words
  // of one row, conflict-free at the odd row stride (16-byte loads would leave 4-word strided writes)
  constexpr int NW1G = (NH * XG + GTB - 1) / GTB, NTLG = (TAIL + GTB - 1) / GTB, NW2F = NH * NH / GTB;
  static_assert(NH * NH % GTB == 0, "staging trip counts");
  float w2f[NW2F];
  float w1r[NW1G], tlr[NTLG];
  // chained update: minibatch k-1's optimiser scalars (lanes 0-7) and KL (lane 8) as VECTOR loads,
  // the first in flight -- scalar loads here would share lgkmcnt with the LDS staging writes and
  // put their latency in front of the first barrier
  float ov = 0.f;
  if constexpr (kChain) ov = lane < 8 ? ch.opt_prev[lane] : ch.grad[PPO_NPARAM];
  // Branch-free: indices clamped, out-of-range values masked after every load is in flight (a
  // conditional load puts a branch -- and, where another path zero-fills the same registers, a
  // full vmcnt wait -- between the loads)
  {
#pragma unroll
    for (int u = 0; u < NW1G; ++u) {
      const int q = min(tid + u * GTB, NH * XG - 1), j = q / XG, k = q % XG;
      w1r[u] = P[PPO_OFF_W1 + j * NIN + min(k, NIN - 1)];
    }
#pragma unroll
    for (int u = 0; u < NTLG; ++u) tlr[u] = P[PPO_OFF_B2 + min(tid + u * GTB, TAIL - 1)];
  }
  const float b1r = P[PPO_OFF_B1 + (tid & (NH - 1))];
  // log-sigma as a vector load too (read out by readlane where the losses use it)
  const float lsv = P[PPO_OFF_SIGMA + (lane & 1)];
  float lsig0 = 0.f, lsig1 = 0.f;
  // chained update: minibatch k-1's chunk squares (its clip norm)
  float csq = 0.f;
  if constexpr (kChain) csq = ch.grad[PPO_NPARAM + 8 + min(tid, RED_BLOCKS - 1)];
  // per-row loss inputs, lane = row (waves 0 and 1 use them: the actor / the critic side)
  RowIn ri;
  {
    const size_t row = (size_t)rb0 + (lane & (RB - 1));
    ri.act0 = row_ld(&e_act[row * 2]); ri.act1 = row_ld(&e_act[row * 2 + 1]);
    ri.nlp = row_ld(&e_nlp[row]); ri.adv = row_ld(&e_adv[row]);
    ri.val = row_ld(&e_val[row]); ri.ret = row_ld(&e_ret[row]);
    ri.mu0 = row_ld(&e_mu[row * 2]); ri.mu1 = row_ld(&e_mu[row * 2 + 1]);
    ri.sg0 = row_ld(&e_sigma[row * 2]); ri.sg1 = row_ld(&e_sigma[row * 2 + 1]);
  }
  // obs rows and the running statistics (always loaded; obs_rms is non-null, checked on the host)
  constexpr int NU = (RB * XG + GTB - 1) / GTB;
  float xo[NU];
  double mu[NU], var[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int q = min(tid + u * GTB, RB * XG - 1), r = q / XG, kc = min(q % XG, NIN - 1);
    xo[u] = row_ld(&e_obs[(size_t)(rb0 + r) * NIN + kc]);
    mu[u] = obs_rms[kc];
    var[u] = obs_rms[NIN + kc];
  }
  // W2 (64 KB of the 85 KB) issued LAST: the staging of x / W1 / biases and layer 1 wait only for the
  // loads ahead of it (counted vmcnt waits), W2 lands during layer 1 and is committed after it
#pragma unroll
  for (int u = 0; u < NW2F; ++u) w2f[u] = P[PPO_OFF_W2 + tid + u * GTB];
  __builtin_amdgcn_sched_barrier(0);   // every load above is issued before anything waits
#pragma unroll
  for (int u = 0; u < NW1G; ++u)
    if ((tid + u * GTB) % XG >= NIN) w1r[u] = 0.f;
  if (kChain && tid >= RED_BLOCKS) csq = 0.f;
  {   // obs rows, normalised on the way into LDS: every value formed unconditionally and selected, so no
      // load is sunk into a branch (a load issued there would come after W2's and wait for all of them)
    const bool norm = c.normalize_input != 0;
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int q = tid + u * GTB;
      const int k = q % XG;
      const float xn = rms_norm(xo[u], mu[u], var[u], c.rms_eps);
      const float xv = (k < NIN && q < RB * XG) ? (norm ? xn : xo[u]) : 0.f;
      s.x[q] = xv;   // q < GX: the slots past RB * XG are never read
    }
  }
#pragma unroll
  for (int u = 0; u < NW1G; ++u)
    if (tid + u * GTB < NH * XG) s.w1[tid + u * GTB] = w1r[u];
#pragma unroll
  for (int u = 0; u < NTLG; ++u)
    if (tid + u * GTB < TAIL) s.tail[tid + u * GTB] = tlr[u];
  if (tid < NH) s.b1[tid] = b1r;
  if (kChain && !kColl && w < 4) {   // k_apply's norm: the same lanes, the same order
    const float t = wave_sum(csq);
    if (lane == 0) s.nrm[w] = t;
  }
  __syncthreads();
  if constexpr (kColl) {   // k_apply<false, ..>'s norm of the all-reduced gradient (waves 0-3)
    if (w < 4) {
      const float t = wave_sum(apply_norm_part(ch.grad, ch.gscale, tid));
      if (lane == 0) s.nrm[w] = t;
    }
    __syncthreads();
  }
  bool slow = false;
  if constexpr (kChain) {
    // (the scalars are read out of ov's lanes only where they are used: readlane ignores exec)
    const auto lane_of = [&](int q) {
      return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ov), q));
    };
    const float total_norm = sqrtf(((s.nrm[0] + s.nrm[1]) + s.nrm[2]) + s.nrm[3]);
    const float coef = clip_coef(c, total_norm);
    const float gscale = kColl ? ch.gscale : 1.0f;
    // (wave 4 of workgroup 0: the kh = 1 waves only commit W2 while layer 1 runs)
    if (blockIdx.x == 0 && tid == 256) {
      float op[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) op[q] = lane_of(q);
      const float kl_prev = kColl ? lane_of(8) * gscale : lane_of(8);   // k_apply: grad[NPARAM] * grad_scale
      opt_store(c, opt_next(c, op, kl_prev), ch.opt_cur, total_norm, kl_prev, ch.kl_out);
    }
    if (kColl || coef < 1.0f) {   // uniform over the launch
      slow = true;
      float op[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) op[q] = lane_of(q);
      redo_step(c, ch, op, coef, gscale, s, lsig0, lsig1);
      __syncthreads();
    }
  }
  USV_PHASE(ppo, 1);
  if (kh == 0) {
    // ---- layer 1 (waves 0-3): h1 = tanh(x W1^T + b1), K = 34 (k = 33 is zero) ----
    f32x16 acc = {};
#pragma unroll
    for (int st = 0; st < 17; ++st) {
      const int k = 2 * st + h;
      acc = mfma32(s.x[i * XG + k], s.w1[(n0 + i) * XG + k], acc);
    }
    const float bj = s.b1[n0 + i];
#pragma unroll
    for (int r = 0; r < 16; ++r) s.h1[crow(r, h) * HS + n0 + i] = fast_tanh(acc[r] + bj);
  }
  USV_PHASE(ppo, 9);
  // W2 into LDS (waves 4-7 do it while 0-3 run layer 1; each thread commits its own loads)
  if (!slow) {
#pragma unroll
    for (int u = 0; u < NW2F; ++u) {
      const int e = tid + u * GTB;
      s.w2[(e >> 7) * HS + (e & (NH - 1))] = w2f[u];
    }
  }
  __syncthreads();
  USV_PHASE(ppo, 10);
  // ---- layer 2: h2 = tanh(h1 W2^T + b2); wave (kh, cb) sums k in [64 kh, 64 kh + 64).  The K-half
  // kh = 1 wave feeds its A-operand rows rotated by 16 (ra), so in BOTH waves of a pair the rows it
  // finishes sit in accumulator registers 0-7 and the rows it hands over in 8-15: every register
  // index is a constant (no per-wave select, no dynamic register indexing) ----
  const int ra = (i + 16 * kh) & (RB - 1);
  {
    f32x16 acc = {};
    if constexpr (kBf) {
#pragma unroll
      for (int st = 0; st < NH / 32; ++st) {
        const int k0 = 64 * kh + 16 * st + 8 * h;
        acc = mfma_bf16(ld8(&s.h1[ra * HS + k0]), ld8(&s.w2[(n0 + i) * HS + k0]), acc);
      }
    } else {
#pragma unroll 16
      for (int st = 0; st < NH / 4; ++st) {
        const int k = 64 * kh + 2 * st + h;
        acc = mfma32(s.h1[ra * HS + k], s.w2[(n0 + i) * HS + k], acc);
      }
    }
    USV_PHASE(ppo, 11);
    // the two K halves meet in LDS as (lower half + upper half) + bias (fp32 addition commutes,
    // so own + other is that sum in both waves)
#pragma unroll
    for (int q = 0; q < 8; ++q) s.xch[cb][8 * kh + q][lane] = acc[8 + q];
    __syncthreads();
    const float bj = s.tail[T_B2 + n0 + i];
#pragma unroll
    for (int q = 0; q < 8; ++q)
      s.h2[(crow(q, h) + 16 * kh) * HS + n0 + i] = fast_tanh((acc[q] + s.xch[cb][8 - 8 * kh + q][lane]) + bj);
  }
  __syncthreads();
  USV_PHASE(ppo, 12);
  constexpr bool kCM = USV_PART_CM != 0 && !kFold;
  const PartOutT<kFold ? AUX_SC1 : USV_PART_AUX, kCM> part_st{
      kCM ? __builtin_amdgcn_make_buffer_rsrc(partials + (size_t)blockIdx.x * RD_P, 0,
                                              (int)(((size_t)RED_BLOCKS * gridDim.x - blockIdx.x) * RD_P * 4), 0x00020000)
          : __builtin_amdgcn_make_buffer_rsrc(partials + (size_t)blockIdx.x * NPART_PAD, 0, NPART * 4, 0x00020000),
      (uint32_t)gridDim.x * RD_P * 4u};
  // ---- heads: mu = Wmu h2 + bmu, value = Wv h2 + bv (16 threads per row, k = part + 16 kk: the 16
  // threads of a row read 16 consecutive words -- no 4-way LDS bank conflicts) ----
  {
    const int r = tid / 16, part = tid % 16;
    float a0 = 0.f, a1 = 0.f, av = 0.f;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int k = part + 16 * kk;
      const float hv = s.h2[r * HS + k];
      a0 = fmaf(s.tail[T_WMU + k], hv, a0);
      a1 = fmaf(s.tail[T_WMU + NH + k], hv, a1);
      av = fmaf(s.tail[T_WV + k], hv, av);
    }
#pragma unroll
    for (int m = 1; m < 16; m <<= 1) {
      a0 += __shfl_xor(a0, m, 64);
      a1 += __shfl_xor(a1, m, 64);
      av += __shfl_xor(av, m, 64);
    }
    if (part == 0) {
      s.out[r * 4 + 0] = a0 + s.tail[T_BMU];
      s.out[r * 4 + 1] = a1 + s.tail[T_BMU + 1];
      s.out[r * 4 + 2] = av + s.tail[T_BV];
    }
  }
  __syncthreads();
  USV_PHASE(ppo, 2);
  // ---- per-row losses and output gradients (lane = row < RB): wave 0 the actor side (ratio, clipped
  // surrogate, dnlp, dmu, dlogstd), wave 1 in parallel the critic loss and dv, wave 2 the bound, entropy and KL
  // terms and the mu / sigma write-back (the same per-row arithmetic and lane sums as one wave doing all) ----
  if (tid < 192) {
    const int r = lane;
    const bool rowok = r < RB;
    const int rr = rowok ? r : 0;
    const size_t row = (size_t)rb0 + rr;
    const float mu0 = s.out[rr * 4], mu1 = s.out[rr * 4 + 1], v = s.out[rr * 4 + 2];
    if (!slow) {
      lsig0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lsv), 0));
      lsig1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, lsv), 1));
    }
    const float ls0 = mu0 * 0.f + lsig0, ls1 = mu1 * 0.f + lsig1;
    const float sg0 = expf(ls0), sg1 = expf(ls1);
    const float bh0 = fmaxf(mu0 - 1.1f, 0.f), bl0 = fminf(mu0 + 1.1f, 0.f);
    const float bh1 = fmaxf(mu1 - 1.1f, 0.f), bl1 = fminf(mu1 + 1.1f, 0.f);
    if (w == 0) {
      float la = 0.f, gs0 = 0.f, gs1 = 0.f;
      if (rowok) {
        const float z0 = (ri.act0 - mu0) / sg0, z1 = (ri.act1 - mu1) / sg1;
        const float nlp = 0.5f * (z0 * z0 + z1 * z1) + kLog2Pi + (ls0 + ls1);
        const float A = ri.adv;
        // actor_loss (common_losses.py:36-46)
        const float ratio = expf(ri.nlp - nlp);
        const float lo = 1.0f - c.e_clip, hi = 1.0f + c.e_clip;
        const float rc = clampt(ratio, lo, hi);
        const float s1 = -(A * ratio), s2 = -(A * rc);
        const float a_loss = fmaxf(s1, s2);
        const float inr = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
        const float g1 = -A, g2 = -A * inr;                // d(-A r)/dr, d(-A clip(r))/dr
        const float g_r = (s1 > s2) ? g1 : ((s1 < s2) ? g2 : 0.5f * (g1 + g2));
        const float dnlp = invB * g_r * (-ratio);          // dr/dnlp = -r
        // + bound_loss (a2c_continuous.py:209-217)
        const float bc = c.bounds_loss_coef * invB;
        const float dmu0 = dnlp * (-z0 / sg0) + bc * 2.f * (bh0 + bl0);
        const float dmu1 = dnlp * (-z1 / sg1) + bc * 2.f * (bh1 + bl1);
        // d nlp / d logstd = 1 - z^2; - entropy_coef * mean(entropy): d entropy / d logstd = 1 per row
        const float dent = -c.entropy_coef * invB;
        gs0 = dnlp * (1.f - z0 * z0) + dent;
        gs1 = dnlp * (1.f - z1 * z1) + dent;
        la = a_loss;
        s.g[r * 4 + 0] = dmu0;
        s.g[r * 4 + 1] = dmu1;
        s.g[r * 4 + 3] = dnlp;
      }
      la = wave_sum(la); gs0 = wave_sum(gs0); gs1 = wave_sum(gs1);
      if (lane == 0) {
        part_st(P_LOSS + 0, la);
        part_st(S_SIG, gs0); part_st(S_SIG + 1, gs1);
      }
    } else if (w == 2) {
      // the KL, entropy and bound terms and the mu / sigma write-back on a wave of their own: they feed the
      // loss sums and the adaptive LR only, not this minibatch's backward
      float le = 0.f, lb = 0.f, lkl = 0.f;
      if (rowok) {
        const float b_loss = (bl0 * bl0 + bh0 * bh0) + (bl1 * bl1 + bh1 * bh1);
        const float ent = (0.5f + 0.5f * logf(USV_2PI_F) + ls0) + (0.5f + 0.5f * logf(USV_2PI_F) + ls1);
        // policy_kl (torch_ext.py:27-36) vs the dataset's mu/sigma, then update_mu_sigma
        const float om0 = ri.mu0, om1 = ri.mu1, os0 = ri.sg0, os1 = ri.sg1;
        const float kl0 = logf(os0 / sg0 + 1e-5f) + (sg0 * sg0 + (om0 - mu0) * (om0 - mu0)) / (2.0f * (os0 * os0 + 1e-5f)) - 0.5f;
        const float kl1 = logf(os1 / sg1 + 1e-5f) + (sg1 * sg1 + (om1 - mu1) * (om1 - mu1)) / (2.0f * (os1 * os1 + 1e-5f)) - 0.5f;
        e_mu[row * 2] = mu0; e_mu[row * 2 + 1] = mu1;
        e_sigma[row * 2] = sg0; e_sigma[row * 2 + 1] = sg1;
        le = ent; lb = b_loss; lkl = kl0 + kl1;
      }
      le = wave_sum(le); lb = wave_sum(lb); lkl = wave_sum(lkl);
      if (lane == 0) {
        part_st(P_LOSS + 2, le); part_st(P_LOSS + 3, lb); part_st(P_LOSS + 4, lkl);
      }
    } else {
      float lc = 0.f;
      if (rowok) {
        // critic_loss (common_losses.py:10-19)
        const float vo = ri.val, R = ri.ret;
        float dv, c_loss;
        if (c.clip_value) {
          const float dvr = v - vo;
          const float dvc = clampt(dvr, -c.e_clip, c.e_clip);
          const float vc = vo + dvc;
          const float l1 = (v - R) * (v - R), l2 = (vc - R) * (vc - R);
          c_loss = fmaxf(l1, l2);
          const float d1 = 2.f * (v - R);
          const float d2 = 2.f * (vc - R) * ((dvr >= -c.e_clip && dvr <= c.e_clip) ? 1.f : 0.f);
          dv = (l1 > l2) ? d1 : ((l1 < l2) ? d2 : 0.5f * (d1 + d2));
        } else {
          c_loss = (R - v) * (R - v);
          dv = 2.f * (v - R);
        }
        dv *= 0.5f * c.critic_coef * invB;
        lc = c_loss;
        s.g[r * 4 + 2] = dv;
      }
      lc = wave_sum(lc);
      if (lane == 0) part_st(P_LOSS + 1, lc);
    }
  }
  __syncthreads();
  USV_PHASE(ppo, 3);
  // ---- heads' grads and dz2 = (dmu Wmu + dv Wv) (1 - h2^2), in place over h2 (quarter qq: 8 rows) ----
  {
    const int j = tid & (NH - 1), qq = tid >> 7;
    const float wm0 = s.tail[T_WMU + j], wm1 = s.tail[T_WMU + NH + j], wv = s.tail[T_WV + j];
    float gw0 = 0.f, gw1 = 0.f, gwv = 0.f, db = 0.f;
#pragma unroll
    for (int q = 0; q < RB / 4; ++q) {
      const int rr = qq * (RB / 4) + q;
      const float hv = s.h2[rr * HS + j];
      const float d0 = s.g[rr * 4], d1 = s.g[rr * 4 + 1], dvv = s.g[rr * 4 + 2];
      gw0 = fmaf(d0, hv, gw0); gw1 = fmaf(d1, hv, gw1); gwv = fmaf(dvv, hv, gwv);
      const float dz = (d0 * wm0 + d1 * wm1 + dvv * wv) * (1.f - hv * hv);
      s.h2[rr * HS + j] = dz;
      db += dz;
    }
    s.hg[qq][0][j] = gw0; s.hg[qq][1][j] = gw1; s.hg[qq][2][j] = gwv; s.hg[qq][3][j] = db;
  }
  __syncthreads();
  USV_PHASE(ppo, 4);
  // ---- the rest of the backward in two concurrent wave groups, no further barrier (round 5; the one-group form
  // before it: K-half exchanges for dh1, a dz1 barrier, dW1 on waves 0-3 after it):
  //   waves 0-3 (column block cb): dh1 = dz2 W2 over the full K = 128 (one accumulator chain), dz1 = dh1 (1 - h1^2)
  //     in registers, then dW1[j in cb][k] = sum_r dz1[r][j] x[r][k] straight from those registers (the A operand's
  //     32 rows are the lane's own accumulator rows), db1 and W1's last column by lane sums;
  //   waves 4-7 (row block t of dW2): the head-weight / b2 / bmu / bv sums, then dW2[n in t][k] = sum_r dz2[r][n]
  //     h1[r][k] (4 tiles, each tile's 16-B partial stores spread over the next tile's chain).
  // The two groups share each SIMD's matrix core, so dW2's 64 KB of partial stores leave over the whole backward
  // (USV_BWD_SYNC = 1 runs dh1 alone first and measured slower: the stores then meet the write bandwidth) ----
  f32x16 dh = {};
  if (w < 4) {
    if constexpr (USV_BWD_PRIO > 0) __builtin_amdgcn_s_setprio(USV_BWD_PRIO);
    if constexpr (kBf) {
#pragma unroll
      for (int st = 0; st < NH / 16; ++st) {
        const int j0 = 16 * st + 8 * h;
        dh = mfma_bf16(ld8(&s.h2[i * HS + j0]), ld8s(&s.w2[j0 * HS + n0 + i], HS), dh);
      }
    } else {
#pragma unroll 16
      for (int st = 0; st < NH / 2; ++st) {
        const int j = 2 * st + h;
        dh = mfma32(s.h2[i * HS + j], s.w2[j * HS + n0 + i], dh);
      }
    }
    USV_PHASE(ppo, 6);
  } else {
    const int tt = tid - 256;
    if (tt < NH) {   // head-weight and b2 gradients: quarter sums in a fixed order
      const int j = tt;
      part_st(tail_slot(PPO_OFF_WMU + j), ((s.hg[0][0][j] + s.hg[1][0][j]) + s.hg[2][0][j]) + s.hg[3][0][j]);
      part_st(tail_slot(PPO_OFF_WMU + NH + j), ((s.hg[0][1][j] + s.hg[1][1][j]) + s.hg[2][1][j]) + s.hg[3][1][j]);
      part_st(tail_slot(PPO_OFF_WV + j), ((s.hg[0][2][j] + s.hg[1][2][j]) + s.hg[2][2][j]) + s.hg[3][2][j]);
      part_st(tail_slot(PPO_OFF_B2 + j), ((s.hg[0][3][j] + s.hg[1][3][j]) + s.hg[2][3][j]) + s.hg[3][3][j]);
    } else if (tt < NH + 3) {   // bmu0, bmu1, bv: the row sums of dmu / dv
      const int q = tt - NH;
      float sacc = 0.f;
      for (int r = 0; r < RB; ++r) sacc += s.g[r * 4 + q];
      part_st(tail_slot(q < 2 ? PPO_OFF_BMU + q : PPO_OFF_BV), sacc);
    }
  }
  if constexpr (USV_BWD_SYNC != 0) __syncthreads();
  if (w < 4) {
    float dz1[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const float hv = s.h1[crow(q, h) * HS + n0 + i];
      dz1[q] = dh[q] * (1.f - hv * hv);
    }
    USV_PHASE(ppo, 7);
    // dW1[n0 + crow(.., h)][k = i]: step q pairs rows crow(q, 0) (lanes h = 0) and crow(q, 1) (h = 1)
    f32x16 acc = {};
#pragma unroll
    for (int q = 0; q < 16; ++q) acc = mfma32(dz1[q], s.x[crow(q, h) * XG + i], acc);
    float sb = 0.f, sc = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      sb += dz1[q];
      sc = fmaf(dz1[q], s.x[crow(q, h) * XG + NIN - 1], sc);
    }
    sb += __shfl_xor(sb, 32, 64);   // rows of h = 0 + rows of h = 1 (the same sum in both lanes)
    sc += __shfl_xor(sc, 32, 64);
#pragma unroll
    for (int a = 0; a < 4; ++a)
      part_st.x4(acc_slot(S_W1, cb, a, lane), acc[4 * a], acc[4 * a + 1], acc[4 * a + 2], acc[4 * a + 3]);
    if (h == 0) {
      part_st(S_B1 + n0 + i, sb);
      part_st(S_W1C + n0 + i, sc);
    }
  } else {
    const int t = w - 4;
    const int nt0 = 32 * t;
    {
    f32x16 prev = {};
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      f32x16 d = {};
      if constexpr (kBf) {
#pragma unroll
        for (int st = 0; st < RB / 16; ++st) {
          const int r0 = 16 * st + 8 * h;
          d = mfma_bf16(ld8s(&s.h2[r0 * HS + nt0 + i], HS), ld8s(&s.h1[r0 * HS + 32 * kb + i], HS), d);
          if (kb > 0) {
#pragma unroll
            for (int a = 2 * st; a < 2 * st + 2; ++a)
              part_st.x4(acc_slot(S_W2, 4 * t + kb - 1, a, lane), prev[4 * a], prev[4 * a + 1], prev[4 * a + 2],
                         prev[4 * a + 3]);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      } else {
#pragma unroll
        for (int st = 0; st < RB / 2; ++st) {
          const int r = st + 16 * h;
          d = mfma32(s.h2[r * HS + nt0 + i], s.h1[r * HS + 32 * kb + i], d);
          if (kb > 0 && (st & 3) == 1) {
            const int a = st >> 2;
            part_st.x4(acc_slot(S_W2, 4 * t + kb - 1, a, lane), prev[4 * a], prev[4 * a + 1], prev[4 * a + 2],
                       prev[4 * a + 3]);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      prev = d;
    }
    USV_PHASE_T(ppo, 13, 256);
#pragma unroll
    for (int a = 0; a < 4; ++a)
      part_st.x4(acc_slot(S_W2, 4 * t + 3, a, lane), prev[4 * a], prev[4 * a + 1], prev[4 * a + 2], prev[4 * a + 3]);
    USV_PHASE_T(ppo, 5, 256);
    }
  }
  USV_PHASE(ppo, 8);
  if constexpr (kFold) {
    // ---- the group fold (see FOLD_G): arrive once every wave's write-through stores are drained ----
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int nblk = (int)gridDim.x, M = nblk / FOLD_G, g = blockIdx.x % FOLD_G, m = blockIdx.x / FOLD_G;
    uint32_t *ctl = fold_ctl(partials, nblk) + g * FOLD_CTL_STRIDE;
    if (tid == 0) {
      // release: the members may sit on other XCDs (separate L2s); the memory model, not the write-through
      // stores' drain alone, then orders this workgroup's row before its arrival
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      const uint32_t old = __hip_atomic_fetch_add(ctl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t gen = old / (uint32_t)M + 1u, target = gen * (uint32_t)M;
      const uint64_t t0 = wall_clock64();
      int ok = 0;
      while (true) {
        const uint32_t v = __hip_atomic_load(ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // sc1 poll
        if ((int32_t)(v - target) >= 0) { ok = 1; __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent"); break; }
        if (wall_clock64() - t0 > FOLD_WAIT_TICKS) break;
        __builtin_amdgcn_s_sleep(1);
      }
      s.fold[0] = ok && !ch.fold_skip;
      s.fold[1] = (int)gen;
    }
    __syncthreads();
    USV_PHASE(ppo, 14);
    if (s.fold[0]) {
      constexpr int NQ = NPART_PAD / 4;
      const int q4 = (NQ + M - 1) / M, qa = m * q4, qb = min(qa + q4, NQ);
      const int h0 = (M + 1) / 2;
      float4 *lds = reinterpret_cast<float4 *>(s.w2);   // the weights are no longer read
      // the group's rows through one buffer descriptor (sc1 loads: served from L2 / memory, never L1)
      const __amdgpu_buffer_rsrc_t rows = __builtin_amdgcn_make_buffer_rsrc(
          partials + (size_t)g * NPART_PAD, 0, (int)((size_t)(nblk - g) * NPART_PAD * 4), 0x00020000);
      float *grow = partials + (size_t)(nblk + g) * NPART_PAD;
      for (int c0 = qa; c0 < qb; c0 += GTB / 2) {
        const int half = tid / (GTB / 2), q = c0 + tid % (GTB / 2);
        const int mb = half ? h0 : 0, me = half ? M : h0;
        const int qc = min(q, NQ - 1);
        f32x4v x[FOLD_MAX_M / 2];
#pragma unroll
        for (int k = 0; k < FOLD_MAX_M / 2; ++k)
          x[k] = ld4_sc1(rows, (uint32_t)((FOLD_G * min(mb + k, M - 1) * NPART_PAD + 4 * qc) * 4));
        f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < FOLD_MAX_M / 2; ++k)
          if (mb + k < me) acc += x[k];
        if (half) lds[tid % (GTB / 2)] = make_float4(acc[0], acc[1], acc[2], acc[3]);
        __syncthreads();
        if (!half && q < qb) {
          const float4 o = lds[tid];
          const f32x4v t = {acc[0] + o.x, acc[1] + o.y, acc[2] + o.z, acc[3] + o.w};
          __builtin_nontemporal_store(t, reinterpret_cast<f32x4v *>(grow + 4 * q));
        }
        __syncthreads();
      }
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) ctl[32 + m] = (uint32_t)s.fold[1];   // this slice of the group row is this launch's
    }
    USV_PHASE(ppo, 15);
  }
}

template <bool kBf, bool kChain, bool kFold, bool kColl = false>
__global__ __launch_bounds__(GTB, 2) void k_mb_grad(ppo_cfg_t c, ChainIn ch, const float *__restrict__ P,
                                                    const double *__restrict__ obs_rms, int row0,
                                                    const float *__restrict__ e_obs, const float *__restrict__ e_act,
                                                    const float *__restrict__ e_nlp, const float *__restrict__ e_val,
                                                    const float *__restrict__ e_ret, const float *__restrict__ e_adv,
                                                    float *e_mu, float *e_sigma, float *partials) {
  __shared__ GradSmem s;
  mb_grad8w<kBf, kChain, kFold, kColl>(c, ch, P, obs_rms, row0, e_obs, e_act, e_nlp, e_val, e_ret, e_adv, e_mu,
                                       e_sigma, partials, s);
}

// k_reduce_partials: the per-workgroup partial rows (stride NPART_PAD floats, 16-B aligned)
// summed in a fixed order (deterministic, independent of the launch) into grad[].
// One 512-thread workgroup per 128 consecutive slots (param_of_slot maps them back to the
// parameter order of grad[]): each half-wave loads a 512-B
// row segment as float4s (32 lanes x 4 params), 16 row groups (wave w, half h: group
// 2w + h takes rows g, g + 16, g + 32, ...) with all 16 loads of a lane in flight,
// then the 16 group sums are added in group order through LDS.  Also writes the KL /
// loss means and the chunk's squared norm (k_apply's clip norm on one rank).
//
// With kSpec (the chained single-GPU update, ppo_minibatch_fused) the workgroup also takes the
// Adam step of its parameters speculatively, with clip coefficient 1 (a.from -> a.to): the clip
// norm needs every chunk, and the next kernel (the next minibatch's gradient kernel or
// k_apply<.., true>) checks it and redoes the step when clipping was due.
//
// With kDP (several ranks, ppo_minibatch_fused_dp) the chunk is all-reduced before that step: a one-shot
// exchange over xGMI peer memory (include/usv_hip.h ppo_dp_t).  Slot q of rank s's chunk goes to every
// rank r's receive buffer x_r[par][s][q] (system-scope sc0 sc1 stores: write-through to the receiver's
// memory), every storing wave waits for its stores, then lane r of wave 0 raises rank r's flag of
// (chunk, sender s) to this minibatch's key v = *dp.clock (par = v & 1: a sender can be at most one
// minibatch ahead of a receiver, so two parities never collide).  Wave 0 polls this rank's flags of
// the chunk (system-scope loads; a wall-clock bound sets dp.err instead of hanging on a lost peer),
// a barrier releases the other waves, and the senders are summed in rank order (sc0 sc1 loads), so
// every rank forms the same bits; / world as the reference's all_grads / rank_size.  The KL rides in
// its loss slot as each rank's minibatch mean (av_kls SUM / rank_size, a2c_common.py:1218-1222).
constexpr int DP_SLOTS = RED_BLOCKS * RD_P;                  // slot space of one sender
constexpr int DP_FLAG_STRIDE = 32;                            // uint32 per flag: one 128-B line each
constexpr long long DP_X_BYTES = 2LL * PPO_DP_MAX * DP_SLOTS * 4;
constexpr long long DP_FLAG_OFF = (DP_X_BYTES + 4095) / 4096 * 4096;
constexpr long long DP_BYTES = DP_FLAG_OFF + (long long)RED_BLOCKS * PPO_DP_MAX * DP_FLAG_STRIDE * 4;
__device__ __forceinline__ void st_sys(float *p, float v) {
  __hip_atomic_store(reinterpret_cast<uint32_t *>(p), __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float ld_sys(const float *p) {
  return __builtin_bit_cast(float, __hip_atomic_load(reinterpret_cast<const uint32_t *>(p), __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_SYSTEM));
}
__device__ __forceinline__ float *dp_x(void *buf, int par, int sender) {
  return reinterpret_cast<float *>(buf) + ((size_t)par * PPO_DP_MAX + sender) * DP_SLOTS;
}
__device__ __forceinline__ uint32_t *dp_flag(void *buf, int chunk, int sender) {
  return reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(buf) + DP_FLAG_OFF) +
         ((size_t)chunk * PPO_DP_MAX + sender) * DP_FLAG_STRIDE;
}

// One chunk of the exchange (every thread of an RD_TB workgroup calls it; tid < RD_P carry slot
// `slot` of chunk `chunk`): this rank's value pv to every rank's receive buffer, the arrival flags,
// the wait for every sender's key, and the senders' values summed in rank order (the same bits on
// every rank).  A wait beyond timeout_ms, or an error another workgroup already flagged, sets / sees
// bit 0 of dp.err and goes on with whatever arrived (the host raises after the epoch), so a lost peer
// costs one timeout per launch, not one per chunk.
// USV_DP_ORDER (bit mask; A/B builds override it): bit 0 = a system-scope RELEASE fence before the flag store
// (every payload store of the workgroup is ordered before the flag in the memory model, not only by the drained
// write-through stores); bit 1 = one system-scope ACQUIRE fence after the poll (the payload loads are ordered
// after the flags seen); 0 = relaxed flag store and poll: the guide's {sc0 sc1 stores and loads both sides}
// form (MI355X_MICROARCH.md, valid hand-off forms) -- every payload store and load is sc0 sc1, every storing wave
// drains its stores (s_waitcnt vmcnt(0)) before the workgroup barrier behind which one lane per receiver
// raises the flag, and every payload load follows the polling wave's match through a workgroup barrier.
// Default 2: the guide keeps the consumer's acquire for a hand-off that matches none of its measured rows
// (these are single-device rows; the exchange crosses xGMI), and the producer then needs sc1 stores drained
// before the flag (its conditions (2)-(3)), which the payload stores are.  Two-rank rehearsal on one box
// (profiles/r04/r04e_dp_order_ab.txt, update us per minibatch): 0: 46.7-46.8, 2: 47.4-48.1, 1: 58.0-58.2,
// 3: 59.2-60.4 -- the system-scope release (buffer_wbl2 sc0 sc1: the XCD L2's dirty lines written back) costs
// ~11 us per minibatch and orders nothing the drained write-through payload stores have not already.
#ifndef USV_DP_ORDER
#define USV_DP_ORDER 2
#endif
__device__ float dp_exchange(const ppo_dp_t &dp, uint32_t key, int chunk, int slot, float pv, int timeout_ms) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int par = (int)(key & 1u);
  if (tid < RD_P)
    for (int r = 0; r < dp.world; ++r) st_sys(dp_x(dp.peer[r], par, dp.rank) + slot, pv);
  __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave: its stores are acknowledged
  __syncthreads();
  if (w == 0) {
    if (lane < dp.world) {   // lane r raises rank r's flag of (this chunk, this sender)
      if constexpr ((USV_DP_ORDER & 1) != 0) {
        // release at system scope: the workgroup's payload stores (drained behind the barrier above) happen
        // before the flag in every rank's view; the explicit wait keeps the flag behind the write-back even
        // where the compiler's scoreboard analysis would drop it (MI355X_MICROARCH.md, compiler hazard)
        // (the guide's producer form: drained stores -> barrier -> release fence -> asm wait -> relaxed flag)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(dp_flag(dp.peer[lane], chunk, dp.rank), key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      } else {
        __hip_atomic_store(dp_flag(dp.peer[lane], chunk, dp.rank), key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    // poll this rank's flags of the chunk: every sender's key >= ours (a sender may be one ahead)
    const uint64_t t0 = wall_clock64(), lim = (uint64_t)timeout_ms * 100000ull;   // 100 MHz
    bool got = lane >= dp.world;
    while (true) {
      if (!got) {
        const uint32_t f = __hip_atomic_load(dp_flag(dp.peer[dp.rank], chunk, lane), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
        got = (int32_t)(f - key) >= 0;
      }
      if (__all(got)) break;
      const int32_t e = __hip_atomic_load(dp.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (e != 0) break;                           // already failed: do not wait again
      if (wall_clock64() - t0 > lim) {             // a lost peer: flag it and go on
        if (lane == 0) atomicOr(dp.err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    // acquire at system scope, once after the poll (polling with acquire loads costs 2-3x per hop): the
    // payload loads below are ordered after every flag this wave saw
    if constexpr ((USV_DP_ORDER & 2) != 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  float t = 0.f;
  if (tid < RD_P) {   // senders in rank order: the same sum on every rank
    const float *xs = dp_x(dp.peer[dp.rank], par, 0);
    for (int r = 0; r < dp.world; ++r) t += ld_sys(xs + (size_t)r * DP_SLOTS + slot);
  }
  return t;
}

// Start-up check of the exchange (ppo_dp_selftest): `rounds` exchanges with keys key0, key0 + 1, ...
// (both parities, each receive region written twice) of a payload that names (sender, round, slot);
// every received value is compared with what its sender wrote.  Bit 0 of dp.err: a flag did not
// arrive; bit 1: a payload arrived wrong or stale (a receive buffer the reader's caches do not see
// the peers' writes in).
__device__ __forceinline__ float dp_probe_value(int sender, int round, int slot) {
  return (float)(sender * 1000003 + round * 65537 + slot);   // exact in fp32 for the sizes here
}
__global__ __launch_bounds__(RD_TB) void k_dp_selftest(ppo_dp_t dp, uint32_t key0, int rounds, int timeout_ms) {
  const int tid = threadIdx.x;
  const int slot = blockIdx.x * RD_P + tid;
  for (int rd = 0; rd < rounds; ++rd) {
    const uint32_t key = key0 + (uint32_t)rd;
    (void)dp_exchange(dp, key, blockIdx.x, slot, dp_probe_value(dp.rank, rd, slot & 0xffff), timeout_ms);
    if (tid < RD_P) {
      const float *xs = dp_x(dp.peer[dp.rank], (int)(key & 1u), 0);
      bool bad = false;
      for (int r = 0; r < dp.world; ++r)
        bad |= ld_sys(xs + (size_t)r * DP_SLOTS + slot) != dp_probe_value(r, rd, slot & 0xffff);
      if (bad) atomicOr(dp.err, 2);
    }
    __syncthreads();
  }
}

template <bool kSpec, bool kDP>
__global__ __launch_bounds__(RD_TB) void k_reduce_partials(const float *__restrict__ partials, int nblk, float *grad,
                                                           float *losses, float inv_b, ppo_cfg_t c, AdamBanks a,
                                                           const float *__restrict__ opt_in, ppo_dp_t dp, int fold) {
  __shared__ float4 red[RD_G][RD_L];
  __shared__ float sqw[RD_TB / 64];
  USV_PHASE(red, 0);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int col = tid % RD_L, grp = tid / RD_L;
  const int p4 = blockIdx.x * RD_L + col;                 // float4 column of the partial rows
  const bool ok = p4 < NPART_PAD / 4;
  const float4 *P4 = reinterpret_cast<const float4 *>(partials);
  // the speculative step's inputs, loaded before the partial rows
  const int myslot = blockIdx.x * RD_P + tid;
  const bool mine = kSpec && tid < RD_P && myslot < S_END;
  const int pq = mine ? param_of_slot(myslot) : 0;
  float p_old = 0.f, m_old = 0.f, v_old = 0.f;
  if (mine) {
    p_old = a.P0[pq]; m_old = a.m0[pq]; v_old = a.v0[pq];
  }
  uint32_t key = 0u;
  if (kDP) key = *dp.clock;   // written by the preceding gradient kernel
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float oin[8] = {};   // the step's scalars: loads issued here, consumed after the row sums
  if (kSpec) {
#pragma unroll
    for (int q = 0; q < 8; ++q) oin[q] = opt_in[q];
  }
  const int p4c = min(p4, NPART_PAD / 4 - 1);
  if (fold) {   // the gradient kernel folded the rows of group g = grp (FOLD_G): one group row per group
    if (grp < FOLD_G) {
      const int M = nblk / FOLD_G;
      const uint32_t *ctl = fold_ctl(partials, nblk) + grp * FOLD_CTL_STRIDE;
      const uint32_t gen = ctl[0] / (uint32_t)M;
      bool folded = true;
      for (int mm = 0; mm < M; ++mm) folded &= ctl[32 + mm] == gen;
      if (folded) {
        acc = P4[(size_t)(nblk + grp) * (NPART_PAD / 4) + p4c];
      } else {   // a member timed out: the same sums from the raw rows, in the fold's order
        const int h0 = (M + 1) / 2;
        float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
        for (int mm = 0; mm < M; ++mm) {
          const float4 x = P4[(size_t)(grp + FOLD_G * mm) * (NPART_PAD / 4) + p4c];
          float4 &t = mm < h0 ? a0 : a1;
          t.x += x.x; t.y += x.y; t.z += x.z; t.w += x.w;
        }
        acc = make_float4(a0.x + a1.x, a0.y + a1.y, a0.z + a1.z, a0.w + a1.w);
      }
    }
  } else
  for (int b0 = grp; b0 < nblk; b0 += RD_G * RD_KB) {
    // branch-free: clamped rows / columns loaded, masked in the sum (every load in flight at once)
    float4 x[RD_KB];
#pragma unroll
    for (int k = 0; k < RD_KB; ++k) {
      const int row = min(b0 + RD_G * k, nblk - 1);
      const float4 *src = USV_PART_CM ? P4 + ((size_t)blockIdx.x * nblk + row) * RD_L + col
                                      : P4 + (size_t)row * (NPART_PAD / 4) + p4c;
#if USV_RD_NT
      const f32x4v v = __builtin_nontemporal_load(reinterpret_cast<const f32x4v *>(src));   // read once
      x[k] = make_float4(v[0], v[1], v[2], v[3]);
#else
      x[k] = *src;
#endif
    }
    // the bias corrections in the shadow of the row loads (they wait on opt_in only)
#pragma unroll
    for (int k = 0; k < RD_KB; ++k) {
      if (ok && b0 + RD_G * k < nblk) {
        acc.x += x[k].x; acc.y += x[k].y; acc.z += x[k].z; acc.w += x[k].w;
      }
    }
  }
  USV_PHASE(red, 1);   // (thread 0's row sums: its loads have landed)
  AdamK ak = {0.f, 1.f};
  if (kSpec)   // uniform: precomputed by the previous step's opt_store (no pow on this path)
    ak = adam_consts_tagged(c, oin[0], oin[1] + 1.0f, oin[4], oin[5], oin[6], oin[7]);
  red[grp][col] = acc;
  __syncthreads();
  float s = 0.f;
  const int slot = blockIdx.x * RD_P + tid;
  if (tid < RD_P) {
#pragma unroll
    for (int g = 0; g < RD_G; ++g) s += reinterpret_cast<const float *>(red[g])[tid];
  }
  USV_PHASE(red, 2);
  float sl = s;   // this rank's value of the slot (the loss means are rank-local)
  if constexpr (kDP) {   // the chunk to every rank (gradient sums; the KL slot as this rank's mean)
    const float pv = slot < S_END ? s : (slot == PPO_NPARAM + 4 ? s * inv_b : 0.f);
    s = dp_exchange(dp, key, blockIdx.x, slot, pv, dp.timeout_ms) / (float)dp.world;   // all_grads / rank_size
  }
  float sq = 0.f;
  if (tid < RD_P) {
    if (slot < S_END) {
      grad[param_of_slot(slot)] = s;
      sq = s * s;
      if (mine) {   // k_apply's step with grad_scale = coef = 1 (g * 1 * 1 == g)
        float pn, mn, vn;
        adam_one(c, ak, s, p_old, m_old, v_old, pn, mn, vn);
        a.P1[pq] = pn; a.m1[pq] = mn; a.v1[pq] = vn;
      }
    } else if (slot < PPO_NPARAM + 5) {
      const int q = slot - PPO_NPARAM;
      if (q == 4) grad[PPO_NPARAM] = kDP ? s : s * inv_b;   // kl mean rides with the gradient (all-reduce)
      if (losses) losses[q] = sl * inv_b;
    }
  }
  USV_PHASE(red, 3);
  if (w < (RD_P + 63) / 64) {
    sq = wave_sum(sq);
    if (lane == 0) sqw[w] = sq;
  }
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < (RD_P + 63) / 64; ++q) t += sqw[q];
    grad[PPO_NPARAM + 8 + blockIdx.x] = t;
  }
  USV_PHASE(red, 4);
}

// clip_grad_norm_ + Adam + AdaptiveScheduler.  Every workgroup forms the same
// total norm (same order) and the same next learning rate, and updates its 256
// parameters (bank a.*0 -> a.*1; the same buffers for an in-place step).  The optimiser
// scalars are double-buffered: the launch reads slot opt_in and workgroup 0 writes the next
// values to slot opt_out, so no workgroup waits for another (no completion counter, no
// device-scope fence).  kFinish closes a chain of ppo_minibatch_fused launches: the last
// reduce kernel already took the unclipped step into bank 1, so parameters are written only
// when clipping was due.
constexpr int AP_TB = 256;
template <bool kNormFromPartials, bool kFinish>
__global__ __launch_bounds__(AP_TB) void k_apply(ppo_cfg_t c, AdamBanks a, const float *__restrict__ grad_in,
                                                 const float *__restrict__ opt_in, float *__restrict__ opt_out,
                                                 float grad_scale, float *kl_out) {
  __shared__ float red[AP_TB / 64];
  const int tid = threadIdx.x;
  const int q = blockIdx.x * AP_TB + tid;
  const int qc = min(q, PPO_NPARAM - 1);
  // every load this thread needs is issued before anything waits: its parameter,
  // moments and gradient, then the norm inputs; the double-precision bias
  // corrections below are computed while they are in flight
  const float g_raw = grad_in[qc], p_old = a.P0[qc], m_old = a.m0[qc], v_old = a.v0[qc];
  // the reduce kernel's per-chunk squares (fixed order; loaded unconditionally: no branch)
  const float s0 = grad_in[PPO_NPARAM + 8 + min(tid, RED_BLOCKS - 1)];
  const float lr = opt_in[0];
  const float step = opt_in[1] + 1.0f;
  const float kl = grad_in[PPO_NPARAM] * grad_scale;
  __builtin_amdgcn_sched_barrier(0);   // the loads above issue first
  const AdamK ak = adam_consts_tagged(c, lr, step, opt_in[4], opt_in[5], opt_in[6], opt_in[7]);
  // the next scalars (workgroup 0's first lane) in the same shadow
  OptNext nx = {};
  if (blockIdx.x == 0 && tid == 0) nx = opt_next(c, opt_in, kl);
  // pin these here, in the shadow of the loads above (the scheduler would otherwise sink
  // them past the norm's barrier onto the critical path)
  __asm__ volatile("" : : "v"(ak.step_size), "v"(ak.bc2s), "v"(nx.nl), "v"(nx.nk.step_size), "v"(nx.nk.bc2s));
  float ss = 0.f;
  if (kNormFromPartials) {
    ss = tid < RED_BLOCKS ? s0 : 0.f;
  } else {
    // total norm of the (all-reduced) gradient: 16-byte aligned, checked on the host
    constexpr int N4 = PPO_NPARAM / 4, U = (N4 + AP_TB - 1) / AP_TB;
    const float4 *g4 = reinterpret_cast<const float4 *>(grad_in);
    float4 gv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) gv[u] = g4[min(tid + u * AP_TB, N4 - 1)];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (tid + u * AP_TB >= N4) continue;
      const float x = gv[u].x * grad_scale, y = gv[u].y * grad_scale;
      const float z = gv[u].z * grad_scale, w = gv[u].w * grad_scale;
      ss = fmaf(x, x, ss); ss = fmaf(y, y, ss); ss = fmaf(z, z, ss); ss = fmaf(w, w, ss);
    }
    for (int r = 4 * N4 + tid; r < PPO_NPARAM; r += AP_TB) {
      const float g = grad_in[r] * grad_scale;
      ss = fmaf(g, g, ss);
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float total_norm = sqrtf(((red[0] + red[1]) + red[2]) + red[3]);
  const float coef = clip_coef(c, total_norm);
  if (q < PPO_NPARAM && (!kFinish || coef < 1.0f)) {
    float pn, mn, vn;
    adam_one(c, ak, g_raw * grad_scale * coef, p_old, m_old, v_old, pn, mn, vn);
    a.P1[q] = pn;
    a.m1[q] = mn;
    a.v1[q] = vn;
  }
  if (blockIdx.x == 0 && tid == 0) opt_store(c, nx, opt_out, total_norm, kl, kl_out);
}

}  // namespace

extern "C" {

int ppo_policy_step(const ppo_cfg_t *cfg, const float *params, const double *obs_rms, const double *val_rms,
                    const float *obs, int t, float *exp_obs, float *exp_act, float *exp_nlp, float *exp_val,
                    float *exp_mu, float *exp_sigma, uint8_t *exp_done, const int64_t *dones_prev,
                    float *actions_out, uint64_t seed, uint64_t step, const uint64_t *step_dev,
                    const float *eps_inject, void *stream) {
  if (!cfg || !params || !obs_rms || !obs || cfg->n_envs <= 0 || t < 0 || t >= cfg->horizon) return 1;
  // USV_POLICY_GRID caps the persistent grid (A/B knob: fewer CUs for the policy kernel leaves the
  // rest to the side stream's field kernels in the overlapped step; results do not depend on it)
  const char *gcap = getenv("USV_POLICY_GRID");
  const int grid_cap = gcap ? atoi(gcap) : 0;
  // USV_POLICY_RW=0: the LDS-staged form (same results)
  const char *rw = getenv("USV_POLICY_RW");
  const bool reg_w = !(rw && atoi(rw) == 0);
  const int ntiles = (cfg->n_envs + RB - 1) / RB;
  int grid = reg_w ? (ntiles < 256 * POL_WPC ? ntiles : 256 * POL_WPC) : policy_grid(cfg->n_envs);
  if (grid_cap > 0 && grid_cap < grid) grid = grid_cap;
  hipLaunchKernelGGL(reg_w ? k_policy_step<true> : k_policy_step<false>, dim3(grid), dim3(TB), 0, (hipStream_t)stream,
                     *cfg, params, obs_rms, val_rms, obs, t, exp_obs, exp_act, exp_nlp, exp_val, exp_mu, exp_sigma,
                     exp_done, dones_prev, actions_out, seed, step, step_dev, eps_inject);
  USV_CHECK_LAUNCH();
  return 0;
}

int ppo_value(const ppo_cfg_t *cfg, const float *params, const double *obs_rms, const double *val_rms,
              const float *obs, float *values, void *stream) {
  if (!cfg || !params || !obs_rms || !obs || !values || cfg->n_envs <= 0) return 1;
  const char *rw = getenv("USV_POLICY_RW");   // 0: the LDS-staged form (same results)
  const bool reg_w = !(rw && atoi(rw) == 0);
  const int ntiles = (cfg->n_envs + RB - 1) / RB;
  const int grid = reg_w ? (ntiles < 256 * POL_WPC ? ntiles : 256 * POL_WPC) : policy_grid(cfg->n_envs);
  hipLaunchKernelGGL(reg_w ? k_value<true> : k_value<false>, dim3(grid), dim3(TB), 0, (hipStream_t)stream, *cfg,
                     params, obs_rms, val_rms, obs, values);
  USV_CHECK_LAUNCH();
  return 0;
}

int ppo_store_reward(const ppo_cfg_t *cfg, const float *rew, const int64_t *dones, int t, float *exp_rew,
                     float *cur_rew, float *cur_shaped, float *cur_len, float *meter, uint64_t *step_dev,
                     void *stream) {
  if (!cfg || !rew || !dones || cfg->n_envs <= 0) return 1;
  const int nblk = (cfg->n_envs + kStoreTB - 1) / kStoreTB;
  hipLaunchKernelGGL(k_store_reward, dim3(nblk), dim3(kStoreTB), 0, (hipStream_t)stream, *cfg, rew,
                     dones, t, exp_rew, cur_rew, cur_shaped, cur_len, meter, step_dev);
  USV_CHECK_LAUNCH();
  if (t == cfg->horizon - 1) {
    hipLaunchKernelGGL(k_meter_fold, dim3((cfg->horizon * 4 + 63) / 64), dim3(64), 0, (hipStream_t)stream, *cfg,
                       meter, nblk);
    USV_CHECK_LAUNCH();
  }
  return 0;
}

int ppo_prepare(const ppo_cfg_t *cfg, const float *params, const double *obs_rms, double *val_rms,
                const float *last_obs, const int64_t *last_dones, const uint8_t *exp_done, float *exp_val,
                const float *exp_rew, float *exp_ret, float *exp_adv, double *work, void *stream) {
  if (!cfg || !params || !work || cfg->n_envs <= 0) return 1;
  hipStream_t s = (hipStream_t)stream;
  // last values (get_values :407-430) into work-adjacent scratch: reuse exp_ret's tail? use a dedicated slice
  float *last_val = reinterpret_cast<float *>(work + 8 + 8 * 4096);
  if (ppo_value(cfg, params, obs_rms, val_rms, last_obs, last_val, stream)) return 2;
  const int nblk = (cfg->n_envs + TB - 1) / TB;
  if (nblk > 4096) return 3;
  // the vector form needs 16-byte aligned rows: H = 16 and 16-byte aligned buffers
  const char *gv = getenv("USV_GAE_VEC");   // 0: the runtime-H loop (tests, A/B)
  const bool vec16 = !(gv && atoi(gv) == 0) && cfg->horizon == 16 &&
                     ((reinterpret_cast<uintptr_t>(exp_val) | reinterpret_cast<uintptr_t>(exp_rew) |
                       reinterpret_cast<uintptr_t>(exp_ret) | reinterpret_cast<uintptr_t>(exp_adv) |
                       reinterpret_cast<uintptr_t>(exp_done)) & 15u) == 0;
  hipLaunchKernelGGL(vec16 ? k_gae<16> : k_gae<0>, dim3(nblk), dim3(TB), 0, s, *cfg, last_val, last_dones, exp_done,
                     exp_val, exp_rew, exp_ret, exp_adv, work);
  USV_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_prepare_finalize, dim3(1), dim3(FIN_TB), 0, s, *cfg, val_rms, work, nblk);
  USV_CHECK_LAUNCH();
  const size_t B = (size_t)cfg->n_envs * cfg->horizon;
  hipLaunchKernelGGL(k_prepare_apply, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, *cfg, work, exp_val,
                     exp_ret, exp_adv);
  USV_CHECK_LAUNCH();
  return 0;
}

// the XCD-group fold of the partial rows (FOLD_G): minibatches of 8 x 1..32 workgroups (the whole grid resident at
// one workgroup per CU).  Off by default: same-box A/B at 131072 envs (profiles/r04/r04c_fold_ab.txt), rocprof
// means fold 22.57 + 5.11 us vs 18.39 + 7.00 us without (write-through partial stores and the group wait
// +1.5 us, the fold's own load / store round 3.6 us, against 1.9 us saved in the reduction, whose time is its
// fixed latency rather than the 21.8 MB it reads).  USV_PPO_FOLD=1 turns it on; USV_PPO_FOLD=2: every member
// arrives but none folds -- the reduction's raw-row path, for the tests.
static int fold_env() {
  const char *e = getenv("USV_PPO_FOLD");
  return e ? atoi(e) : 0;
}
static bool fold_on(int nblk) {
  return fold_env() != 0 && nblk % FOLD_G == 0 && nblk / FOLD_G >= 1 && nblk / FOLD_G <= FOLD_MAX_M;
}

int ppo_minibatch_grad(const ppo_cfg_t *cfg, const float *params, double *obs_rms, const double *val_rms,
                       int update_obs_rms, int mb_index, const float *exp_obs, const float *exp_act,
                       const float *exp_nlp, const float *exp_val, const float *exp_ret, const float *exp_adv,
                       float *exp_mu, float *exp_sigma, float *grad, float *losses, float *partials, double *work,
                       void *stream) {
  (void)val_rms;
  if (!cfg || !params || !obs_rms || !grad || !partials || !work) return 1;
  if (cfg->minibatch % RB != 0 || ppo_partials_floats(cfg->minibatch) <= 0) return 2;   // no partial layout
  if (reinterpret_cast<uintptr_t>(params) & 15u) return 4;   // 16-byte weight staging loads
  hipStream_t s = (hipStream_t)stream;
  const int row0 = mb_index * cfg->minibatch;
  if (update_obs_rms && cfg->normalize_input) {
    // RunningMeanStd.train on the minibatch obs (mini-epoch 0 only, a2c_common.py:1243-1244);
    // partials at work[8..], completion counter in the bits of work[7]
    const int nb = 64;
    hipLaunchKernelGGL(k_obs_stats, dim3(nb), dim3(TB), 0, s, *cfg, exp_obs, row0, cfg->minibatch, work + 8, obs_rms,
                       reinterpret_cast<unsigned *>(work + 7));
    USV_CHECK_LAUNCH();
  }
  if (reinterpret_cast<uintptr_t>(partials) & 15u) return 3;
  const int nblk = cfg->minibatch / RB;
  const bool fold = fold_on(nblk);
  ChainIn ch{};
  ch.fold_skip = fold_env() == 2;
  hipLaunchKernelGGL((cfg->bf16_gemm ? (fold ? k_mb_grad<true, false, true> : k_mb_grad<true, false, false>)
                                     : (fold ? k_mb_grad<false, false, true> : k_mb_grad<false, false, false>)),
                     dim3(nblk), dim3(GTB), 0, s, *cfg, ch, params, obs_rms, row0, exp_obs, exp_act, exp_nlp,
                     exp_val, exp_ret, exp_adv, exp_mu, exp_sigma, partials);
  USV_CHECK_LAUNCH();
  hipLaunchKernelGGL((k_reduce_partials<false, false>), dim3(RED_BLOCKS), dim3(RD_TB), 0, s, partials, nblk, grad,
                     losses, 1.0f / (float)cfg->minibatch, *cfg, AdamBanks{}, nullptr, ppo_dp_t{}, (int)fold);
  USV_CHECK_LAUNCH();
  return 0;
}

static bool banks_ok(const ppo_adam_banks_t *b) {
  if (!b || !b->opt) return false;
  for (int i = 0; i < 2; ++i) {
    if (!b->params[i] || !b->m[i] || !b->v[i]) return false;
    if (reinterpret_cast<uintptr_t>(b->params[i]) & 15u) return false;   // 16-byte weight staging loads
  }
  return true;
}

static int fused_launch(const ppo_cfg_t *cfg, const ppo_adam_banks_t *banks, const ppo_dp_t *dp, int seq,
                        double *obs_rms, int update_obs_rms, int mb_index, const float *exp_obs, const float *exp_act,
                        const float *exp_nlp, const float *exp_val, const float *exp_ret, const float *exp_adv,
                        float *exp_mu, float *exp_sigma, float *grad, float *losses, float *partials, double *work,
                        float *kl_prev_out, void *stream) {
  if (!cfg || !obs_rms || !grad || !partials || !work || seq < 0) return 1;
  if (!banks_ok(banks)) return 4;
  if (cfg->minibatch % RB != 0 || ppo_partials_floats(cfg->minibatch) <= 0) return 2;   // no partial layout
  if (reinterpret_cast<uintptr_t>(partials) & 15u) return 3;
  if (dp) {
    if (dp->world < 1 || dp->world > PPO_DP_MAX || dp->rank < 0 || dp->rank >= dp->world || !dp->clock || !dp->err)
      return 5;
    for (int r = 0; r < dp->world; ++r)
      if (!dp->peer[r]) return 5;
  }
  hipStream_t s = (hipStream_t)stream;
  const int cur = seq & 1, prv = cur ^ 1, nblk = cfg->minibatch / RB, row0 = mb_index * cfg->minibatch;
  if (update_obs_rms && cfg->normalize_input) {
    hipLaunchKernelGGL(k_obs_stats, dim3(64), dim3(TB), 0, s, *cfg, exp_obs, row0, cfg->minibatch, work + 8, obs_rms,
                       reinterpret_cast<unsigned *>(work + 7));
    USV_CHECK_LAUNCH();
  }
  const float *P = banks->params[cur];
  const dim3 gg(nblk), gb(GTB);
  uint32_t *clk = dp ? dp->clock : nullptr;
  const bool fold = fold_on(nblk);
  if (seq == 0) {
    ChainIn ch{};
    ch.dp_clock = clk;
    ch.fold_skip = fold_env() == 2;
    hipLaunchKernelGGL((cfg->bf16_gemm ? (fold ? k_mb_grad<true, false, true> : k_mb_grad<true, false, false>)
                                       : (fold ? k_mb_grad<false, false, true> : k_mb_grad<false, false, false>)),
                       gg, gb, 0, s, *cfg, ch, P, obs_rms, row0, exp_obs, exp_act, exp_nlp, exp_val, exp_ret, exp_adv,
                       exp_mu, exp_sigma, partials);
  } else {
    const ChainIn ch{banks->params[prv], banks->m[prv], banks->v[prv], banks->params[cur], banks->m[cur],
                     banks->v[cur], grad, banks->opt + 8 * prv, banks->opt + 8 * cur, kl_prev_out, clk,
                     fold_env() == 2};
    hipLaunchKernelGGL((cfg->bf16_gemm ? (fold ? k_mb_grad<true, true, true> : k_mb_grad<true, true, false>)
                                       : (fold ? k_mb_grad<false, true, true> : k_mb_grad<false, true, false>)),
                       gg, gb, 0, s, *cfg, ch, P, obs_rms, row0, exp_obs, exp_act, exp_nlp, exp_val, exp_ret, exp_adv,
                       exp_mu, exp_sigma, partials);
  }
  USV_CHECK_LAUNCH();
  const AdamBanks a{banks->params[cur], banks->m[cur], banks->v[cur], banks->params[prv], banks->m[prv],
                    banks->v[prv]};
  if (dp)
    hipLaunchKernelGGL((k_reduce_partials<true, true>), dim3(RED_BLOCKS), dim3(RD_TB), 0, s, partials, nblk, grad,
                       losses, 1.0f / (float)cfg->minibatch, *cfg, a, banks->opt + 8 * cur, *dp, (int)fold);
  else
    hipLaunchKernelGGL((k_reduce_partials<true, false>), dim3(RED_BLOCKS), dim3(RD_TB), 0, s, partials, nblk, grad,
                       losses, 1.0f / (float)cfg->minibatch, *cfg, a, banks->opt + 8 * cur, ppo_dp_t{}, (int)fold);
  USV_CHECK_LAUNCH();
  return 0;
}

int ppo_minibatch_fused(const ppo_cfg_t *cfg, const ppo_adam_banks_t *banks, int seq, double *obs_rms,
                        int update_obs_rms, int mb_index, const float *exp_obs, const float *exp_act,
                        const float *exp_nlp, const float *exp_val, const float *exp_ret, const float *exp_adv,
                        float *exp_mu, float *exp_sigma, float *grad, float *losses, float *partials, double *work,
                        float *kl_prev_out, void *stream) {
  return fused_launch(cfg, banks, nullptr, seq, obs_rms, update_obs_rms, mb_index, exp_obs, exp_act, exp_nlp, exp_val,
                      exp_ret, exp_adv, exp_mu, exp_sigma, grad, losses, partials, work, kl_prev_out, stream);
}

int ppo_minibatch_fused_dp(const ppo_cfg_t *cfg, const ppo_adam_banks_t *banks, const ppo_dp_t *dp, int seq,
                           double *obs_rms, int update_obs_rms, int mb_index, const float *exp_obs,
                           const float *exp_act, const float *exp_nlp, const float *exp_val, const float *exp_ret,
                           const float *exp_adv, float *exp_mu, float *exp_sigma, float *grad, float *losses,
                           float *partials, double *work, float *kl_prev_out, void *stream) {
  if (!dp) return 5;
  return fused_launch(cfg, banks, dp, seq, obs_rms, update_obs_rms, mb_index, exp_obs, exp_act, exp_nlp, exp_val,
                      exp_ret, exp_adv, exp_mu, exp_sigma, grad, losses, partials, work, kl_prev_out, stream);
}

// Several ranks without the peer exchange (the RCCL fallback): two launches per minibatch and an in-stream SUM
// all-reduce of grad[0, PPO_NPARAM] by the caller in between.  Minibatch seq's gradient kernel first takes
// minibatch seq - 1's step in every workgroup (redo_step: the all-reduced gradient x grad_scale, k_apply's clip
// norm of it) from bank (seq - 1) % 2 into bank seq % 2 and trains on the result; its reduction writes the plain
// gradient sum (ppo_minibatch_grad's); ppo_minibatch_coll_finish takes the last step (k_apply).  The same bits as
// ppo_minibatch_grad + all-reduce + ppo_minibatch_apply(grad_scale, norm_from_partials = 0).
int ppo_minibatch_coll(const ppo_cfg_t *cfg, const ppo_adam_banks_t *banks, int seq, float grad_scale,
                       double *obs_rms, int update_obs_rms, int mb_index, const float *exp_obs, const float *exp_act,
                       const float *exp_nlp, const float *exp_val, const float *exp_ret, const float *exp_adv,
                       float *exp_mu, float *exp_sigma, float *grad, float *losses, float *partials, double *work,
                       float *kl_prev_out, void *stream) {
  if (!cfg || !obs_rms || !grad || !partials || !work || seq < 0 || !(grad_scale > 0.f)) return 1;
  if (!banks_ok(banks)) return 4;
  if (cfg->minibatch % RB != 0 || ppo_partials_floats(cfg->minibatch) <= 0) return 2;   // no partial layout
  if ((reinterpret_cast<uintptr_t>(partials) | reinterpret_cast<uintptr_t>(grad)) & 15u) return 3;
  hipStream_t s = (hipStream_t)stream;
  const int cur = seq & 1, prv = cur ^ 1, nblk = cfg->minibatch / RB, row0 = mb_index * cfg->minibatch;
  if (update_obs_rms && cfg->normalize_input) {
    hipLaunchKernelGGL(k_obs_stats, dim3(64), dim3(TB), 0, s, *cfg, exp_obs, row0, cfg->minibatch, work + 8, obs_rms,
                       reinterpret_cast<unsigned *>(work + 7));
    USV_CHECK_LAUNCH();
  }
  const float *P = banks->params[cur];
  if (seq == 0) {
    ChainIn ch{};
    hipLaunchKernelGGL((cfg->bf16_gemm ? k_mb_grad<true, false, false> : k_mb_grad<false, false, false>), dim3(nblk),
                       dim3(GTB), 0, s, *cfg, ch, P, obs_rms, row0, exp_obs, exp_act, exp_nlp, exp_val, exp_ret,
                       exp_adv, exp_mu, exp_sigma, partials);
  } else {
    const ChainIn ch{banks->params[prv], banks->m[prv], banks->v[prv], banks->params[cur], banks->m[cur],
                     banks->v[cur], grad, banks->opt + 8 * prv, banks->opt + 8 * cur, kl_prev_out, nullptr, 0,
                     grad_scale};
    hipLaunchKernelGGL((cfg->bf16_gemm ? k_mb_grad<true, true, false, true> : k_mb_grad<false, true, false, true>),
                       dim3(nblk), dim3(GTB), 0, s, *cfg, ch, P, obs_rms, row0, exp_obs, exp_act, exp_nlp, exp_val,
                       exp_ret, exp_adv, exp_mu, exp_sigma, partials);
  }
  USV_CHECK_LAUNCH();
  hipLaunchKernelGGL((k_reduce_partials<false, false>), dim3(RED_BLOCKS), dim3(RD_TB), 0, s, partials, nblk, grad,
                     losses, 1.0f / (float)cfg->minibatch, *cfg, AdamBanks{}, nullptr, ppo_dp_t{}, 0);
  USV_CHECK_LAUNCH();
  return 0;
}

int ppo_minibatch_coll_finish(const ppo_cfg_t *cfg, const ppo_adam_banks_t *banks, int count, const float *grad,
                              float grad_scale, float *kl_out, void *stream) {
  if (!cfg || !grad || count < 1 || !(grad_scale > 0.f)) return 1;
  if (!banks_ok(banks)) return 4;
  if (reinterpret_cast<uintptr_t>(grad) & 15u) return 2;
  const int prv = (count - 1) & 1, cur = count & 1;
  const AdamBanks a{banks->params[prv], banks->m[prv], banks->v[prv], banks->params[cur], banks->m[cur],
                    banks->v[cur]};
  hipLaunchKernelGGL((k_apply<false, false>), dim3((PPO_NPARAM + AP_TB - 1) / AP_TB), dim3(AP_TB), 0,
                     (hipStream_t)stream, *cfg, a, grad, banks->opt + 8 * prv, banks->opt + 8 * cur, grad_scale,
                     kl_out);
  USV_CHECK_LAUNCH();
  return 0;
}

long long ppo_dp_buffer_bytes(void) { return DP_BYTES; }

int ppo_dp_selftest(const ppo_dp_t *dp, unsigned key0, int rounds, int timeout_ms, void *stream) {
  if (!dp || dp->world < 1 || dp->world > PPO_DP_MAX || dp->rank < 0 || dp->rank >= dp->world || !dp->err ||
      rounds < 1 || timeout_ms < 1)
    return 1;
  for (int r = 0; r < dp->world; ++r)
    if (!dp->peer[r]) return 2;
  hipLaunchKernelGGL(k_dp_selftest, dim3(RED_BLOCKS), dim3(RD_TB), 0, (hipStream_t)stream, *dp, (uint32_t)key0,
                     rounds, timeout_ms);
  USV_CHECK_LAUNCH();
  return 0;
}

int ppo_dp_alloc(void **dptr, void *ipc_handle) {
  if (!dptr || !ipc_handle) return 1;
  static_assert(sizeof(hipIpcMemHandle_t) == 64, "ipc handle size");
  // uncached device memory (as RCCL's IPC buffers): the peers' xGMI writes land in HBM, and no L2 of the
  // reading device can hold a stale copy of a flag or payload line it polled before; plain device memory
  // (hipMalloc) only if that allocation is refused.  USV_DP_MALLOC=plain forces hipMalloc (A/B).
  const char *mode = getenv("USV_DP_MALLOC");
  const bool plain = mode && strcmp(mode, "plain") == 0;
  if (plain || hipExtMallocWithFlags(dptr, (size_t)DP_BYTES, hipDeviceMallocUncached) != hipSuccess) {
    (void)hipGetLastError();
    if (hipMalloc(dptr, (size_t)DP_BYTES) != hipSuccess) return 2;
  }
  if (hipMemset(*dptr, 0, (size_t)DP_BYTES) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 3;
  hipIpcMemHandle_t h;
  if (hipIpcGetMemHandle(&h, *dptr) != hipSuccess) return 4;
  memcpy(ipc_handle, &h, sizeof(h));
  return 0;
}

int ppo_dp_open(const void *ipc_handle, void **dptr) {
  if (!dptr || !ipc_handle) return 1;
  hipIpcMemHandle_t h;
  memcpy(&h, ipc_handle, sizeof(h));
  return hipIpcOpenMemHandle(dptr, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess ? 0 : 2;
}

int ppo_dp_close(void *dptr) { return hipIpcCloseMemHandle(dptr) == hipSuccess ? 0 : 1; }
int ppo_dp_free(void *dptr) { return hipFree(dptr) == hipSuccess ? 0 : 1; }

int ppo_minibatch_finish(const ppo_cfg_t *cfg, const ppo_adam_banks_t *banks, int count, const float *grad,
                         float *kl_out, void *stream) {
  if (!cfg || !grad || count <= 0) return 1;
  if (!banks_ok(banks)) return 4;
  const int last = (count - 1) & 1, nxt = last ^ 1;
  const AdamBanks a{banks->params[last], banks->m[last], banks->v[last], banks->params[nxt], banks->m[nxt],
                    banks->v[nxt]};
  hipLaunchKernelGGL((k_apply<true, true>), dim3((PPO_NPARAM + AP_TB - 1) / AP_TB), dim3(AP_TB), 0,
                     (hipStream_t)stream, *cfg, a, grad, banks->opt + 8 * last, banks->opt + 8 * nxt, 1.0f, kl_out);
  USV_CHECK_LAUNCH();
  return 0;
}

int ppo_rms_seq_doubles(const ppo_cfg_t *cfg, int rows) {
  if (!cfg || cfg->minibatch <= 0 || rows < cfg->minibatch) return -1;
  const int nmb = rows / cfg->minibatch;
  return nmb * 2 * NIN + nmb * OM_CH * 2 * NIN;
}

int ppo_obs_rms_epoch(const ppo_cfg_t *cfg, const float *exp_obs, int rows, double *obs_rms, double *rms_seq,
                      void *stream) {
  if (!cfg || !exp_obs || !obs_rms || !rms_seq || cfg->minibatch <= 1 || rows < cfg->minibatch) return 1;
  const int nmb = rows / cfg->minibatch;
  hipStream_t s = (hipStream_t)stream;
  double *part = rms_seq + (size_t)nmb * 2 * NIN;
  hipLaunchKernelGGL(k_obs_moments, dim3(nmb, OM_CH), dim3(TB), 0, s, *cfg, exp_obs, part);
  USV_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_obs_rms_seq, dim3(1), dim3(RS_TB), 0, s, *cfg, part, nmb, obs_rms, rms_seq);
  USV_CHECK_LAUNCH();
  return 0;
}

int ppo_minibatch_apply(const ppo_cfg_t *cfg, float *params, float *grad, float *adam_m, float *adam_v, float *opt,
                        int opt_slot, float grad_scale, float *kl_out, int norm_from_partials, void *stream) {
  if (!cfg || !params || !grad || !adam_m || !adam_v || !opt) return 1;
  if (reinterpret_cast<uintptr_t>(grad) & 15u) return 2;
  if (opt_slot != 0 && opt_slot != 1) return 3;
  const AdamBanks a{params, adam_m, adam_v, params, adam_m, adam_v};
  hipLaunchKernelGGL((norm_from_partials ? k_apply<true, false> : k_apply<false, false>),
                     dim3((PPO_NPARAM + AP_TB - 1) / AP_TB), dim3(AP_TB), 0, (hipStream_t)stream, *cfg, a, grad,
                     opt + 8 * opt_slot, opt + 8 * (1 - opt_slot), grad_scale, kl_out);
  USV_CHECK_LAUNCH();
  return 0;
}

// per-workgroup rows, the fold's group rows and its control lines (zero-initialised by the caller)
int ppo_partials_floats(int minibatch) {
  static_assert(RED_BLOCKS * RD_P >= NPART_PAD, "chunk-major rows cover a partial row");
  if (minibatch < RB || minibatch % RB != 0) return -1;
  const long long f = (long long)part_body_floats(minibatch / RB) + FOLD_G * FOLD_CTL_STRIDE;
  return f > 0x7fffffffLL ? -1 : (int)f;
}
int ppo_grad_floats(void) { return PPO_NPARAM + 8 + RED_BLOCKS; }
int ppo_meter_floats(int n_envs, int horizon) {
  return horizon * 4 + horizon * ((n_envs + kStoreTB - 1) / kStoreTB) * 4;
}

}  // extern "C"
