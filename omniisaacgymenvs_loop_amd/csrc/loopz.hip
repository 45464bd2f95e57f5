// loopz trainer hot path (the reference's default trainer, scripts/rlgames_train.py:273-484)
// for MI355X (gfx950), fp32 end to end.
//
// Replaces (omniisaacgymenvs/algo/ppo/...):
//   module.py:184-361  MLPEncode / MLPEncode_wrap (mass encoder 8-64-16-8 + main MLP, LeakyReLU)
//   module.py:517-659  SquashedGaussianDiagonalCovariance.sample / evaluate / enforce_minimum_std
//   ppo.py:102-153     PPO.observe / PPO.step (actor.sample, critic.predict, storage.add_transitions)
//   storage.py:92-121  RolloutStorage.compute_returns (GAE, advantage normalisation)
//   ppo.py:237-321     PPO._train_step (in-order minibatches, clipped surrogate + clipped value loss,
//                      clip_grad_norm_, torch.optim.Adam, non-finite loss skip)
//
// Layout: the flat parameter vector is the optimizer's param order (actor net | std | critic net);
// rollout storage is time-major [T][N] as RolloutStorage keeps it, so an in-order minibatch is a
// contiguous row range.  Each network's 32-row tile runs the main MLP on the f32 matrix cores
// (v_mfma_f32_32x32x2_f32, weights staged once per workgroup in LDS, activations in LDS) and the
// tiny mass encoder on the VALU.  The gradient kernel is persistent over the minibatch's tiles:
// every weight gradient accumulates in registers (matrix-core accumulators for the two big
// layers) across the workgroup's tiles and leaves once as a per-workgroup partial, summed in a
// fixed order (deterministic) by the reduction kernel before clip + Adam.
#include "usv_device.h"

namespace {

constexpr int NH = LZ_NH, MS = LZ_MASS, LT = LZ_LAT, E1 = LZ_E1, E2 = LZ_E2, NA = LZ_NA;
constexpr int RB = 32;     // rows per tile
constexpr int TB = 256;    // threads per workgroup: wave w owns output columns 32w..32w+31
constexpr int XS = 36;     // row stride of the main input z / W1 in LDS (>= obs_dim, zero padded)
constexpr int HS = 130;    // row stride of h1 / h2 / W2 in LDS
constexpr float kSlope = 0.01f;             // nn.LeakyReLU negative_slope
constexpr float kSqEps = 1e-6f;             // SquashedGaussian eps (module.py:519)
constexpr float kHalfLog2Pi = 0.91893853320467274178f;   // log(sqrt(2 pi)) (torch Normal.log_prob)

typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
// C/D layout of a 32x32 tile: lane l holds column l&31, rows (r&3) + 8(r>>2) + 4(l>>5)
__device__ __forceinline__ int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
__device__ __forceinline__ float lrelu(float x) { return x > 0.f ? x : x * kSlope; }
__device__ __forceinline__ float dlrelu(float y) { return y > 0.f ? 1.f : kSlope; }   // y > 0 <=> x > 0

// offsets of one MLPEncode inside the flat vector (module order: mass_encoder, then action_mlp)
struct NetOff {
  int e0w, e0b, e2w, e2b, e4w, e4b, m0w, m0b, m2w, m2b, m4w, m4b, size;
};
__host__ __device__ inline NetOff net_off(int obs_dim, int nout) {
  NetOff o{};
  int p = 0;
  o.e0w = p; p += E1 * MS; o.e0b = p; p += E1;
  o.e2w = p; p += E2 * E1; o.e2b = p; p += E2;
  o.e4w = p; p += LT * E2; o.e4b = p; p += LT;
  o.m0w = p; p += NH * obs_dim; o.m0b = p; p += NH;
  o.m2w = p; p += NH * NH; o.m2b = p; p += NH;
  o.m4w = p; p += nout * NH; o.m4b = p; p += nout;
  o.size = p;
  return o;
}
__host__ __device__ inline int actor_base() { return 0; }
__host__ __device__ inline int std_base(int obs_dim) { return net_off(obs_dim, NA).size; }
__host__ __device__ inline int critic_base(int obs_dim) { return std_base(obs_dim) + NA; }
__host__ __device__ inline int nparam(int obs_dim) { return critic_base(obs_dim) + net_off(obs_dim, 1).size; }
// per-workgroup partial row of one network: its parameters, then 4 extra slots
// (actor: dstd0, dstd1, surrogate sum, log-prob sum; critic: value-loss sum, 0, 0, 0)
__host__ __device__ inline int part_stride(int obs_dim) { return (net_off(obs_dim, NA).size + 5 + 3) & ~3; }

constexpr int ENC_N = E1 * MS + E1 + E2 * E1 + E2 + LT * E2 + LT;   // 1752
struct NetSmem {
  float w2[NH * HS];        // W2[j][k]
  float w1[NH * XS];        // W1[j][k], k >= obs_dim zero
  float enc[ENC_N];         // mass encoder, flat in parameter order
  float b1[NH], b2[NH];
  float w3[NA * NH], b3[NA];
  float x[RB * XS];         // main input z = [speed | task | latent], zero padded
  float m[RB * MS];         // mass / CoM inputs of the encoder
  float e1[RB * E1];        // encoder activations (backward: de1 in place)
  float e2[RB * E2];
  float de2[RB * E2];
  float dl[RB * LT];        // d latent
  float h1[RB * HS];        // layer 1 (backward: dz1 in place)
  float h2[RB * HS];        // layer 2 (backward: dz2 in place)
  float out[RB * NA];       // head outputs (pre-activation)
  float g[RB * NA];         // d head outputs
  float red[TB];
};

// Stage one network's weights into LDS (once per workgroup).
__device__ void stage_net(const float *__restrict__ P, const NetOff &o, int obs_dim, int nout, NetSmem &s) {
  const int tid = threadIdx.x;
  for (int q = tid; q < NH * NH; q += TB) s.w2[(q >> 7) * HS + (q & (NH - 1))] = P[o.m2w + q];
  for (int q = tid; q < NH * XS; q += TB) {
    const int j = q / XS, k = q % XS;
    s.w1[q] = k < obs_dim ? P[o.m0w + j * obs_dim + k] : 0.f;
  }
  for (int q = tid; q < ENC_N; q += TB) s.enc[q] = P[o.e0w + q];
  if (tid < NH) { s.b1[tid] = P[o.m0b + tid]; s.b2[tid] = P[o.m2b + tid]; }
  for (int q = tid; q < NA * NH; q += TB) s.w3[q] = q < nout * NH ? P[o.m4w + q] : 0.f;
  if (tid < NA) s.b3[tid] = tid < nout ? P[o.m4b + tid] : 0.f;
}

// Rows [row0, row0 + nrows) of obs (row stride obs_dim) into s.m / s.x (nan_to_num, as
// storage.add_transitions and PPO.observe sanitise); rows past nrows repeat the last row.  With ridx
// (the shuffle sampler's minibatch indices) tile row r is storage row ridx[r] instead of row0 + r.
__device__ void stage_rows(const float *__restrict__ obs, size_t row0, int nrows, int obs_dim, NetSmem &s,
                           const int32_t *__restrict__ ridx = nullptr) {
  const int tid = threadIdx.x;
  const int nsp = obs_dim - MS;
  for (int q = tid; q < RB * XS; q += TB) {
    const int r = q / XS, k = q % XS;
    const int rc = r < nrows ? r : nrows - 1;
    const size_t row = ridx ? (size_t)ridx[rc] : row0 + rc;
    float v = 0.f;
    if (k < obs_dim) {
      v = obs[row * (size_t)obs_dim + k];
      if (!isfinite(v)) v = 0.f;
    }
    if (k < nsp) s.x[q] = v;
    else if (k < obs_dim) s.m[r * MS + (k - nsp)] = v;
    if (k >= nsp) s.x[q] = 0.f;   // latent slots are written by the encoder, padding stays 0
  }
}

// Forward of the staged tile: mass encoder (VALU), main MLP (MFMA), head pre-activations in s.out.
__device__ void tile_forward(int obs_dim, int nout, NetSmem &s) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 31, h = lane >> 5, n0 = 32 * w;
  const int nsp = obs_dim - MS;
  const float *We0 = s.enc, *be0 = We0 + E1 * MS, *We2 = be0 + E1, *be2 = We2 + E2 * E1, *We4 = be2 + E2,
              *be4 = We4 + LT * E2;
  __syncthreads();
  // mass encoder layer 0: 32 rows x 64 units, 8 per thread (k-ordered fmaf)
#pragma unroll
  for (int u = 0; u < RB * E1 / TB; ++u) {
    const int q = tid + u * TB, r = q / E1, j = q % E1;
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < MS; ++k) a = fmaf(s.m[r * MS + k], We0[j * MS + k], a);
    s.e1[q] = lrelu(a + be0[j]);
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < RB * E2 / TB; ++u) {
    const int q = tid + u * TB, r = q / E2, j = q % E2;
    float a = 0.f;
#pragma unroll 16
    for (int k = 0; k < E1; ++k) a = fmaf(s.e1[r * E1 + k], We2[j * E1 + k], a);
    s.e2[q] = lrelu(a + be2[j]);
  }
  __syncthreads();
  {
    const int r = tid / LT, j = tid % LT;   // 32 x 8 = TB
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < E2; ++k) a = fmaf(s.e2[r * E2 + k], We4[j * E2 + k], a);
    s.x[r * XS + nsp + j] = lrelu(a + be4[j]);
  }
  __syncthreads();
  // main layer 0: h1 = lrelu(z W1^T + b1), K = XS (zero padded)
  {
    f32x16 acc = {};
#pragma unroll
    for (int st = 0; st < XS / 2; ++st) {
      const int k = 2 * st + h;
      acc = mfma32(s.x[i * XS + k], s.w1[(n0 + i) * XS + k], acc);
    }
    const float bj = s.b1[n0 + i];
#pragma unroll
    for (int r = 0; r < 16; ++r) s.h1[crow(r, h) * HS + n0 + i] = lrelu(acc[r] + bj);
  }
  __syncthreads();
  {
    f32x16 acc = {};
#pragma unroll 16
    for (int st = 0; st < NH / 2; ++st) {
      const int k = 2 * st + h;
      acc = mfma32(s.h1[i * HS + k], s.w2[(n0 + i) * HS + k], acc);
    }
    const float bj = s.b2[n0 + i];
#pragma unroll
    for (int r = 0; r < 16; ++r) s.h2[crow(r, h) * HS + n0 + i] = lrelu(acc[r] + bj);
  }
  __syncthreads();
  // head: 8 threads per row, 16 k each
  {
    const int r = tid / 8, part = tid % 8;
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int k = part * 16; k < part * 16 + 16; ++k) {
      const float hv = s.h2[r * HS + k];
      a0 = fmaf(s.w3[k], hv, a0);
      a1 = fmaf(s.w3[NH + k], hv, a1);
    }
#pragma unroll
    for (int mm = 1; mm < 8; mm <<= 1) {
      a0 += __shfl_xor(a0, mm, 64);
      a1 += __shfl_xor(a1, mm, 64);
    }
    if (part == 0) {
      s.out[r * NA] = a0 + s.b3[0];
      if (nout > 1) s.out[r * NA + 1] = a1 + s.b3[1];
    }
  }
  __syncthreads();
}

__device__ __forceinline__ float normal_log_prob(float u, float mu, float sd) {
  // torch Normal.log_prob: -((value - loc) ** 2) / (2 * var) - log(scale) - log(sqrt(2 pi))
  const float d = u - mu;
  return ((-(d * d)) / (2.0f * (sd * sd)) - logf(sd)) - kHalfLog2Pi;
}
__device__ __forceinline__ float squash_log_det(const lz_cfg_t &c, float u0, float u1) {
  // log(action_scale + eps).sum() + log(1 - tanh(u)^2 + eps).sum(1) (module.py:563)
  const float t0 = tanhf(u0), t1 = tanhf(u1);
  return (logf(c.action_scale[0] + kSqEps) + logf(c.action_scale[1] + kSqEps)) +
         (logf((1.0f - t0 * t0) + kSqEps) + logf((1.0f - t1 * t1) + kSqEps));
}

__host__ __device__ inline int fwd_grid(int n) { return (n + RB - 1) / RB < 256 ? (n + RB - 1) / RB : 256; }

// ------------------------------------------------------------------ rollout
template <bool kActor>
__global__ __launch_bounds__(TB) void k_lz_forward(lz_cfg_t c, const float *__restrict__ P, const float *__restrict__ obs,
                                                   int t, float *st_obs, float *st_act, float *st_logp, float *st_val,
                                                   float *actions_out, float *values_out, uint64_t seed, uint64_t step,
                                                   const float *__restrict__ eps_inject) {
  __shared__ NetSmem s;
  const int n = c.n_envs, D = c.obs_dim;
  const int nout = kActor ? NA : 1;
  const NetOff o = net_off(D, nout);
  const float *Pn = P + (kActor ? actor_base() : critic_base(D));
  stage_net(Pn, o, D, nout, s);
  const float sd0 = P[std_base(D)], sd1 = P[std_base(D) + 1];
  const int ntiles = (n + RB - 1) / RB;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int row0 = tile * RB, nrows = min(RB, n - row0);
    stage_rows(obs, row0, nrows, D, s);
    tile_forward(D, nout, s);
    const int r = threadIdx.x;
    if (r < nrows) {
      const int e = row0 + r;
      const size_t slot = (size_t)t * n + e;
      if (kActor) {
        const float mu0 = tanhf(s.out[r * NA]), mu1 = tanhf(s.out[r * NA + 1]);
        float z0, z1;
        if (eps_inject) {
          z0 = eps_inject[2 * e];
          z1 = eps_inject[2 * e + 1];
        } else {   // Normal.sample: Box-Muller on Philox(site 0x300)
          float u[4];
          philox_u4(seed, (uint32_t)e, step, 0x300u, u);
          const float rr0 = sqrtf(-2.0f * logf(1.0f - u[0])), rr1 = sqrtf(-2.0f * logf(1.0f - u[2]));
          z0 = rr0 * cosf(USV_2PI_F * u[1]);
          z1 = rr1 * cosf(USV_2PI_F * u[3]);
        }
        const float u0 = mu0 + sd0 * z0, u1 = mu1 + sd1 * z1;
        const float a0 = tanhf(u0) * c.action_scale[0], a1 = tanhf(u1) * c.action_scale[1];
        const float lp = (normal_log_prob(u0, mu0, sd0) + normal_log_prob(u1, mu1, sd1)) - squash_log_det(c, u0, u1);
        actions_out[2 * e] = a0;
        actions_out[2 * e + 1] = a1;
        if (st_act) {
          st_act[slot * 2] = isfinite(a0) ? a0 : 0.f;
          st_act[slot * 2 + 1] = isfinite(a1) ? a1 : 0.f;
          st_logp[slot] = isfinite(lp) ? lp : 0.f;
        }
      } else {
        const float v = s.out[r * NA];
        if (values_out) values_out[e] = isfinite(v) ? v : 0.f;
        if (st_val) st_val[slot] = isfinite(v) ? v : 0.f;
      }
    }
    if (kActor && st_obs) {   // the sanitised observation row into storage
      for (int q = threadIdx.x; q < nrows * D; q += TB) {
        const int rr = q / D, k = q % D;
        const float v = obs[(size_t)(row0 + rr) * D + k];
        st_obs[((size_t)t * n + row0 + rr) * D + k] = isfinite(v) ? v : 0.f;
      }
    }
    __syncthreads();
  }
}

__global__ void k_lz_store(lz_cfg_t c, const float *__restrict__ rew, const int64_t *__restrict__ dones, int t,
                           float *st_rew, uint8_t *st_done) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= c.n_envs) return;
  const float r = rew[e];
  st_rew[(size_t)t * c.n_envs + e] = isfinite(r) ? r : 0.f;
  st_done[(size_t)t * c.n_envs + e] = (uint8_t)(dones[e] != 0);
}

// ------------------------------------------------------------------ returns
// RolloutStorage.compute_returns: one thread per env walks t = T-1 .. 0 (time-major rows are
// coalesced across the wave); per-block fp64 sums of the raw advantages for the normalisation.
__global__ __launch_bounds__(256) void k_lz_gae(lz_cfg_t c, const float *__restrict__ last_values,
                                                const float *__restrict__ st_rew, const uint8_t *__restrict__ st_done,
                                                const float *__restrict__ st_val, float *st_ret, float *st_adv,
                                                double *work) {
  __shared__ double s1[4], s2[4];
  const int n = c.n_envs, T = c.horizon;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  double a_sum = 0.0, a_sq = 0.0;
  if (e < n) {
    const float g = c.gamma, gl = c.lam;
    float lv = last_values[e];
    if (!isfinite(lv)) lv = 0.f;
    float adv = 0.f;
    for (int t = T - 1; t >= 0; --t) {
      const size_t q = (size_t)t * n + e;
      const float nv = (t == T - 1) ? lv : st_val[q + n];
      const float nnt = 1.0f - (float)st_done[q];
      const float v = st_val[q];
      const float delta = (st_rew[q] + (nnt * g) * nv) - v;
      adv = delta + ((nnt * g) * gl) * adv;
      const float ret = adv + v;
      st_ret[q] = ret;
      const float a = ret - v;
      st_adv[q] = a;
      a_sum += (double)a;
      a_sq += (double)a * (double)a;
    }
  }
  // fixed-order block reduction
  for (int off = 32; off > 0; off >>= 1) {
    a_sum += __shfl_xor(a_sum, off, 64);
    a_sq += __shfl_xor(a_sq, off, 64);
  }
  if ((threadIdx.x & 63) == 0) { s1[threadIdx.x >> 6] = a_sum; s2[threadIdx.x >> 6] = a_sq; }
  __syncthreads();
  if (threadIdx.x == 0) {
    work[8 + 2 * blockIdx.x] = ((s1[0] + s1[1]) + s1[2]) + s1[3];
    work[8 + 2 * blockIdx.x + 1] = ((s2[0] + s2[1]) + s2[2]) + s2[3];
  }
}

__global__ void k_lz_adv_finalize(lz_cfg_t c, double *work, int nblk) {
  if (threadIdx.x != 0) return;
  double s = 0.0, q = 0.0;
  for (int b = 0; b < nblk; ++b) { s += work[8 + 2 * b]; q += work[8 + 2 * b + 1]; }
  const double cnt = (double)c.n_envs * (double)c.horizon;
  const double mean = s / cnt;
  double var = cnt > 1.0 ? (q - cnt * mean * mean) / (cnt - 1.0) : 0.0;
  if (var < 0.0) var = 0.0;
  double sd = sqrt(var);
  if (!isfinite(sd)) sd = 0.0;   // adv_std nan_to_num (storage.py:117)
  work[0] = mean;
  work[1] = sd;
}

__global__ void k_lz_adv_apply(lz_cfg_t c, const double *__restrict__ work, float *st_ret, float *st_adv) {
  const size_t q = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (size_t)c.n_envs * c.horizon) return;
  const float mean = (float)work[0], sd = (float)work[1];
  float a = (st_adv[q] - mean) / (sd + 1e-8f);
  if (!isfinite(a)) a = 0.f;
  st_adv[q] = a;
  const float r = st_ret[q];
  if (!isfinite(r)) st_ret[q] = 0.f;
}

// ------------------------------------------------------------ minibatch grad
// blockIdx < G: actor workgroups, blockIdx >= G: critic workgroups; each loops over the
// minibatch's tiles g, g + G, ... and writes one partial row.
template <bool kActor>
__device__ void grad_net(const lz_cfg_t &c, const float *__restrict__ P, int wg, int G, size_t mb_row0, int M,
                         const float *__restrict__ st_obs, const float *__restrict__ st_act,
                         const float *__restrict__ st_logp, const float *__restrict__ st_val,
                         const float *__restrict__ st_ret, const float *__restrict__ st_adv, float *part,
                         NetSmem &s, const int32_t *__restrict__ ridx) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int i = lane & 31, h = lane >> 5, n0 = 32 * w;
  const int D = c.obs_dim, nsp = D - MS, nx = D - 32;   // nx: W1 columns past the first 32 (1..4)
  const int nout = kActor ? NA : 1;
  const NetOff o = net_off(D, nout);
  const float *Pn = P + (kActor ? actor_base() : critic_base(D));
  stage_net(Pn, o, D, nout, s);
  const float sd0 = P[std_base(D)], sd1 = P[std_base(D) + 1];
  const float invB = 1.0f / (float)M;
  const float *We2 = s.enc + E1 * MS + E1, *We4 = We2 + E2 * E1 + E2;
  // register accumulators, carried across the tiles of this workgroup
  f32x16 acc2[4] = {}, acc1 = {};
  const int j = tid & (NH - 1), hf = tid >> 7;            // (unit, row half) for the VALU reductions
  float gw3[NA] = {}, gb2 = 0.f, gb1 = 0.f, gw1x[4] = {}, gb3[NA] = {};
  float ge4w = 0.f, ge4b = 0.f, ge2w[4] = {}, ge2b = 0.f, ge0w[2] = {}, ge0b = 0.f;
  float l_a = 0.f, l_b = 0.f, l_im = 0.f, gsd0 = 0.f, gsd1 = 0.f;   // loss sums (thread r < 32)
  const int ntiles = (M + RB - 1) / RB;
  for (int tile = wg; tile < ntiles; tile += G) {
    const int rt0 = tile * RB, nrows = min(RB, M - rt0);
    const size_t row0 = mb_row0 + rt0;
    const int32_t *tidx = ridx ? ridx + rt0 : nullptr;   // shuffle sampler: this tile's storage rows
    stage_rows(st_obs, row0, nrows, D, s, tidx);
    tile_forward(D, nout, s);
    // ---- losses and head gradients (one thread per row) ----
    if (tid < RB) {
      const int r = tid;
      float d0 = 0.f, d1 = 0.f;
      if (r < nrows) {
        const size_t q = tidx ? (size_t)tidx[r] : row0 + r;
        if (kActor) {
          const float mu0 = tanhf(s.out[r * NA]), mu1 = tanhf(s.out[r * NA + 1]);
          // SquashedGaussian.evaluate (module.py:586-637): u = atanh(clamp(a / (scale + eps)))
          float as0 = st_act[2 * q] / (c.action_scale[0] + kSqEps), as1 = st_act[2 * q + 1] / (c.action_scale[1] + kSqEps);
          as0 = clampt(as0, -1.0f + kSqEps, 1.0f - kSqEps);
          as1 = clampt(as1, -1.0f + kSqEps, 1.0f - kSqEps);
          const float u0 = 0.5f * (log1pf(as0) - log1pf(-as0)), u1 = 0.5f * (log1pf(as1) - log1pf(-as1));
          const float lp = (normal_log_prob(u0, mu0, sd0) + normal_log_prob(u1, mu1, sd1)) - squash_log_det(c, u0, u1);
          const float A = st_adv[q];
          const float ratio = expf(lp - st_logp[q]);
          const float lo = 1.0f - c.clip, hi = 1.0f + c.clip;
          const float s1 = -A * ratio, s2 = -A * clampt(ratio, lo, hi);
          const float inr = (ratio >= lo && ratio <= hi) ? 1.f : 0.f;
          const float g1 = -A, g2 = -A * inr;
          const float g_r = (s1 > s2) ? g1 : ((s1 < s2) ? g2 : 0.5f * (g1 + g2));
          // loss = mean(surr + c_v vl - c_e entropy), entropy = -log_prob
          const float dlp = (g_r * ratio + c.entropy_coef) * invB;
          const float var0 = sd0 * sd0, var1 = sd1 * sd1;
          float dmu0 = dlp * (u0 - mu0) / var0, dmu1 = dlp * (u1 - mu1) / var1;
          if (c.expert_act) {   // imitation: (1 - rl) * sum_a (expert_a - mu_a)^2, row mean (ppo.py:279-282)
            const float e0 = c.expert_act[2 * q], e1 = c.expert_act[2 * q + 1];
            dmu0 = dmu0 + c.im_coef * (2.0f * (mu0 - e0)) * invB;
            dmu1 = dmu1 + c.im_coef * (2.0f * (mu1 - e1)) * invB;
            l_im += c.im_coef * ((e0 - mu0) * (e0 - mu0) + (e1 - mu1) * (e1 - mu1));
          }
          d0 = dmu0 * (1.0f - mu0 * mu0);
          d1 = dmu1 * (1.0f - mu1 * mu1);
          gsd0 += dlp * ((u0 - mu0) * (u0 - mu0) / (var0 * sd0) - 1.0f / sd0);
          gsd1 += dlp * ((u1 - mu1) * (u1 - mu1) / (var1 * sd1) - 1.0f / sd1);
          l_a += fmaxf(s1, s2);
          l_b += lp;
        } else {
          const float v = s.out[r * NA], vo = st_val[q], R = st_ret[q];
          float dv, vl;
          if (c.use_clipped_value_loss) {
            const float dvr = v - vo;
            const float vc = vo + clampt(dvr, -c.clip, c.clip);
            const float l1 = (v - R) * (v - R), l2 = (vc - R) * (vc - R);
            vl = fmaxf(l1, l2);
            const float e1 = 2.f * (v - R);
            const float e2 = 2.f * (vc - R) * ((dvr >= -c.clip && dvr <= c.clip) ? 1.f : 0.f);
            dv = (l1 > l2) ? e1 : ((l1 < l2) ? e2 : 0.5f * (e1 + e2));
          } else {
            vl = (R - v) * (R - v);
            dv = 2.f * (v - R);
          }
          d0 = dv * c.value_loss_coef * invB;
          l_a += vl;
        }
      }
      s.g[r * NA] = d0;
      s.g[r * NA + 1] = d1;
    }
    __syncthreads();
    // ---- head weight grads, dz2 = (dout W3) lrelu'(h2) in place over h2 ----
    {
      const float w30 = s.w3[j], w31 = s.w3[NH + j];
      float dbsum = 0.f;
#pragma unroll 4
      for (int q = 0; q < RB / 2; ++q) {
        const int r = hf * (RB / 2) + q;
        const float hv = s.h2[r * HS + j];
        const float g0 = s.g[r * NA], g1 = s.g[r * NA + 1];
        gw3[0] = fmaf(g0, hv, gw3[0]);
        gw3[1] = fmaf(g1, hv, gw3[1]);
        const float dz = (g0 * w30 + g1 * w31) * dlrelu(hv);
        s.h2[r * HS + j] = dz;
        dbsum += dz;
        if (j == 0) { gb3[0] += g0; gb3[1] += g1; }
      }
      gb2 += dbsum;
    }
    __syncthreads();
    // ---- dW2[n][k] += sum_r dz2[r][n] h1[r][k]: wave w owns n block w, all 4 k blocks ----
#pragma unroll 4
    for (int st = 0; st < RB / 2; ++st) {
      const int r = st + (RB / 2) * h;
      const float a = s.h2[r * HS + n0 + i];
#pragma unroll
      for (int kb = 0; kb < 4; ++kb) acc2[kb] = mfma32(a, s.h1[r * HS + 32 * kb + i], acc2[kb]);
    }
    // ---- dh1[r][k] = sum_n dz2[r][n] W2[n][k]: wave w owns k block w ----
    f32x16 dh = {};
#pragma unroll 16
    for (int st = 0; st < NH / 2; ++st) {
      const int jn = 2 * st + h;
      dh = mfma32(s.h2[i * HS + jn], s.w2[jn * HS + n0 + i], dh);
    }
    __syncthreads();   // every read of h1 (dW2 operand) is done
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int idx = crow(q, h) * HS + n0 + i;
      s.h1[idx] = dh[q] * dlrelu(s.h1[idx]);   // h1 := dz1
    }
    __syncthreads();
    // ---- dW1 += dz1^T z: k < 32 on the matrix cores (wave w: n block w), k >= 32 and b1 on the VALU ----
#pragma unroll
    for (int st = 0; st < RB / 2; ++st) {
      const int r = st + (RB / 2) * h;
      acc1 = mfma32(s.h1[r * HS + n0 + i], s.x[r * XS + i], acc1);
    }
    {
      float db = 0.f;
      for (int q = 0; q < RB / 2; ++q) {
        const int r = hf * (RB / 2) + q;
        const float dz = s.h1[r * HS + j];
        db += dz;
#pragma unroll
        for (int cx = 0; cx < 4; ++cx)
          if (cx < nx) gw1x[cx] = fmaf(dz, s.x[r * XS + 32 + cx], gw1x[cx]);
      }
      gb1 += db;
    }
    // ---- d latent: (dz1 W1[:, nsp:]) lrelu'(lat), 32 rows x 8 ----
    {
      const int r = tid / LT, qq = tid % LT;
      float a = 0.f;
#pragma unroll 8
      for (int jj = 0; jj < NH; ++jj) a = fmaf(s.h1[r * HS + jj], s.w1[jj * XS + nsp + qq], a);
      s.dl[tid] = a * dlrelu(s.x[r * XS + nsp + qq]);
    }
    __syncthreads();
    // ---- encoder layer 4 grads, de2 ----
    if (tid < LT * E2) {
      const int qq = tid / E2, cc = tid % E2;
      float a = 0.f;
      for (int r = 0; r < RB; ++r) a = fmaf(s.dl[r * LT + qq], s.e2[r * E2 + cc], a);
      ge4w += a;
    } else if (tid < LT * E2 + LT) {
      const int qq = tid - LT * E2;
      float a = 0.f;
      for (int r = 0; r < RB; ++r) a += s.dl[r * LT + qq];
      ge4b += a;
    }
#pragma unroll
    for (int u = 0; u < RB * E2 / TB; ++u) {
      const int q = tid + u * TB, r = q / E2, cc = q % E2;
      float a = 0.f;
#pragma unroll
      for (int qq = 0; qq < LT; ++qq) a = fmaf(s.dl[r * LT + qq], We4[qq * E2 + cc], a);
      s.de2[q] = a * dlrelu(s.e2[q]);
    }
    __syncthreads();
    // ---- encoder layer 2 grads (reads e1), then de1 in place over e1 ----
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int p = tid + u * TB, cc = p / E1, k = p % E1;   // 16 x 64
      float a = 0.f;
      for (int r = 0; r < RB; ++r) a = fmaf(s.de2[r * E2 + cc], s.e1[r * E1 + k], a);
      ge2w[u] += a;
    }
    if (tid < E2) {
      float a = 0.f;
      for (int r = 0; r < RB; ++r) a += s.de2[r * E2 + tid];
      ge2b += a;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < RB * E1 / TB; ++u) {
      const int q = tid + u * TB, r = q / E1, k = q % E1;
      float a = 0.f;
#pragma unroll
      for (int cc = 0; cc < E2; ++cc) a = fmaf(s.de2[r * E2 + cc], We2[cc * E1 + k], a);
      s.e1[q] = a * dlrelu(s.e1[q]);   // e1 := de1
    }
    __syncthreads();
    // ---- encoder layer 0 grads ----
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = tid + u * TB, k = p / MS, cc = p % MS;   // 64 x 8
      float a = 0.f;
      for (int r = 0; r < RB; ++r) a = fmaf(s.e1[r * E1 + k], s.m[r * MS + cc], a);
      ge0w[u] += a;
    }
    if (tid < E1) {
      float a = 0.f;
      for (int r = 0; r < RB; ++r) a += s.e1[r * E1 + tid];
      ge0b += a;
    }
    __syncthreads();   // the next tile restages s.x / s.m / s.e1
  }
  // ---- the partial row (network parameter order, then the extra slots) ----
  float *pr = part;
#pragma unroll
  for (int kb = 0; kb < 4; ++kb)
#pragma unroll
    for (int q = 0; q < 16; ++q) pr[o.m2w + (n0 + crow(q, h)) * NH + 32 * kb + i] = acc2[kb][q];
#pragma unroll
  for (int q = 0; q < 16; ++q) pr[o.m0w + (n0 + crow(q, h)) * D + i] = acc1[q];
  // the two row halves of the VALU accumulators meet in LDS (half 0 + half 1)
  float *red = s.red;
  auto fold = [&](float v) -> float {   // thread (j, hf): returns half0 + half1 in hf == 0 threads
    __syncthreads();
    red[tid] = v;
    __syncthreads();
    return hf == 0 ? red[j] + red[NH + j] : 0.f;
  };
  {
    const float t0 = fold(gw3[0]);
    if (hf == 0) pr[o.m4w + j] = t0;
    const float t1 = fold(gw3[1]);
    if (hf == 0 && nout > 1) pr[o.m4w + NH + j] = t1;
    const float b2v = fold(gb2);
    if (hf == 0) pr[o.m2b + j] = b2v;
    const float b1v = fold(gb1);
    if (hf == 0) pr[o.m0b + j] = b1v;
    for (int cx = 0; cx < 4; ++cx) {
      const float v = fold(gw1x[cx]);
      if (hf == 0 && cx < nx) pr[o.m0w + j * D + 32 + cx] = v;
    }
    const float bb0 = fold(gb3[0]), bb1 = fold(gb3[1]);
    if (tid == 0) {
      pr[o.m4b] = bb0;
      if (nout > 1) pr[o.m4b + 1] = bb1;
    }
  }
  if (tid < LT * E2) pr[o.e4w + tid] = ge4w;
  else if (tid < LT * E2 + LT) pr[o.e4b + tid - LT * E2] = ge4b;
#pragma unroll
  for (int u = 0; u < 4; ++u) pr[o.e2w + tid + u * TB] = ge2w[u];
  if (tid < E2) pr[o.e2b + tid] = ge2b;
#pragma unroll
  for (int u = 0; u < 2; ++u) pr[o.e0w + tid + u * TB] = ge0w[u];
  if (tid < E1) pr[o.e0b + tid] = ge0b;
  // extras: wave 0 sums the per-row loss terms (lanes 32..63 hold zeros)
  if (w == 0) {
    const float sa = wave_sum(l_a), sb = wave_sum(l_b), q0 = wave_sum(gsd0), q1 = wave_sum(gsd1);
    const float si = wave_sum(l_im);
    if (lane == 0) {
      const int x = o.size;
      if (kActor) { pr[x] = q0; pr[x + 1] = q1; pr[x + 2] = sa; pr[x + 3] = sb; pr[x + 4] = si; }
      else { pr[x] = sa; pr[x + 1] = 0.f; pr[x + 2] = 0.f; pr[x + 3] = 0.f; }
    }
  }
}

__global__ __launch_bounds__(TB) void k_lz_grad(lz_cfg_t c, const float *__restrict__ P, int G, size_t mb_row0, int M,
                                                const float *__restrict__ st_obs, const float *__restrict__ st_act,
                                                const float *__restrict__ st_logp, const float *__restrict__ st_val,
                                                const float *__restrict__ st_ret, const float *__restrict__ st_adv,
                                                float *part_a, float *part_c, const int32_t *__restrict__ ridx) {
  __shared__ NetSmem s;
  const int stride = part_stride(c.obs_dim);
  if ((int)blockIdx.x < G)
    grad_net<true>(c, P, blockIdx.x, G, mb_row0, M, st_obs, st_act, st_logp, st_val, st_ret, st_adv,
                   part_a + (size_t)blockIdx.x * stride, s, ridx);
  else
    grad_net<false>(c, P, blockIdx.x - G, G, mb_row0, M, st_obs, st_act, st_logp, st_val, st_ret, st_adv,
                    part_c + (size_t)(blockIdx.x - G) * stride, s, ridx);
}

// Fixed-order sum of the G partial rows of each network into grad[] (parameter order), the loss
// sums into grad[np .. np + 4) (surrogate, log-prob, value loss, imitation) and each chunk's squared norm
// into grad[np + 8 + chunk].  One thread per parameter, 16 row loads in flight.
constexpr int RD_TB = 256;
__global__ __launch_bounds__(RD_TB) void k_lz_reduce(lz_cfg_t c, const float *__restrict__ part_a,
                                                     const float *__restrict__ part_c, int G, float *grad) {
  __shared__ float sq[RD_TB / 64];
  const int D = c.obs_dim, np = nparam(D), stride = part_stride(D);
  const int na = net_off(D, NA).size, cb = critic_base(D);
  const int p = blockIdx.x * RD_TB + threadIdx.x;
  // parameter p's column: actor rows hold [actor net | dstd], critic rows the critic net
  const float *src = nullptr;
  int col = 0;
  if (p < cb) { src = part_a; col = p; }            // actor net, then dstd at columns na, na + 1
  else if (p < np) { src = part_c; col = p - cb; }
  float acc = 0.f;
  if (src) {
    for (int b0 = 0; b0 < G; b0 += 16) {
      float x[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) x[k] = src[(size_t)min(b0 + k, G - 1) * stride + col];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (b0 + k < G) acc += x[k];
    }
    grad[p] = acc;
  }
  float s2 = wave_sum(acc * acc);
  if ((threadIdx.x & 63) == 0) sq[threadIdx.x >> 6] = s2;
  __syncthreads();
  if (threadIdx.x == 0) grad[np + 8 + blockIdx.x] = ((sq[0] + sq[1]) + sq[2]) + sq[3];
  if (blockIdx.x == 0 && threadIdx.x < 4) {   // loss sums: surrogate, log-prob, value loss, imitation
    const float *s_ = threadIdx.x == 2 ? part_c : part_a;
    const int cc = threadIdx.x == 0 ? na + 2 : (threadIdx.x == 1 ? na + 3 : (threadIdx.x == 2 ? net_off(D, 1).size
                                                                                                : na + 4));
    float a = 0.f;
    for (int b = 0; b < G; ++b) a += s_[(size_t)b * stride + cc];
    grad[np + threadIdx.x] = a;
  }
}

// clip_grad_norm_ + torch.optim.Adam over the whole loopz parameter vector; skipped (no step)
// when the minibatch loss is not finite (ppo.py:290-296).  opt double-buffered as in ppo.hip.
constexpr int AP_TB = 256;
__global__ __launch_bounds__(AP_TB) void k_lz_apply(lz_cfg_t c, float *P, const float *__restrict__ grad, float *m,
                                                    float *v, const float *__restrict__ opt_in,
                                                    float *__restrict__ opt_out, int M, int nchunks) {
  __shared__ float red[AP_TB / 64];
  const int D = c.obs_dim, np = nparam(D);
  const int tid = threadIdx.x;
  const int q = blockIdx.x * AP_TB + tid;
  const int qc = min(q, np - 1);
  const float g_raw = grad[qc], p_old = P[qc], m_old = m[qc], v_old = v[qc];
  float ss = 0.f;
  for (int k = tid; k < nchunks; k += AP_TB) ss += grad[np + 8 + k];
  const float invB = 1.0f / (float)M;
  const float surr = grad[np] * invB, lps = grad[np + 1] * invB, vl = grad[np + 2] * invB;
  // rl_loss + im_loss (ppo.py:276-283); only its finiteness is used (the non-finite skip)
  const float loss = ((surr + c.value_loss_coef * vl) + c.entropy_coef * lps) + (c.expert_act ? grad[np + 3] * invB : 0.f);
  const bool ok = isfinite(loss);
  const float step = opt_in[1] + (ok ? 1.0f : 0.0f);
  const float lr = opt_in[0];
  const double bc1 = 1.0 - pow((double)c.adam_b1, (double)step);
  const double bc2 = 1.0 - pow((double)c.adam_b2, (double)step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2s = (float)sqrt(bc2);
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float total_norm = sqrtf(((red[0] + red[1]) + red[2]) + red[3]);
  const float coef = fminf(c.max_grad_norm / (total_norm + 1e-6f), 1.0f);
  if (ok && q < np) {
    const float g = g_raw * coef;
    const float mi = m_old + (1.0f - c.adam_b1) * (g - m_old);
    const float vi = v_old * c.adam_b2 + (1.0f - c.adam_b2) * g * g;
    const float denom = sqrtf(vi) / bc2s + c.adam_eps;
    P[q] = p_old - step_size * (mi / denom);
    m[q] = mi;
    v[q] = vi;
  }
  if (blockIdx.x == 0 && tid == 0) {
    opt_out[0] = lr;
    opt_out[1] = step;
    opt_out[2] = vl;
    opt_out[3] = surr;
    opt_out[4] = total_norm;
    opt_out[5] = ok ? 1.0f : 0.0f;
    opt_out[6] = opt_in[6];
    opt_out[7] = opt_in[7];
  }
}

__global__ void k_lz_min_std(lz_cfg_t c, float *P) {
  const int d = threadIdx.x;
  if (d >= NA) return;
  float s = P[std_base(c.obs_dim) + d];
  if (!isfinite(s)) s = c.min_std;
  P[std_base(c.obs_dim) + d] = fmaxf(s, c.min_std);
}

bool cfg_ok(const lz_cfg_t *c) {
  // the main input (obs_dim wide) fills the first 32-column matrix-core block and at most 4 more
  // columns: obs_dim 33 (priv_dim 8, mass_dim 8 as the loopz cfg.yaml uses) .. 36
  return c && c->n_envs > 0 && c->horizon > 0 && c->obs_dim >= 33 && c->obs_dim <= LZ_MAX_OBS &&
         c->mini_batches > 0 && c->epochs > 0;
}

int grad_groups(int M) {
  const int ntiles = (M + RB - 1) / RB;
  return ntiles < 128 ? ntiles : 128;
}

}  // namespace

extern "C" {

int lz_nparam(int obs_dim) { return nparam(obs_dim); }
int lz_grad_floats(int obs_dim) { return nparam(obs_dim) + 8 + (nparam(obs_dim) + RD_TB - 1) / RD_TB; }
int lz_partials_floats(const lz_cfg_t *cfg) {
  if (!cfg_ok(cfg)) return -1;
  const int M = cfg->n_envs * cfg->horizon / cfg->mini_batches;
  return 2 * grad_groups(M) * part_stride(cfg->obs_dim);
}

int lz_act(const lz_cfg_t *cfg, const float *params, const float *obs, int t, float *st_obs, float *st_act,
           float *st_logp, float *st_val, float *actions_out, uint64_t seed, uint64_t step,
           const float *eps_inject, void *stream) {
  if (!cfg_ok(cfg) || !params || !obs || !actions_out || t < 0 || t >= cfg->horizon) return 1;
  hipStream_t s = (hipStream_t)stream;
  const int grid = fwd_grid(cfg->n_envs);
  hipLaunchKernelGGL(k_lz_forward<true>, dim3(grid), dim3(TB), 0, s, *cfg, params, obs, t, st_obs, st_act, st_logp,
                     st_val, actions_out, (float *)nullptr, seed, step, eps_inject);
  USV_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_lz_forward<false>, dim3(grid), dim3(TB), 0, s, *cfg, params, obs, t, st_obs, st_act, st_logp,
                     st_val, actions_out, (float *)nullptr, seed, step, eps_inject);
  USV_CHECK_LAUNCH();
  return 0;
}

int lz_value(const lz_cfg_t *cfg, const float *params, const float *obs, float *values, void *stream) {
  if (!cfg_ok(cfg) || !params || !obs || !values) return 1;
  hipLaunchKernelGGL(k_lz_forward<false>, dim3(fwd_grid(cfg->n_envs)), dim3(TB), 0, (hipStream_t)stream, *cfg, params,
                     obs, 0, (float *)nullptr, (float *)nullptr, (float *)nullptr, (float *)nullptr,
                     (float *)nullptr, values, (uint64_t)0, (uint64_t)0, (const float *)nullptr);
  USV_CHECK_LAUNCH();
  return 0;
}

int lz_store(const lz_cfg_t *cfg, const float *rew, const int64_t *dones, int t, float *st_rew, uint8_t *st_done,
             void *stream) {
  if (!cfg_ok(cfg) || !rew || !dones || !st_rew || !st_done || t < 0 || t >= cfg->horizon) return 1;
  hipLaunchKernelGGL(k_lz_store, dim3((cfg->n_envs + 255) / 256), dim3(256), 0, (hipStream_t)stream, *cfg, rew, dones,
                     t, st_rew, st_done);
  USV_CHECK_LAUNCH();
  return 0;
}

int lz_returns(const lz_cfg_t *cfg, const float *last_values, const float *st_rew, const uint8_t *st_done,
               const float *st_val, float *st_ret, float *st_adv, double *work, void *stream) {
  if (!cfg_ok(cfg) || !last_values || !st_rew || !st_done || !st_val || !st_ret || !st_adv || !work) return 1;
  hipStream_t s = (hipStream_t)stream;
  const int nblk = (cfg->n_envs + 255) / 256;
  hipLaunchKernelGGL(k_lz_gae, dim3(nblk), dim3(256), 0, s, *cfg, last_values, st_rew, st_done, st_val, st_ret, st_adv,
                     work);
  USV_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_lz_adv_finalize, dim3(1), dim3(64), 0, s, *cfg, work, nblk);
  USV_CHECK_LAUNCH();
  const size_t B = (size_t)cfg->n_envs * cfg->horizon;
  hipLaunchKernelGGL(k_lz_adv_apply, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, *cfg, work, st_ret, st_adv);
  USV_CHECK_LAUNCH();
  return 0;
}

int lz_minibatch(const lz_cfg_t *cfg, float *params, float *adam_m, float *adam_v, float *opt, int opt_slot, int mb,
                 const float *st_obs, const float *st_act, const float *st_logp, const float *st_val,
                 const float *st_ret, const float *st_adv, float *partials, float *grad, void *stream) {
  return lz_minibatch_rows(cfg, params, adam_m, adam_v, opt, opt_slot, mb, st_obs, st_act, st_logp, st_val, st_ret,
                           st_adv, nullptr, partials, grad, stream);
}

int lz_minibatch_rows(const lz_cfg_t *cfg, float *params, float *adam_m, float *adam_v, float *opt, int opt_slot,
                      int mb, const float *st_obs, const float *st_act, const float *st_logp, const float *st_val,
                      const float *st_ret, const float *st_adv, const int32_t *rows, float *partials, float *grad,
                      void *stream) {
  if (!cfg_ok(cfg) || !params || !adam_m || !adam_v || !opt || !partials || !grad) return 1;
  if (opt_slot != 0 && opt_slot != 1) return 2;
  const int B = cfg->n_envs * cfg->horizon, M = B / cfg->mini_batches;
  if (M <= 0 || mb < 0 || mb >= cfg->mini_batches) return 3;
  hipStream_t s = (hipStream_t)stream;
  const int G = grad_groups(M);
  const int stride = part_stride(cfg->obs_dim);
  float *part_a = partials, *part_c = partials + (size_t)G * stride;
  hipLaunchKernelGGL(k_lz_grad, dim3(2 * G), dim3(TB), 0, s, *cfg, params, G, (size_t)mb * M, M, st_obs, st_act,
                     st_logp, st_val, st_ret, st_adv, part_a, part_c, rows);
  USV_CHECK_LAUNCH();
  const int np = nparam(cfg->obs_dim), nch = (np + RD_TB - 1) / RD_TB;
  hipLaunchKernelGGL(k_lz_reduce, dim3(nch), dim3(RD_TB), 0, s, *cfg, part_a, part_c, G, grad);
  USV_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_lz_apply, dim3((np + AP_TB - 1) / AP_TB), dim3(AP_TB), 0, s, *cfg, params, grad, adam_m, adam_v,
                     opt + 8 * opt_slot, opt + 8 * (1 - opt_slot), M, nch);
  USV_CHECK_LAUNCH();
  return 0;
}

int lz_enforce_min_std(const lz_cfg_t *cfg, float *params, void *stream) {
  if (!cfg_ok(cfg) || !params) return 1;
  hipLaunchKernelGGL(k_lz_min_std, dim3(1), dim3(64), 0, (hipStream_t)stream, *cfg, params);
  USV_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
