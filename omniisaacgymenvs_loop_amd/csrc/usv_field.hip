// Potential field of the reset batch on MI355X (gfx950).
//
// Replaces BatchedMapGPU (tasks/USV/d_multi_gemini.py:66-271), called from
// CaptureXYTask.get_spawns (USV_capture_xy_static_obs.py:1054-1057):
//   occupancy/SDF over 16 obstacles + border, 8-neighbour wavefront cost-to-go
//   (costs 1 / 1.414, obstacles = inf), repulsion J = eta (1/d - 1/r0)^2 masked
//   by clamp(dist_to_goal/3, 0, 1), batch-global max of finite costs and of J,
//   per-env min/max normalisation, potential = g_norm + 0.5 J_norm.
//
// k_field_wave (one 256-thread workgroup per reset env, persistent over the
// device-side reset count):
//   1. SDF + occupancy of the 150x150 grid (SDF to a per-slot HBM scratch, the
//      cost grid initialised in LDS, 90 KB);
//   2. cost-to-go: 225 threads each own a 10x10 tile in registers and relax it
//      with a raster forward + backward chamfer sweep against a halo ring read
//      from LDS; one barrier per iteration with a block-wide "changed" vote.
//      The reference runs 225 synchronous Jacobi sweeps; both iterate to the
//      same unique fixed point (every cell = min over paths of the fp32 path
//      sums), so the result is the reference's bit for bit whenever its 225
//      sweeps have converged (they do: the hop depth of a 150x150 grid with 16
//      r = 0.5 m obstacles is < 120; checked on the golden fixtures).  An
//      occupied target cell is seeded exactly as the reference's first Jacobi
//      sweep does (its neighbours get 1 / 1.414);
//   3. raw cost to the field buffer + per-env statistics, split by finite and
//      infinite cost so that the batch constant inf_val (unknown until every
//      env is done) enters only through one monotone scalar per batch.
// k_field_batch (one workgroup): batch max of finite costs -> inf_val, the
//   repulsion mask of infinite cells, batch J max, any-inside flag.
// k_field_final (grid-stride over (slot, 2048-cell chunk)): normalisation.
#include "usv_device.h"

namespace {

constexpr int G = USV_GRID;
constexpr int G2 = USV_GRID2;
constexpr int T = 10;            // tile edge
constexpr int NT = G / T;        // 15 tiles per edge
constexpr int GP = G + 2;        // LDS cost grid padded with an +inf ring (no halo bounds checks)
constexpr int kWaveThreads = 256;
constexpr int kMaxIters = 4096;  // safety cap (never reached)
constexpr int kChunk = 2048;     // cells per k_field_final work item
constexpr int kChunks = (G2 + kChunk - 1) / kChunk;

// slot_stats layout (per reset slot)
enum {
  SS_GMIN_F = 0, SS_GMAX_F, SS_ANY_INF,        // finite-cost extrema, any infinite cell
  SS_JMIN_F_NI, SS_JMAX_F_NI, SS_JMAX_F_ALL,   // J over finite cells: non-inside min/max, max of all
  SS_JRMIN_I_NI, SS_JRMAX_I_NI, SS_JRMAX_I_ALL,  // eta (1/d - 1/r0)^2 over infinite cells (mask applied later)
  SS_INSIDE, SS_ITERS
};

__device__ __forceinline__ float grid_coord(const float *lin, float map_size, int i) {
  if (lin) return lin[i];
  const double cell_d = (double)map_size / G;
  const float start = (float)(-(double)map_size / 2 + cell_d / 2);
  const float end = (float)((double)map_size / 2 - cell_d / 2);
  const float step = (end - start) / (float)(G - 1);
  return (i < G / 2) ? start + step * (float)i : end - step * (float)(G - i - 1);
}

__device__ __forceinline__ float min_dist(const float *so, float gx, float gy) {
  float m2 = INFINITY;
#pragma unroll
  for (int o = 0; o < USV_NOBST; ++o) {
    const float dx = gx - so[2 * o], dy = gy - so[2 * o + 1];
    m2 = fminf(m2, fmaf(dy, dy, dx * dx));
  }
  return sqrtf(m2);   // sqrt is monotone: sqrt(min) == min(sqrt), bit-exact
}

// +inf for an occupied cell, 0 for a free one (costs are >= 0: max(m, wall) keeps
// free cells and pins occupied ones), from the tile's free bit mask without a
// per-cell lane mask
__device__ __forceinline__ float wall(const uint32_t *freem, int bit) {
  const uint32_t f = (freem[bit >> 5] >> (bit & 31)) & 1u;
  return __uint_as_float((f - 1u) & 0x7f800000u);
}

// eta (1/d - 1/r0)^2 before the goal mask, 0 outside the influence radius
__device__ __forceinline__ float j_raw(const usv_cfg_t &c, float dte, float inv_r) {
  if (!(dte < c.influence_radius)) return 0.f;
  const float d = maxf(dte, 1e-3f);
  const float t = 1.0f / d - inv_r;
  return c.eta * (t * t);
}
__device__ __forceinline__ float goal_mask(const usv_cfg_t &c, float cv, float cell) {
  return clampt((cv * cell) / c.safe_radius, 0.f, 1.f);
}

// ---------------------------------------------------------------- pass B ---
__global__ __launch_bounds__(kWaveThreads) void k_field_wave(usv_cfg_t c, usv_bufs_t b) {
  __shared__ float cost[GP * GP];
  __shared__ uint8_t occ[G2];
  __shared__ float so[2 * USV_NOBST];
  __shared__ float slin[G];
  __shared__ float red[12][kWaveThreads / 64];
  const int n = b.n;
  const int count = b.ctl[USV_CTL_RESET_COUNT];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const bool owner = tid < NT * NT;
  const int tr = owner ? tid / NT : 0, tc = owner ? tid % NT : 0;
  const int r0 = tr * T, c0 = tc * T;
  const float cell = (float)((double)c.map_size / G);
  const float half_map = (float)((double)c.map_size / 2);
  const float inv_r = (float)(1.0 / (double)c.influence_radius);
  for (int slot = blockIdx.x; slot < count; slot += gridDim.x) {
    const int e = b.reset_ids[slot];
    if (tid < 2 * USV_NOBST) so[tid] = b.obst[(size_t)tid * n + e];
    if (tid < G) slin[tid] = grid_coord(b.grid_lin, c.map_size, tid);
    __syncthreads();
    // target cell (compute_cost_field_wavefront :148-154)
    const float tx = b.field_old_tgt[e], ty = b.field_old_tgt[n + e];
    int ix = (int)((tx + half_map) / cell), iy = (int)((ty + half_map) / cell);
    ix = min(max(ix, 0), G - 1);
    iy = min(max(iy, 0), G - 1);
    const bool tgt_free = !((min_dist(so, slin[ix], slin[iy]) - c.obstacle_radius) <= 0.f) && ix > 0 &&
                          ix < G - 1 && iy > 0 && iy < G - 1;
    for (int q = tid; q < 4 * GP; q += kWaveThreads) {   // the +inf ring
      const int side = q / GP, k = q % GP;
      const int idx = side == 0 ? k : side == 1 ? (GP - 1) * GP + k : side == 2 ? k * GP : k * GP + GP - 1;
      cost[idx] = INFINITY;
    }
    // ---- 1. occupancy / SDF (compute_occupancy_and_sdf :66-104) + initial cost ----
    float *sdf_s = b.sdf + (size_t)slot * G2;
    for (int q = tid; q < G2; q += kWaveThreads) {
      const int r = q / G, cc = q % G;
      const float sdf = min_dist(so, slin[cc], slin[r]) - c.obstacle_radius;
      sdf_s[q] = sdf;
      const bool border = r == 0 || r == G - 1 || cc == 0 || cc == G - 1;
      const bool o = border || sdf <= 0.f;
      occ[q] = o ? 1 : 0;
      float init = INFINITY;
      if (tgt_free) {
        if (r == iy && cc == ix) init = 0.f;
      } else if (!o) {
        // reference's first synchronous sweep from an occupied target cell
        const int di = r - iy, dj = cc - ix;
        if (abs(di) <= 1 && abs(dj) <= 1 && (di || dj)) init = (di && dj) ? 1.414f : 1.0f;
      }
      cost[(r + 1) * GP + cc + 1] = init;
    }
    __syncthreads();
    // ---- 2. cost-to-go: tiled chamfer sweeps until nothing changes ----
    // h holds the tile (interior, persistent across iterations) and its halo
    // ring (reloaded every iteration).  Updates only ever lower a value, so a
    // cell changed iff its new value is below the old one; only the tile's
    // edge cells are read by other threads, so only they go back to LDS.
    float h[T + 2][T + 2];
    uint32_t freem[4] = {0u, 0u, 0u, 0u};
    if (owner) {
#pragma unroll
      for (int i = 0; i < T; ++i)
#pragma unroll
        for (int j = 0; j < T; ++j) {
          const int q = (r0 + i) * G + c0 + j;
          h[i + 1][j + 1] = cost[(r0 + i + 1) * GP + c0 + j + 1];
          if (!occ[q]) freem[(i * T + j) >> 5] |= 1u << ((i * T + j) & 31);
        }
    }
    int it = 0;
    for (; it < kMaxIters; ++it) {
      int changed = 0;
      if (owner) {
#pragma unroll
        for (int i = 0; i < T + 2; ++i)
#pragma unroll
          for (int j = 0; j < T + 2; ++j) {
            if (i >= 1 && i <= T && j >= 1 && j <= T) continue;
            h[i][j] = cost[(r0 + i) * GP + c0 + j];   // padded coordinates
          }
        // forward raster sweep (up-left, up, up-right, left), then backward (mirror)
#pragma unroll
        for (int i = 1; i <= T; ++i)
#pragma unroll
          for (int j = 1; j <= T; ++j) {
            float m = h[i][j];
            m = fminf(m, h[i - 1][j - 1] + 1.414f);
            m = fminf(m, h[i - 1][j] + 1.0f);
            m = fminf(m, h[i - 1][j + 1] + 1.414f);
            m = fminf(m, h[i][j - 1] + 1.0f);
            const float nv = fmaxf(m, wall(freem, (i - 1) * T + (j - 1)));
            changed |= nv < h[i][j];
            h[i][j] = nv;
          }
#pragma unroll
        for (int i = T; i >= 1; --i)
#pragma unroll
          for (int j = T; j >= 1; --j) {
            float m = h[i][j];
            m = fminf(m, h[i + 1][j + 1] + 1.414f);
            m = fminf(m, h[i + 1][j] + 1.0f);
            m = fminf(m, h[i + 1][j - 1] + 1.414f);
            m = fminf(m, h[i][j + 1] + 1.0f);
            const float nv = fmaxf(m, wall(freem, (i - 1) * T + (j - 1)));
            changed |= nv < h[i][j];
            h[i][j] = nv;
          }
        if (changed) {
#pragma unroll
          for (int i = 1; i <= T; ++i)
#pragma unroll
            for (int j = 1; j <= T; ++j)
              if (i == 1 || i == T || j == 1 || j == T) cost[(r0 + i) * GP + c0 + j] = h[i][j];
        }
      }
      if (!__syncthreads_or(changed)) break;
    }
    if (owner) {
#pragma unroll
      for (int i = 1; i <= T; ++i)
#pragma unroll
        for (int j = 1; j <= T; ++j) cost[(r0 + i) * GP + c0 + j] = h[i][j];
    }
    __syncthreads();
    // ---- 3. raw cost out + per-env statistics (finite / infinite split) ----
    float gmin = INFINITY, gmax = -INFINITY, jmin_f = INFINITY, jmax_f = -INFINITY, jall_f = 0.f;
    float jrmin_i = INFINITY, jrmax_i = -INFINITY, jrall_i = 0.f;
    int any_inf = 0, inside = 0;
    float *Fe = b.field + (size_t)e * G2;
    for (int q = tid; q < G2; q += kWaveThreads) {
      const float g = cost[(q / G + 1) * GP + q % G + 1];
      Fe[q] = g;
      const float dte = sdf_s[q] - c.obstacle_radius;   // this thread's own phase-1 write
      const bool ins = dte <= 0.f;
      inside |= ins;
      const float jr = j_raw(c, dte, inv_r);
      if (isinf(g)) {
        any_inf = 1;
        jrall_i = fmaxf(jrall_i, jr);
        if (!ins) { jrmin_i = fminf(jrmin_i, jr); jrmax_i = fmaxf(jrmax_i, jr); }
      } else {
        gmin = fminf(gmin, g);
        gmax = fmaxf(gmax, g);
        const float j = jr == 0.f && !(dte < c.influence_radius) ? 0.f : jr * goal_mask(c, g, cell);
        jall_f = fmaxf(jall_f, j);
        if (!ins) { jmin_f = fminf(jmin_f, j); jmax_f = fmaxf(jmax_f, j); }
      }
    }
    float vals[10] = {wave_min(gmin), wave_max(gmax), 0.f, wave_min(jmin_f), wave_max(jmax_f), wave_max(jall_f),
                      wave_min(jrmin_i), wave_max(jrmax_i), wave_max(jrall_i), 0.f};
    if (lane == 0)
      for (int k = 0; k < 10; ++k) red[k][wid] = vals[k];
    const int has_inf = __syncthreads_or(any_inf);
    const int has_inside = __syncthreads_or(inside);
    if (tid == 0) {
      float a[10];
      for (int k = 0; k < 10; ++k) a[k] = red[k][0];
      for (int w = 1; w < kWaveThreads / 64; ++w) {
        a[SS_GMIN_F] = fminf(a[SS_GMIN_F], red[SS_GMIN_F][w]);
        a[SS_GMAX_F] = fmaxf(a[SS_GMAX_F], red[SS_GMAX_F][w]);
        a[SS_JMIN_F_NI] = fminf(a[SS_JMIN_F_NI], red[SS_JMIN_F_NI][w]);
        a[SS_JMAX_F_NI] = fmaxf(a[SS_JMAX_F_NI], red[SS_JMAX_F_NI][w]);
        a[SS_JMAX_F_ALL] = fmaxf(a[SS_JMAX_F_ALL], red[SS_JMAX_F_ALL][w]);
        a[SS_JRMIN_I_NI] = fminf(a[SS_JRMIN_I_NI], red[SS_JRMIN_I_NI][w]);
        a[SS_JRMAX_I_NI] = fmaxf(a[SS_JRMAX_I_NI], red[SS_JRMAX_I_NI][w]);
        a[SS_JRMAX_I_ALL] = fmaxf(a[SS_JRMAX_I_ALL], red[SS_JRMAX_I_ALL][w]);
      }
      float *st = b.slot_stats + (size_t)slot * 16;
      for (int k = 0; k < 9; ++k) st[k] = a[k];
      st[SS_ANY_INF] = has_inf ? 1.f : 0.f;
      st[SS_INSIDE] = has_inside ? 1.f : 0.f;
      st[SS_ITERS] = (float)it;   // iterations (diagnostic)
      if (isfinite(a[SS_GMAX_F])) {
        atomic_max_f32(&b.fscratch[0], a[SS_GMAX_F]);
        atomicOr(&b.ctl[USV_CTL_ANY_FINITE], 1);
      }
    }
    __syncthreads();
  }
}

// batch constants given every slot's statistics
struct BatchK {
  float inf_val, mask_inf;
};
__device__ __forceinline__ BatchK batch_k(const usv_cfg_t &c, const usv_bufs_t &b) {
  const float max_val = b.ctl[USV_CTL_ANY_FINITE] ? b.fscratch[0] : 100.0f;
  const float inf_val = max_val * 1.5f;
  const float cell = (float)((double)c.map_size / G);
  return BatchK{inf_val, goal_mask(c, inf_val, cell)};
}

// ---------------------------------------------------------------- pass C ---
__global__ __launch_bounds__(1024) void k_field_batch(usv_cfg_t c, usv_bufs_t b) {
  __shared__ float red[16];
  __shared__ int ins;
  const int count = b.ctl[USV_CTL_RESET_COUNT];
  const int tid = threadIdx.x;
  if (count <= 0) return;
  const BatchK k = batch_k(c, b);
  if (tid == 0) ins = 0;
  __syncthreads();
  float jm = 0.f;
  int inside = 0;
  for (int s = tid; s < count; s += 1024) {
    const float *st = b.slot_stats + (size_t)s * 16;
    jm = fmaxf(jm, st[SS_JMAX_F_ALL]);
    if (st[SS_ANY_INF] != 0.f) jm = fmaxf(jm, st[SS_JRMAX_I_ALL] * k.mask_inf);   // monotone in the raw value
    inside |= st[SS_INSIDE] != 0.f;
  }
  jm = wave_max(jm);
  if ((tid & 63) == 0) red[tid >> 6] = jm;
  if (inside) ins = 1;
  __syncthreads();
  if (tid == 0) {
    float m = 0.f;
    for (int w = 0; w < 16; ++w) m = fmaxf(m, red[w]);
    b.fscratch[1] = m;                                   // J.max() over the batch (:257)
    b.ctl[USV_CTL_ANY_INSIDE] = ins;
  }
}

// ---------------------------------------------------------------- pass D ---
__global__ __launch_bounds__(256) void k_field_final(usv_cfg_t c, usv_bufs_t b) {
  const int count = b.ctl[USV_CTL_RESET_COUNT];
  const BatchK k = batch_k(c, b);
  const float cell = (float)((double)c.map_size / G);
  const float inv_r = (float)(1.0 / (double)c.influence_radius);
  const bool any_inside = b.ctl[USV_CTL_ANY_INSIDE] != 0;
  const float cur_max = b.fscratch[1];
  const float high = (cur_max > 1e-6f) ? cur_max * 10.0f : 100.0f;
  const int items = count * kChunks;
  for (int w = blockIdx.x; w < items; w += gridDim.x) {
    const int slot = w / kChunks, ch = w % kChunks;
    const int e = b.reset_ids[slot];
    const float *st = b.slot_stats + (size_t)slot * 16;
    const bool has_inf = st[SS_ANY_INF] != 0.f;
    const bool has_inside = st[SS_INSIDE] != 0.f;
    const float gmin = has_inf ? fminf(st[SS_GMIN_F], k.inf_val) : st[SS_GMIN_F];
    const float gmax = has_inf ? fmaxf(st[SS_GMAX_F], k.inf_val) : st[SS_GMAX_F];
    float jmn = st[SS_JMIN_F_NI], jmx = st[SS_JMAX_F_NI];
    if (isfinite(st[SS_JRMIN_I_NI])) {       // some infinite-cost, not-inside cell exists
      jmn = fminf(jmn, st[SS_JRMIN_I_NI] * k.mask_inf);
      jmx = fmaxf(jmx, st[SS_JRMAX_I_NI] * k.mask_inf);
    }
    if (any_inside && has_inside) { jmn = fminf(jmn, high); jmx = fmaxf(jmx, high); }
    const float gden = (gmax - gmin) + 1e-6f;
    const float jden = (jmx - jmn) + 1e-6f;
    float *Fe = b.field + (size_t)e * G2;
    const float *sdf_s = b.sdf + (size_t)slot * G2;
    const int q1 = min(G2, (ch + 1) * kChunk);
    for (int q = ch * kChunk + threadIdx.x; q < q1; q += 256) {
      const float g = Fe[q];
      const float cv = isinf(g) ? k.inf_val : g;
      const float dte = sdf_s[q] - c.obstacle_radius;
      const float jr = j_raw(c, dte, inv_r);
      const float j = (dte < c.influence_radius) ? jr * goal_mask(c, cv, cell) : 0.f;
      const float jv = (any_inside && dte <= 0.f) ? high : j;
      const float gn = (cv - gmin) / gden;
      const float jn = (jv - jmn) / jden;
      Fe[q] = gn + c.field_alpha * jn;
    }
  }
}

}  // namespace

extern "C" int usv_potential_field(const usv_cfg_t *cfg, const usv_bufs_t *b, void *stream) {
  if (!cfg || !b || b->n <= 0 || !b->slot_stats || !b->field || !b->sdf) return 1;
  hipStream_t s = (hipStream_t)stream;
  // the reset count lives on the device: launch persistent grids, blocks loop over slots
  const int grid_b = b->n < 512 ? b->n : 512;
  const int grid_d = b->n * kChunks < 4096 ? b->n * kChunks : 4096;
  hipLaunchKernelGGL(k_field_wave, dim3(grid_b), dim3(kWaveThreads), 0, s, *cfg, *b);
  USV_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_field_batch, dim3(1), dim3(1024), 0, s, *cfg, *b);
  USV_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_field_final, dim3(grid_d), dim3(256), 0, s, *cfg, *b);
  USV_CHECK_LAUNCH();
  return 0;
}
