// Potential field of the reset batch on MI355X (gfx950).
//
// Replaces BatchedMapGPU (tasks/USV/d_multi_gemini.py:66-271), called from
// CaptureXYTask.get_spawns (USV_capture_xy_static_obs.py:1054-1057):
//   occupancy/SDF over 16 obstacles + border, 8-neighbour wavefront cost-to-go
//   (costs 1 / 1.414, obstacles = inf), repulsion J = eta (1/d - 1/r0)^2 masked
//   by clamp(dist_to_goal/3, 0, 1), batch-global max of finite costs and of J,
//   per-env min/max normalisation, potential = g_norm + 0.5 J_norm.
//
// k_field_wave / k_field_wave_pack (one 256-thread workgroup per reset env,
// persistent over the device-side reset count; _pack holds two envs per CU):
//   1. occupancy of the 150x150 grid as a 2.8 KB bit map in LDS, splatted per
//      obstacle over its bounding box with the exact per-cell distance test (the
//      SDF itself is computed by k_field_stats, off this kernel's critical path);
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
//   3. raw cost into the env's field tiles (b.field: the threads' own 10 x 10 tiles).
// k_field_stats (per slot and 30-row band): the SDF (recomputed from the obstacles)
//   and the cost tiles -> per-env statistics, split by finite and infinite cost so that the batch
//   constant inf_val (unknown until every env is done) enters only through one
//   monotone scalar per batch.
// k_field_batch (one workgroup): batch max of finite costs -> inf_val, the
//   repulsion mask of infinite cells, batch J max, any-inside flag.
// k_field_norm (one thread per slot): the env's normalisation constants (b.fnorm); the field itself is
//   never materialised -- readers form texels from the SDF, the cost and the constants (field_value).
#include "usv_device.h"

USV_PROBE_DEFINE(field)

namespace {

constexpr int G = USV_GRID;
constexpr int G2 = USV_GRID2;
constexpr int FS = USV_FIELD_STRIDE;   // floats per env of the tiled field / SDF buffers
constexpr int T = 10;            // tile edge
constexpr int NT = G / T;        // 15 tiles per edge
constexpr int kWaveThreads = 256;
constexpr int kMaxIters = 4096;  // safety cap (never reached)
constexpr int kSlotStride = USV_FIELD_SLOT_STATS;   // floats per reset slot: 16 final + 12 per chunk + obstacles
constexpr int kSlotObst = 160;                      // the slot's 16 obstacle centres (x, y interleaved)
static_assert(kSlotObst + 2 * USV_NOBST <= kSlotStride, "slot_stats layout");
constexpr int kFieldPackMinEnvs = 32768;           // k_field_wave_pack (two envs per CU) from this many envs
// USV_SWEEP_WAVES: waves per SIMD the packed sweep kernel is compiled for (2: two reset envs per CU at <= 256
// VGPRs; 3: three envs per CU, 3 x 51.7 KB of LDS, <= 168 VGPRs) and its persistent grid (256 CUs x that)
#ifndef USV_SWEEP_WAVES
#define USV_SWEEP_WAVES 2
#endif
constexpr int kPackGrid = 256 * USV_SWEEP_WAVES;

// slot_stats layout (per reset slot)
enum {
  SS_GMIN_F = 0, SS_GMAX_F, SS_ANY_INF,        // finite-cost extrema, any infinite cell
  SS_JMIN_F_NI, SS_JMAX_F_NI, SS_JMAX_F_ALL,   // J over finite cells: non-inside min/max, max of all
  SS_JRMIN_I_NI, SS_JRMAX_I_NI, SS_JRMAX_I_ALL,  // eta (1/d - 1/r0)^2 over infinite cells (mask applied later)
  SS_INSIDE, SS_ITERS, SS_EXACT
};

// +inf for an occupied cell, 0 for a free one (costs are >= 0: max(m, wall) keeps
// free cells and pins occupied ones), from the tile's free bit mask without a
// per-cell lane mask
__device__ __forceinline__ float wall(const uint32_t *freem, int bit) {
  const uint32_t f = (freem[bit >> 5] >> (bit & 31)) & 1u;
  return __uint_as_float((f - 1u) & 0x7f800000u);
}

// ---------------------------------------------------------------- pass B ---
// LDS: the SDF grid (90 KB, also the occupancy source), the four edge rows /
// columns of every tile (the only cells other threads read; a ring of +inf
// tiles around the 15x15 tile grid removes bounds checks), the per-row
// obstacle dy table of the separable SDF, and each tile's last-changed
// iteration (a tile is swept only while it or a neighbour still changes).
constexpr int NTP = NT + 2;                     // padded tile grid edge
constexpr uint32_t kInfBits = 0x7f800000u;      // +inf
constexpr uint32_t kOcc = 0xFFFFFFFFu;          // occupied cell marker (a NaN above +inf in u32 order)
enum { E_TOP = 0, E_BOT, E_LEFT, E_RIGHT };
// occupancy (sdf <= 0) bit map, column-major: column cc owns words [cc * kOccColWords, +5)
constexpr int kOccColWords = (G + 31) / 32;
__device__ __forceinline__ bool occ_bit(const uint32_t *occ, int r, int cc) {
  return (occ[cc * kOccColWords + (r >> 5)] >> (r & 31)) & 1u;
}

// compute_cost_field_wavefront (d_multi_gemini.py:135-192) as written: int(1.5 G) = 225
// synchronous sweeps of min(self, 8 rolled neighbours + move cost) with the rolled-in edge at
// +inf, occupied cells forced to +inf after every sweep, the target cell seeded with 0.  Run
// only for an env whose tile-sweep fixed point is not certified equal to it (see below):
// ping-pong through the env's field row (k_field_stats writes the SDF there later) and the
// slot's scratch, where the result ends as k_field_wave leaves its raw cost, one block barrier per sweep; all waves of the block share the CU's L1, so plain
// global loads see the other waves' stores after the barrier.
constexpr int kRefSweeps = (G * 3) / 2;
template <int NT>
__device__ __forceinline__ void cost_sweeps_exact(const uint32_t *occ, int ix, int iy, float *A, float *B) {
  const int tid = threadIdx.x;
  for (int q = tid; q < G2; q += NT) A[q] = (q == iy * G + ix) ? 0.f : INFINITY;
  __syncthreads();
  for (int it = 0; it < kRefSweeps; ++it) {
    for (int q = tid; q < G2; q += NT) {
      const int r = q / G, cc = q % G;
      float m = A[q];
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          if (!dx && !dy) continue;
          const int rr = r - dy, c2 = cc - dx;   // torch.roll(shifts=(dy, dx)): shifted[r][c] = A[r-dy][c-dx]
          if (rr < 0 || rr >= G || c2 < 0 || c2 >= G) continue;
          m = fminf(m, A[rr * G + c2] + ((dx && dy) ? 1.414f : 1.0f));
        }
      const bool o = r == 0 || r == G - 1 || cc == 0 || cc == G - 1 || occ_bit(occ, r, cc);
      B[q] = o ? INFINITY : m;
    }
    __syncthreads();
    float *t = A; A = B; B = t;
  }
}

// CaptureXYTask.get_spawns obstacle part (static_obs.py:968-1048) for every reset env whose
// obstacles usv_reset handed over (ctl[PLACE], keys of its draws): one wave per reset env runs
// the rejection sampling around the previous-episode target (usv_reset left the spawn in
// px / py and that target in field_old_tgt) and stores the centres.  A launch of its own, so the
// sweep kernel's four waves do not wait on one wave's sampling for every slot.
constexpr int kPlaceTB = 256;
__global__ __launch_bounds__(kPlaceTB) void k_field_place(usv_cfg_t c, usv_bufs_t b) {
  if (b.ctl[USV_CTL_PLACE] == 0) return;
  const int n = b.n;
  const int count = min(b.ctl[USV_CTL_RESET_COUNT], n);
  const uint64_t h_seed = (uint64_t)(uint32_t)b.ctl[USV_CTL_H_SEED_LO] | ((uint64_t)(uint32_t)b.ctl[USV_CTL_H_SEED_HI] << 32);
  const uint64_t h_step = (uint64_t)(uint32_t)b.ctl[USV_CTL_H_STEP_LO] | ((uint64_t)(uint32_t)b.ctl[USV_CTL_H_STEP_HI] << 32);
  const float *h_inj = reinterpret_cast<const float *>(
      (uintptr_t)((uint64_t)(uint32_t)b.ctl[USV_CTL_H_INJ_LO] | ((uint64_t)(uint32_t)b.ctl[USV_CTL_H_INJ_HI] << 32)));
  const int lane = threadIdx.x & 63;
  const int waves = (int)gridDim.x * (kPlaceTB / 64);
  for (int slot = (int)blockIdx.x * (kPlaceTB / 64) + (int)(threadIdx.x >> 6); slot < count; slot += waves) {
    const int e = b.reset_ids[slot];
    const float2 oc = place_obstacles(c, e, b.px[e], b.py[e], b.field_old_tgt[e], b.field_old_tgt[n + e], h_seed,
                                      h_step, h_inj);
    if (lane < USV_NOBST) {
      b.obst[(size_t)(2 * lane) * n + e] = oc.x;
      b.obst[(size_t)(2 * lane + 1) * n + e] = oc.y;
    }
  }
}

// LDS holds the tile edges and a 2.8 KB occupancy bit map (the SDF itself goes to
// the per-slot HBM scratch only): 51 KB.  Two launch shapes of the same body:
// k_field_wave_pack is held to 256 registers (its spills sit in the per-slot
// prologue, not in the sweep), so two reset envs share a CU -- one wave of each per
// SIMD -- for batches that fill the chip more than once; k_field_wave keeps the
// compiler's 256 + 76 registers and one env per CU, for small batches, where the
// kernel is latency-bound and a shared CU would only slow the slowest env.
// USV_SWEEP_CHG 1: a sweep notes a lowered cell by OR-ing the old ^ new bit patterns into a per-lane VGPR
// (updates only ever lower a value, so the tile changed iff the OR is non-zero); 0: a per-cell compare into a
// lane mask (one VALU compare + one SALU OR per cell, the SALU op waiting on the compare)
// 2: the same OR as ONE v_bitop3_b32 per cell (chg | (old ^ new), truth table 0xF6 over the operand constants
// 0xF0 / 0xCC / 0xAA) where the compiler emits an XOR per cell plus an OR3 per two cells
#ifndef USV_SWEEP_CHG
#define USV_SWEEP_CHG 2
#endif
#ifndef USV_SWEEP_FNOTE_EDGE
#define USV_SWEEP_FNOTE_EDGE 1
#endif
#if USV_SWEEP_CHG == 2
#define USV_SWEEP_NOTE(hb, m) (chg = __builtin_amdgcn_bitop3_b32(chg, (uint32_t)(hb), (uint32_t)(m), 0xF6))
#elif USV_SWEEP_CHG
#define USV_SWEEP_NOTE(hb, m) (chg |= (uint32_t)((hb) ^ (m)))
#else
#define USV_SWEEP_NOTE(hb, m) (changed |= (m) < (hb))
#endif
// TH x TW tiles (10 x 10: the packed and plain kernels; 10 x 5: the small-batch kernel, two waves per SIMD for one
// env) over NTHR threads; the field buffer keeps its 10 x 10 tiles (a 10 x 5 tile stores into half of one)
template <bool kPlace, int TH = T, int TW = T, int NTHR = kWaveThreads>
__device__ __forceinline__ void field_wave_body(const usv_cfg_t &c, const usv_bufs_t &b) {
  constexpr int NTR = G / TH, NTC = G / TW;        // tile rows / columns
  constexpr int NPR = NTR + 2, NPC = NTC + 2;      // with the +inf ring
  constexpr int WC = NTHR / 128;                   // wave regions per band (two bands of <= 8 tile rows)
  static_assert(G % TH == 0 && G % TW == 0 && NTR <= 16 && NTC <= 8 * WC && NTHR % 128 == 0, "sweep tiling");
  static_assert(USV_FIELD_TH == TH && USV_FIELD_TW % TW == 0, "sweep tiles inside the field tiles");
  __shared__ uint32_t occ[G * kOccColWords];
  __shared__ float edgeh[2][NPR * NPC][TW];   // top / bottom row of every tile
  __shared__ float edgev[2][NPR * NPC][TH];   // left / right column
  __shared__ int lastc[NPR * NPC];
  __shared__ float so[2 * USV_NOBST];
  __shared__ float slin[G];
  const int n = b.n;
  const int count = min(b.ctl[USV_CTL_RESET_COUNT], n);   // slots index reset_ids[0, n)
  const int tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  // obstacle placement handed over by usv_reset (keys of its draws): done here only with kPlace
  const bool place = kPlace && b.ctl[USV_CTL_PLACE] != 0;
  uint64_t h_seed = 0, h_step = 0;
  const float *h_inj = nullptr;
  if (kPlace) {
    h_seed = (uint64_t)(uint32_t)b.ctl[USV_CTL_H_SEED_LO] | ((uint64_t)(uint32_t)b.ctl[USV_CTL_H_SEED_HI] << 32);
    h_step = (uint64_t)(uint32_t)b.ctl[USV_CTL_H_STEP_LO] | ((uint64_t)(uint32_t)b.ctl[USV_CTL_H_STEP_HI] << 32);
    h_inj = reinterpret_cast<const float *>(
        (uintptr_t)((uint64_t)(uint32_t)b.ctl[USV_CTL_H_INJ_LO] | ((uint64_t)(uint32_t)b.ctl[USV_CTL_H_INJ_HI] << 32)));
  }
  // tile of this thread; waves own compact quadrants of the tile grid (8x8,
  // 8x7, 7x8, 7x7 tiles) so a wave idles as a whole while its region is ahead
  // of / behind the front
  const int quad = tid >> 6, qk = tid & 63;
  const int qr = quad / WC, qc = quad % WC;
  const int qw = min(8, NTC - 8 * qc), qh = min(8, NTR - 8 * qr);
  const bool tile_ok = qk < qw * qh;
  const int tr = tile_ok ? qr * 8 + qk / qw : 0;
  const int tc = tile_ok ? qc * 8 + qk % qw : 0;
  const int r0 = tr * TH, c0 = tc * TW;
  const int tp = (tr + 1) * NPC + tc + 1;
  const float cell = (float)((double)c.map_size / G);
  const float half_map = (float)((double)c.map_size / 2);
  const float inv_r = (float)(1.0 / (double)c.influence_radius);
  // the +inf ring of tiles (constant for the launch)
  for (int q = tid; q < 2 * NPR * NPC * TW; q += NTHR) {
    const int t = (q / TW) % (NPR * NPC);
    const int rr = t / NPC, cc = t % NPC;
    if (rr == 0 || rr == NPR - 1 || cc == 0 || cc == NPC - 1) (&edgeh[0][0][0])[q] = INFINITY;
  }
  for (int q = tid; q < 2 * NPR * NPC * TH; q += NTHR) {
    const int t = (q / TH) % (NPR * NPC);
    const int rr = t / NPC, cc = t % NPC;
    if (rr == 0 || rr == NPR - 1 || cc == 0 || cc == NPC - 1) (&edgev[0][0][0])[q] = INFINITY;
  }
  for (int q = tid; q < NPR * NPC; q += NTHR) lastc[q] = -1000;
  for (int slot = blockIdx.x; slot < count; slot += gridDim.x) {
    USV_PHASE(field, 0);
    const int e = b.reset_ids[slot];
    if (kPlace && place) {
      // CaptureXYTask.get_spawns obstacle part (static_obs.py:968-1048) for this reset env, as
      // k_field_place does it: wave 0 samples and publishes the centres (small batches: one
      // round of workgroups, where a separate launch would add its latency to the step)
      if (wid == 0) {
        const float2 oc = place_obstacles(c, e, b.px[e], b.py[e], b.field_old_tgt[e], b.field_old_tgt[n + e],
                                          h_seed, h_step, h_inj);
        if (lane < USV_NOBST) {
          so[2 * lane] = oc.x;
          so[2 * lane + 1] = oc.y;
          b.obst[(size_t)(2 * lane) * n + e] = oc.x;
          b.obst[(size_t)(2 * lane + 1) * n + e] = oc.y;
        }
      }
    } else if (tid < 2 * USV_NOBST) {
      // the obstacle centres (placed for this reset by k_field_place, or the env's own)
      so[tid] = b.obst[(size_t)tid * n + e];
    }
    if (tid < G) slin[tid] = grid_coord(b.grid_lin, c.map_size, tid);
    for (int q = tid; q < G * kOccColWords; q += NTHR) occ[q] = 0u;
    __syncthreads();
#ifdef USV_PHASE_PROBE
    if (tid == 0 && blockIdx.x < 4096) g_probe_field[blockIdx.x][12] = wall_clock64();
#endif
    // ---- 1. occupancy (compute_occupancy_and_sdf :66-104): sdf <= 0 <=> some obstacle has
    // sqrt(d^2) - r <= 0 (sqrt and the subtraction are monotone), so each obstacle marks the
    // cells of its bounding box that pass the exact test with its own distance ----
    if (tid < 2 * USV_NOBST) b.slot_stats[(size_t)slot * kSlotStride + kSlotObst + tid] = so[tid];
    {
      const float half_m = (float)((double)c.map_size / 2);
      const float cellf = (float)((double)c.map_size / G);
      const int reach = (int)ceilf(c.obstacle_radius / cellf) + 2;   // cells either side, with margin
      const int bw = 2 * reach + 1;
      for (int q = tid; q < USV_NOBST * bw * bw; q += NTHR) {
        const int o = q / (bw * bw), k = q % (bw * bw);
        const float ox = so[2 * o], oy = so[2 * o + 1];
        const float ic = (ox + half_m) / cellf - 0.5f, jc = (oy + half_m) / cellf - 0.5f;
        if (!(fabsf(ic) < 4.0f * G && fabsf(jc) < 4.0f * G)) continue;   // parked obstacles (999, 999)
        const int cc = (int)floorf(ic) - reach + k % bw, r = (int)floorf(jc) - reach + k / bw;
        if (cc < 0 || cc >= G || r < 0 || r >= G) continue;
        const float dx = slin[cc] - ox, dy = slin[r] - oy;
        if (sqrtf(fmaf(dy, dy, dx * dx)) - c.obstacle_radius <= 0.f)
          atomicOr(&occ[cc * kOccColWords + (r >> 5)], 1u << (r & 31));
      }
    }
    __syncthreads();
    USV_PHASE(field, 1);
#ifdef USV_PHASE_PROBE
    if (tid == 0 && blockIdx.x < 4096) g_probe_field[blockIdx.x][13] = clock64();
#endif
    // target cell (compute_cost_field_wavefront :148-154)
    const float tx = b.field_old_tgt[e], ty = b.field_old_tgt[n + e];
    int ix = (int)((tx + half_map) / cell), iy = (int)((ty + half_map) / cell);
    ix = min(max(ix, 0), G - 1);
    iy = min(max(iy, 0), G - 1);
    const bool tgt_free = !occ_bit(occ, iy, ix) && ix > 0 && ix < G - 1 && iy > 0 && iy < G - 1;
    // ---- 2. cost-to-go: tiled chamfer sweeps until nothing changes ----
    // Costs are >= 0, so float order == signed order of the bit patterns: the
    // relaxation runs on i32 min (no NaN canonicalisation).  An occupied cell
    // holds 0xFFFFFFFF (a negative NaN, -1 as i32): it is the smallest value in
    // its own min, so it keeps itself with no extra instruction, and neighbours
    // read it as |h| + w -- a positive NaN whatever payload the add returns, above
    // +inf, so it drops out of their min.  Updates only ever lower a value.
    float h[TH + 2][TW + 2];
    if (tile_ok) {
#pragma unroll
      for (int i = 0; i < TH; ++i)
#pragma unroll
        for (int j = 0; j < TW; ++j) {
          const int r = r0 + i, cc = c0 + j;
          const bool border = r == 0 || r == G - 1 || cc == 0 || cc == G - 1;
          const bool o = border || occ_bit(occ, r, cc);
          float init = INFINITY;
          if (o) {
            init = __uint_as_float(kOcc);
          } else if (tgt_free) {
            if (r == iy && cc == ix) init = 0.f;
          } else {
            // reference's first synchronous sweep from an occupied target cell
            const int di = r - iy, dj = cc - ix;
            if (abs(di) <= 1 && abs(dj) <= 1 && (di || dj)) init = (di && dj) ? 1.414f : 1.0f;
          }
          h[i + 1][j + 1] = init;
        }
#pragma unroll
      for (int k = 0; k < TW; ++k) {
        edgeh[E_TOP][tp][k] = h[1][k + 1];
        edgeh[E_BOT][tp][k] = h[TH][k + 1];
      }
#pragma unroll
      for (int k = 0; k < TH; ++k) {
        edgev[E_LEFT - 2][tp][k] = h[k + 1][1];
        edgev[E_RIGHT - 2][tp][k] = h[k + 1][TW];
      }
      lastc[tp] = 0;
    }
    __syncthreads();
    int it = 0;
    for (; it < kMaxIters; ++it) {
      int changed = 0;
#if USV_SWEEP_CHG
      uint32_t chg = 0u;   // OR of (old ^ new) over the tile's cells: a VGPR, no per-cell lane-mask SALU op
#endif
      bool dirty = false;
      if (tile_ok) {
#pragma unroll
        for (int dr = -1; dr <= 1; ++dr)
#pragma unroll
          for (int dc = -1; dc <= 1; ++dc) dirty |= lastc[tp + dr * NPC + dc] >= it - 1;
      }
      if (dirty) {
#pragma unroll
        for (int k = 0; k < TW; ++k) {
          h[0][k + 1] = edgeh[E_BOT][tp - NPC][k];
          h[TH + 1][k + 1] = edgeh[E_TOP][tp + NPC][k];
        }
#pragma unroll
        for (int k = 0; k < TH; ++k) {
          h[k + 1][0] = edgev[E_RIGHT - 2][tp - 1][k];
          h[k + 1][TW + 1] = edgev[E_LEFT - 2][tp + 1][k];
        }
        h[0][0] = edgeh[E_BOT][tp - NPC - 1][TW - 1];
        h[0][TW + 1] = edgeh[E_BOT][tp - NPC + 1][0];
        h[TH + 1][0] = edgeh[E_TOP][tp + NPC - 1][TW - 1];
        h[TH + 1][TW + 1] = edgeh[E_TOP][tp + NPC + 1][0];
        // forward raster sweep (up-left, up, up-right, left), then backward (mirror).
        // Cell (i, j) of the forward sweep depends on (i, j-1) and row i-1 up to
        // column j+1, so cells with equal 2i + j are independent: emitting the
        // sweep level by level gives the scheduler 3-5 independent chains (a
        // single wave's dependent VALU op costs ~7 cycles on gfx950, an
        // independent one ~4).  Same updates in a dependency-respecting order
        // (each cell still sees exactly the raster sweep's operands).
#pragma unroll
        for (int L = 0; L < 2 * TH + TW - 2; ++L)
#pragma unroll
          for (int i = 1; i <= TH; ++i) {
            const int j = L - 2 * (i - 1) + 1;
            if (j < 1 || j > TW) continue;
            const int32_t hb = __float_as_int(h[i][j]);
            int32_t m = min(hb, __float_as_int(fabsf(h[i - 1][j - 1]) + 1.414f));
            m = min(m, __float_as_int(fabsf(h[i - 1][j]) + 1.0f));
            m = min(m, __float_as_int(fabsf(h[i - 1][j + 1]) + 1.414f));
            m = min(m, __float_as_int(fabsf(h[i][j - 1]) + 1.0f));
            // USV_SWEEP_FNOTE_EDGE: the forward pass notes only the tile's edge cells (the halos its neighbours
            // read).  The backward pass notes every cell, and a backward pass that lowers nothing leaves the tile
            // at its fixed point under the current halos (after the forward pass every forward constraint holds;
            // the unchanged backward pass keeps them and adds the backward ones), so an interior cell lowered by
            // the forward pass alone needs no further sweep of this tile or of its neighbours
            if (USV_SWEEP_FNOTE_EDGE == 0 || i == 1 || i == TH || j == 1 || j == TW) USV_SWEEP_NOTE(hb, m);
            h[i][j] = __int_as_float(m);
          }
#pragma unroll
        for (int L = 0; L < 2 * TH + TW - 2; ++L)
#pragma unroll
          for (int i = TH; i >= 1; --i) {
            const int j = TW - (L - 2 * (TH - i));
            if (j < 1 || j > TW) continue;
            const int32_t hb = __float_as_int(h[i][j]);
            int32_t m = min(hb, __float_as_int(fabsf(h[i + 1][j + 1]) + 1.414f));
            m = min(m, __float_as_int(fabsf(h[i + 1][j]) + 1.0f));
            m = min(m, __float_as_int(fabsf(h[i + 1][j - 1]) + 1.414f));
            m = min(m, __float_as_int(fabsf(h[i][j + 1]) + 1.0f));
            USV_SWEEP_NOTE(hb, m);
            h[i][j] = __int_as_float(m);
          }
#if USV_SWEEP_CHG
        // opaque to the optimiser: otherwise it folds (OR of old ^ new) != 0 back into per-cell compares
        __asm__("" : "+v"(chg));
        changed = chg != 0u;
#endif
        if (changed) {
#pragma unroll
          for (int k = 0; k < TW; ++k) {
            edgeh[E_TOP][tp][k] = h[1][k + 1];
            edgeh[E_BOT][tp][k] = h[TH][k + 1];
          }
#pragma unroll
          for (int k = 0; k < TH; ++k) {
            edgev[E_LEFT - 2][tp][k] = h[k + 1][1];
            edgev[E_RIGHT - 2][tp][k] = h[k + 1][TW];
          }
          lastc[tp] = it;
        }
      }
      if (!__syncthreads_or(changed)) break;
    }
    USV_PHASE(field, 2);
#ifdef USV_PHASE_PROBE
    if (tid == 0 && blockIdx.x < 4096) g_probe_field[blockIdx.x][14] = clock64();
#endif
    // ---- certificate: the reference stops after 225 Jacobi sweeps, whose result at a cell is the
    // minimum over paths of at most 225 hops.  Every hop adds >= 1 to an fp32 path sum, so a cell
    // whose fixed-point cost is <= kPinnedCost has an optimal path of <= 225 hops and the two agree.
    // If some finite cost exceeds it (long detours; never for the packaged spawn ranges, possible
    // for replayed scenes) or the sweep cap was reached, the env takes the reference's sweeps. ----
    constexpr float kPinnedCost = 224.0f;
    float hmax = 0.f;
    if (tile_ok) {
#pragma unroll
      for (int i = 0; i < TH; ++i)
#pragma unroll
        for (int j = 0; j < TW; ++j) {
          const uint32_t hb = __float_as_uint(h[i + 1][j + 1]);
          if (hb < kInfBits) hmax = fmaxf(hmax, h[i + 1][j + 1]);
        }
    }
    const bool exact = __syncthreads_or((hmax > kPinnedCost) || (it >= kMaxIters)) != 0;
    // ---- 3. raw cost out (occupied marker -> +inf) into the env's field tile: the field's 10 x 10 tiles are
    // these threads' tiles, so the 100 stores are immediate offsets of one base (no per-thread offsets, no
    // scratch copy).  Statistics and the SDF in k_field_stats, the constants in k_field_norm ----
    // (a TH x TW sweep tile is the column part (tc % kSub) of field tile (tr, tc / kSub))
    constexpr int kSub = USV_FIELD_TW / TW;
    static_assert(USV_FIELD_TCOLS * USV_FIELD_TW == G && USV_FIELD_TCOLS == NTC / kSub, "field tiles = sweep tiles");
    if (tile_ok) {
      float *Ft = b.field + (size_t)e * FS + (tr * USV_FIELD_TCOLS + tc / kSub) * (USV_FIELD_TH * USV_FIELD_TW) +
                  (tc % kSub) * TW;
#pragma unroll
      for (int i = 0; i < TH; ++i)
#pragma unroll
        for (int j = 0; j < TW; ++j)
          Ft[i * USV_FIELD_TW + j] = __float_as_uint(h[i + 1][j + 1]) > kInfBits ? INFINITY : h[i + 1][j + 1];
    }
    if (tile_ok) lastc[tp] = -1000;   // ready for the next slot
    if (exact) {   // (uniform) the reference's 225 literal sweeps for this env, over the tiles just stored
      // (rare: never for the packaged spawn ranges; in the sweep kernel itself rather than a launch of its own,
      // whose workgroups had to wait for CUs the concurrent policy step held: ~50 us on the field chain per step)
      __syncthreads();
      float *Fe = b.field + (size_t)e * FS;          // overwritten: the ping-pong buffer, then the cost tiles
      float *scratch = b.sdf + (size_t)e * FS;      // the other ping-pong buffer
      cost_sweeps_exact<NTHR>(occ, ix, iy, Fe, scratch);   // 225 (odd) sweeps: result in scratch
      for (int q = tid; q < G2; q += NTHR) Fe[field_idx(q / G, q % G)] = scratch[q];
      if (tid == 0) atomicAdd(&b.ctl[USV_CTL_FIELD_EXACT], 1);
    }
    if (tid == 0) {
      b.slot_stats[(size_t)slot * kSlotStride + SS_ITERS] = (float)it;   // iterations (diagnostic)
      b.slot_stats[(size_t)slot * kSlotStride + SS_EXACT] = exact ? 1.f : 0.f;   // took the reference's sweeps
#ifdef USV_PHASE_PROBE
      if (blockIdx.x < 4096) g_probe_field[blockIdx.x][15] = (unsigned long long)it;
#endif
    }
    __syncthreads();
    USV_PHASE(field, 3);
  }
}

__global__ __launch_bounds__(kWaveThreads) void k_field_wave(usv_cfg_t c, usv_bufs_t b) { field_wave_body<true>(c, b); }
__global__ __launch_bounds__(kWaveThreads, USV_SWEEP_WAVES) void k_field_wave_pack(usv_cfg_t c, usv_bufs_t b) {
  field_wave_body<false>(c, b);
}
// small batches (fewer reset envs than CUs): one env per CU either way, so 10 x 5 tiles over 450 threads (two waves
// per SIMD instead of one) trade more tile hops per sweep for twice the issue rate (USV_FIELD_HALF)
constexpr int kHalfThreads = 512;
__global__ __launch_bounds__(kHalfThreads) void k_field_wave_half(usv_cfg_t c, usv_bufs_t b) {
  field_wave_body<false, T, T / 2, kHalfThreads>(c, b);
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

// ------------------------------------------------------------- pass C1 ---
// Per (slot, band of kBandRows grid rows): statistics split by finite / infinite cost so
// the batch constant inf_val (known only when every env is done) enters
// through one monotone scalar per batch.  Partials at slot_stats[slot][16 + 12 band].
// The SDF is formed separably with cell_sdf's rounded operations: a thread owns two
// adjacent columns, keeps (gx - ox)^2 of both for the obstacles in registers and,
// per row, forms gy - oy once for the two cells -- fmaf(dy, dy, dx * dx), the same
// min tree, sqrt, minus the radius: the same bits in about half the instructions.
// Every statistic is a min / max (any grouping gives the same value), so the cells can be
// dealt to threads in any shape: each wave owns a compact 38-column x 30-row block of the band
// (19 column pairs x 3 row groups), so the obstacles that can reach it are few (a per-wave mask)
// and many of its row strips lie out of every obstacle's reach, where the SDF cannot enter the
// statistics and a cell contributes only through its cost (the "far" path below).
// USV_STATS_PIPE=1: k_field_stats loads the next item's costs during the current one (0: at the item's start)
#ifndef USV_STATS_PIPE
#define USV_STATS_PIPE 0
#endif
// USV_STATS_REG_OBST=1: every obstacle's (gx - ox)^2 and oy in registers across the band (0: the mask's from LDS,
// 48 fewer VGPRs: with USV_STATS_WAVES 5 waves per SIMD instead of 4, -5% on the kernel late in training)
#ifndef USV_STATS_REG_OBST
#define USV_STATS_REG_OBST 0
#endif
// USV_STATS_WAVES: k_field_stats' minimum waves per SIMD (its register budget: 5 -> 96 VGPRs, no spills with the LDS
// obstacles; 6 spills)
#ifndef USV_STATS_WAVES
#define USV_STATS_WAVES 5
#endif
constexpr int kBandRows = 30, kBands = G / kBandRows;       // row bands of a slot
constexpr int kRowGroups = 3;                               // row groups per wave (rows rg, rg + 3, ...)
constexpr int kWavePairs = 19;                              // column pairs per wave: 4 waves x 38 >= 150 columns
constexpr int kBandIters = kBandRows / kRowGroups;          // rows per thread and band
static_assert(G % kBandRows == 0 && kBandRows % kRowGroups == 0 && kWavePairs * kRowGroups <= 64 &&
              4 * 2 * kWavePairs >= G && G % 2 == 0, "k_field_stats geometry");
static_assert(kSlotObst >= 16 + 12 * kBands, "slot_stats band partials");
__global__ __launch_bounds__(256, USV_STATS_WAVES) void k_field_stats(usv_cfg_t c, usv_bufs_t b) {
  __shared__ float red[10][4];
  __shared__ int flags[2];
  __shared__ float slin[G];
  __shared__ float so[2 * USV_NOBST];
  const int count = min(b.ctl[USV_CTL_RESET_COUNT], b.n);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int cbase = wid * 2 * kWavePairs;                    // first column of this wave's block
  const int cpl = lane % kWavePairs, rg = lane / kWavePairs;
  const int c0u = cbase + 2 * cpl;
  const bool act = rg < kRowGroups && c0u < G;               // other lanes only join the reductions
  const int c0 = act ? c0u : 0;                              // (even: the pair is one tile row)
  const int rgc = act ? rg : 0;
  const int chi = min(cbase + 2 * kWavePairs - 1, G - 1);    // last column of the block
  const float cell = (float)((double)c.map_size / G);
  const float inv_r = (float)(1.0 / (double)c.influence_radius);
  const float inv_safe = 1.0f / c.safe_radius;   // goal_mask's quotient as div_rn (field_value's form)
  // a cell whose squared distance to every obstacle in reach is >= far_d^2 has dte >= R + 1e-3 (jr = 0, not
  // inside) whatever the rounding of the sqrt and the two subtractions: it enters only through its cost
  const float far_d = c.influence_radius + 2.0f * c.obstacle_radius + 0.01f * cell + 1e-3f;
  const uint32_t far2 = __float_as_uint(far_d * far_d);
  const int items = count * kBands;
  if (tid < G) slin[tid] = grid_coord(b.grid_lin, c.map_size, tid);
  // the band's raw costs (two adjacent cells per row: one 8-byte load), all in flight at once
  const auto load_costs = [&](int wq, int eq, float2 *dst) {
    const float *F = b.field + (size_t)eq * FS;     // the raw cost tiles (k_field_wave / k_field_exact)
#pragma unroll
    for (int k = 0; k < kBandIters; ++k) {
      const int r = (wq % kBands) * kBandRows + rgc + kRowGroups * k;
      dst[k] = *reinterpret_cast<const float2 *>(F + field_idx(r, c0));
    }
  };
  // USV_STATS_PIPE: a software pipeline over the workgroup's items -- the next item's obstacle coordinates and slot
  // index load at the top of an item, its costs after the current SDF, so they arrive during this item's statistics
  float2 gA[kBandIters], gB[kBandIters];
  float so_nx = 0.f;
#if USV_STATS_PIPE
  if ((int)blockIdx.x < items) {
    const int sl = (int)blockIdx.x / kBands;
    load_costs((int)blockIdx.x, b.reset_ids[sl], gA);
    if (tid < 2 * USV_NOBST) so_nx = b.slot_stats[(size_t)sl * kSlotStride + kSlotObst + tid];
  }
#endif
  // one item: the statistics of band w % kBands of slot w / kBands from the costs in gv (pipelined: loaded by
  // the previous item) while the next item's costs load into gnx
  const auto item = [&](const int w, float2 (&gv)[kBandIters], float2 (&gnx)[kBandIters]) {
    const int slot = w / kBands, band = w % kBands;
#if USV_STATS_PIPE
    if (tid < 2 * USV_NOBST) so[tid] = so_nx;
    if (tid < 2) flags[tid] = 0;
    __syncthreads();
    // the next item (this one again after the last: loads without a branch, so the wait counts stay exact)
    const int wn = w + (int)gridDim.x < items ? w + (int)gridDim.x : w;
    const int en = b.reset_ids[wn / kBands];
    if (tid < 2 * USV_NOBST) so_nx = b.slot_stats[(size_t)(wn / kBands) * kSlotStride + kSlotObst + tid];
#else
    if (tid < 2 * USV_NOBST) so[tid] = b.slot_stats[(size_t)slot * kSlotStride + kSlotObst + tid];
    if (tid < 2) flags[tid] = 0;
    __syncthreads();
    load_costs(w, b.reset_ids[slot], gv);
#endif
#if USV_STATS_REG_OBST
    float dxa[USV_NOBST], dxb[USV_NOBST], oy[USV_NOBST];
    {
      const float gxa = slin[c0], gxb = slin[c0 + 1];
#pragma unroll
      for (int o = 0; o < USV_NOBST; ++o) {
        const float ox = so[2 * o];
        const float da = gxa - ox, db = gxb - ox;
        dxa[o] = da * da;
        dxb[o] = db * db;
        oy[o] = so[2 * o + 1];
      }
    }
#else
    const float gxa = slin[c0], gxb = slin[c0 + 1];
#endif
    // Obstacles that can matter to this wave's block: the SDF enters the statistics only through j_raw (0
    // unless dist - 2 r_obs < influence_radius) and the inside test (dist <= 2 r_obs), so an obstacle farther
    // than far_d from the whole block (in x or in y) can only be the minimum of a cell whose SDF is irrelevant
    // (jr = 0, not inside, with the exact SDF and with the smaller set alike).  Uniform per wave.
    uint32_t omask;
    {
      const float ylo = slin[band * kBandRows], yhi = slin[band * kBandRows + kBandRows - 1];
      const float xlo = slin[cbase], xhi = slin[chi];
      const int ol = lane & (USV_NOBST - 1);
      const float oxl = so[2 * ol], oyl = so[2 * ol + 1];
      const float dyb = fmaxf(fmaxf(ylo - oyl, oyl - yhi), 0.f);
      const float dxb_ = fmaxf(fmaxf(xlo - oxl, oxl - xhi), 0.f);
      omask = (uint32_t)(__ballot(lane < USV_NOBST && !(dyb > far_d) && !(dxb_ > far_d)) & 0xFFFFull);
      omask = __builtin_amdgcn_readfirstlane(omask);
    }
    float gmin = INFINITY, gmax = -INFINITY, jmin_f = INFINITY, jmax_f = -INFINITY, jall_f = 0.f;
    float jrmin_i = INFINITY, jrmax_i = -INFINITY, jrall_i = 0.f;
    int any_inf = 0, inside = 0;
    // branch-free: each statistic takes its cell's value or the neutral element of its min / max
    const auto stat = [&](float g, float sv) {
      const float dte = sv - c.obstacle_radius;
      const bool ins = dte <= 0.f;
      inside |= ins;
      const float jr = j_raw(c, dte, inv_r);
      const bool gi = isinf(g);
      any_inf |= gi;
      // goal_mask(c, g, cell) as div_rn by the correctly rounded reciprocal: the same bits for every finite
      // g (usv_device.h div_rn); an infinite g gives NaN here, and j is only read where g is finite
      const float j = jr * clampt(div_rn(g * cell, c.safe_radius, inv_safe), 0.f, 1.f);
      jrall_i = fmaxf(jrall_i, gi ? jr : 0.f);
      jrmin_i = fminf(jrmin_i, (gi && !ins) ? jr : INFINITY);
      jrmax_i = fmaxf(jrmax_i, (gi && !ins) ? jr : -INFINITY);
      gmin = fminf(gmin, gi ? INFINITY : g);
      gmax = fmaxf(gmax, gi ? -INFINITY : g);
      jall_f = fmaxf(jall_f, gi ? 0.f : j);
      jmin_f = fminf(jmin_f, (!gi && !ins) ? j : INFINITY);
      jmax_f = fmaxf(jmax_f, (!gi && !ins) ? j : -INFINITY);
    };
    // the same statistics for a cell out of every obstacle's reach (jr = +0, not inside): what stat() gives
    // there, without the sqrt and the divisions (jall_f and jrall_i take max(., +0), a no-op from their +0 start)
    const auto stat_far = [&](float g) {
      const bool gi = isinf(g);
      any_inf |= gi;
      jrmin_i = fminf(jrmin_i, gi ? 0.f : INFINITY);
      jrmax_i = fmaxf(jrmax_i, gi ? 0.f : -INFINITY);
      gmin = fminf(gmin, gi ? INFINITY : g);
      gmax = fmaxf(gmax, gi ? -INFINITY : g);
      jmin_f = fminf(jmin_f, gi ? INFINITY : 0.f);
      jmax_f = fmaxf(jmax_f, gi ? -INFINITY : 0.f);
    };
    // squared distances (non-negative: u32 min of the bit patterns is the float min, exact in any
    // order), obstacle-outer so a skipped obstacle is one scalar branch for the block's rows
    float gy[kBandIters];
    uint32_t a[kBandIters], bb[kBandIters];
#pragma unroll
    for (int k = 0; k < kBandIters; ++k) {
      gy[k] = slin[band * kBandRows + rgc + kRowGroups * k];
      a[k] = bb[k] = 0x7F800000u;
    }
#if USV_STATS_REG_OBST
#pragma unroll
    for (int o = 0; o < USV_NOBST; ++o) {
      if (!((omask >> o) & 1u)) continue;   // uniform
#pragma unroll
      for (int k = 0; k < kBandIters; ++k) {
        const float dy = gy[k] - oy[o];
        a[k] = min(a[k], __float_as_uint(fmaf(dy, dy, dxa[o])));
        bb[k] = min(bb[k], __float_as_uint(fmaf(dy, dy, dxb[o])));
      }
    }
#else
    // the mask's obstacles only (a scalar loop over its set bits; the coordinates are LDS broadcasts): no
    // per-obstacle registers
    for (uint32_t om = omask; om != 0u; om &= om - 1u) {
      const int o = __builtin_ctz(om);
      const float ox = so[2 * o], oyo = so[2 * o + 1];
      const float da = gxa - ox, db = gxb - ox;
      const float dxa = da * da, dxb = db * db;
#pragma unroll
      for (int k = 0; k < kBandIters; ++k) {
        const float dy = gy[k] - oyo;
        a[k] = min(a[k], __float_as_uint(fmaf(dy, dy, dxa)));
        bb[k] = min(bb[k], __float_as_uint(fmaf(dy, dy, dxb)));
      }
    }
#endif
#if USV_STATS_PIPE
    load_costs(wn, en, gnx);
#endif
#pragma unroll
    for (int k = 0; k < kBandIters; ++k) {
      // a row strip of the block whose cells all lie out of reach takes the far path (uniform branch)
      const bool near = act && (a[k] < far2 || bb[k] < far2);
      if (__ballot(near) != 0ull) {
        const float sva = sqrtf(__uint_as_float(a[k])) - c.obstacle_radius;
        const float svb = sqrtf(__uint_as_float(bb[k])) - c.obstacle_radius;
        if (act) {
          stat(gv[k].x, sva);
          stat(gv[k].y, svb);
        }
      } else if (act) {
        stat_far(gv[k].x);
        stat_far(gv[k].y);
      }
    }
    float vals[9] = {wave_min(gmin), wave_max(gmax), wave_min(jmin_f), wave_max(jmax_f), wave_max(jall_f),
                     wave_min(jrmin_i), wave_max(jrmax_i), wave_max(jrall_i), 0.f};
    __syncthreads();   // flags reset visible
    if (lane == 0)
      for (int k = 0; k < 8; ++k) red[k][wid] = vals[k];
    if (any_inf) flags[0] = 1;
    if (inside) flags[1] = 1;
    __syncthreads();
    if (tid == 0) {
      float a[8];
      for (int k = 0; k < 8; ++k) a[k] = red[k][0];
      for (int v = 1; v < 4; ++v) {
        a[0] = fminf(a[0], red[0][v]); a[1] = fmaxf(a[1], red[1][v]);
        a[2] = fminf(a[2], red[2][v]); a[3] = fmaxf(a[3], red[3][v]); a[4] = fmaxf(a[4], red[4][v]);
        a[5] = fminf(a[5], red[5][v]); a[6] = fmaxf(a[6], red[6][v]); a[7] = fmaxf(a[7], red[7][v]);
      }
      float *pp = b.slot_stats + (size_t)slot * kSlotStride + 16 + 12 * band;
      pp[SS_GMIN_F] = a[0]; pp[SS_GMAX_F] = a[1]; pp[SS_ANY_INF] = flags[0] ? 1.f : 0.f;
      pp[SS_JMIN_F_NI] = a[2]; pp[SS_JMAX_F_NI] = a[3]; pp[SS_JMAX_F_ALL] = a[4];
      pp[SS_JRMIN_I_NI] = a[5]; pp[SS_JRMAX_I_NI] = a[6]; pp[SS_JRMAX_I_ALL] = a[7];
      pp[SS_INSIDE] = flags[1] ? 1.f : 0.f;
      // the batch max of finite costs (:205-210) is folded from these band maxima by
      // k_field_batch (one atomic per band on a single address serialised this kernel)
    }
    __syncthreads();
  };
#if USV_STATS_PIPE
  // the two cost buffers in turn: no register copies between items (a copy would wait for the loads)
  for (int w = blockIdx.x; w < items;) {
    item(w, gA, gB);
    w += (int)gridDim.x;
    if (w >= items) break;
    item(w, gB, gA);
    w += (int)gridDim.x;
  }
#else
  for (int w = blockIdx.x; w < items; w += gridDim.x) item(w, gA, gB);
#endif
}

// ------------------------------------------------------------- pass C2 ---
// fold each slot's chunk partials (chunk order), then the batch maxima: the max of
// finite costs (d_multi_gemini.py:205-210), J.max() (:257-260) and the any-inside
// flag.  Six slots per wave (lane 10 g + q folds statistic q of the wave's slot g over the chunks: one cache
// line per chunk row instead of a scattered load per statistic and slot), waves of
// kBatchBlocks workgroups loop over the slots; the batch maxima leave through max
// atomics (exact in any order, one set per workgroup) and the last workgroup forms
// J.max() = max(J over finite cells, mask(inf_val) * raw J over infinite cells) --
// the multiplication by the non-negative mask is monotone, so the max of the
// products is the product with the max.
// USV_BATCH_BLOCKS: the batch fold's workgroups (64; 256 measured slower: the per-workgroup max atomics
// contend).  USV_BATCH_SLOTS_PER_WAVE: slots per wave and round (6: lanes 0-59; 1: lanes 0-9, one dependent round of
// band-partial loads per slot, ~8 rounds at ~2,000 resets per step)
#ifndef USV_BATCH_BLOCKS
#define USV_BATCH_BLOCKS 64
#endif
#ifndef USV_BATCH_SLOTS_PER_WAVE
#define USV_BATCH_SLOTS_PER_WAVE 6
#endif
constexpr int kBatchBlocks = USV_BATCH_BLOCKS;
constexpr int kBatchSpw = USV_BATCH_SLOTS_PER_WAVE;
static_assert(kBatchSpw >= 1 && 10 * kBatchSpw <= 64, "k_field_batch lane groups");
__global__ __launch_bounds__(256) void k_field_batch(usv_cfg_t c, usv_bufs_t b) {
  __shared__ float wred[4][4];
  __shared__ bool last;
  const int count = min(b.ctl[USV_CTL_RESET_COUNT], b.n);
  if (count <= 0) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = lane / 10, q = lane % 10, l0 = 10 * grp;   // slot group of this lane, its statistic
  const int nw = (int)gridDim.x * 4;
  // the lane's running maxima over its groups' slots (max-neutral starts: costs and J are >= 0)
  float gfin = -INFINITY, jf = 0.f, jr = 0.f, ins = 0.f;
  const bool is_min = q == SS_GMIN_F || q == SS_JMIN_F_NI || q == SS_JRMIN_I_NI;
  for (int sl0 = ((int)blockIdx.x * 4 + wid) * kBatchSpw; sl0 < count; sl0 += nw * kBatchSpw) {
    const int sl = sl0 + grp;
    const bool ok = grp < kBatchSpw && sl < count;
    float a = 0.f;
    if (ok) {
      float *st = b.slot_stats + (size_t)sl * kSlotStride;
      float x[kBands];
#pragma unroll
      for (int ch = 0; ch < kBands; ++ch) x[ch] = st[16 + 12 * ch + q];
      a = x[0];
#pragma unroll
      for (int ch = 1; ch < kBands; ++ch) a = is_min ? fminf(a, x[ch]) : fmaxf(a, x[ch]);
      st[q] = a;
    }
    // the slot's folded statistics from its group's lanes (lanes without a slot read themselves, unused)
    const float s_gmax = __shfl(a, ok ? l0 + SS_GMAX_F : lane, 64);
    const float s_anyinf = __shfl(a, ok ? l0 + SS_ANY_INF : lane, 64);
    const float s_jf = __shfl(a, ok ? l0 + SS_JMAX_F_ALL : lane, 64);
    const float s_jr = __shfl(a, ok ? l0 + SS_JRMAX_I_ALL : lane, 64);
    const float s_in = __shfl(a, ok ? l0 + SS_INSIDE : lane, 64);
    if (ok) {
      gfin = fmaxf(gfin, s_gmax);             // -inf: no finite cell in the slot
      jf = fmaxf(jf, s_jf);
      if (s_anyinf != 0.f) jr = fmaxf(jr, s_jr);
      ins = fmaxf(ins, s_in);
    }
  }
  // wave maxima over the lanes (max is exact in any order)
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) {
    gfin = fmaxf(gfin, __shfl_xor(gfin, off, 64));
    jf = fmaxf(jf, __shfl_xor(jf, off, 64));
    jr = fmaxf(jr, __shfl_xor(jr, off, 64));
    ins = fmaxf(ins, __shfl_xor(ins, off, 64));
  }
  if (lane == 0) { wred[wid][0] = gfin; wred[wid][1] = jf; wred[wid][2] = jr; wred[wid][3] = ins; }
  __syncthreads();
  if (tid == 0) {
    float g = wred[0][0], f = wred[0][1], r = wred[0][2], in = wred[0][3];
    for (int w = 1; w < 4; ++w) {
      g = fmaxf(g, wred[w][0]); f = fmaxf(f, wred[w][1]); r = fmaxf(r, wred[w][2]); in = fmaxf(in, wred[w][3]);
    }
    // fscratch[0], [2], [3] and the two flags start at 0 (k_step_begin); costs and J are >= 0
    if (isfinite(g)) {
      atomic_max_f32(&b.fscratch[0], g);
      atomicOr(&b.ctl[USV_CTL_ANY_FINITE], 1);
    }
    atomic_max_f32(&b.fscratch[2], f);
    atomic_max_f32(&b.fscratch[3], r);
    if (in != 0.f) atomicOr(&b.ctl[USV_CTL_ANY_INSIDE], 1);
    __threadfence();
    last = atomicAdd(&b.ctl[USV_CTL_BATCH_DONE], 1) == (int)gridDim.x - 1;
  }
  __syncthreads();
  if (!last || tid != 0) return;
  __threadfence();
  const BatchK k = batch_k(c, b);
  b.fscratch[1] = fmaxf(b.fscratch[2], b.fscratch[3] * k.mask_inf);   // J.max() over the batch (:257)
  b.ctl[USV_CTL_BATCH_DONE] = 0;
}

// ---------------------------------------------------------------- pass D ---
// The per-env normalisation (d_multi_gemini.py:211-223, 262-271) as constants: the env's cost range
// with inf_val for unreachable cells, its J range with the batch's `high` for inside cells, and the batch
// values a texel needs (inf_val, high, any-inside) -> usv_bufs_t.fnorm.  The field is never materialised:
// its readers form texels with field_value (usv_device.h) from the SDF, the cost and these constants
// (the reference materialises 150 x 150 floats per reset env that the env step samples at 4 texels).
__global__ __launch_bounds__(256) void k_field_norm(usv_cfg_t c, usv_bufs_t b) {
  const int count = min(b.ctl[USV_CTL_RESET_COUNT], b.n);
  const BatchK k = batch_k(c, b);
  const bool any_inside = b.ctl[USV_CTL_ANY_INSIDE] != 0;
  const float cur_max = b.fscratch[1];
  const float high = (cur_max > 1e-6f) ? cur_max * 10.0f : 100.0f;
  for (int slot = (int)(blockIdx.x * blockDim.x + threadIdx.x); slot < count; slot += (int)(gridDim.x * blockDim.x)) {
    const int e = b.reset_ids[slot];
    const float *st = b.slot_stats + (size_t)slot * kSlotStride;
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
    float4 *fn = reinterpret_cast<float4 *>(b.fnorm + (size_t)e * USV_FNORM);
    const float gden = (gmax - gmin) + 1e-6f, jden = (jmx - jmn) + 1e-6f;
    fn[0] = make_float4(gmin, gden, jmn, jden);
    fn[1] = make_float4(k.inf_val, any_inside ? high : -high, 1.0f / gden, 1.0f / jden);   // (field_norm_of)
  }
}

// usv_field_view: the materialised fields of `count` envs, row-major [count][G][G] (tests, host views)
__global__ __launch_bounds__(256) void k_field_view(usv_cfg_t c, usv_bufs_t b, const int32_t *ids, int count,
                                                    float *out) {
  const float cell = (float)((double)c.map_size / G);
  const float inv_r = (float)(1.0 / (double)c.influence_radius);
  const float inv_safe = 1.0f / c.safe_radius;
  const long long total = (long long)count * G2;
  for (long long q = (long long)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (long long)gridDim.x * blockDim.x) {
    const int i = (int)(q / G2), cell_i = (int)(q % G2), r = cell_i / G, cc = cell_i % G;
    const int e = ids[i];
    const float4 *fn = reinterpret_cast<const float4 *>(b.fnorm + (size_t)e * USV_FNORM);
    const FieldNorm k = field_norm_of(fn[0], fn[1]);
    const float *ob = b.obst + e;   // [16][2][n]
    const float sv = cell_sdf([&](int o) { return make_float2(ob[(size_t)(2 * o) * b.n], ob[(size_t)(2 * o + 1) * b.n]); },
                              grid_coord(b.grid_lin, c.map_size, cc), grid_coord(b.grid_lin, c.map_size, r),
                              c.obstacle_radius);
    out[q] = field_value(c, k, sv, b.field[(size_t)e * FS + field_idx(r, cc)], cell, inv_r, inv_safe);
  }
}

}  // namespace

namespace {
// stage 1: the obstacle placement alone (k_field_place); stage 2: the rest after it (sweeps, exactness
// fallback, statistics, batch fold, constants) = stage 3 (sweeps, fallback, statistics) + stage 4 (batch fold,
// constants)
// k_field_stats' grid: workgroups loop over (slot, band) items; USV_STATS_GRID caps it (default 4096)
static int stats_grid(int n) {
  static const int cap = [] {
    const char *v = getenv("USV_STATS_GRID");
    const int x = v ? atoi(v) : 0;
    return x > 0 ? x : 4096;
  }();
  return n * kBands < cap ? n * kBands : cap;
}

int field_stages(const usv_cfg_t *cfg, const usv_bufs_t *b, int stage, hipStream_t s) {
  const int grid_b = b->n < 512 ? b->n : 512;
  const int grid_n = (b->n + 255) / 256 < 64 ? (b->n + 255) / 256 : 64;
  const int grid_p = (b->n + kPlaceTB / 64 - 1) / (kPlaceTB / 64) < 1024 ? (b->n + kPlaceTB / 64 - 1) / (kPlaceTB / 64) : 1024;
  if (stage == 1) {
    hipLaunchKernelGGL(k_field_place, dim3(grid_p), dim3(kPlaceTB), 0, s, *cfg, *b);
    USV_CHECK_LAUNCH();
    return 0;
  }
  if (stage == 2 || stage == 3) {
    // USV_FIELD_HALF=1/0 forces the small-batch sweep kernel on / off; unset: on below kFieldPackMinEnvs envs
    const char *half_env = getenv("USV_FIELD_HALF");
    const bool half = half_env ? atoi(half_env) != 0 : b->n < kFieldPackMinEnvs;
    if (half) {
      hipLaunchKernelGGL(k_field_wave_half, dim3(b->n < 256 ? b->n : 256), dim3(kHalfThreads), 0, s, *cfg, *b);
    } else {
      const int grid_w = b->n < kPackGrid ? b->n : kPackGrid;
      hipLaunchKernelGGL(k_field_wave_pack, dim3(grid_w), dim3(kWaveThreads), 0, s, *cfg, *b);
    }
    USV_CHECK_LAUNCH();
    const int grid_s = stats_grid(b->n);
    hipLaunchKernelGGL(k_field_stats, dim3(grid_s), dim3(256), 0, s, *cfg, *b);
    USV_CHECK_LAUNCH();
  }
  if (stage == 2 || stage == 4) {
    hipLaunchKernelGGL(k_field_batch, dim3(kBatchBlocks), dim3(256), 0, s, *cfg, *b);
    USV_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_field_norm, dim3(grid_n), dim3(256), 0, s, *cfg, *b);
    USV_CHECK_LAUNCH();
  }
  return 0;
}
}  // namespace

extern "C" int usv_field_stage(const usv_cfg_t *cfg, const usv_bufs_t *b, int stage, void *stream) {
  if (!cfg || !b || b->n <= 0 || !b->slot_stats || !b->field || !b->sdf || !b->fnorm || stage < 1 || stage > 4) return 1;
  return field_stages(cfg, b, stage, (hipStream_t)stream);
}

extern "C" int usv_field_view(const usv_cfg_t *cfg, const usv_bufs_t *b, const int32_t *env_ids, int count,
                              float *out, void *stream) {
  if (!cfg || !b || b->n <= 0 || !b->field || !b->sdf || !b->fnorm || !env_ids || !out || count < 0) return 1;
  if (count == 0) return 0;
  const long long total = (long long)count * G2;
  const int grid = (int)((total + 255) / 256 < 8192 ? (total + 255) / 256 : 8192);
  hipLaunchKernelGGL(k_field_view, dim3(grid), dim3(256), 0, (hipStream_t)stream, *cfg, *b, env_ids, count, out);
  USV_CHECK_LAUNCH();
  return 0;
}

extern "C" int usv_potential_field(const usv_cfg_t *cfg, const usv_bufs_t *b, void *stream) {
  if (!cfg || !b || b->n <= 0 || !b->slot_stats || !b->field || !b->sdf || !b->fnorm) return 1;
  hipStream_t s = (hipStream_t)stream;
  // the reset count lives on the device: launch persistent grids, blocks loop over slots
  const int grid_b = b->n < 512 ? b->n : 512;
  const int grid_n = (b->n + 255) / 256 < 64 ? (b->n + 255) / 256 : 64;
  // two reset envs per CU only when the batch fills the chip more than once (a few hundred
  // resets per step); USV_FIELD_PACK=0/1 forces either layout (A/B runs, tests)
  const char *pack_env = getenv("USV_FIELD_PACK");
  const bool pack = pack_env ? atoi(pack_env) != 0 : b->n >= kFieldPackMinEnvs;
  if (pack) {
    // large batches: placement first, one wave per reset env (the grid covers n envs at most;
    // the count lives on the device); k_field_wave places in-kernel
    const int grid_p = (b->n + kPlaceTB / 64 - 1) / (kPlaceTB / 64) < 1024 ? (b->n + kPlaceTB / 64 - 1) / (kPlaceTB / 64) : 1024;
    hipLaunchKernelGGL(k_field_place, dim3(grid_p), dim3(kPlaceTB), 0, s, *cfg, *b);
    USV_CHECK_LAUNCH();
  }
  if (pack) hipLaunchKernelGGL(k_field_wave_pack, dim3(b->n < kPackGrid ? b->n : kPackGrid), dim3(kWaveThreads), 0, s,
                              *cfg, *b);
  else hipLaunchKernelGGL(k_field_wave, dim3(grid_b), dim3(kWaveThreads), 0, s, *cfg, *b);
  USV_CHECK_LAUNCH();
  const int grid_s = stats_grid(b->n);
  hipLaunchKernelGGL(k_field_stats, dim3(grid_s), dim3(256), 0, s, *cfg, *b);
  USV_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_field_batch, dim3(kBatchBlocks), dim3(256), 0, s, *cfg, *b);
  USV_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_field_norm, dim3(grid_n), dim3(256), 0, s, *cfg, *b);
  USV_CHECK_LAUNCH();
  return 0;
}
