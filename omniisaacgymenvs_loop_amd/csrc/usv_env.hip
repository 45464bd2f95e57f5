// USV CaptureXY env hot path for MI355X (gfx950): thruster LUT, reset path
// (compaction + domain randomisation + spawn/obstacle rejection sampling) and
// the fused control step (action mapping, 10 substeps of 3-DoF hydrodynamics
// with semi-implicit Euler, observation, reward, penalties, kills, stats).
//
// One thread per env, struct-of-arrays state in HBM: every per-env field is a
// coalesced 4-byte-per-lane stream.  The step kernel keeps the 10 substeps in
// registers (state is read once and written once per control step).
//
// Reference call chains replaced (loop-Z/omniisaacgymenvs_loop):
//   envs/vec_env_rlgames.py:120-217          VecEnvRLGames.step
//   tasks/USV_Virtual.py:1042-1133            pre_physics_step, apply_forces
//   tasks/USV_Virtual.py:771-986              update_state, get_observations
//   tasks/USV_Virtual.py:1223-1237,1628-1652  is_done, calculate_metrics
//   tasks/USV_Virtual.py:1502-1618            reset_idx
//   tasks/USV/USV_capture_xy_static_obs.py    get_state_observations, compute_reward,
//                                             update_kills, get_spawns, get_goals
//   envs/USV/{Hydrodynamics,ThrusterDynamics}.py  damping + thruster LUT/lag
// The rigid-body integrator replaces PhysX (no reference implementation).
#include "usv_device.h"

namespace {

constexpr int kBlock = 256;

// ------------------------------------------------------------------------
// Thruster LUT: F.interpolate(linear, align_corners=True) 21 -> 1000 points
// (ThrusterDynamics.py:152-177).  The CPU build of the reference contracts
// l0*t[i0] + l1*t[i1] into fma(l0, t[i0], l1*t[i1]).
// ------------------------------------------------------------------------
__global__ void k_build_lut(const float *__restrict__ tl, const float *__restrict__ tr, int n_in,
                            float *__restrict__ lut) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= USV_LUT_N) return;
  const float scale = (float)(n_in - 1) / (float)(USV_LUT_N - 1);
  const float src = scale * (float)i;
  int i0 = (int)src;
  if (i0 > n_in - 1) i0 = n_in - 1;
  const int off = (i0 < n_in - 1) ? 1 : 0;
  const float l1 = src - (float)i0;
  const float l0 = 1.0f - l1;
  lut[i] = fmaf(l0, tl[i0], l1 * tl[i0 + off]);
  lut[USV_LUT_N + i] = fmaf(l0, tr[i0], l1 * tr[i0 + off]);
}

// step index / action bias of this step: the device clock when present
__device__ __forceinline__ uint64_t step_of(const usv_bufs_t &b, uint64_t step) { return b.clock ? b.clock[2] : step; }
__device__ __forceinline__ float bias_of(const usv_cfg_t &c, const usv_bufs_t &b, float bias) {
  if (!b.clock) return bias;
  return (c.act_bias_steps > 0 && b.clock[3] < (uint64_t)c.act_bias_steps) ? c.act_bias : 0.f;
}

// reset-slot uniform i of env e (injected row e, or Philox site 0x100)
struct ResetRng {
  const float *inj;
  uint64_t seed, step;
  uint32_t env;
  int cached_blk = -1;
  float buf[4];
  __device__ float operator()(int i) {
    if (inj) return inj[(size_t)env * USV_NU_RESET + i];
    const int blk = i >> 2;
    if (blk != cached_blk) {
      philox_u4(seed, env, step, 0x100u + (uint32_t)blk, buf);
      cached_blk = blk;
    }
    return buf[i & 3];
  }
};

// ------------------------------------------------------------------------
// Per-step scratch reset (reset count, field maxima, extras sums): one tiny
// kernel instead of four memset nodes.
// ------------------------------------------------------------------------
__global__ void k_step_begin(usv_bufs_t b) {
  const int t = threadIdx.x;
  if (t == 0 && b.clock) {   // device step clock: this step's index and bias-call count
    b.clock[2] = b.clock[0]++;
    b.clock[3] = b.clock[1]++;
  }
  if (t == 0) b.ctl[USV_CTL_RESET_COUNT] = 0;
  if (t == 1) b.ctl[USV_CTL_ANY_INSIDE] = 0;
  if (t == 2) b.ctl[USV_CTL_ANY_FINITE] = 0;
  if (t < 4) b.fscratch[t] = 0.f;
  if (t < USV_NSTAT) b.extras_acc[t] = 0.f;
}

// ------------------------------------------------------------------------
// Reset path (USVVirtual.reset_idx, USV_Virtual.py:1502-1618).  One thread per
// env; threads of envs with reset_buf==1 do the work.  The reset list is
// compacted with a wave ballot + one atomic per wave (order is irrelevant:
// draws are keyed by env id, the potential-field batch statistics are maxima).
// Obstacle rejection sampling follows in the same kernel, one whole wave per
// reset env (place_obstacles).
// ------------------------------------------------------------------------
// 64-lane (whole wave) obstacle placement for reset env ee (CaptureXYTask.get_spawns
// obstacle part, static_obs.py:968-1048).  Lane (q, o) = (lane >> 4, lane & 15) holds
// obstacle o (replicated over the four 16-lane groups) and draws the candidate of
// iteration 4r + q of round r, so the Philox work of four rejection iterations runs in
// parallel; the iterations themselves stay sequential and pick candidates by shuffle.
// Box around the previous-episode target; an obstacle is redrawn while it is closer
// than min_dist_safe to the spawn or the target, or closer than min_obs_sep to a
// lower-index obstacle; after USV_SPAWN_ITERS redraws the leftovers go to limbo
// (999, 999).  Same uniforms as the per-env restatement (reset slots RU_OBST + 2o,
// RU_RESAMPLE + 32 it + 2o (+1)).
__device__ void place_obstacles(const usv_cfg_t &c, const usv_bufs_t &b, int ee, float sx, float sy, float tx,
                                float ty, uint64_t seed, uint64_t step, const float *__restrict__ inj) {
  static_assert(USV_NOBST == 16, "16-lane groups");
  const int n = b.n;
  const int lane = threadIdx.x & 63, o = lane & 15, q = lane >> 4, gbase = lane & 48;
  auto Ue = [&](int i) -> float {
    if (inj) return inj[(size_t)ee * USV_NU_RESET + i];
    float u4[4];
    philox_u4(seed, (uint32_t)ee, step, 0x100u + (uint32_t)(i >> 2), u4);
    return u4[i & 3];
  };
  const float mnx = tx - c.obst_box, mny = ty - c.obst_box;
  const float dx_ = (tx + c.obst_box) - mnx, dy_ = (ty + c.obst_box) - mny;
  float ox = Ue(RU_OBST + 2 * o) * dx_ + mnx;
  float oy = Ue(RU_OBST + 2 * o + 1) * dy_ + mny;
  const float sep2 = c.min_obs_sep * c.min_obs_sep;
  bool done = false;
  for (int r = 0; !done; ++r) {
    const int itq = 4 * r + q;
    float cx = 0.f, cy = 0.f;
    if (itq < USV_SPAWN_ITERS) {
      const int rb = RU_RESAMPLE + itq * USV_NOBST * 2;
      cx = Ue(rb + 2 * o) * dx_ + mnx;
      cy = Ue(rb + 2 * o + 1) * dy_ + mny;
    }
    for (int qq = 0; qq < 4; ++qq) {
      const int it = 4 * r + qq;
      const float ds = tnorm2(ox - sx, oy - sy);
      const float dt = tnorm2(ox - tx, oy - ty);
      bool bad = (ds < c.min_dist_safe) || (dt < c.min_dist_safe);
      const bool vo = ox < 900.f;
#pragma unroll
      for (int i = 0; i < USV_NOBST - 1; ++i) {
        const float xi = __shfl(ox, gbase + i, 64), yi = __shfl(oy, gbase + i, 64);
        const float ddx = xi - ox, ddy = yi - oy;
        if (i < o && vo && (xi < 900.f) && (ddx * ddx + ddy * ddy) < sep2) bad = true;
      }
      const uint32_t inval = (uint32_t)((__ballot(bad) >> gbase) & 0xFFFFull);   // same in every group
      if (inval == 0) { done = true; break; }
      if (it == USV_SPAWN_ITERS) {  // leftovers to limbo (:1042-1048)
        if (bad) { ox = 999.0f; oy = 999.0f; }
        done = true;
        break;
      }
      const float nx = __shfl(cx, 16 * qq + o, 64), ny = __shfl(cy, 16 * qq + o, 64);
      if (bad) { ox = nx; oy = ny; }
    }
  }
  if (q == 0) {
    b.obst[(size_t)(2 * o) * n + ee] = ox;
    b.obst[(size_t)(2 * o + 1) * n + ee] = oy;
  }
}

__global__ __launch_bounds__(kBlock) void k_reset(usv_cfg_t c, usv_bufs_t b, uint64_t seed, uint64_t step,
                                                  const float *__restrict__ inj) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = b.n;
  const bool active = (e < n) && (b.reset_buf[e] != 0);
  const int lane = threadIdx.x & 63;
  step = step_of(b, step);
  // ---- compaction: reset_buf.nonzero() (USV_Virtual.py:1045) ----
  const uint64_t mask = __ballot(active);
  if (mask != 0) {
    const int leader = __ffsll((long long)mask) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(&b.ctl[USV_CTL_RESET_COUNT], __popcll(mask));
    base = __shfl(base, leader, 64);
    // ---- episode extras: sums of the envs being reset (:1591-1612), one atomic per wave ----
    if (c.stats_on) {
      for (int q = 0; q < USV_NSTAT; ++q) {
        float v = 0.f;
        if (active) {
          v = b.stats[(size_t)q * n + e];
          if (q == ST_SUCCESS) v = (float)b.done_succ[e];
          if (q == ST_COLLISION) v = (float)b.done_coll[e];
          b.stats[(size_t)q * n + e] = 0.f;
        }
        v = wave_sum(v);
        if (lane == leader) atomicAdd(&b.extras_acc[q], v);
      }
    }
    float sx = 0.f, sy = 0.f, tx = 0.f, ty = 0.f;
    if (active) {
      const int slot = base + __popcll(mask & ((1ull << lane) - 1ull));
      b.reset_ids[slot] = e;
      ResetRng U{inj, seed, step, (uint32_t)e};
      // ---- CaptureXYTask.reset (static_obs.py:767-778) ----
      b.goal_cnt[e] = 0;
      b.done_succ[e] = 0;
      b.done_coll[e] = 0;
      b.just_reset[e] = 1;
      // ---- MassDistributionDisturbances.randomize_masses / _randomize_com (USV_disturbances.py:94-150) ----
      float mass;
      if (c.mass_dr_on) mass = U(RU_MASS) * (float)((double)c.mass_max - (double)c.mass_min) + c.mass_min;
      else mass = U(RU_MASS) * 0.0f + c.base_mass;
      float cx = c.base_com[0], cy = c.base_com[1], cz = c.base_com[2];
      if (c.mass_dr_on && c.com_mode == 1) {
        cx = c.base_com[0] + (U(RU_COM + 0) * 2.0f - 1.0f) * c.com_disp[0];
        cy = c.base_com[1] + (U(RU_COM + 1) * 2.0f - 1.0f) * c.com_disp[1];
        cz = c.base_com[2] + (U(RU_COM + 2) * 2.0f - 1.0f) * c.com_disp[2];
      } else if (c.mass_dr_on && c.com_mode == 2 && c.com_legacy_r > 0.f) {
        const float r = U(RU_COM) * c.com_legacy_r;
        const float th = U(RU_COM + 1) * USV_PI_F * 2.0f;
        cx = c.base_com[0] + cosf(th) * r;
        cy = c.base_com[1] + sinf(th) * r;
      }
      b.mass[e] = mass;
      b.com_x[e] = cx;
      b.com_y[e] = cy;
      b.com_z[e] = cz;
      // ---- independent randomisations (yaw inertia :193-240, drag :136-174, thrusters :112-127) ----
      if (c.indep_kiz_on && !c.couple_kiz) {
        const float u = U(RU_KIZ);
        b.k_iz[e] = c.kiz_log ? expf(logf(c.kiz_min) + u * (logf(c.kiz_max) - logf(c.kiz_min)))
                              : c.kiz_min + u * (c.kiz_max - c.kiz_min);
      }
      if (c.drag_rand_on && b.lin_damp) {
        for (int a = 0; a < 3; ++a) {
          b.lin_damp[(size_t)a * n + e] = c.lin_damp[a] + (U(RU_DRAG + a) * 2.0f - 1.0f) * c.lin_rand[a];
          b.quad_damp[(size_t)a * n + e] = c.quad_damp[a] + (U(RU_DRAG + 6 + a) * 2.0f - 1.0f) * c.quad_rand[a];
        }
      }
      if (c.indep_kdrag_on) {
        const float u = U(RU_KDRAG);
        b.k_drag[e] = c.kdrag_log ? expf(logf(c.kdrag_min) + u * (logf(c.kdrag_max) - logf(c.kdrag_min)))
                                  : c.kdrag_min + u * (c.kdrag_max - c.kdrag_min);
      }
      if (c.indep_thr_on) {
        if (c.thr_separate) {
          b.thr_l[e] = U(RU_THR) * 2.0f * c.left_rand + (1.0f - c.left_rand);
          b.thr_r[e] = U(RU_THR + 1) * 2.0f * c.right_rand + (1.0f - c.right_rand);
        } else {
          const float m = U(RU_THR) * 2.0f * c.thr_rand + (1.0f - c.thr_rand);
          b.thr_l[e] = m;
          b.thr_r[e] = m;
        }
      }
      // ---- _apply_mass_driven_coupling (USV_Virtual.py:988-1040) ----
      if (c.couple_drag || c.couple_thr || c.couple_kiz) {
        const double den_d = (double)c.mass_max - (double)c.base_mass;
        const float den = (float)(den_d > 1e-6 ? den_d : 1e-6);
        const float r = clampt((mass - c.base_mass) / den, 0.f, 1.f);
        b.mass_r[e] = r;
        if (c.couple_drag) b.k_drag[e] = c.kdrag_min + r * (float)((double)c.kdrag_max - (double)c.kdrag_min);
        if (c.couple_thr) {
          const float s = clampt(1.0f - r * c.thr_rand, (float)(1.0 - (double)c.thr_rand), 1.0f);
          b.thr_l[e] = s;
          b.thr_r[e] = s;
        }
        if (c.couple_kiz) b.k_iz[e] = c.kiz_min + r * (float)((double)c.kiz_max - (double)c.kiz_min);
      }
      // ---- CaptureXYTask.get_spawns (static_obs.py:936-1060), previous-episode target ----
      const float r = U(RU_SPAWN_R) * (c.spawn_rmax - c.spawn_rmin) + c.spawn_rmin;
      const float th = U(RU_SPAWN_TH) * 2.0f * USV_PI_F;
      sx = r * cosf(th);
      sy = r * sinf(th);
      const float yaw0 = U(RU_YAW) * USV_PI_F;
      tx = b.tgt_x[e];
      ty = b.tgt_y[e];
      b.field_old_tgt[e] = tx;
      b.field_old_tgt[n + e] = ty;
      // ---- pose / velocities / bookkeeping (USV_Virtual.py:1541-1579) ----
      b.px[e] = sx;
      b.py[e] = sy;
      b.yaw[e] = yaw0;
      b.vx[e] = U(RU_VX) * 3.0f - 1.5f;
      b.vy[e] = U(RU_VY) * 3.0f - 1.5f;
      b.wz[e] = 0.f;
      b.reset_buf[e] = 0;
      b.progress[e] = 0;
      b.prev_cmd[e] = 0.f;
      b.prev_cmd[n + e] = 0.f;
      // ---- set_targets -> get_goals (static_obs.py:913-930) ----
      const float g = c.goal_random_position;
      b.tgt_x[e] = U(RU_GOAL) * g * 2.0f - g;
      b.tgt_y[e] = U(RU_GOAL + 1) * g * 2.0f - g;
    }
    // ---- obstacles: the whole wave places each of its reset envs in turn ----
    for (uint64_t mm = mask; mm; mm &= mm - 1) {
      const int src = __ffsll((long long)mm) - 1;
      const int ee = blockIdx.x * blockDim.x + (threadIdx.x & ~63) + src;
      place_obstacles(c, b, ee, __shfl(sx, src, 64), __shfl(sy, src, 64), __shfl(tx, src, 64),
                      __shfl(ty, src, 64), seed, step, inj);
    }
  }
  // ---- the last workgroup finalises extras["episode"] = means over this step's resets (:1591-1612) ----
  __shared__ bool last;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(&b.ctl[USV_CTL_OBST_DONE], 1) == (int)gridDim.x - 1;
    __threadfence();
  }
  __syncthreads();
  if (!last) return;
  const int count = b.ctl[USV_CTL_RESET_COUNT];
  const int qs = threadIdx.x;
  if (qs < USV_NSTAT && count > 0) {
    float m = b.extras_acc[qs] / (float)count;
    if (qs != ST_SUCCESS && qs != ST_COLLISION) m = m / (float)c.max_episode_length;
    b.extras[qs] = isnan(m) ? 0.f : m;
  }
  if (qs == 0) b.ctl[USV_CTL_OBST_DONE] = 0;
}

// ------------------------------------------------------------------------
// grid_sample(field, 2*pos/map, bilinear, border, align_corners=False)
// (static_obs.py:302-326) in the arithmetic of PyTorch's CPU kernel.
// ------------------------------------------------------------------------
__device__ __forceinline__ float sample_field(const float *__restrict__ F, float map_size, float x, float y) {
  constexpr int G = USV_GRID;
  const float gx = 2.0f * x / map_size, gy = 2.0f * y / map_size;
  const float half = (float)G / 2.0f;
  float ix = fmaf(gx + 1.f, half, -0.5f);
  float iy = fmaf(gy + 1.f, half, -0.5f);
  ix = minf((float)(G - 1), maxf(ix, 0.f));
  iy = minf((float)(G - 1), maxf(iy, 0.f));
  const float xw = floorf(ix), yn = floorf(iy);
  const float w = ix - xw, ee = 1.f - w;
  const float nn = iy - yn, ss = 1.f - nn;
  const float nw = ss * ee, ne = ss * w, sw = nn * ee, se = nn * w;
  const int i0 = (int)xw, j0 = (int)yn, i1 = i0 + 1, j1 = j0 + 1;
  const float v_nw = F[j0 * G + i0];
  const float v_ne = (i1 < G) ? F[j0 * G + i1] : 0.f;
  const float v_sw = (j1 < G) ? F[j1 * G + i0] : 0.f;
  const float v_se = (i1 < G && j1 < G) ? F[j1 * G + i1] : 0.f;
  return fmaf(v_se, se, fmaf(v_sw, sw, fmaf(v_ne, ne, v_nw * nw)));
}

__device__ __forceinline__ float pen_scalar(int kind, float k, float x0, float cc, float x) {
  if (kind == PEN_DEADZONE) return -maxf(fabsf(x) - x0, 0.f) * k + cc;
  if (kind == PEN_EXPABS) return (expf(x0 * fabsf(x)) - 1.0f) * k + cc;
  return 0.f;
}

__device__ __forceinline__ float enc_centered(float x, float xmin, float xmax, float nominal) {
  double s = fabs((double)xmin - nominal);
  if (fabs((double)xmax - nominal) > s) s = fabs((double)xmax - nominal);
  if (1e-6 > s) s = 1e-6;
  return clampt((x - nominal) / (float)s, -1.f, 1.f);
}
__device__ __forceinline__ float enc_minmax(float x, float xmin, float xmax) {
  if ((double)xmax - (double)xmin <= 1e-6) return 0.f;
  const float z = (x - xmin) / (float)((double)xmax - (double)xmin);
  return clampt(2.0f * z - 1.0f, -1.f, 1.f);
}

// ------------------------------------------------------------------------
// Fused control step.  Reads per env: state (6) + lag (2) + DR params (6) +
// task/history (~12) + obstacles (32) + 4 texels of the field; writes state,
// lag, history, obs row (33), reward, done, stats.
// ------------------------------------------------------------------------
template <bool kStats>
__global__ __launch_bounds__(kBlock) void k_env_step(usv_cfg_t c, usv_bufs_t b, const float *__restrict__ actions,
                                                     const float *__restrict__ lut, float bias, uint64_t seed,
                                                     uint64_t step, const float *__restrict__ inj, int part) {
  __shared__ float sobs[kBlock * USV_NOBS];
  __shared__ uint8_t keep[kBlock];
  const int n = b.n;
  const int e = blockIdx.x * kBlock + threadIdx.x;
  // part 0: every env; 1: envs not reset this step (they do not read this step's new
  // fields, so this part can run concurrently with the potential-field kernels);
  // 2: the envs reset this step, after their fields are built
  bool mine = e < n;
  if (mine && part != 0) {
    const bool jr = b.just_reset[e] != 0;
    mine = (part == 1) ? !jr : jr;
  }
  keep[threadIdx.x] = mine ? 1 : 0;
  const int32_t *ctl = b.ctl;
  const bool pot_none = ctl[USV_CTL_POT_VALID] == 0 || ctl[USV_CTL_RESET_COUNT] > 0;
  const bool pen_valid = ctl[USV_CTL_PEN_VALID] != 0;
  const bool rew_valid = ctl[USV_CTL_REW_VALID] != 0;
  // obs row staged straight into LDS (odd row stride: conflict-free), clamped on write
  // (_process_data clamp, vec_env_rlgames.py:85-95)
  step = step_of(b, step);
  bias = bias_of(c, b, bias);
  float *obs = sobs + threadIdx.x * USV_NOBS;
  const float clip = c.clip_obs;
  auto put = [&](int q, float v) { obs[q] = clampt(v, -clip, clip); };
#pragma unroll
  for (int q = 0; q < USV_NOBS; ++q) obs[q] = 0.f;
  if (mine) {
    // ---- every per-env input that does not depend on this step's results is loaded
    // here, up front, so the HBM latencies overlap each other and the physics (only
    // the 4 field texels and the 2 LUT entries are data-dependent gathers) ----
    const bool was_reset = b.just_reset[e] != 0;
    const float2 a2 = reinterpret_cast<const float2 *>(actions)[e];
    float px = b.px[e], py = b.py[e], yaw = b.yaw[e];
    float vx = b.vx[e], vy = b.vy[e], wz = b.wz[e];
    float fl = b.fl[e], fr = b.fr[e];
    const float m = b.mass[e];
    const float k_iz = b.k_iz[e], k_drag = b.k_drag[e], thr_l = b.thr_l[e], thr_r = b.thr_r[e];
    const float comx = b.com_x[e], comy = b.com_y[e], comz = b.com_z[e];
    float lin0 = c.lin_damp[0], lin1 = c.lin_damp[1], lin2 = c.lin_damp[2];
    float qd0 = c.quad_damp[0], qd1 = c.quad_damp[1], qd2 = c.quad_damp[2];
    if (b.lin_damp) {
      lin0 = b.lin_damp[e]; lin1 = b.lin_damp[n + e]; lin2 = b.lin_damp[2 * n + e];
      qd0 = b.quad_damp[e]; qd1 = b.quad_damp[n + e]; qd2 = b.quad_damp[2 * n + e];
    }
    const int progress0 = b.progress[e];
    const float tgx = b.tgt_x[e], tgy = b.tgt_y[e];
    float obx[USV_NOBST], oby[USV_NOBST];
#pragma unroll
    for (int o = 0; o < USV_NOBST; ++o) {
      obx[o] = b.obst[(size_t)(2 * o) * n + e];
      oby[o] = b.obst[(size_t)(2 * o + 1) * n + e];
    }
    const int goal_cnt0 = b.goal_cnt[e];
    const float prev_d_mem = b.prev_dist[e], prev_head_mem = b.prev_head[e];
    const float prev_pot_mem = b.prev_pot[e], prev_wz_mem = b.prev_wz[e];
    float sums[USV_NSTAT];
    if (kStats) {
#pragma unroll
      for (int q = 0; q < USV_NSTAT; ++q) sums[q] = b.stats[(size_t)q * n + e];
    }
    // ---- uniforms of this step (SU_* layout) ----
    float u[USV_NU_STEP];
    if (inj) {
#pragma unroll
      for (int i = 0; i < USV_NU_STEP; ++i) u[i] = inj[(size_t)e * USV_NU_STEP + i];
    } else {
      philox_u4(seed, (uint32_t)e, step, 0u, u);
      philox_u4(seed, (uint32_t)e, step, 1u, u + 4);
    }
    // ---- VecEnvRLGames.step clamp (:136-140) + pre_physics_step (:1050-1099) ----
    const float cmd0 = clampt(a2.x, -c.clip_actions, c.clip_actions);
    const float cmd1 = clampt(a2.y, -c.clip_actions, c.clip_actions);
    const float prev_cmd0 = was_reset ? 0.f : cmd0;
    const float prev_cmd1 = was_reset ? 0.f : cmd1;
    float t0 = cmd0, t1 = cmd1;
    if (bias != 0.f) { t0 = t0 + bias; t1 = t1 + bias; }
    if (c.act_noise_on) {
      const float rng = (float)((double)c.act_noise_max - (double)c.act_noise_min);
      t0 = t0 + (u[SU_ACT] * rng + c.act_noise_min);
      t1 = t1 + (u[SU_ACT + 1] * rng + c.act_noise_min);
    }
    t0 = clampt(t0, -1.f, 1.f);
    t1 = clampt(t1, -1.f, 1.f);
    float unit0 = c.affine_thrust ? 0.5f * (t0 + 1.0f) : clampt(t0, 0.f, 1.f);
    float unit1 = c.affine_thrust ? 0.5f * (t1 + 1.0f) : clampt(t1, 0.f, 1.f);
    unit0 = clampt(unit0, 0.f, 1.f);
    unit1 = clampt(unit1, 0.f, 1.f);
    const float uu0 = was_reset ? 0.f : unit0, uu1 = was_reset ? 0.f : unit1;
    // ---- DynamicsFirstOrder.get_cmd_interpolated (ThrusterDynamics.py:179-219) ----
    int i0 = (int)rintf(((uu0 + 1.0f) / 2.0f) * (float)(USV_LUT_N - 1));
    int i1 = (int)rintf(((uu1 + 1.0f) / 2.0f) * (float)(USV_LUT_N - 1));
    i0 = min(max(i0, 0), USV_LUT_N - 1);
    i1 = min(max(i1, 0), USV_LUT_N - 1);
    float tgt0 = lut[i0], tgt1 = lut[USV_LUT_N + i1];
    if (c.use_thr_mult) { tgt0 = tgt0 * thr_l; tgt1 = tgt1 * thr_r; }
    // ---- 10 substeps: thruster lag, planar forces, semi-implicit Euler ----
    const float izz = c.izz0 * k_iz;
    const float kd = c.use_drag_scale ? k_drag : 1.0f;
    const float al = c.thr_alpha, oma = 1.0f - c.thr_alpha;
    const float dt = c.dt;
    for (int s = 0; s < c.substeps; ++s) {
      fl = fl * al + oma * tgt0;                      // ThrusterDynamics.py:133-136
      fr = fr * al + oma * tgt1;
      float sy_, cy_;
      sincosf(yaw, &sy_, &cy_);
      const float ub = cy_ * vx + sy_ * vy;           // R^T v (Utils.py:8-12)
      const float vb = -sy_ * vx + cy_ * vy;
      const float rb = wz;
      float D0 = lin0 + qd0 * fabsf(ub), D1 = lin1 + qd1 * fabsf(vb), D2 = lin2 + qd2 * fabsf(rb);
      D0 = D0 * c.scaling_damping; D1 = D1 * c.scaling_damping; D2 = D2 * c.scaling_damping;
      if (c.use_drag_scale) { D0 = D0 * kd; D1 = D1 * kd; D2 = D2 * kd; }
      const float X = fl + fr + (-D0 * ub);           // Hydrodynamics.py:243
      const float Y = -D1 * vb;
      const float N = -(c.thr_y - comy) * fl + (c.thr_y + comy) * fr + (-D2 * rb);
      const float ax = (cy_ * X - sy_ * Y) / m;
      const float ay = (sy_ * X + cy_ * Y) / m;
      const float aw = N / izz;
      vx = vx + ax * dt;
      vy = vy + ay * dt;
      wz = wz + aw * dt;
      px = px + vx * dt;
      py = py + vy * dt;
      float yw = yaw + wz * dt;
      if (yw > USV_PI_F) yw -= USV_2PI_F;
      else if (yw <= -USV_PI_F) yw += USV_2PI_F;
      yaw = yw;
    }
    b.px[e] = px; b.py[e] = py; b.yaw[e] = yaw;
    b.vx[e] = vx; b.vy[e] = vy; b.wz[e] = wz;
    b.fl[e] = fl; b.fr[e] = fr;
    // ---- post_physics_step: progress, update_state noise (USV_Virtual.py:771-813) ----
    const int progress = progress0 + 1;
    b.progress[e] = progress;
    float pxn = px, pyn = py;
    if (c.pos_noise_on) {
      const float rng = (float)((double)c.pos_noise_max - (double)c.pos_noise_min);
      pxn = pxn + (u[SU_PX] * rng + c.pos_noise_min);
      pyn = pyn + (u[SU_PX + 1] * rng + c.pos_noise_min);
    }
    float vxn = vx, vyn = vy, wzn = wz;
    if (c.vel_noise_on) {
      const float rng = (float)((double)c.vel_noise_max - (double)c.vel_noise_min);
      vxn = vxn + (u[SU_VX] * rng + c.vel_noise_min);
      vyn = vyn + (u[SU_VY] * rng + c.vel_noise_min);
      wzn = wzn + (u[SU_WZ] * rng + c.vel_noise_min);
    }
    float yawn = yaw;
    if (c.head_noise_on) {
      const float rng = (float)((double)c.head_noise_max - (double)c.head_noise_min);
      yawn = yawn + (u[SU_HEAD] * rng + c.head_noise_min);
    }
    const float hc = cosf(yawn), hs = sinf(yawn);
    // ---- get_state_observations (static_obs.py:193-299) ----
    const float ex = tgx - pxn, ey = tgy - pyn;
    const float theta = atan2f(hs, hc);
    const float beta = atan2f(ey, ex);
    const float alpha = fmodf((beta - theta) + USV_PI_F, USV_2PI_F) - USV_PI_F;
    const float herr = fabsf(alpha);
    const float dist = sqrtf(ex * ex + ey * ey);
    const float dist_n = tnorm2(ex, ey);
    const float ct = cosf(theta), st = sinf(theta);
    // 16 obstacle distances, running top-5 (torch.topk largest=False, ascending)
    float bd[USV_NCLOSE], bx[USV_NCLOSE], by[USV_NCLOSE];
#pragma unroll
    for (int q = 0; q < USV_NCLOSE; ++q) { bd[q] = INFINITY; bx[q] = 0.f; by[q] = 0.f; }
    float min_od = INFINITY, coll = 0.f;
#pragma unroll
    for (int o = 0; o < USV_NOBST; ++o) {
      const float rx = obx[o] - pxn;
      const float ry = oby[o] - pyn;
      const float d = tnorm2(rx, ry);
      min_od = fminf(min_od, d);
      coll += (float)(d < c.collision_threshold) * (-10.0f) * 10.0f;
      // insertion (strict <: ties keep the lower obstacle index first)
      float cd = d, cx = rx, cy = ry;
#pragma unroll
      for (int q = 0; q < USV_NCLOSE; ++q) {
        if (cd < bd[q]) {
          const float td = bd[q], tx = bx[q], ty = by[q];
          bd[q] = cd; bx[q] = cx; by[q] = cy;
          cd = td; cx = tx; cy = ty;
        }
      }
    }
    if (c.obs_local) {
      put(0, hc * vxn + hs * vyn);
      put(1, -hs * vxn + hc * vyn);
    } else {
      put(0, vxn);
      put(1, vyn);
    }
    put(2, wzn);
    put(3, cosf(alpha));
    put(4, sinf(alpha));
    put(5, dist_n);
#pragma unroll
    for (int q = 0; q < USV_NCLOSE; ++q) {
      const float vbx = bx[q] * ct + by[q] * st;
      const float vby = -bx[q] * st + by[q] * ct;
      const float nf = sqrtf(vbx * vbx + vby * vby + 1e-6f);
      put(8 + 3 * q, bd[q] - c.obstacle_radius);
      put(9 + 3 * q, -vbx / nf);
      put(10 + 3 * q, -vby / nf);
    }
    const int pa = USV_NOBS - c.priv_dim - 2;
    put(pa, prev_cmd0);
    put(pa + 1, prev_cmd1);
    b.prev_cmd[e] = prev_cmd0;
    b.prev_cmd[n + e] = prev_cmd1;
    // ---- privileged tail (USV_Virtual.py:840-976) ----
    {
      float mass_o, co0, co1, co2;
      if (c.masscom_base) {
        mass_o = c.mass_relative ? 0.f : c.base_mass;
        co0 = c.com_scaled ? c.base_com[0] / (c.com_scale[0] + 1e-6f) : c.base_com[0];
        co1 = c.com_scaled ? c.base_com[1] / (c.com_scale[1] + 1e-6f) : c.base_com[1];
        co2 = c.com_scaled ? c.base_com[2] / (c.com_scale[2] + 1e-6f) : c.base_com[2];
      } else {
        const float den = (float)(fabs((double)c.base_mass) > 1e-6 ? fabs((double)c.base_mass) : 1e-6);
        mass_o = c.mass_relative ? (m - c.base_mass) / den : m;
        const float cx = comx, cz = comz;
        co0 = c.com_scaled ? cx / (c.com_scale[0] + 1e-6f) : cx;
        co1 = c.com_scaled ? comy / (c.com_scale[1] + 1e-6f) : comy;
        co2 = c.com_scaled ? cz / (c.com_scale[2] + 1e-6f) : cz;
      }
      const int pt = USV_NOBS - c.priv_dim;
      put(pt, mass_o); put(pt + 1, co0); put(pt + 2, co1); put(pt + 3, co2);
      if (c.priv_dim == 8) {
        float kdv, tl, tr, kz;
        if (c.masscom_base) {
          if (c.priv_mode == 2) {
            kdv = 0.5f * (c.kdrag_min + c.kdrag_max);
            tl = tr = c.couple_thr ? (1.0f - 0.5f * c.thr_rand) : 1.0f;
            kz = 0.5f * (c.kiz_min + c.kiz_max);
          } else { kdv = tl = tr = kz = 1.0f; }
        } else {
          kdv = k_drag; tl = thr_l; tr = thr_r; kz = k_iz;
        }
        if (c.priv_mode == 1) {
          kdv = enc_centered(kdv, c.kdrag_min, c.kdrag_max, c.priv_nominal);
          tl = enc_centered(tl, c.thr_min, c.thr_max, c.priv_nominal);
          tr = enc_centered(tr, c.thr_min, c.thr_max, c.priv_nominal);
          kz = enc_centered(kz, c.kiz_min, c.kiz_max, c.priv_nominal);
        } else if (c.priv_mode == 2) {
          kdv = c.priv_drag_on ? enc_minmax(kdv, c.kdrag_min, c.kdrag_max) : 0.f;
          tl = c.priv_thr_on ? enc_minmax(tl, c.thr_min, c.thr_max) : 0.f;
          tr = c.priv_thr_on ? enc_minmax(tr, c.thr_min, c.thr_max) : 0.f;
          kz = c.priv_kiz_on ? enc_minmax(kz, c.kiz_min, c.kiz_max) : 0.f;
        }
        put(pt + 4, kdv); put(pt + 5, tl); put(pt + 6, tr); put(pt + 7, kz);
      }
    }
    // ---- compute_reward (static_obs.py:335-657) ----
    const float bover = maxf(dist - c.kill_dist, 0.f);
    const float bpen = -expm1f(minf(bover / 0.25f, 20.0f)) * c.boundary_cost;
    const int gir = dist < c.position_tolerance;
    const int goal_cnt = goal_cnt0 * gir + gir;
    b.goal_cnt[e] = goal_cnt;
    const float prev_err = rew_valid ? prev_d_mem : dist;
    float dist_r;
    if (c.reward_mode == 0) dist_r = c.position_scale * (prev_err - dist);
    else if (c.reward_mode == 1) dist_r = c.position_scale * (prev_err * prev_err - dist * dist);
    else dist_r = c.position_scale * (expf(-dist / c.exp_coeff) - expf(-prev_err / c.exp_coeff));
    const float h2 = herr * herr;
    float align_r = c.align_la1 * (expf(c.align_la2 * (h2 * h2)) + expf(c.align_la3 * h2));
    if (was_reset) dist_r = 0.f;
    const float prev_dist = was_reset ? dist : (rew_valid ? prev_d_mem : dist);
    const float pot = sample_field(b.field + (size_t)e * USV_GRID2, c.map_size, pxn, pyn);
    const float pn = clampt(pot, 0.f, 1.f);
    const float xs = clampt((pn - 0.6f) / (0.3f + 1e-6f), 0.f, 1.f);
    const float danger = xs * xs * (3.0f - 2.0f * xs);
    align_r = align_r * maxf(0.3f, 1.0f - danger);
    dist_r = dist_r * maxf(0.6f, 1.0f - danger * 0.5f);
    const float g = clampt(cosf(herr), 0.f, 1.f);
    dist_r = minf(dist_r, 0.f) + g * maxf(dist_r, 0.f);
    const float prev_h = (rew_valid && !was_reset) ? prev_head_mem : herr;
    const float hi = clampt(prev_h - herr, -0.4f, 0.4f);
    const float hi_r = hi * 0.05f;
    b.prev_head[e] = herr;
    const float prev_pot = (pot_none || was_reset) ? pot : prev_pot_mem;
    float praw = (prev_pot - pot) * 100.0f;
    if (fabsf(praw) < 0.01f) praw = 0.f;
    const float pa1 = 2.0f * tanhf(praw / (2.0f + 1e-6f));
    const float gdx = ex / (dist + 1e-6f), gdy = ey / (dist + 1e-6f);
    const float vtp = maxf(vxn * gdx + vyn * gdy, 0.f);
    const float ddp = maxf(prev_dist - dist, 0.f);
    const float gv = clampt((vtp - 0.02f) / ((0.15f - 0.02f) + 1e-6f), 0.f, 1.f);
    const float gd = clampt(ddp / (0.01f + 1e-6f), 0.f, 1.f);
    const float ggate = maxf(gv, gd) * g;
    const float ppos = maxf(pa1, 0.f), pneg = minf(pa1, 0.f);
    const float gate_pos = (ppos < 0.5f) ? 1.0f : ggate;
    const float shaping = gate_pos * ppos + pneg;
    const bool worsening = shaping < -0.05f;
    const bool turning = fabsf(wzn) > 0.2f;
    const float vfwd = vxn * hc + vyn * hs;
    const float sf = clampt((fabsf(vfwd) - 0.15f) / ((0.60f - 0.15f) + 1e-6f), 0.f, 1.f);
    const float turn_haz = (float)(worsening && turning) * (-10.0f) * (g * g) * sf;
    b.prev_pot[e] = pot;
    const float speed_r = (1.0f - expf(-vtp / (0.8f + 1e-6f))) * 0.05f;
    const float sgn = (alpha > 0.f) ? 1.f : ((alpha < 0.f) ? -1.f : 0.f);
    const float tang = (herr > 1.0f) ? sgn * 1.0f : sgn * 0.2f;
    const float dw = wzn - tang;
    const float ang_r = expf(-(dw * dw) / 0.2f) * 0.03f;
    const float goal_r = ((float)goal_cnt * c.goal_reward) * 5.0f;
    b.prev_dist[e] = dist;
    const float total = dist_r * 0.5f + align_r * 0.5f + shaping * 2.0f + turn_haz + goal_r + c.time_reward +
                        coll + speed_r + ang_r + hi_r;
    // ---- Penalties.compute_penalty (USV_task_rewards.py:440-523) ----
    const float pact0 = c.pen_use_u ? unit0 : cmd0, pact1 = c.pen_use_u ? unit1 : cmd1;
    float p_lin = 0.f, p_ang = 0.f, p_angv = 0.f, p_en = 0.f;
    if (c.pen_lin_kind == PEN_NORM) p_lin = -tnorm2(vxn, vyn) * c.pen_lin_k + c.pen_lin_c;
    if (c.pen_ang_kind) p_ang = pen_scalar(c.pen_ang_kind, c.pen_ang_k, c.pen_ang_x0, c.pen_ang_c, wzn);
    if (c.pen_angv_kind) {
      const float prev_w = pen_valid ? prev_wz_mem : wzn;
      p_angv = pen_scalar(c.pen_angv_kind, c.pen_angv_k, c.pen_angv_x0, c.pen_angv_c, wzn - prev_w);
    }
    if (c.pen_en_kind == PEN_SUM) p_en = -(pact0 + pact1) * c.pen_en_k + c.pen_en_c;
    else if (c.pen_en_kind == PEN_SUMSQ) p_en = -(pact0 * pact0 + pact1 * pact1) * c.pen_en_k + c.pen_en_c;
    b.prev_wz[e] = wzn;
    b.rew[e] = total + (((p_lin + p_ang) + p_angv) + p_en);
    // ---- update_kills / is_done (static_obs.py:661-706, USV_Virtual.py:1223-1237) ----
    const bool dkill = dist > c.kill_dist;
    const bool ckill = min_od < c.collision_threshold;
    const bool skill = goal_cnt >= c.kill_after_n;
    const bool die = dkill || ckill || skill;
    if (die) {
      b.done_coll[e] = ckill;
      b.done_succ[e] = skill && !ckill;
    }
    const int tout = progress >= c.max_episode_length - 1;
    const int rb = c.fixed_horizon_eval ? tout : (tout ? 1 : (int)die);
    b.reset_buf[e] = rb;
    b.dones[e] = (int64_t)rb;
    b.just_reset[e] = 0;
    if (kStats) {
      float *S = b.stats;
#define ADDS(k, v) sums[k] += (v)
      ADDS(ST_TOTAL_REWARD, total); ADDS(ST_DISTANCE_REWARD, dist_r); ADDS(ST_ALIGNMENT_REWARD, align_r);
      ADDS(ST_HEADING_IMPROVE_REWARD, hi_r); ADDS(ST_POTENTIAL_SHAPING_REWARD, shaping);
      ADDS(ST_SPEED_REWARD, speed_r); ADDS(ST_ANGULAR_REWARD, ang_r); ADDS(ST_TURN_HAZARD_PENALTY, turn_haz);
      ADDS(ST_GOAL_REWARD, goal_r); ADDS(ST_TIME_REWARD, c.time_reward); ADDS(ST_COLLISION_REWARD, coll);
      ADDS(ST_DANGER_MEAN, danger); ADDS(ST_DANGER_HI_RATE, (float)(danger > 0.5f));
      ADDS(ST_G_GATE_MEAN, gate_pos); ADDS(ST_POSITION_ERROR, dist); ADDS(ST_BOUNDARY_PENALTY, bpen);
      if (c.pen_ang_kind) ADDS(ST_ANGULAR_VEL_PENALTY, p_ang);
      if (c.pen_angv_kind) ADDS(ST_ANGULAR_VEL_VARIATION_PENALTY, p_angv);
      if (c.pen_en_kind) ADDS(ST_ENERGY_PENALTY, p_en);
      ADDS(ST_NORMED_LINEAR_VEL, tnorm2(vxn, vyn));
      ADDS(ST_NORMED_ANGULAR_VEL, fabsf(wzn));
      ADDS(ST_CMD_NEG_RATE, ((float)(t0 < 0.f) + (float)(t1 < 0.f)) / 2.0f);
      ADDS(ST_U_MEAN, (unit0 + unit1) / 2.0f);
      ADDS(ST_U_LOW_RATE, ((float)(unit0 < 0.05f) + (float)(unit1 < 0.05f)) / 2.0f);
      ADDS(ST_U_SUM, unit0 + unit1);
#undef ADDS
#pragma unroll
      for (int q = 0; q < USV_NSTAT; ++q) S[(size_t)q * n + e] = sums[q];
    }
  }
  // ---- coalesced obs store: rows of 33 floats staged through LDS ----
  __syncthreads();
  const int row0 = blockIdx.x * kBlock;
  const int rows = min(kBlock, n - row0);
  float *dst = b.obs + (size_t)row0 * USV_NOBS;
  for (int i = threadIdx.x; i < rows * USV_NOBS; i += kBlock)
    if (keep[i / USV_NOBS]) dst[i] = sobs[i];
  // ---- global flags: the step has consumed the Nones (:361, :448, USV_task_rewards.py:450) ----
  if (part != 1 && blockIdx.x == 0 && threadIdx.x == 0) {
    b.ctl[USV_CTL_POT_VALID] = 1;
    b.ctl[USV_CTL_PEN_VALID] = 1;
    b.ctl[USV_CTL_REW_VALID] = 1;
  }
}

// planar forces only (parity with Hydrodynamics.ComputeHydrodynamicsEffects)
__global__ void k_forces(usv_cfg_t c, usv_bufs_t b, float *__restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = b.n;
  if (e >= n) return;
  float sy_, cy_;
  sincosf(b.yaw[e], &sy_, &cy_);
  const float vx = b.vx[e], vy = b.vy[e], wz = b.wz[e];
  const float ub = cy_ * vx + sy_ * vy, vb = -sy_ * vx + cy_ * vy;
  float lin0 = c.lin_damp[0], lin1 = c.lin_damp[1], lin2 = c.lin_damp[2];
  float qd0 = c.quad_damp[0], qd1 = c.quad_damp[1], qd2 = c.quad_damp[2];
  if (b.lin_damp) {
    lin0 = b.lin_damp[e]; lin1 = b.lin_damp[n + e]; lin2 = b.lin_damp[2 * n + e];
    qd0 = b.quad_damp[e]; qd1 = b.quad_damp[n + e]; qd2 = b.quad_damp[2 * n + e];
  }
  float D0 = (lin0 + qd0 * fabsf(ub)) * c.scaling_damping;
  float D1 = (lin1 + qd1 * fabsf(vb)) * c.scaling_damping;
  float D2 = (lin2 + qd2 * fabsf(wz)) * c.scaling_damping;
  if (c.use_drag_scale) { const float k = b.k_drag[e]; D0 *= k; D1 *= k; D2 *= k; }
  const float fl = b.fl[e], fr = b.fr[e], comy = b.com_y[e];
  out[3 * e] = fl + fr + (-D0 * ub);
  out[3 * e + 1] = -D1 * vb;
  out[3 * e + 2] = -(c.thr_y - comy) * fl + (c.thr_y + comy) * fr + (-D2 * wz);
}

}  // namespace

extern "C" {

int usv_build_lut(const float *table_l21, const float *table_r21, int n_table, float *lut_dev, void *stream) {
  if (!table_l21 || !table_r21 || !lut_dev || n_table < 2) return 1;
  hipLaunchKernelGGL(k_build_lut, dim3((USV_LUT_N + 255) / 256), dim3(256), 0, (hipStream_t)stream, table_l21,
                     table_r21, n_table, lut_dev);
  USV_CHECK_LAUNCH();
  return 0;
}

int usv_reset(const usv_cfg_t *cfg, const usv_bufs_t *b, uint64_t seed, uint64_t step, const float *u_inject,
              void *stream) {
  if (!cfg || !b || b->n <= 0) return 1;
  hipStream_t s = (hipStream_t)stream;
  // per-step scratch: reset count, field maxima, extras sums
  hipLaunchKernelGGL(k_step_begin, dim3(1), dim3(64), 0, s, *b);
  USV_CHECK_LAUNCH();
  const int grid = (b->n + kBlock - 1) / kBlock;
  hipLaunchKernelGGL(k_reset, dim3(grid), dim3(kBlock), 0, s, *cfg, *b, seed, step, u_inject);
  USV_CHECK_LAUNCH();
  return 0;
}

int usv_env_step_part(const usv_cfg_t *cfg, const usv_bufs_t *b, const float *actions, const float *lut_dev,
                      float action_bias, uint64_t seed, uint64_t step, const float *u_inject, int part,
                      void *stream) {
  if (!cfg || !b || !actions || !lut_dev || b->n <= 0 || part < 0 || part > 2) return 1;
  if (cfg->priv_dim != 4 && cfg->priv_dim != 8) return 3;
  const int grid = (b->n + kBlock - 1) / kBlock;
  hipStream_t s = (hipStream_t)stream;
  if (cfg->stats_on)
    hipLaunchKernelGGL(k_env_step<true>, dim3(grid), dim3(kBlock), 0, s, *cfg, *b, actions, lut_dev, action_bias,
                       seed, step, u_inject, part);
  else
    hipLaunchKernelGGL(k_env_step<false>, dim3(grid), dim3(kBlock), 0, s, *cfg, *b, actions, lut_dev, action_bias,
                       seed, step, u_inject, part);
  USV_CHECK_LAUNCH();
  return 0;
}

int usv_env_step(const usv_cfg_t *cfg, const usv_bufs_t *b, const float *actions, const float *lut_dev,
                 float action_bias, uint64_t seed, uint64_t step, const float *u_inject, void *stream) {
  return usv_env_step_part(cfg, b, actions, lut_dev, action_bias, seed, step, u_inject, 0, stream);
}

int usv_forces(const usv_cfg_t *cfg, const usv_bufs_t *b, float *out, void *stream) {
  if (!cfg || !b || !out || b->n <= 0) return 1;
  hipLaunchKernelGGL(k_forces, dim3((b->n + 255) / 256), dim3(256), 0, (hipStream_t)stream, *cfg, *b, out);
  USV_CHECK_LAUNCH();
  return 0;
}

int usv_hip_version(void) { return 1; }

}  // extern "C"
