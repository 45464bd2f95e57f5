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
#include "usv_layout_gen.h"

#include <algorithm>
#include <cmath>
#include <cstddef>

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
// USVVirtual.step at this step's reset (which = 4) or after its calculate_metrics (which = 5); without the device
// clock, from the step index (exact for power-of-two horizons)
__device__ __forceinline__ double ref_step_of(const usv_cfg_t &c, const usv_bufs_t &b, uint64_t step, int which) {
  if (b.clock) return __longlong_as_double((long long)b.clock[which]);
  return (double)(step + (which == 5 ? 1 : 0)) * c.step_inc;
}
// GoToPoseTask's spawn curriculum (USV_go_to_pose.py:266-290 radii, :188-202 kill distance): linear in the
// reference step between warmup and end, in the reference's double arithmetic
__device__ __forceinline__ double curriculum_lerp(const usv_cfg_t &c, double st, double cur, double fin) {
  if (st < c.cur_warmup) return cur;
  if (st > c.cur_end) return fin;
  const double r = (st - c.cur_warmup) / (c.cur_end - c.cur_warmup);
  return r * (fin - cur) + cur;
}
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
// USV_RESET_FOLD_KERNEL: the episode-extras fold of the reset path in a one-workgroup launch of its own
// (k_extras_fold) instead of by the last k_reset workgroup behind a device-scope counter and fences
#ifndef USV_RESET_FOLD_KERNEL
#define USV_RESET_FOLD_KERNEL 1
#endif

__global__ void k_step_begin(usv_bufs_t b, double step_inc) {
  const int t = threadIdx.x;
  if (t == 0 && b.clock) {   // device step clock: this step's index and bias-call count
    b.clock[2] = b.clock[0]++;
    b.clock[3] = b.clock[1]++;
    // USVVirtual.step (a double, += 1 / horizon_length per calculate_metrics, USV_Virtual.py:1633): its value
    // at this step's reset_idx and after this step's calculate_metrics, accumulated as the reference does
    const uint64_t after = b.clock[5];
    b.clock[4] = after;
    b.clock[5] = (uint64_t)__double_as_longlong(__longlong_as_double((long long)after) + step_inc);
  }
  if (t == 0) b.ctl[USV_CTL_RESET_COUNT] = 0;
  if (t == 3 && b.ctl[USV_CTL_STEPPED]) {   // a step has run: prev_* are no longer None
    b.ctl[USV_CTL_POT_VALID] = 1;
    b.ctl[USV_CTL_PEN_VALID] = 1;
    b.ctl[USV_CTL_REW_VALID] = 1;
  }
  if (t == 1) b.ctl[USV_CTL_ANY_INSIDE] = 0;
  if (t == 2) b.ctl[USV_CTL_ANY_FINITE] = 0;
  if (t < 4) b.fscratch[t] = 0.f;
  // completion counters of this step's kernels: their last workgroup also returns them to 0,
  // but a step never depends on that (a counter left non-zero by an aborted launch would
  // otherwise make every later "last workgroup" test fail silently)
  if (t == 4) b.ctl[USV_CTL_OBST_DONE] = 0;
  if (t == 5) b.ctl[USV_CTL_BATCH_DONE] = 0;
}

// ------------------------------------------------------------------------
// Reset path (USVVirtual.reset_idx, USV_Virtual.py:1502-1618).  One thread per
// env; threads of envs with reset_buf==1 do the work.  The reset list is
// compacted with a wave ballot + one atomic per wave (order is irrelevant:
// draws are keyed by env id, the potential-field batch statistics are maxima).
// Obstacle rejection sampling follows in the same kernel, one whole wave per
// reset env (place_obstacles).
// ------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_reset(usv_cfg_t c, usv_bufs_t b, uint64_t seed, uint64_t step,
                                                  const float *__restrict__ inj) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = b.n;
  const bool active = (e < n) && (b.reset_buf[e] != 0);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  // episode-extras sums of this workgroup's resetting envs, per wave (fixed order)
  __shared__ float wsum[kBlock / 64][USV_NSTAT];
  step = step_of(b, step);
  // ---- compaction: reset_buf.nonzero() (USV_Virtual.py:1045): wave ballots, a workgroup
  // prefix in LDS and one atomic per workgroup (slots are workgroup-contiguous) ----
  const uint64_t mask = __ballot(active);
  __shared__ int wbase[kBlock / 64];
  if (lane == 0) wbase[wid] = __popcll(mask);
  if (c.stats_on && mask == 0 && lane < USV_NSTAT) wsum[wid][lane] = 0.f;
  __syncthreads();
  if (threadIdx.x == 0) {
    int tot = 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) { const int k = wbase[w]; wbase[w] = tot; tot += k; }
    const int base0 = tot ? atomicAdd(&b.ctl[USV_CTL_RESET_COUNT], tot) : 0;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) wbase[w] += base0;
  }
  __syncthreads();
  if (mask != 0) {
    const int leader = __ffsll((long long)mask) - 1;
    const int base = wbase[wid];
    // ---- episode extras: sums of the envs being reset (:1591-1612): wave sums here, the
    // workgroup's partial at the end, folded in workgroup order by the last workgroup ----
    if (c.stats_on) {
      // all 28 loads first, then 28 independent wave sums (their shuffles interleave)
      const int ec = min(e, n - 1);
      float v[USV_NSTAT];
#pragma unroll
      for (int q = 0; q < USV_NSTAT; ++q) v[q] = b.stats[(size_t)q * n + ec];
      v[ST_SUCCESS] = (float)b.done_succ[ec];
      v[ST_COLLISION] = (float)b.done_coll[ec];
      if (active) {
#pragma unroll
        for (int q = 0; q < USV_NSTAT; ++q) b.stats[(size_t)q * n + e] = 0.f;
      }
#pragma unroll
      for (int q = 0; q < USV_NSTAT; ++q) v[q] = wave_sum(active ? v[q] : 0.f);
      if (lane == leader) {
#pragma unroll
        for (int q = 0; q < USV_NSTAT; ++q) wsum[wid][q] = v[q];
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
        float sth, cth;
        usv_sincos_cr(th, &sth, &cth);
        cx = c.base_com[0] + cth * r;
        cy = c.base_com[1] + sth * r;
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
      // ---- ForceDisturbance.generate_force / TorqueDisturbance.generate_torque
      // (USV_disturbances.py:327-508, called from reset_idx:1517-1518) ----
      if (b.dist) {
        float *D = b.dist;
        const size_t nn = (size_t)n;
        if (c.fdist_on && c.fsin_on) {
          const float fr_ = (float)((double)c.ffreq_max - (double)c.ffreq_min);
          const float sr_ = (float)((double)c.fshift_max - (double)c.fshift_min);
          D[DI_FXF * nn + e] = U(RU_FSIN) * fr_ + c.ffreq_min;
          D[DI_FYF * nn + e] = U(RU_FSIN + 1) * fr_ + c.ffreq_min;
          D[DI_FXS * nn + e] = U(RU_FSIN + 2) * sr_ + c.fshift_min;
          D[DI_FYS * nn + e] = U(RU_FSIN + 3) * sr_ + c.fshift_min;
          D[DI_FAMP * nn + e] = U(RU_FSIN + 4) * (float)((double)c.fsin_max - (double)c.fsin_min) + c.fsin_min;
        }
        if (c.fdist_on && c.fconst_on) {
          const float r = U(RU_FCONST) * (float)((double)c.fconst_max - (double)c.fconst_min) + c.fconst_min;
          const float th = U(RU_FCONST + 1) * USV_PI_F * 2.0f;
          float sth, cth;
          usv_sincos_cr(th, &sth, &cth);
          if (c.inj_trig && inj) { cth = U(RU_TRIG + 4); sth = U(RU_TRIG + 5); }
          D[DI_FCX * nn + e] = cth * r;
          D[DI_FCY * nn + e] = sth * r;
        }
        if (c.tdist_on && c.tsin_on) {
          D[DI_TF * nn + e] = U(RU_TSIN) * (float)((double)c.tfreq_max - (double)c.tfreq_min) + c.tfreq_min;
          D[DI_TS * nn + e] = U(RU_TSIN + 1) * (float)((double)c.tshift_max - (double)c.tshift_min) + c.tshift_min;
          D[DI_TAMP * nn + e] = U(RU_TSIN + 2) * (float)((double)c.tsin_max - (double)c.tsin_min) + c.tsin_min;
        }
        if (c.tdist_on && c.tconst_on) {
          float r = U(RU_TCONST) * (float)((double)c.tconst_max - (double)c.tconst_min) + c.tconst_min;
          if (U(RU_TCONST + 1) > 0.5f) r = r * -1.0f;   // half of the envs at random (:505-507)
          D[DI_TC * nn + e] = r;
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
      // ---- task.get_spawns, previous-episode target (get_goals runs later, USV_Virtual.py:1618) ----
      tx = b.tgt_x[e];
      ty = b.tgt_y[e];
      // the spawn heading reaches the stand-in as the quaternion (cos(yaw0 / 2), 0, 0, sin(yaw0 / 2))
      // (static_obs.py:959-961) and set_world_poses turns it into its yaw (usv_yaw_of_quat)
      const bool inj_trig = c.inj_trig && inj;   // parity tests: the reference's recorded torch.cos / sin values
      float qz0, qw0;
      usv_sincos_cr(U(RU_YAW) * USV_PI_F * 0.5f, &qz0, &qw0);
      if (inj_trig) { qw0 = U(RU_TRIG + 2); qz0 = U(RU_TRIG + 3); }
      const float yaw0 = usv_yaw_of_quat(qw0, qz0);
      if (c.task_kind == USV_TASK_CAPTURE_XY) {   // CaptureXYTask.get_spawns (static_obs.py:936-1060)
        const float r = U(RU_SPAWN_R) * (c.spawn_rmax - c.spawn_rmin) + c.spawn_rmin;
        const float th = U(RU_SPAWN_TH) * 2.0f * USV_PI_F;
        float sth, cth;
        usv_sincos_cr(th, &sth, &cth);
        if (inj_trig) { cth = U(RU_TRIG); sth = U(RU_TRIG + 1); }
        sx = r * cth;
        sy = r * sth;
        b.field_old_tgt[e] = tx;
        b.field_old_tgt[n + e] = ty;
      } else if (c.task_kind == USV_TASK_GO_TO_POSE) {   // GoToPoseTask.get_spawns (USV_go_to_pose.py:256-319)
        double rmax = c.spawn_rmax, rmin = c.spawn_rmin;
        if (c.curriculum_on) {   // :266-290, with the step the reference passes (USV_Virtual.py:1546)
          const double st = ref_step_of(c, b, step, 4);
          rmax = curriculum_lerp(c, st, c.cur_max_dist, c.max_spawn_d);
          rmin = curriculum_lerp(c, st, c.cur_min_dist, c.min_spawn_d);
        }
        const float r = U(RU_SPAWN_R) * (float)(rmax - rmin) + (float)rmin;
        const float th = U(RU_SPAWN_TH) * 2.0f * USV_PI_F;
        float sth, cth;
        usv_sincos_cr(th, &sth, &cth);
        if (inj_trig) { cth = U(RU_TRIG); sth = U(RU_TRIG + 1); }
        sx = r * cth + tx;
        sy = r * sth + ty;
        b.prev_dist[e] = 0.f;                            // GoToPoseTask.reset: prev_position_dist = 0 (:227)
      } else {                                           // TrackXYOVelocityTask.get_spawns (:203-219): env origin
        sx = 0.f;
        sy = 0.f;
      }
      // ---- the reference's cached root state still holds this pre-reset pose when the first substep
      // computes its drag and disturbances (USV_Virtual.py:1103-1117): keep those inputs ----
      if (c.stale_root) {
        const float opx = b.px[e], opy = b.py[e], ovx = b.vx[e], ovy = b.vy[e];
        const QuatRot qr = usv_quat_rot(b.yaw[e]);
        const float so = qr.S, co = qr.C;
        float ub = co * ovx + so * ovy;               // R^T v (Utils.py:10-14, Hydrodynamics.py:209-217)
        float vb = -so * ovx + co * ovy;
        if (c.current_on) {                           // relative to the water (Hydrodynamics.py:224-237)
          ub = ub - (co * c.flow_vel[0] + so * c.flow_vel[1]);
          vb = vb - (-so * c.flow_vel[0] + co * c.flow_vel[1]);
        }
        b.stale[USV_STALE_UB * (size_t)n + e] = ub;
        b.stale[USV_STALE_VB * (size_t)n + e] = vb;
        b.stale[USV_STALE_RB * (size_t)n + e] = b.wz[e];
        b.stale[USV_STALE_PX * (size_t)n + e] = opx;
        b.stale[USV_STALE_PY * (size_t)n + e] = opy;
      }
      // ---- pose / velocities / bookkeeping (USV_Virtual.py:1541-1579) ----
      if (b.scene) {
        // scene replay (_scene_replay_take_scene_indices / _scene_replay_apply, USV_Virtual.py:1372-1457,
        // CaptureXYTask.apply_scene static_obs.py:785-863): pose, velocity, goal and obstacles from the
        // env's next scene; the field is built for the NEW goal; no spawn / velocity / goal draws
        int idx = b.scene_next[e];
        b.scene_next[e] = idx + 1;
        const int ns = b.n_scenes;
        if (b.scene_cycle) {
          idx %= ns;
          if (idx < 0) idx += ns;   // torch's floor modulo
        } else if (idx < 0 || idx >= ns) {
          atomicOr(&b.ctl[USV_CTL_SCENE_ERR], 1);   // the reference raises IndexError (:1387-1391)
          idx = min(max(idx, 0), ns - 1);
        }
        b.scene_last[e] = idx;
        const float *sc = b.scene + (size_t)idx * USV_SCENE_STRIDE;
#pragma unroll
        for (int q = 0; q < 2 * USV_NOBST; ++q) b.obst[(size_t)q * n + e] = sc[USV_SC_OBST + q];
        b.px[e] = sc[USV_SC_START];
        b.py[e] = sc[USV_SC_START + 1];
        {   // the yaw-only quaternion of the scene's start yaw (USV_Virtual.py:1447-1450) through set_world_poses
          float hz, hw;
          usv_sincos_cr(0.5f * sc[USV_SC_YAW], &hz, &hw);
          if (inj_trig) { hw = U(RU_TRIG + 2); hz = U(RU_TRIG + 3); }
          b.yaw[e] = usv_yaw_of_quat(hw, hz);
        }
        b.vx[e] = sc[USV_SC_VEL];
        b.vy[e] = sc[USV_SC_VEL + 1];
        b.tgt_x[e] = sc[USV_SC_GOAL];
        b.tgt_y[e] = sc[USV_SC_GOAL + 1];
        b.field_old_tgt[e] = sc[USV_SC_GOAL];
        b.field_old_tgt[n + e] = sc[USV_SC_GOAL + 1];
      } else {
        b.px[e] = sx;
        b.py[e] = sy;
        b.yaw[e] = yaw0;
        b.vx[e] = U(RU_VX) * 3.0f - 1.5f;
        b.vy[e] = U(RU_VY) * 3.0f - 1.5f;
      }
      b.wz[e] = 0.f;
      b.reset_buf[e] = 0;
      b.progress[e] = 0;
      b.prev_cmd[e] = 0.f;
      b.prev_cmd[n + e] = 0.f;
      // ---- set_targets -> task.get_goals (not called under scene replay, :1613-1616) ----
      if (b.scene) {
      } else if (c.task_kind != USV_TASK_TRACK_XYO) {   // static_obs.py:913-930, USV_go_to_pose.py:229-254
        const float g = c.goal_random_position;
        b.tgt_x[e] = U(RU_GOAL) * g * 2.0f - g;
        b.tgt_y[e] = U(RU_GOAL + 1) * g * 2.0f - g;
        if (c.task_kind == USV_TASK_GO_TO_POSE) b.tgt_h[e] = U(RU_GOAL_H) * USV_PI_F * 2.0f;
      } else {                                   // USV_track_xyo_velocity.py:178-199: target velocities
        const float gl = c.tk_goal_rand[0], ga = c.tk_goal_rand[1];
        b.tgt_x[e] = U(RU_GOAL) * gl * 2.0f - gl;
        b.tgt_y[e] = U(RU_GOAL + 1) * gl * 2.0f - gl;
        b.tgt_h[e] = U(RU_GOAL_H) * ga * 2.0f - ga;
      }
    }
    (void)sx; (void)sy; (void)tx; (void)ty;
  }
  // ---- obstacles: placed by the potential-field kernel, one workgroup per reset env
  // (place_obstacles, usv_device.h); this kernel hands over the draw keys ----
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    b.ctl[USV_CTL_H_SEED_LO] = (int32_t)(uint32_t)seed;
    b.ctl[USV_CTL_H_SEED_HI] = (int32_t)(uint32_t)(seed >> 32);
    b.ctl[USV_CTL_H_STEP_LO] = (int32_t)(uint32_t)step;
    b.ctl[USV_CTL_H_STEP_HI] = (int32_t)(uint32_t)(step >> 32);
    b.ctl[USV_CTL_H_INJ_LO] = (int32_t)(uint32_t)(uintptr_t)inj;
    b.ctl[USV_CTL_H_INJ_HI] = (int32_t)(uint32_t)((uint64_t)(uintptr_t)inj >> 32);
    b.ctl[USV_CTL_PLACE] = b.scene ? 0 : 1;   // scene replay: obstacles come from the scene
  }
  // ---- the last workgroup finalises extras["episode"] = means over this step's resets (:1591-1612).
  // Per-workgroup partials (no float atomics: one address per statistic would serialise
  // every wave of the grid on it, and the sum order would vary run to run) ----
  __syncthreads();
  const int qs = threadIdx.x;
  if (c.stats_on && qs < USV_NSTAT) {
    float a = wsum[0][qs];
#pragma unroll
    for (int w = 1; w < kBlock / 64; ++w) a += wsum[w][qs];
    b.extras_acc[(size_t)blockIdx.x * USV_NSTAT + qs] = a;
#if !USV_RESET_FOLD_KERNEL
    __threadfence();
#endif
  }
#if USV_RESET_FOLD_KERNEL
  // the fold runs as k_extras_fold right behind this launch (stream order publishes the partials)
}

__global__ __launch_bounds__(kBlock) void k_extras_fold(usv_cfg_t c, usv_bufs_t b, int nblk) {
  const int qs = threadIdx.x;
  __shared__ float fold[8][32];
  const int count = min(b.ctl[USV_CTL_RESET_COUNT], b.n);
  const int G = nblk;
#else
  __shared__ bool last;
  __shared__ float fold[8][32];
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(&b.ctl[USV_CTL_OBST_DONE], 1) == (int)gridDim.x - 1;
    __threadfence();
  }
  __syncthreads();
  if (!last) return;
  const int count = b.ctl[USV_CTL_RESET_COUNT];
  const int G = (int)gridDim.x;
#endif
  if (c.stats_on && count > 0) {
    // 8 interleaved block subsets per statistic, each summed in block order, then combined in order
    static_assert(USV_NSTAT <= 32 && kBlock == 256, "fold layout");
    const int q = qs & 31, k = qs >> 5;
    float a = 0.f;
    if (q < USV_NSTAT) {
      // blocks k, k+8, k+16, ... in that order; 16 loads in flight per batch
      for (int b0 = k; b0 < G; b0 += 128) {
        float x[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) x[u] = b.extras_acc[(size_t)min(b0 + 8 * u, G - 1) * USV_NSTAT + q];
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (b0 + 8 * u < G) a += x[u];
      }
    }
    fold[k][q] = a;
    __syncthreads();
    if (qs < USV_NSTAT) {
      float tot = fold[0][qs];
#pragma unroll
      for (int kk = 1; kk < 8; ++kk) tot += fold[kk][qs];
      float m = tot / (float)count;
      if (qs != ST_SUCCESS && qs != ST_COLLISION) m = m / (float)c.max_episode_length;
      // USV_NAN_PROBE: the reference raises on a NaN extra before zeroing it (USV_Virtual.py:1601-1605)
      if (c.nan_probe && isnan(m)) atomicOr(&b.ctl[USV_CTL_NAN_FLAG], (int)USV_NAN_EXTRAS);
      b.extras[qs] = isnan(m) ? 0.f : m;
    }
  }
  if (qs == 0) b.ctl[USV_CTL_OBST_DONE] = 0;
}

// ------------------------------------------------------------------------
// grid_sample(field, 2*pos/map, bilinear, border, align_corners=False)
// (static_obs.py:302-326) in the arithmetic of PyTorch's CPU kernel.  Split in
// two: field_taps issues the 4 texel loads as soon as the position is known,
// field_blend combines them where the reward needs the potential.
// ------------------------------------------------------------------------
struct FieldTaps {
  float g_nw, g_ne, g_sw, g_se;    // raw costs of the 4 texels (the env's tiles)
  float4 fn0, fn1;                 // the env's normalisation constants (usv_bufs_t.fnorm)
  float nw, ne, sw, se;
  int i0, i1c, j0, j1c;
  bool i_out, j_out;
};
// F: the env's cost tiles, FN: its USV_FNORM constants
__device__ __forceinline__ FieldTaps field_taps(const float *__restrict__ F, const float *__restrict__ FN,
                                                float map_size, float x, float y) {
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
  FieldTaps t;
  t.nw = ss * ee; t.ne = ss * w; t.sw = nn * ee; t.se = nn * w;
  const int i0 = (int)xw, j0 = (int)yn, i1 = i0 + 1, j1 = j0 + 1;
  // border clamp: i1/j1 == G only when the weight of that tap is 0 (ix, iy <= G-1);
  // the tap then reads the last column/row (any finite value) and is replaced by 0
  const int i1c = min(i1, G - 1), j1c = min(j1, G - 1);
  t.g_nw = F[field_idx(j0, i0)];
  t.g_ne = F[field_idx(j0, i1c)];
  t.g_sw = F[field_idx(j1c, i0)];
  t.g_se = F[field_idx(j1c, i1c)];
  t.fn0 = reinterpret_cast<const float4 *>(FN)[0];
  t.fn1 = reinterpret_cast<const float4 *>(FN)[1];
  t.i0 = i0; t.i1c = i1c; t.j0 = j0; t.j1c = j1c;
  t.i_out = i1 >= G;
  t.j_out = j1 >= G;
  return t;
}
// the field's grid coordinates from the host-derived (start, end, step) or the override table
struct GridK {
  float start, end, step;
  const float *lin;
  __device__ __forceinline__ float operator()(int i) const { return lin ? lin[i] : grid_coord_k(start, end, step, i); }
};
// the texels from their parts (the SDF from the env's obstacles ob(o), field_value: the reference's
// normalisation), then the bilinear blend
template <class Ob>
__device__ __forceinline__ float field_blend(const usv_cfg_t &c, const FieldTaps &t, Ob ob, const GridK &gk, float cell,
                                             float inv_r, float inv_safe) {
  const FieldNorm k = field_norm_of(t.fn0, t.fn1);
  const float x0 = gk(t.i0), x1 = gk(t.i1c), y0 = gk(t.j0), y1 = gk(t.j1c);
  const float r = c.obstacle_radius;
  const float v_nw = field_value(c, k, cell_sdf(ob, x0, y0, r), t.g_nw, cell, inv_r, inv_safe);
  float v_ne = field_value(c, k, cell_sdf(ob, x1, y0, r), t.g_ne, cell, inv_r, inv_safe);
  float v_sw = field_value(c, k, cell_sdf(ob, x0, y1, r), t.g_sw, cell, inv_r, inv_safe);
  float v_se = field_value(c, k, cell_sdf(ob, x1, y1, r), t.g_se, cell, inv_r, inv_safe);
  if (t.i_out) { v_ne = 0.f; v_se = 0.f; }
  if (t.j_out) { v_sw = 0.f; v_se = 0.f; }
  return fmaf(v_se, t.se, fmaf(v_sw, t.sw, fmaf(v_ne, t.ne, v_nw * t.nw)));
}

__device__ __forceinline__ float pen_scalar(int kind, float k, float x0, float cc, float x) {
  if (kind == PEN_DEADZONE) return -maxf(fabsf(x) - x0, 0.f) * k + cc;
  if (kind == PEN_EXPABS) return (usv_exp(x0 * fabsf(x)) - 1.0f) * k + cc;
  return 0.f;
}

// ------------------------------------------------------------------------
// Fused control step.  One thread per env.  Every per-env array lives in one
// <2 GiB window of HBM (StepWin: byte offsets from the window base), so all
// per-env loads/stores are buffer instructions with ONE shared 32-bit lane
// offset and a scalar per-array offset: no per-access 64-bit address VALU work.
// ------------------------------------------------------------------------
// reward terms of compute_reward (static_obs.py:335-657) that do not depend on the
// potential, and the potential-dependent tail
struct RewardPre {
  float dist_r0, align0, g, ggate, turning, sf, goal_r, coll, speed_r, ang_r, hi_r, pen_sum;
};
struct RewardOut {
  float pot, total, rew, dist_r, align_r, shaping, turn_haz, danger, gate_pos;
};
__device__ __forceinline__ RewardOut reward_tail(const usv_cfg_t &c, const RewardPre &p, float pot, bool pot_is_prev,
                                                 float prev_pot_mem) {
  constexpr float kXs = 0.3f + 1e-6f, kPa = 2.0f + 1e-6f;
  RewardOut o;
  o.pot = pot;
  const float pn = clampt(pot, 0.f, 1.f);
  const float xs = clampt(div_rn(pn - 0.6f, kXs, 1.0f / kXs), 0.f, 1.f);
  o.danger = xs * xs * (3.0f - 2.0f * xs);
  o.align_r = p.align0 * maxf(0.3f, 1.0f - o.danger);
  float dist_r = p.dist_r0 * maxf(0.6f, 1.0f - o.danger * 0.5f);
  dist_r = minf(dist_r, 0.f) + p.g * maxf(dist_r, 0.f);
  o.dist_r = dist_r;
  const float prev_pot = pot_is_prev ? pot : prev_pot_mem;
  float praw = (prev_pot - pot) * 100.0f;
  if (fabsf(praw) < 0.01f) praw = 0.f;
  const float pa1 = 2.0f * usv_tanh(div_rn(praw, kPa, 1.0f / kPa));
  const float ppos = maxf(pa1, 0.f), pneg = minf(pa1, 0.f);
  o.gate_pos = (ppos < 0.5f) ? 1.0f : p.ggate;
  o.shaping = o.gate_pos * ppos + pneg;
  const bool worsening = o.shaping < -0.05f;
  o.turn_haz = (float)(worsening && p.turning != 0.f) * (-10.0f) * (p.g * p.g) * p.sf;
  o.total = dist_r * 0.5f + o.align_r * 0.5f + o.shaping * 2.0f + o.turn_haz + p.goal_r + c.time_reward + p.coll +
            p.speed_r + p.ang_r + p.hi_r;
  o.rew = o.total + p.pen_sum;
  return o;
}

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

struct StepWin {
  uint32_t px, py, yaw, vx, vy, wz, fl, fr, mass, k_iz, k_drag, thr_l, thr_r, com_x, com_y, com_z;
  uint32_t lin_damp, quad_damp, progress, tgt_x, tgt_y, obst, goal_cnt, prev_dist, prev_head, prev_pot, prev_wz;
  uint32_t stats, prev_cmd, rew, reset_buf, dones, done_coll, done_succ, just_reset, obs;
  uint32_t dist, env_org, stale;
  uint32_t n4;      // bytes of one [n] f32 row
  uint32_t bytes;   // window size
};
// The same offsets as compile-time constants for the canonical slab (include/usv_hip.h USV_SLAB_*) with
// 2^kShift-byte rows: the general StepWin keeps ~45 offsets live in scalar registers across the kernel and the
// compiler spills them into VGPR lanes (~560 v_readlane / v_writelane per wave); constants are rematerialised
template <int kShift>
struct FixedWin {
  static constexpr uint32_t R(int row) { return (uint32_t)row << kShift; }
  static constexpr uint32_t px = R(USV_SLAB_STATE), py = R(USV_SLAB_STATE + 1), yaw = R(USV_SLAB_STATE + 2),
                            vx = R(USV_SLAB_STATE + 3), vy = R(USV_SLAB_STATE + 4), wz = R(USV_SLAB_STATE + 5),
                            fl = R(USV_SLAB_STATE + 6), fr = R(USV_SLAB_STATE + 7);
  static constexpr uint32_t mass = R(USV_SLAB_PARAMS), com_x = R(USV_SLAB_PARAMS + 1), com_y = R(USV_SLAB_PARAMS + 2),
                            com_z = R(USV_SLAB_PARAMS + 3), k_drag = R(USV_SLAB_PARAMS + 4),
                            thr_l = R(USV_SLAB_PARAMS + 5), thr_r = R(USV_SLAB_PARAMS + 6), k_iz = R(USV_SLAB_PARAMS + 7);
  static constexpr uint32_t lin_damp = R(USV_SLAB_LIN_DAMP), quad_damp = R(USV_SLAB_QUAD_DAMP);
  static constexpr uint32_t tgt_x = R(USV_SLAB_TGT), tgt_y = R(USV_SLAB_TGT + 1), obst = R(USV_SLAB_OBST);
  static constexpr uint32_t prev_cmd = R(USV_SLAB_PREV_CMD);
  static constexpr uint32_t prev_dist = R(USV_SLAB_HIST), prev_head = R(USV_SLAB_HIST + 1),
                            prev_pot = R(USV_SLAB_HIST + 2), prev_wz = R(USV_SLAB_HIST + 3);
  static constexpr uint32_t goal_cnt = R(USV_SLAB_IBUF), progress = R(USV_SLAB_IBUF + 1),
                            reset_buf = R(USV_SLAB_IBUF + 2), done_succ = R(USV_SLAB_IBUF + 3),
                            done_coll = R(USV_SLAB_IBUF + 4);
  static constexpr uint32_t just_reset = R(USV_SLAB_JUST_RESET), stats = R(USV_SLAB_STATS), obs = R(USV_SLAB_OBS),
                            rew = R(USV_SLAB_REW), dones = R(USV_SLAB_DONES), dist = R(USV_SLAB_DIST),
                            env_org = R(USV_SLAB_ENV_ORG), stale = R(USV_SLAB_STALE);
  static constexpr uint32_t n4 = 1u << kShift;
  static constexpr uint32_t bytes = (uint32_t)USV_SLAB_ROWS << kShift;
  static_assert((unsigned long long)USV_SLAB_ROWS << kShift < 0x80000000ull, "window < 2 GiB");
};
constexpr int kFixedShiftMin = 13, kFixedShiftMax = 22;   // n in (1024, 1048576]

// uniform constants derived on the host from usv_cfg_t (float/double arithmetic of the
// reference done once; divisors with their correctly rounded reciprocals for div_rn)
struct StepK {
  float act_rng, pos_rng, vel_rng, head_rng;
  float mass_den, inv_mass_den;
  float com_div[3], inv_com_div[3];
  float priv_base[8];             // the 8 privileged values when they do not depend on the env
  float enc_lo[3], enc_r[3], inv_enc_r[3];   // kdrag, thr, kiz: minmax range / centered scale
  int enc_ok[3];
  float inv_exp_coeff;
  float cell, inv_r, inv_safe;    // the potential field's cell size, 1 / influence radius, RN(1 / safe_radius)
  float gstart, gend, gstep;      // its grid coordinates (grid_coord's float values)
};

// privileged observation tail (USV_Virtual.py:840-976): raw / centered / minmax encoders
template <class Put>
__device__ __forceinline__ void write_priv_tail(const usv_cfg_t &c, const StepK &K, float m, float comx, float comy,
                                                float comz, float k_drag, float thr_l, float thr_r, float k_iz,
                                                Put put) {
  const int pt = USV_NOBS_BASE;
  if (c.masscom_base) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < c.priv_dim) put(pt + q, K.priv_base[q]);
    return;
  }
  put(pt, c.mass_relative ? div_rn(m - c.base_mass, K.mass_den, K.inv_mass_den) : m);
  put(pt + 1, c.com_scaled ? div_rn(comx, K.com_div[0], K.inv_com_div[0]) : comx);
  put(pt + 2, c.com_scaled ? div_rn(comy, K.com_div[1], K.inv_com_div[1]) : comy);
  put(pt + 3, c.com_scaled ? div_rn(comz, K.com_div[2], K.inv_com_div[2]) : comz);
  if (c.priv_dim == 8) {
    float v[4] = {k_drag, thr_l, thr_r, k_iz};
    const bool on[4] = {c.priv_drag_on != 0, c.priv_thr_on != 0, c.priv_thr_on != 0, c.priv_kiz_on != 0};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = q == 0 ? 0 : (q == 3 ? 2 : 1);
      if (c.priv_mode == 1) {          // enc_centered
        v[q] = clampt(div_rn(v[q] - c.priv_nominal, K.enc_r[j], K.inv_enc_r[j]), -1.f, 1.f);
      } else if (c.priv_mode == 2) {   // enc_minmax
        if (!on[q] || !K.enc_ok[j]) {
          v[q] = 0.f;
        } else {
          const float z = div_rn(v[q] - K.enc_lo[j], K.enc_r[j], K.inv_enc_r[j]);
          v[q] = clampt(2.0f * z - 1.0f, -1.f, 1.f);
        }
      }
      put(pt + 4 + q, v[q]);
    }
  }
}

__device__ __forceinline__ float bld(__amdgpu_buffer_rsrc_t R, uint32_t so, uint32_t vo) {
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(R, vo, so, 0));
}
__device__ __forceinline__ int32_t bldi(__amdgpu_buffer_rsrc_t R, uint32_t so, uint32_t vo) {
  return (int32_t)__builtin_amdgcn_raw_buffer_load_b32(R, vo, so, 0);
}
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t R, uint32_t so, uint32_t vo, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), R, vo, so, 0);
}
__device__ __forceinline__ void bsti(__amdgpu_buffer_rsrc_t R, uint32_t so, uint32_t vo, int32_t v) {
  __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, R, vo, so, 0);
}

// 64-bit (distance bits, obstacle index) compare-exchange for the top-5 network:
// keys are distinct, so the network reproduces torch.topk(largest=False)'s
// order exactly (ties -> lower index first)
__device__ __forceinline__ void cx64(uint64_t &a, uint64_t &b) {
  const uint64_t lo = a < b ? a : b, hi = a < b ? b : a;
  a = lo; b = hi;
}
__device__ __forceinline__ void mn64(uint64_t &a, uint64_t b) { a = a < b ? a : b; }
__device__ __forceinline__ void mx64(uint64_t a, uint64_t &b) { b = a < b ? b : a; }

// the 5 smallest of 16 keys in ascending order in k[0..4]: Batcher's odd-even
// merge sort pruned to the comparators that reach outputs 0..4 (50 of 63;
// checked exhaustively by the 0-1 principle)
__device__ __forceinline__ void top5_of_16(uint64_t k[16]) {
  cx64(k[0], k[1]); cx64(k[2], k[3]); cx64(k[0], k[2]); cx64(k[1], k[3]); cx64(k[1], k[2]);
  cx64(k[4], k[5]); cx64(k[6], k[7]); cx64(k[4], k[6]); cx64(k[5], k[7]); cx64(k[5], k[6]);
  cx64(k[0], k[4]); cx64(k[2], k[6]); cx64(k[2], k[4]); cx64(k[1], k[5]); mn64(k[3], k[7]);
  cx64(k[3], k[5]); cx64(k[1], k[2]); cx64(k[3], k[4]); mn64(k[5], k[6]);
  cx64(k[8], k[9]); cx64(k[10], k[11]); cx64(k[8], k[10]); cx64(k[9], k[11]); cx64(k[9], k[10]);
  cx64(k[12], k[13]); cx64(k[14], k[15]); cx64(k[12], k[14]); cx64(k[13], k[15]); cx64(k[13], k[14]);
  cx64(k[8], k[12]); cx64(k[10], k[14]); cx64(k[10], k[12]); cx64(k[9], k[13]); mn64(k[11], k[15]);
  cx64(k[11], k[13]); cx64(k[9], k[10]); cx64(k[11], k[12]); mn64(k[13], k[14]);
  cx64(k[0], k[8]); mn64(k[4], k[12]); mn64(k[4], k[8]); mn64(k[2], k[10]); cx64(k[2], k[4]);
  cx64(k[1], k[9]); mn64(k[5], k[13]); mn64(k[5], k[9]); mn64(k[3], k[11]); mn64(k[3], k[5]);
  cx64(k[1], k[2]); cx64(k[3], k[4]);
}

// the episode sums whose step value comes out of reward_tail (the potential-dependent part of the reward)
__device__ __forceinline__ constexpr bool stat_of_reward(int key) {
  return key == ST_TOTAL_REWARD || key == ST_DISTANCE_REWARD || key == ST_ALIGNMENT_REWARD ||
         key == ST_POTENTIAL_SHAPING_REWARD || key == ST_TURN_HAZARD_PENALTY || key == ST_DANGER_MEAN ||
         key == ST_DANGER_HI_RATE || key == ST_G_GATE_MEAN;
}

// The config and the host-derived constants travel as ONE first kernel argument, so the kernel can re-read
// them from the kernel-argument segment (scalar loads through a laundered pointer) at the start of a section:
// values loaded at the top stay live in scalar registers across the whole kernel otherwise, and the ~50 of
// them that do not fit were spilled to VGPR lanes (371 v_readlane + the s_nop hazards they bring)
struct StepCfg {
  usv_cfg_t c;
  StepK K;
};
typedef __attribute__((address_space(4))) const StepCfg KStepCfg;
__device__ __forceinline__ StepCfg step_cfg_reload() {
#if defined(__HIP_DEVICE_COMPILE__)
  KStepCfg *p = (KStepCfg *)__builtin_amdgcn_kernarg_segment_ptr();
  __asm__ volatile("" : "+s"(p));   // a new pointer value: nothing loaded before this point is reused
  return *p;
#else
  return StepCfg{};   // (host pass: never called)
#endif
}

template <bool kStats, bool kInj, bool kDist, class Win>
__global__ __launch_bounds__(kBlock) void k_env_step(StepCfg ck, usv_bufs_t b, Win w,
                                                     const char *__restrict__ wbase, const float *__restrict__ actions,
                                                     const float *__restrict__ lut, float bias, uint64_t seed,
                                                     uint64_t step, const float *__restrict__ inj, int part) {
  __shared__ float sobs[kBlock * USV_NOBS];
  __shared__ float2 sob[USV_NOBST][kBlock];
  __shared__ float slut[2 * USV_LUT_N];
  __shared__ uint8_t keep[kBlock];
  const usv_cfg_t &c = ck.c;
  const StepK &K = ck.K;
  const int n = b.n;
  const int tid = threadIdx.x;
  const int e = blockIdx.x * kBlock + tid;
  const __amdgpu_buffer_rsrc_t R = __builtin_amdgcn_make_buffer_rsrc((void *)wbase, 0, (int)w.bytes, 0x00020000);
  // thruster LUT -> registers first (the oldest loads in flight: waiting for them before
  // the LDS write below does not wait for the per-env loads issued after them)
  static_assert(2 * USV_LUT_N / 4 <= 2 * kBlock, "LUT staging: two float4 per thread");
  const float4 *lut4 = reinterpret_cast<const float4 *>(lut);
  const bool lut_hi = tid + kBlock < 2 * USV_LUT_N / 4;
  const float4 lut_a = lut4[tid];
  const float4 lut_b = lut4[min(tid + kBlock, 2 * USV_LUT_N / 4 - 1)];   // unconditional: no branch, no early wait
  // part 0: every env; 1: envs not reset this step (they do not read this step's new
  // fields, so this part can run concurrently with the potential-field kernels);
  // 2: the envs reset this step, after their fields are built
  // Every lane runs the whole step (lanes past n on env n-1); the stores of lanes that
  // are not `mine` go to an offset past the window, which the buffer range check drops.
  const int ec = min(e, n - 1);
  const uint32_t v4 = (uint32_t)ec * 4u;
  // loads in the order they are consumed (vmcnt waits retire loads in issue order):
  // action + reset flag (LUT index), state and parameters (substeps), then the rest
  const float2 a2 = reinterpret_cast<const float2 *>(actions)[ec];
  const bool was_reset = __builtin_amdgcn_raw_buffer_load_b8(R, (uint32_t)ec, w.just_reset, 0) != 0;
  __builtin_amdgcn_sched_barrier(0);
  constexpr uint32_t kDrop = 0x80000000u;   // > w.bytes
  const int32_t *ctl = b.ctl;
  // control words: plain (non-short-circuit) scalar reads, so no branch waits on memory here
  const int32_t ctl_pot = ctl[USV_CTL_POT_VALID], ctl_cnt = ctl[USV_CTL_RESET_COUNT];
  const bool pot_none = (ctl_pot == 0) | (ctl_cnt > 0);
  const bool pen_valid = ctl[USV_CTL_PEN_VALID] != 0;
  const bool rew_valid = ctl[USV_CTL_REW_VALID] != 0;
  step = step_of(b, step);
  bias = bias_of(c, b, bias);
  // obs row staged in LDS (odd row stride: conflict-free), clamped on write
  // (_process_data clamp, vec_env_rlgames.py:85-95); slots no branch writes are zeroed
  float *obs = sobs + tid * USV_NOBS;
  const float clip = c.clip_obs;
  auto put = [&](int q, float v) { obs[q] = clampt(v, -clip, clip); };
  obs[6] = 0.f;
  obs[7] = 0.f;
  if (c.priv_dim == 4) { obs[29] = 0.f; obs[30] = 0.f; obs[31] = 0.f; obs[32] = 0.f; }   // input padding
  {
    // ---- every per-env input that does not depend on this step's results is loaded
    // up front, so the HBM latencies overlap each other and the physics ----
    float px = bld(R, w.px, v4), py = bld(R, w.py, v4), yaw = bld(R, w.yaw, v4);
    float vx = bld(R, w.vx, v4), vy = bld(R, w.vy, v4), wz = bld(R, w.wz, v4);
    float fl = bld(R, w.fl, v4), fr = bld(R, w.fr, v4);
    const float m = bld(R, w.mass, v4);
    const float k_iz = bld(R, w.k_iz, v4), k_drag = bld(R, w.k_drag, v4);
    const float thr_l = bld(R, w.thr_l, v4), thr_r = bld(R, w.thr_r, v4);
    const float comx = bld(R, w.com_x, v4), comy = bld(R, w.com_y, v4), comz = bld(R, w.com_z, v4);
    // per-env damping (drag DR) or the config's: loaded unconditionally (offset 0 is inside
    // the window when absent) and selected, so no branch sits between the loads
    const bool dr = b.lin_damp != nullptr;
    const float l0 = bld(R, w.lin_damp, v4), l1 = bld(R, w.lin_damp + w.n4, v4), l2 = bld(R, w.lin_damp + 2 * w.n4, v4);
    const float q0 = bld(R, w.quad_damp, v4), q1 = bld(R, w.quad_damp + w.n4, v4);
    const float q2 = bld(R, w.quad_damp + 2 * w.n4, v4);
    const float lin0 = dr ? l0 : c.lin_damp[0], lin1 = dr ? l1 : c.lin_damp[1], lin2 = dr ? l2 : c.lin_damp[2];
    const float qd0 = dr ? q0 : c.quad_damp[0], qd1 = dr ? q1 : c.quad_damp[1], qd2 = dr ? q2 : c.quad_damp[2];
    // disturbance parameters (drawn at reset) and the env origin (root_pos is world-frame)
    float dp[USV_NDIST], orgx = 0.f, orgy = 0.f;
    if (kDist) {
#pragma unroll
      for (int q = 0; q < USV_NDIST; ++q) dp[q] = bld(R, w.dist + (uint32_t)q * w.n4, v4);
      const float ox_ = bld(R, w.env_org, v4), oy_ = bld(R, w.env_org + w.n4, v4);
      orgx = b.env_org ? ox_ : 0.f;
      orgy = b.env_org ? oy_ : 0.f;
    }
    // a reset env's first substep: the pre-reset inputs usv_reset kept; the other lanes
    // read past the window (no memory access, 0)
    const bool stl = c.stale_root && was_reset;
    const uint32_t vst = stl ? v4 : kDrop;
    const float st_ub = bld(R, w.stale + USV_STALE_UB * w.n4, vst), st_vb = bld(R, w.stale + USV_STALE_VB * w.n4, vst);
    const float st_rb = bld(R, w.stale + USV_STALE_RB * w.n4, vst);
    float st_px = 0.f, st_py = 0.f;
    if (kDist) {
      st_px = bld(R, w.stale + USV_STALE_PX * w.n4, vst);
      st_py = bld(R, w.stale + USV_STALE_PY * w.n4, vst);
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the substep inputs ahead of the loads below
    const int progress0 = bldi(R, w.progress, v4);
    const float tgx = bld(R, w.tgt_x, v4), tgy = bld(R, w.tgt_y, v4);
    float obx[USV_NOBST], oby[USV_NOBST];
#pragma unroll
    for (int o = 0; o < USV_NOBST; ++o) {
      obx[o] = bld(R, w.obst + (uint32_t)(2 * o) * w.n4, v4);
      oby[o] = bld(R, w.obst + (uint32_t)(2 * o + 1) * w.n4, v4);
    }
    const int goal_cnt0 = bldi(R, w.goal_cnt, v4);

    const float prev_d_mem = bld(R, w.prev_dist, v4), prev_head_mem = bld(R, w.prev_head, v4);
    const float prev_pot_mem = bld(R, w.prev_pot, v4), prev_wz_mem = bld(R, w.prev_wz, v4);
    // episode sums that this step adds to (the other keys are written by the reset path only)
    constexpr int kSum[25] = {ST_TOTAL_REWARD, ST_DISTANCE_REWARD, ST_ALIGNMENT_REWARD, ST_HEADING_IMPROVE_REWARD,
                              ST_POTENTIAL_SHAPING_REWARD, ST_SPEED_REWARD, ST_ANGULAR_REWARD,
                              ST_TURN_HAZARD_PENALTY, ST_GOAL_REWARD, ST_TIME_REWARD, ST_COLLISION_REWARD,
                              ST_DANGER_MEAN, ST_DANGER_HI_RATE, ST_G_GATE_MEAN, ST_POSITION_ERROR,
                              ST_BOUNDARY_PENALTY, ST_ANGULAR_VEL_PENALTY, ST_ANGULAR_VEL_VARIATION_PENALTY,
                              ST_ENERGY_PENALTY, ST_NORMED_LINEAR_VEL, ST_NORMED_ANGULAR_VEL, ST_CMD_NEG_RATE,
                              ST_U_MEAN, ST_U_LOW_RATE, ST_U_SUM};
    const bool sum_on[25] = {true, true, true, true, true, true, true, true, true, true, true, true, true,
                             true, true, true, c.pen_ang_kind != 0, c.pen_angv_kind != 0, c.pen_en_kind != 0,
                             true, true, true, true, true, true};
    float sums[25];
    if (kStats) {
#pragma unroll
      for (int q = 0; q < 25; ++q) sums[q] = bld(R, w.stats + (uint32_t)kSum[q] * w.n4, v4);
    }
    // ---- uniforms of this step (SU_* layout; the second Philox block only when drawn from) ----
    float u[USV_NU_STEP];
    if (kInj) {
#pragma unroll
      for (int i = 0; i < USV_NU_STEP; ++i) u[i] = inj[(size_t)ec * USV_NU_STEP + i];
    } else {
      philox_u4(seed, (uint32_t)e, step, 0u, u);
      if (c.pos_noise_on || c.act_noise_on) philox_u4(seed, (uint32_t)e, step, 1u, u + 4);
      else u[4] = u[5] = u[6] = u[7] = 0.f;
    }
    // ---- VecEnvRLGames.step clamp (:136-140) + pre_physics_step (:1050-1099) ----
    const float cmd0 = clampt(a2.x, -c.clip_actions, c.clip_actions);
    const float cmd1 = clampt(a2.y, -c.clip_actions, c.clip_actions);
    const float prev_cmd0 = was_reset ? 0.f : cmd0;
    const float prev_cmd1 = was_reset ? 0.f : cmd1;
    float t0 = cmd0, t1 = cmd1;
    if (bias != 0.f) { t0 = t0 + bias; t1 = t1 + bias; }
    if (c.act_noise_on) {
      t0 = t0 + (u[SU_ACT] * K.act_rng + c.act_noise_min);
      t1 = t1 + (u[SU_ACT + 1] * K.act_rng + c.act_noise_min);
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
    bool mine = e < n;
    if (part == 1 || part == 2) mine = mine && ((part == 1) ? !was_reset : was_reset);
    // part 3: every env, but the envs reset this step leave their potential-dependent reward to
    // usv_env_step_late (their fields are still being built): stash + no rew / prev_pot / reward sums
    const bool defer = part == 3 && was_reset;
    keep[tid] = mine ? 1 : 0;
    const uint32_t vs = mine ? v4 : kDrop;
    reinterpret_cast<float4 *>(slut)[tid] = lut_a;
    if (lut_hi) reinterpret_cast<float4 *>(slut)[tid + kBlock] = lut_b;
    __syncthreads();   // LUT staged
    float tgt0 = slut[i0], tgt1 = slut[USV_LUT_N + i1];
    if (c.use_thr_mult) { tgt0 = tgt0 * thr_l; tgt1 = tgt1 * thr_r; }
    // ---- 10 substeps: thruster lag, planar forces, semi-implicit Euler.  The
    // integrator is this build's own (it replaces PhysX): accelerations divide by
    // m and Izz through their reciprocals with one correction step (div_rn == the
    // IEEE quotient for quotients in [2^-90, 2^120]) ----
    const float izz = c.izz0 * k_iz;
    const float inv_m = 1.0f / m, inv_izz = 1.0f / izz;
    const float kd = c.use_drag_scale ? k_drag : 1.0f;
    const float al = c.thr_alpha, oma = 1.0f - c.thr_alpha;
    const float dt = c.dt;
    const float arm_l = -(c.thr_y - comy), arm_r = c.thr_y + comy;
    for (int s = 0; s < c.substeps; ++s) {
      fl = fl * al + oma * tgt0;                      // ThrusterDynamics.py:133-136
      fr = fr * al + oma * tgt1;
      // the attitude the reference reads back: R = quaternion_to_matrix(q(yaw)) (usv_quat_rot)
      const QuatRot qr = usv_quat_rot(yaw);
      const float sy_ = qr.S, cy_ = qr.C;
      float ub = cy_ * vx + sy_ * vy;                 // R^T v (Utils.py:10-14, Hydrodynamics.py:209-217)
      float vb = -sy_ * vx + cy_ * vy;
      float rb = wz;
      float hpx = px, hpy = py;
      if (kDist && c.current_on) {                    // relative to the water (Hydrodynamics.py:224-237)
        ub = ub - (cy_ * c.flow_vel[0] + sy_ * c.flow_vel[1]);
        vb = vb - (-sy_ * c.flow_vel[0] + cy_ * c.flow_vel[1]);
      }
      if (s == 0) {                                   // the cached pre-reset root state
        ub = stl ? st_ub : ub;
        vb = stl ? st_vb : vb;
        rb = stl ? st_rb : rb;
        hpx = stl ? st_px : hpx;
        hpy = stl ? st_py : hpy;
      }
      float dfx = 0.f, dfy = 0.f, dtz = 0.f;
      if (kDist) {
        // get_disturbance_forces / get_torque_disturbance at root_pos (USV_disturbances.py:386-410,510-530)
        const float wx = hpx + orgx, wy = hpy + orgy;
        dfx = dp[DI_FCX];
        dfy = dp[DI_FCY];
        dtz = dp[DI_TC];
        if (c.fsin_on) {
          dfx = dfx + usv_sin_cr(wx * dp[DI_FXF] + dp[DI_FXS]) * dp[DI_FAMP];
          dfy = dfy + usv_sin_cr(wy * dp[DI_FYF] + dp[DI_FYS]) * dp[DI_FAMP];
        }
        if (c.tsin_on) dtz = dtz + usv_sin_cr((wx + wy) * dp[DI_TF] + dp[DI_TS]) * dp[DI_TAMP];
      }
      float D0 = lin0 + qd0 * fabsf(ub), D1 = lin1 + qd1 * fabsf(vb), D2 = lin2 + qd2 * fabsf(rb);
      D0 = D0 * c.scaling_damping; D1 = D1 * c.scaling_damping; D2 = D2 * c.scaling_damping;
      if (c.use_drag_scale) { D0 = D0 * kd; D1 = D1 * kd; D2 = D2 * kd; }
      // base force = disturbance + drag (+ hydrostatics, 0 in the plane), thrusters (USV_Virtual.py:1118-1132)
      const float X = kDist ? fl + fr + (dfx + (-D0 * ub)) : fl + fr + (-D0 * ub);   // Hydrodynamics.py:243
      const float Y = kDist ? dfy + (-D1 * vb) : -D1 * vb;
      const float N = kDist ? arm_l * fl + arm_r * fr + (dtz + (-D2 * rb)) : arm_l * fl + arm_r * fr + (-D2 * rb);
      const float ax = div_rn(cy_ * X - sy_ * Y, m, inv_m);
      const float ay = div_rn(sy_ * X + cy_ * Y, m, inv_m);
      const float aw = div_rn(N, izz, inv_izz);
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
    bst(R, w.px, vs, px); bst(R, w.py, vs, py); bst(R, w.yaw, vs, yaw);
    bst(R, w.vx, vs, vx); bst(R, w.vy, vs, vy); bst(R, w.wz, vs, wz);
    bst(R, w.fl, vs, fl); bst(R, w.fr, vs, fr);
    // the rest of the step reads its config afresh (see StepCfg)
    const StepCfg ck2 = step_cfg_reload();
    const usv_cfg_t &c = ck2.c;
    const StepK &K = ck2.K;
    // ---- post_physics_step: progress, update_state noise (USV_Virtual.py:771-813) ----
    const int progress = progress0 + 1;
    bsti(R, w.progress, vs, progress);
    float pxn = px, pyn = py;
    if (c.pos_noise_on) {
      pxn = pxn + (u[SU_PX] * K.pos_rng + c.pos_noise_min);
      pyn = pyn + (u[SU_PX + 1] * K.pos_rng + c.pos_noise_min);
    }
    // the potential sample only needs the position: issue its 4 texel loads now
    const FieldTaps taps = field_taps(b.field + (size_t)ec * USV_FIELD_STRIDE, b.fnorm + (size_t)ec * USV_FNORM,
                                      c.map_size, pxn, pyn);
    float vxn = vx, vyn = vy, wzn = wz;
    if (c.vel_noise_on) {
      vxn = vxn + (u[SU_VX] * K.vel_rng + c.vel_noise_min);
      vyn = vyn + (u[SU_VY] * K.vel_rng + c.vel_noise_min);
      wzn = wzn + (u[SU_WZ] * K.vel_rng + c.vel_noise_min);
    }
    // update_state's heading: atan2 of the read-back quaternion (USV_Virtual.py:776-786), then its noise
    float yawn = usv_heading(usv_quat_rot(yaw));
    if (c.head_noise_on) yawn = yawn + (u[SU_HEAD] * K.head_rng + c.head_noise_min);
    float hs, hc;
    usv_sincos(yawn, &hs, &hc);
    // ---- get_state_observations (static_obs.py:193-299) ----
    const float ex = tgx - pxn, ey = tgy - pyn;
    const float theta = usv_atan2(hs, hc);
    const float beta = usv_atan2(ey, ex);
    const float alpha = fmodf((beta - theta) + USV_PI_F, USV_2PI_F) - USV_PI_F;
    const float herr = fabsf(alpha);
    const float dist = sqrtf(ex * ex + ey * ey);
    const float dist_n = tnorm2(ex, ey);
    float st, ct, sa, ca;
    usv_sincos(theta, &st, &ct);
    usv_sincos(alpha, &sa, &ca);     // usv_sincos's cos is exactly even: ca == cos(herr) as well
    // 16 obstacle distances; the 5 nearest (torch.topk largest=False, ascending) by a
    // selection network over (distance bits, index) keys -- distances are >= 0 so
    // their bit patterns order like the floats
    uint64_t key[USV_NOBST];
    float min_od = INFINITY, coll = 0.f;
#pragma unroll
    for (int o = 0; o < USV_NOBST; ++o) {
      const float d = tnorm2(obx[o] - pxn, oby[o] - pyn);
      min_od = fminf(min_od, d);
      coll += (float)(d < c.collision_threshold) * (-10.0f) * 10.0f;
      key[o] = ((uint64_t)__float_as_uint(d) << 4) | (uint64_t)o;
      sob[o][tid] = make_float2(obx[o], oby[o]);
    }
    top5_of_16(key);
    if (c.obs_local) {
      put(0, hc * vxn + hs * vyn);
      put(1, -hs * vxn + hc * vyn);
    } else {
      put(0, vxn);
      put(1, vyn);
    }
    put(2, wzn);
    put(3, ca);
    put(4, sa);
    put(5, dist_n);
#pragma unroll
    for (int q = 0; q < USV_NCLOSE; ++q) {
      const int o = (int)(key[q] & 15u);
      const float2 ob = sob[o][tid];
      const float bx = ob.x - pxn, by = ob.y - pyn;
      const float bd = __uint_as_float((uint32_t)(key[q] >> 4));
      const float vbx = bx * ct + by * st;
      const float vby = -bx * st + by * ct;
      const float nf = sqrtf(vbx * vbx + vby * vby + 1e-6f);
      const float inv_nf = 1.0f / nf;
      put(8 + 3 * q, bd - c.obstacle_radius);
      put(9 + 3 * q, div_rn(-vbx, nf, inv_nf));
      put(10 + 3 * q, div_rn(-vby, nf, inv_nf));
    }
    const int pa = USV_NOBS_BASE - 2;
    put(pa, prev_cmd0);
    put(pa + 1, prev_cmd1);
    bst(R, w.prev_cmd, vs, prev_cmd0);
    bst(R, w.prev_cmd + w.n4, vs, prev_cmd1);
    // ---- privileged tail (USV_Virtual.py:840-976) ----
    write_priv_tail(c, K, m, comx, comy, comz, k_drag, thr_l, thr_r, k_iz, put);
    {   // the reward / kill / statistics section reads its config afresh too (see StepCfg)
    const StepCfg ck3 = step_cfg_reload();
    const usv_cfg_t &c = ck3.c;
    const StepK &K = ck3.K;
    // ---- compute_reward (static_obs.py:335-657): the potential-independent terms first ----
    constexpr float kGv = (0.15f - 0.02f) + 1e-6f, kGd = 0.01f + 1e-6f;
    constexpr float kSf = (0.60f - 0.15f) + 1e-6f, kSp = 0.8f + 1e-6f, kAn = 0.2f;
    const float bover = maxf(dist - c.kill_dist, 0.f);
    const float bpen = -expm1f(minf(bover / 0.25f, 20.0f)) * c.boundary_cost;
    const int gir = dist < c.position_tolerance;
    const int goal_cnt = goal_cnt0 * gir + gir;
    bsti(R, w.goal_cnt, vs, goal_cnt);
    const float prev_err = rew_valid ? prev_d_mem : dist;
    RewardPre rp;
    if (c.reward_mode == 0) rp.dist_r0 = c.position_scale * (prev_err - dist);
    else if (c.reward_mode == 1) rp.dist_r0 = c.position_scale * (prev_err * prev_err - dist * dist);
    else rp.dist_r0 = c.position_scale * (usv_exp(div_rn(-dist, c.exp_coeff, K.inv_exp_coeff)) -
                                          usv_exp(div_rn(-prev_err, c.exp_coeff, K.inv_exp_coeff)));
    const float h2 = herr * herr;
    rp.align0 = c.align_la1 * (usv_exp(c.align_la2 * (h2 * h2)) + usv_exp(c.align_la3 * h2));
    if (was_reset) rp.dist_r0 = 0.f;
    const float prev_dist = was_reset ? dist : (rew_valid ? prev_d_mem : dist);
    rp.g = clampt(ca, 0.f, 1.f);
    const float prev_h = (rew_valid && !was_reset) ? prev_head_mem : herr;
    const float hi = clampt(prev_h - herr, -0.4f, 0.4f);
    rp.hi_r = hi * 0.05f;
    bst(R, w.prev_head, vs, herr);
    const float dd = dist + 1e-6f, inv_dd = 1.0f / dd;
    const float gdx = div_rn(ex, dd, inv_dd), gdy = div_rn(ey, dd, inv_dd);
    const float vtp = maxf(vxn * gdx + vyn * gdy, 0.f);
    const float ddp = maxf(prev_dist - dist, 0.f);
    const float gv = clampt(div_rn(vtp - 0.02f, kGv, 1.0f / kGv), 0.f, 1.f);
    const float gd = clampt(div_rn(ddp, kGd, 1.0f / kGd), 0.f, 1.f);
    rp.ggate = maxf(gv, gd) * rp.g;
    rp.turning = fabsf(wzn) > 0.2f ? 1.f : 0.f;
    const float vfwd = vxn * hc + vyn * hs;
    rp.sf = clampt(div_rn(fabsf(vfwd) - 0.15f, kSf, 1.0f / kSf), 0.f, 1.f);
    rp.speed_r = (1.0f - usv_exp(div_rn(-vtp, kSp, 1.0f / kSp))) * 0.05f;
    const float sgn = (alpha > 0.f) ? 1.f : ((alpha < 0.f) ? -1.f : 0.f);
    const float tang = (herr > 1.0f) ? sgn * 1.0f : sgn * 0.2f;
    const float dw = wzn - tang;
    rp.ang_r = usv_exp(div_rn(-(dw * dw), kAn, 1.0f / kAn)) * 0.03f;
    rp.goal_r = ((float)goal_cnt * c.goal_reward) * 5.0f;
    rp.coll = coll;
    bst(R, w.prev_dist, vs, dist);
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
    bst(R, w.prev_wz, vs, wzn);
    rp.pen_sum = ((p_lin + p_ang) + p_angv) + p_en;
    // ---- the potential-dependent tail ----
    const RewardOut ro = reward_tail(c, rp, field_blend(c, taps, [&](int o) { return sob[o][tid]; }, GridK{K.gstart, K.gend, K.gstep, b.grid_lin},
                                                 K.cell, K.inv_r, K.inv_safe), pot_none || was_reset, prev_pot_mem);
    const uint32_t vr = defer ? kDrop : vs;   // the potential-dependent outputs
    bst(R, w.prev_pot, vr, ro.pot);
    bst(R, w.rew, vr, ro.rew);
    if (defer && mine) {
      const float st[USV_RSTASH_ROWS] = {rp.dist_r0, rp.align0, rp.g, rp.ggate, rp.turning, rp.sf, rp.goal_r, rp.coll,
                                         rp.speed_r, rp.ang_r, rp.hi_r, rp.pen_sum, pxn, pyn};
#pragma unroll
      for (int q = 0; q < USV_RSTASH_ROWS; ++q) b.rstash[(size_t)q * n + e] = st[q];
    }
    // ---- update_kills / is_done (static_obs.py:661-706, USV_Virtual.py:1223-1237) ----
    const bool dkill = dist > c.kill_dist;
    const bool ckill = min_od < c.collision_threshold;
    const bool skill = goal_cnt >= c.kill_after_n;
    const bool die = dkill || ckill || skill;
    if (die) {
      bsti(R, w.done_coll, vs, ckill);
      bsti(R, w.done_succ, vs, skill && !ckill);
    }
    const int tout = progress >= c.max_episode_length - 1;
    const int rb = c.fixed_horizon_eval ? tout : (tout ? 1 : (int)die);
    bsti(R, w.reset_buf, vs, rb);
    const u32x2_t rb64 = {(uint32_t)rb, 0u};
    __builtin_amdgcn_raw_buffer_store_b64(rb64, R, mine ? (uint32_t)ec * 8u : kDrop, w.dones, 0);
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, R, mine ? (uint32_t)ec : kDrop, w.just_reset, 0);
    if (c.nan_probe) {   // clamped actions, the observed state, the reward (obs: at the row store below)
      uint32_t bits = ((nonfinite(cmd0) | nonfinite(cmd1)) ? USV_NAN_ACTIONS : 0u) |
                      ((nonfinite(pxn) | nonfinite(pyn) | nonfinite(yawn) | nonfinite(vxn) | nonfinite(vyn) |
                        nonfinite(wzn)) ? USV_NAN_STATE : 0u) |
                      ((!defer && nonfinite(ro.rew)) ? USV_NAN_REWARD : 0u);
      nan_report(&b.ctl[USV_CTL_NAN_FLAG], mine ? bits : 0u);
    }
    if (kStats) {
      const float add[25] = {ro.total, ro.dist_r, ro.align_r, rp.hi_r, ro.shaping, rp.speed_r, rp.ang_r, ro.turn_haz,
                             rp.goal_r, c.time_reward, coll, ro.danger, (float)(ro.danger > 0.5f), ro.gate_pos, dist,
                             bpen, p_ang, p_angv, p_en, tnorm2(vxn, vyn), fabsf(wzn),
                             ((float)(t0 < 0.f) + (float)(t1 < 0.f)) / 2.0f, (unit0 + unit1) / 2.0f,
                             ((float)(unit0 < 0.05f) + (float)(unit1 < 0.05f)) / 2.0f, unit0 + unit1};
#pragma unroll
      for (int q = 0; q < 25; ++q)
        if (sum_on[q]) bst(R, w.stats + (uint32_t)kSum[q] * w.n4, stat_of_reward(kSum[q]) ? vr : vs, sums[q] + add[q]);
    }
    }
  }
  // ---- coalesced obs store: rows of 33 floats staged through LDS ----
  __syncthreads();
  const int row0 = blockIdx.x * kBlock;
  const int rows = min(kBlock, n - row0);
  const uint32_t obase = (uint32_t)row0 * (uint32_t)(USV_NOBS * 4);
  // obs entries are clamped to +-clip_obs, so only a NaN is non-finite: x != x
  uint32_t obad = 0u;
  if (part == 0 || part == 3) {
    const int nv = rows * USV_NOBS / 4;       // whole float4s (row0 * 33 * 4 B is 16-B aligned)
    for (int i = tid; i < nv; i += kBlock) {
      const float4 v = reinterpret_cast<const float4 *>(sobs)[i];
      obad |= (uint32_t)((v.x != v.x) | (v.y != v.y) | (v.z != v.z) | (v.w != v.w));
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4_t, v),
                                             R, obase + (uint32_t)i * 16u, w.obs, 0);
    }
    for (int i = nv * 4 + tid; i < rows * USV_NOBS; i += kBlock) {
      obad |= (uint32_t)(sobs[i] != sobs[i]);
      bst(R, w.obs, obase + (uint32_t)i * 4u, sobs[i]);
    }
  } else {
    for (int i = tid; i < rows * USV_NOBS; i += kBlock)
      if (keep[i / USV_NOBS]) {
        obad |= (uint32_t)(sobs[i] != sobs[i]);
        bst(R, w.obs, obase + (uint32_t)i * 4u, sobs[i]);
      }
  }
  if (c.nan_probe) nan_report(&b.ctl[USV_CTL_NAN_FLAG], obad ? USV_NAN_OBS : 0u);
  // ---- the step has consumed the Nones (:361, :448, USV_task_rewards.py:450): marked here,
  // promoted to the POT/PEN/REW_VALID flags by the next usv_reset, so the flags never change
  // while a step kernel that reads them runs ----
  if (blockIdx.x == 0 && tid == 0) b.ctl[USV_CTL_STEPPED] = 1;
}


// usv_env_step_late: the potential-dependent reward of the envs reset this step, once their fields
// exist (after usv_env_step_part(.., 3) and the field kernels): the stashed potential-independent terms,
// the field sample at the stashed position, reward_tail with prev_potential None (a reset env), the
// reward, prev_pot and the reward sums -- the operations part 0 runs for these envs, in the same order.
#ifndef USV_LATE_GRID
#define USV_LATE_GRID 256
#endif
constexpr int kLateGrid = USV_LATE_GRID;
__global__ __launch_bounds__(64) void k_env_reward_late(usv_cfg_t c, usv_bufs_t b) {
  const int n = b.n;
  const float cell = (float)((double)c.map_size / USV_GRID);
  const float inv_r = (float)(1.0 / (double)c.influence_radius);
  const float inv_safe = 1.0f / c.safe_radius;
  const double cell_d = (double)c.map_size / USV_GRID;
  const float g_start = (float)(-(double)c.map_size / 2 + cell_d / 2), g_end = (float)((double)c.map_size / 2 - cell_d / 2);
  const GridK gk{g_start, g_end, (g_end - g_start) / (float)(USV_GRID - 1), b.grid_lin};
  const int count = min(b.ctl[USV_CTL_RESET_COUNT], n);
  // slots spread thinly over many one-wave workgroups (lane l of workgroup g takes slot g + G l, ...): every
  // lane's loads are gathers from scattered envs, so a wave with few active lanes issues them in few cycles
  // and every CU takes a share (64 consecutive slots per wave put ~74 x 64 scattered lines on one CU)
  const int G = (int)gridDim.x;
  for (int slot = (int)blockIdx.x + G * (int)threadIdx.x; slot < count; slot += G * (int)blockDim.x) {
    const int e = b.reset_ids[slot];
    float st[USV_RSTASH_ROWS];
#pragma unroll
    for (int q = 0; q < USV_RSTASH_ROWS; ++q) st[q] = b.rstash[(size_t)q * n + e];
    const RewardPre rp{st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7], st[8], st[9], st[10], st[11]};
    const FieldTaps taps = field_taps(b.field + (size_t)e * USV_FIELD_STRIDE, b.fnorm + (size_t)e * USV_FNORM,
                                      c.map_size, st[12], st[13]);
    float2 obs_c[USV_NOBST];
#pragma unroll
    for (int o = 0; o < USV_NOBST; ++o)
      obs_c[o] = make_float2(b.obst[(size_t)(2 * o) * n + e], b.obst[(size_t)(2 * o + 1) * n + e]);
    const RewardOut ro = reward_tail(c, rp, field_blend(c, taps, [&](int o) { return obs_c[o]; }, gk, cell, inv_r, inv_safe),
                                     true, 0.f);
    b.prev_pot[e] = ro.pot;
    b.rew[e] = ro.rew;
    if (c.stats_on) {
      const float add[8] = {ro.total, ro.dist_r, ro.align_r, ro.shaping, ro.turn_haz, ro.danger,
                            (float)(ro.danger > 0.5f), ro.gate_pos};
      constexpr int key[8] = {ST_TOTAL_REWARD, ST_DISTANCE_REWARD, ST_ALIGNMENT_REWARD, ST_POTENTIAL_SHAPING_REWARD,
                              ST_TURN_HAZARD_PENALTY, ST_DANGER_MEAN, ST_DANGER_HI_RATE, ST_G_GATE_MEAN};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float *p = b.stats + (size_t)key[q] * n + e;
        *p = *p + add[q];
      }
    }
    if (c.nan_probe && nonfinite(ro.rew)) atomicOr(&b.ctl[USV_CTL_NAN_FLAG], (int)USV_NAN_REWARD);
  }
}

// ------------------------------------------------------------------------
// GoToPose / TrackXYOVelocity control step.  Same physics, action
// mapping, noise, penalties and privileged tail as the CaptureXY step; the task
// part follows GoToPoseTask (tasks/USV/USV_go_to_pose.py:89-209) and
// TrackXYOVelocityTask (USV_track_xyo_velocity.py:75-166) with their rewards
// (USV_task_rewards.py:160-249, 328-393).  Glue where the reference cannot run
// these tasks: the task_data block is the Core layout's 20 columns
// (unwritten columns 0), update_kills(step) is the task's own, the reward is
// task.compute_reward(current_state, actions) + penalties as calculate_metrics
// (USV_Virtual.py:1628-1652) does for every task.
// TrackXYOVelocity's angular error is reduced over ALL envs
// (torch.square(err).sum(-1) of a 1-D tensor, :121-123), so its step is two
// launches: this kernel writes per-block partial sums, k_track_finish completes.
// ------------------------------------------------------------------------
__device__ __forceinline__ float task_term(int mode, float x, float coeff) {
  if (mode == 0) return 1.0f / (1.0f + x);
  if (mode == 1) return 1.0f / (1.0f + x * x);
  return usv_exp(-x / coeff);
}

template <int kKind, bool kStats, bool kInj>
__global__ __launch_bounds__(kBlock) void k_env_step_task(StepCfg ck, usv_bufs_t b,
                                                          const float *__restrict__ actions,
                                                          const float *__restrict__ lut, float bias, uint64_t seed,
                                                          uint64_t step, const float *__restrict__ inj) {
  __shared__ float sobs[kBlock * USV_NOBS];
  __shared__ float sred[kBlock / 64];
  const usv_cfg_t &c = ck.c;
  const StepK &K = ck.K;
  const int n = b.n;
  const int tid = threadIdx.x;
  const int e = blockIdx.x * kBlock + tid;
  const int ec = min(e, n - 1);
  const bool mine = e < n;
  const size_t nn = (size_t)n;
  step = step_of(b, step);
  bias = bias_of(c, b, bias);
  const bool pen_valid = b.ctl[USV_CTL_PEN_VALID] != 0;
  float *obs = sobs + tid * USV_NOBS;
  const float clip = c.clip_obs;
  auto put = [&](int q, float v) { obs[q] = clampt(v, -clip, clip); };
  // ---- loads ----
  const float2 a2 = reinterpret_cast<const float2 *>(actions)[ec];
  const bool was_reset = b.just_reset[ec] != 0;
  float px = b.px[ec], py = b.py[ec], yaw = b.yaw[ec], vx = b.vx[ec], vy = b.vy[ec], wz = b.wz[ec];
  float fl = b.fl[ec], fr = b.fr[ec];
  const float m = b.mass[ec], k_iz = b.k_iz[ec], k_drag = b.k_drag[ec];
  const float thr_l = b.thr_l[ec], thr_r = b.thr_r[ec];
  const float comx = b.com_x[ec], comy = b.com_y[ec], comz = b.com_z[ec];
  float lin0 = c.lin_damp[0], lin1 = c.lin_damp[1], lin2 = c.lin_damp[2];
  float qd0 = c.quad_damp[0], qd1 = c.quad_damp[1], qd2 = c.quad_damp[2];
  if (b.lin_damp) {
    lin0 = b.lin_damp[ec]; lin1 = b.lin_damp[nn + ec]; lin2 = b.lin_damp[2 * nn + ec];
    qd0 = b.quad_damp[ec]; qd1 = b.quad_damp[nn + ec]; qd2 = b.quad_damp[2 * nn + ec];
  }
  float dp[USV_NDIST], orgx = 0.f, orgy = 0.f;
  const bool has_dist = b.dist != nullptr;
  if (has_dist) {
#pragma unroll
    for (int q = 0; q < USV_NDIST; ++q) dp[q] = b.dist[q * nn + ec];
    if (b.env_org) { orgx = b.env_org[ec]; orgy = b.env_org[nn + ec]; }
  }
  const int progress0 = b.progress[ec], goal_cnt0 = b.goal_cnt[ec];
  const float tgx = b.tgt_x[ec], tgy = b.tgt_y[ec], tgh = b.tgt_h[ec];
  const float prev_pd = b.prev_dist[ec], prev_wz_mem = b.prev_wz[ec];
  // a reset env's first substep: the pre-reset inputs usv_reset kept
  const bool stl = c.stale_root && was_reset;
  float st_ub = 0.f, st_vb = 0.f, st_rb = 0.f, st_px = 0.f, st_py = 0.f;
  if (stl) {
    st_ub = b.stale[USV_STALE_UB * nn + ec];
    st_vb = b.stale[USV_STALE_VB * nn + ec];
    st_rb = b.stale[USV_STALE_RB * nn + ec];
    st_px = b.stale[USV_STALE_PX * nn + ec];
    st_py = b.stale[USV_STALE_PY * nn + ec];
  }
  float sums[USV_NSTAT];
  if (kStats) {
#pragma unroll
    for (int q = 0; q < USV_NSTAT; ++q) sums[q] = b.stats[q * nn + ec];
  }
  float u[USV_NU_STEP];
  if (kInj) {
#pragma unroll
    for (int i = 0; i < USV_NU_STEP; ++i) u[i] = inj[(size_t)ec * USV_NU_STEP + i];
  } else {
    philox_u4(seed, (uint32_t)e, step, 0u, u);
    if (c.pos_noise_on || c.act_noise_on) philox_u4(seed, (uint32_t)e, step, 1u, u + 4);
    else u[4] = u[5] = u[6] = u[7] = 0.f;
  }
  // ---- VecEnvRLGames.step clamp + pre_physics_step (USV_Virtual.py:1050-1099) ----
  const float cmd0 = clampt(a2.x, -c.clip_actions, c.clip_actions);
  const float cmd1 = clampt(a2.y, -c.clip_actions, c.clip_actions);
  const float prev_cmd0 = was_reset ? 0.f : cmd0, prev_cmd1 = was_reset ? 0.f : cmd1;
  float t0 = cmd0, t1 = cmd1;
  if (bias != 0.f) { t0 = t0 + bias; t1 = t1 + bias; }
  if (c.act_noise_on) {
    t0 = t0 + (u[SU_ACT] * K.act_rng + c.act_noise_min);
    t1 = t1 + (u[SU_ACT + 1] * K.act_rng + c.act_noise_min);
  }
  t0 = clampt(t0, -1.f, 1.f);
  t1 = clampt(t1, -1.f, 1.f);
  float unit0 = c.affine_thrust ? 0.5f * (t0 + 1.0f) : clampt(t0, 0.f, 1.f);
  float unit1 = c.affine_thrust ? 0.5f * (t1 + 1.0f) : clampt(t1, 0.f, 1.f);
  unit0 = clampt(unit0, 0.f, 1.f);
  unit1 = clampt(unit1, 0.f, 1.f);
  const float uu0 = was_reset ? 0.f : unit0, uu1 = was_reset ? 0.f : unit1;
  int i0 = (int)rintf(((uu0 + 1.0f) / 2.0f) * (float)(USV_LUT_N - 1));
  int i1 = (int)rintf(((uu1 + 1.0f) / 2.0f) * (float)(USV_LUT_N - 1));
  i0 = min(max(i0, 0), USV_LUT_N - 1);
  i1 = min(max(i1, 0), USV_LUT_N - 1);
  float tgt0 = lut[i0], tgt1 = lut[USV_LUT_N + i1];
  if (c.use_thr_mult) { tgt0 = tgt0 * thr_l; tgt1 = tgt1 * thr_r; }
  // ---- substeps: the CaptureXY step's integrator (thruster lag, planar forces, semi-implicit Euler) ----
  const float izz = c.izz0 * k_iz;
  const float inv_m = 1.0f / m, inv_izz = 1.0f / izz;
  const float kd = c.use_drag_scale ? k_drag : 1.0f;
  const float al = c.thr_alpha, oma = 1.0f - c.thr_alpha;
  const float dt = c.dt;
  const float arm_l = -(c.thr_y - comy), arm_r = c.thr_y + comy;
  for (int s = 0; s < c.substeps; ++s) {
    fl = fl * al + oma * tgt0;
    fr = fr * al + oma * tgt1;
    const QuatRot qr = usv_quat_rot(yaw);   // R = quaternion_to_matrix(q(yaw)), as the CaptureXY step
    const float sy_ = qr.S, cy_ = qr.C;
    float ub = cy_ * vx + sy_ * vy;
    float vb = -sy_ * vx + cy_ * vy;
    float rb = wz;
    float hpx = px, hpy = py;
    if (has_dist && c.current_on) {
      ub = ub - (cy_ * c.flow_vel[0] + sy_ * c.flow_vel[1]);
      vb = vb - (-sy_ * c.flow_vel[0] + cy_ * c.flow_vel[1]);
    }
    if (s == 0 && stl) { ub = st_ub; vb = st_vb; rb = st_rb; hpx = st_px; hpy = st_py; }
    float dfx = 0.f, dfy = 0.f, dtz = 0.f;
    if (has_dist) {
      const float wx = hpx + orgx, wy = hpy + orgy;
      dfx = dp[DI_FCX];
      dfy = dp[DI_FCY];
      dtz = dp[DI_TC];
      if (c.fsin_on) {
        dfx = dfx + usv_sin_cr(wx * dp[DI_FXF] + dp[DI_FXS]) * dp[DI_FAMP];
        dfy = dfy + usv_sin_cr(wy * dp[DI_FYF] + dp[DI_FYS]) * dp[DI_FAMP];
      }
      if (c.tsin_on) dtz = dtz + usv_sin_cr((wx + wy) * dp[DI_TF] + dp[DI_TS]) * dp[DI_TAMP];
    }
    float D0 = lin0 + qd0 * fabsf(ub), D1 = lin1 + qd1 * fabsf(vb), D2 = lin2 + qd2 * fabsf(rb);
    D0 = D0 * c.scaling_damping; D1 = D1 * c.scaling_damping; D2 = D2 * c.scaling_damping;
    if (c.use_drag_scale) { D0 = D0 * kd; D1 = D1 * kd; D2 = D2 * kd; }
    const float X = has_dist ? fl + fr + (dfx + (-D0 * ub)) : fl + fr + (-D0 * ub);
    const float Y = has_dist ? dfy + (-D1 * vb) : -D1 * vb;
    const float N = has_dist ? arm_l * fl + arm_r * fr + (dtz + (-D2 * rb)) : arm_l * fl + arm_r * fr + (-D2 * rb);
    const float ax = div_rn(cy_ * X - sy_ * Y, m, inv_m);
    const float ay = div_rn(sy_ * X + cy_ * Y, m, inv_m);
    const float aw = div_rn(N, izz, inv_izz);
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
  if (mine) {
    b.px[e] = px; b.py[e] = py; b.yaw[e] = yaw; b.vx[e] = vx; b.vy[e] = vy; b.wz[e] = wz;
    b.fl[e] = fl; b.fr[e] = fr;
  }
  {   // the rest of the step reads its config afresh (see StepCfg)
  const StepCfg ck2 = step_cfg_reload();
  const usv_cfg_t &c = ck2.c;
  const StepK &K = ck2.K;
  // ---- post_physics_step: progress, update_state noise (USV_Virtual.py:771-813) ----
  const int progress = progress0 + 1;
  float pxn = px, pyn = py;
  if (c.pos_noise_on) {
    pxn = pxn + (u[SU_PX] * K.pos_rng + c.pos_noise_min);
    pyn = pyn + (u[SU_PX + 1] * K.pos_rng + c.pos_noise_min);
  }
  float vxn = vx, vyn = vy, wzn = wz;
  if (c.vel_noise_on) {
    vxn = vxn + (u[SU_VX] * K.vel_rng + c.vel_noise_min);
    vyn = vyn + (u[SU_VY] * K.vel_rng + c.vel_noise_min);
    wzn = wzn + (u[SU_WZ] * K.vel_rng + c.vel_noise_min);
  }
  float yawn = usv_heading(usv_quat_rot(yaw));   // update_state's heading (USV_Virtual.py:776-786)
  if (c.head_noise_on) yawn = yawn + (u[SU_HEAD] * K.head_rng + c.head_noise_min);
  float hs, hc;
  usv_sincos(yawn, &hs, &hc);
  // ---- Core.update_observation_tensor (USV_core.py:55-121) ----
  if (c.obs_local) {
    put(0, hc * vxn + hs * vyn);
    put(1, -hs * vxn + hc * vyn);
  } else {
    put(0, vxn);
    put(1, vyn);
  }
  put(2, wzn);
#pragma unroll
  for (int q = 3; q < USV_NOBS - 10; ++q) obs[q] = 0.f;   // task_data columns no task writes
  const int pa = USV_NOBS_BASE - 2;
  if (c.priv_dim == 4) { obs[29] = 0.f; obs[30] = 0.f; obs[31] = 0.f; obs[32] = 0.f; }   // input padding
  put(pa, prev_cmd0);
  put(pa + 1, prev_cmd1);
  write_priv_tail(c, K, m, comx, comy, comz, k_drag, thr_l, thr_r, k_iz, put);
  {
  const StepCfg ck3 = step_cfg_reload();
  const usv_cfg_t &c = ck3.c;
  const StepK &K = ck3.K;
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
  const float pen_sum = ((p_lin + p_ang) + p_angv) + p_en;
  const int tout = progress >= c.max_episode_length - 1;
  float t_add[4];
  float overall = 0.f;
  int goal_cnt = goal_cnt0, die = 0;
  if (kKind == USV_TASK_GO_TO_POSE) {
    // GoToPoseTask.get_state_observations (:89-130)
    const float ex = tgx - pxn, ey = tgy - pyn;
    const float theta = usv_atan2(hs, hc);
    const float beta = usv_atan2(ey, ex);
    const float alpha = fmodf((beta - theta) + USV_PI_F, USV_2PI_F) - USV_PI_F;
    const float hraw = fmodf((tgh - theta) + USV_PI_F, USV_2PI_F) - USV_PI_F;
    float shr, chr;
    usv_sincos(hraw, &shr, &chr);
    const float herr = usv_atan2(shr, chr);
    float sa, ca, sh, ch;
    usv_sincos(alpha, &sa, &ca);
    usv_sincos(herr, &sh, &ch);
    put(3, ca);
    put(4, sa);
    put(5, tnorm2(ex, ey));
    put(6, ch);
    put(7, sh);
    // compute_reward (:134-181)
    const float pdist = sqrtf(ex * ex + ey * ey);
    const float hdist = fabsf(herr);
    const float prog_r = 2.0f * clampt(prev_pd - pdist, -2.0f, 2.0f);
    if (mine) b.prev_dist[e] = pdist;
    const float speed = tnorm2(vxn, vyn);
    const int gir = (pdist < c.position_tolerance) & (speed < 0.1f);
    goal_cnt = goal_cnt0 * gir + gir;
    // GoToPoseReward.compute_reward (USV_task_rewards.py:190-233)
    const float hw = 1.0f - 1.0f / (1.0f + usv_exp(-c.sig_gain * (pdist - 2.0f)));
    const float pos_r = c.tk_scale[0] * task_term(c.tk_mode[0], pdist, c.tk_coeff[0]);
    const float head_r = hw * c.tk_scale[1] * task_term(c.tk_mode[1], hdist, c.tk_coeff[1]);
    const float act_pen = -0.05f * (fabsf(cmd0) + fabsf(cmd1));
    overall = (((pos_r + head_r) + prog_r) + 2.0f * (float)gir) + act_pen;
    // update_kills (:183-209): kill_dist (the curriculum's at the step after calculate_metrics) / goal counter
    const float kd = c.curriculum_on ? (float)curriculum_lerp(c, ref_step_of(c, b, step, 5), c.cur_kill_dist,
                                                              c.kill_dist_d)
                                     : c.kill_dist;
    die = (pdist > kd) || (goal_cnt >= c.kill_after_n);
    t_add[0] = pos_r; t_add[1] = head_r; t_add[2] = pdist; t_add[3] = speed;   // update_statistics (:211-219)
  } else {
    // TrackXYOVelocityTask.get_state_observations (:75-101)
    const float lex = tgx - vxn, ley = tgy - vyn, aerr = tgh - wzn;
    put(3, lex);
    put(4, ley);
    put(5, aerr);
    // compute_reward (:103-141): the angular part waits for the all-env sum
    const float pos_d = sqrtf(pxn * pxn + pyn * pyn);
    const float lin_d = sqrtf(lex * lex + ley * ley);
    const float lin_r = task_term(c.tk_mode[0], lin_d, c.tk_coeff[0]) * c.tk_scale[0];
    float part = mine ? aerr * aerr : 0.f;
    part = wave_sum(part);
    if ((tid & 63) == 0) sred[tid >> 6] = part;
    float *ts = b.task_scratch;
    if (mine) {
      ts[USV_TS_LIN_REW * nn + e] = lin_r;
      ts[USV_TS_PEN * nn + e] = pen_sum;
      ts[USV_TS_LIN_OK * nn + e] = (float)(lin_d < c.tk_tol[0]);
      ts[USV_TS_POS_KILL * nn + e] = (float)(pos_d > c.kill_dist);
    }
    t_add[0] = lin_r; t_add[1] = lin_d; t_add[2] = 0.f; t_add[3] = 0.f;
  }
  if (mine) {
    b.progress[e] = progress;
    b.prev_cmd[e] = prev_cmd0;
    b.prev_cmd[nn + e] = prev_cmd1;
    b.prev_wz[e] = wzn;
    b.just_reset[e] = 0;
    if (kKind == USV_TASK_GO_TO_POSE) {
      const float rew = overall + pen_sum;
      const int rb = c.fixed_horizon_eval ? tout : (tout ? 1 : die);
      b.goal_cnt[e] = goal_cnt;
      b.rew[e] = rew;
      b.reset_buf[e] = rb;
      b.dones[e] = rb;
    }
    if (kStats) {
      const float vn = tnorm2(vxn, vyn);
      float add[USV_NSTAT];
#pragma unroll
      for (int q = 0; q < USV_NSTAT; ++q) add[q] = 0.f;
      add[0] = t_add[0]; add[1] = t_add[1]; add[2] = t_add[2]; add[3] = t_add[3];
      add[ST_ANGULAR_VEL_PENALTY] = p_ang;
      add[ST_ANGULAR_VEL_VARIATION_PENALTY] = p_angv;
      add[ST_ENERGY_PENALTY] = p_en;
      add[ST_NORMED_LINEAR_VEL] = vn;
      add[ST_NORMED_ANGULAR_VEL] = fabsf(wzn);
      add[ST_CMD_NEG_RATE] = ((float)(t0 < 0.f) + (float)(t1 < 0.f)) / 2.0f;
      add[ST_U_MEAN] = (unit0 + unit1) / 2.0f;
      add[ST_U_LOW_RATE] = ((float)(unit0 < 0.05f) + (float)(unit1 < 0.05f)) / 2.0f;
      add[ST_U_SUM] = unit0 + unit1;
#pragma unroll
      for (int q = 0; q < USV_NSTAT; ++q)
        if (q != ST_SUCCESS && q != ST_COLLISION && (kKind == USV_TASK_GO_TO_POSE || (q != 2 && q != 3)))
          b.stats[q * nn + e] = sums[q] + add[q];
    }
  }
  __syncthreads();
  if (kKind == USV_TASK_TRACK_XYO && tid == 0) {
    float sblk = 0.f;
#pragma unroll
    for (int w = 0; w < kBlock / 64; ++w) sblk += sred[w];
    b.task_scratch[USV_TS_ROWS * nn + blockIdx.x] = sblk;
  }
  // ---- coalesced obs store ----
  const int row0 = blockIdx.x * kBlock;
  const int rows = min(kBlock, n - row0);
  float *ob = b.obs + (size_t)row0 * USV_NOBS;
  uint32_t obad = 0u;
  for (int i = tid; i < rows * USV_NOBS; i += kBlock) {
    obad |= (uint32_t)(sobs[i] != sobs[i]);
    ob[i] = sobs[i];
  }
  if (c.nan_probe) {   // clamped actions, the observed state, the reward (TrackXYO: k_track_finish), obs
    uint32_t bits = ((nonfinite(cmd0) | nonfinite(cmd1)) ? USV_NAN_ACTIONS : 0u) |
                    ((nonfinite(pxn) | nonfinite(pyn) | nonfinite(yawn) | nonfinite(vxn) | nonfinite(vyn) |
                      nonfinite(wzn)) ? USV_NAN_STATE : 0u) |
                    ((kKind == USV_TASK_GO_TO_POSE && nonfinite(overall + pen_sum)) ? USV_NAN_REWARD : 0u);
    nan_report(&b.ctl[USV_CTL_NAN_FLAG], (mine ? bits : 0u) | (obad ? USV_NAN_OBS : 0u));
  }
  if (blockIdx.x == 0 && tid == 0) b.ctl[USV_CTL_STEPPED] = 1;
  }
  }
}

// TrackXYOVelocity, phase 2: angular velocity distance over all envs, then the
// angular reward, goal counter, kills and dones of every env (:103-166)
template <bool kStats>
__global__ __launch_bounds__(kBlock) void k_track_finish(usv_cfg_t c, usv_bufs_t b, int nblk) {
  __shared__ float sred[kBlock];
  const int n = b.n;
  const size_t nn = (size_t)n;
  const int tid = threadIdx.x;
  const float *part = b.task_scratch + USV_TS_ROWS * nn;
  float acc = 0.f;
  for (int i = tid; i < nblk; i += kBlock) acc += part[i];   // fixed order: every block gets the same sum
  sred[tid] = acc;
  __syncthreads();
  for (int w = kBlock / 2; w > 0; w >>= 1) {
    if (tid < w) sred[tid] += sred[tid + w];
    __syncthreads();
  }
  const float ang_d = sqrtf(sred[0]);
  const int e = blockIdx.x * kBlock + tid;
  if (c.nan_probe) {   // the reward of every env (one wave-uniform probe ahead of the per-env tail)
    const int ec = min(e, n - 1);
    const float *ts = b.task_scratch;
    const float ang_r = task_term(c.tk_mode[1], ang_d, c.tk_coeff[1]) * c.tk_scale[1];
    const float rew = (ts[USV_TS_LIN_REW * nn + ec] + ang_r) + ts[USV_TS_PEN * nn + ec];
    nan_report(&b.ctl[USV_CTL_NAN_FLAG], (e < n && nonfinite(rew)) ? USV_NAN_REWARD : 0u);
  }
  if (e >= n) return;
  const float *ts = b.task_scratch;
  const int ang_ok = ang_d < c.tk_tol[1];
  const int gir = (int)ts[USV_TS_LIN_OK * nn + e] * ang_ok;
  const int goal_cnt = b.goal_cnt[e] * gir + gir;
  const float ang_r = task_term(c.tk_mode[1], ang_d, c.tk_coeff[1]) * c.tk_scale[1];
  const float rew = (ts[USV_TS_LIN_REW * nn + e] + ang_r) + ts[USV_TS_PEN * nn + e];
  const int die = (ts[USV_TS_POS_KILL * nn + e] != 0.f) || (goal_cnt > c.kill_after_n);
  const int tout = b.progress[e] >= c.max_episode_length - 1;
  const int rb = c.fixed_horizon_eval ? tout : (tout ? 1 : die);
  b.goal_cnt[e] = goal_cnt;
  b.rew[e] = rew;
  b.reset_buf[e] = rb;
  b.dones[e] = rb;
  if (kStats) {
    b.stats[2 * nn + e] += ang_r;
    b.stats[3 * nn + e] += ang_d;
  }
}

// planar forces only (parity with Hydrodynamics.ComputeHydrodynamicsEffects)
// Hydrostatic wrench (usv_hydrostatics): one thread per env, the reference's operation order.
__global__ void k_hydrostatics(usv_hydro_t h, int n, const float *__restrict__ quat, const float *__restrict__ root_z,
                               float *__restrict__ volume, float *__restrict__ euler, float *__restrict__ wrench) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const float4 q = reinterpret_cast<const float4 *>(quat)[e];
  const float w = q.x, x = q.y, y = q.z, z = q.w;
  // USVVirtual.update_state (USV_Virtual.py:791-798)
  const float high = clampt(h.zero_height - root_z[e], 0.f, h.zero_height + 20.0f);
  const float vol = clampt(high * h.waterplane_area, 0.f, h.max_volume);
  // get_euler_angles (:815-835): the rotation-matrix entries as the reference forms them
  const float r00 = 1.0f - 2.0f * (y * y) - 2.0f * (z * z);
  const float r10 = 2.0f * x * y + 2.0f * w * z;
  const float r20 = 2.0f * x * z - 2.0f * w * y;
  const float r21 = 2.0f * y * z + 2.0f * w * x;
  const float r22 = 1.0f - 2.0f * (x * x) - 2.0f * (y * y);
  const float roll = atan2f(r21, r22), pitch = asinf(-r20), yaw = atan2f(r10, r00);
  // compute_archimedes_metacentric_global (Hydrostatics.py:63-98); the Python scalars fold first
  const float fz = (-h.water_density * h.gravity) * vol;
  const float tx = (-1.0f * h.metacentric_width) * (sinf(roll) * h.avg_force);
  const float ty = (-1.0f * h.metacentric_length) * (sinf(pitch) * h.avg_force);
  // _local (:100-133): R = quaternion_to_matrix(q) (pytorch3d, real first); F_local = R^T (0, 0, fz)
  const float two_s = 2.0f / (((w * w + x * x) + y * y) + z * z);
  const float R20 = two_s * (x * z - y * w), R21 = two_s * (y * z + x * w), R22 = 1.0f - two_s * (x * x + y * y);
  float *out = wrench + (size_t)e * 6;
  out[0] = R20 * fz;
  out[1] = R21 * fz;
  out[2] = R22 * fz;
  out[3] = tx * h.amplify_torque;   // torque not rotated (:123)
  out[4] = ty * h.amplify_torque;
  out[5] = 0.0f * h.amplify_torque;
  volume[e] = vol;
  euler[(size_t)e * 3 + 0] = roll;
  euler[(size_t)e * 3 + 1] = pitch;
  euler[(size_t)e * 3 + 2] = yaw;
}

__global__ void k_forces(usv_cfg_t c, usv_bufs_t b, float *__restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = b.n;
  if (e >= n) return;
  const QuatRot qr = usv_quat_rot(b.yaw[e]);   // R = quaternion_to_matrix(q(yaw)) (Hydrodynamics.py:209-217)
  const float sy_ = qr.S, cy_ = qr.C;
  const float vx = b.vx[e], vy = b.vy[e], wz = b.wz[e];
  float ub = cy_ * vx + sy_ * vy, vb = -sy_ * vx + cy_ * vy;
  if (c.current_on) {   // relative to the water (Hydrodynamics.py:224-237)
    ub = ub - (cy_ * c.flow_vel[0] + sy_ * c.flow_vel[1]);
    vb = vb - (-sy_ * c.flow_vel[0] + cy_ * c.flow_vel[1]);
  }
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

// ---- host side of the step launch ----
// byte offsets of the step kernel's per-env arrays inside one window; status 2 when
// they span 2 GiB or more (allocate them from one slab, as tasks/usv_virtual.py does)
int step_window(const usv_cfg_t &c, const usv_bufs_t &b, const char **base, StepWin *w) {
  const size_t n = (size_t)b.n, f = n * 4;
  struct Arr {
    const void *p;
    size_t bytes;
    uint32_t *off;
    bool required;
  };
  const Arr arr[] = {
      {b.px, f, &w->px, true}, {b.py, f, &w->py, true}, {b.yaw, f, &w->yaw, true}, {b.vx, f, &w->vx, true},
      {b.vy, f, &w->vy, true}, {b.wz, f, &w->wz, true}, {b.fl, f, &w->fl, true}, {b.fr, f, &w->fr, true},
      {b.mass, f, &w->mass, true}, {b.k_iz, f, &w->k_iz, true}, {b.k_drag, f, &w->k_drag, true},
      {b.thr_l, f, &w->thr_l, true}, {b.thr_r, f, &w->thr_r, true}, {b.com_x, f, &w->com_x, true},
      {b.com_y, f, &w->com_y, true}, {b.com_z, f, &w->com_z, true}, {b.lin_damp, 3 * f, &w->lin_damp, false},
      {b.lin_damp ? b.quad_damp : nullptr, 3 * f, &w->quad_damp, b.lin_damp != nullptr},
      {b.progress, f, &w->progress, true}, {b.tgt_x, f, &w->tgt_x, true}, {b.tgt_y, f, &w->tgt_y, true},
      {b.obst, 2 * USV_NOBST * f, &w->obst, true}, {b.goal_cnt, f, &w->goal_cnt, true},
      {b.prev_dist, f, &w->prev_dist, true}, {b.prev_head, f, &w->prev_head, true},
      {b.prev_pot, f, &w->prev_pot, true}, {b.prev_wz, f, &w->prev_wz, true},
      {c.stats_on ? b.stats : nullptr, USV_NSTAT * f, &w->stats, c.stats_on != 0},
      {b.prev_cmd, 2 * f, &w->prev_cmd, true}, {b.rew, f, &w->rew, true}, {b.reset_buf, f, &w->reset_buf, true},
      {b.dones, 2 * f, &w->dones, true}, {b.done_coll, f, &w->done_coll, true},
      {b.done_succ, f, &w->done_succ, true}, {b.just_reset, n, &w->just_reset, true},
      {b.obs, USV_NOBS * f, &w->obs, true}, {b.dist, USV_NDIST * f, &w->dist, false},
      {b.dist ? b.env_org : nullptr, 2 * f, &w->env_org, false},
      {c.stale_root ? b.stale : nullptr, USV_STALE_ROWS * f, &w->stale, c.stale_root != 0}};
  uintptr_t lo = UINTPTR_MAX, hi = 0;
  for (const Arr &a : arr) {
    if (!a.p) {
      if (a.required) return 1;
      continue;
    }
    lo = std::min(lo, (uintptr_t)a.p);
    hi = std::max(hi, (uintptr_t)a.p + a.bytes);
  }
  if (hi - lo >= 0x7FFFFFFFull) return 2;
  for (const Arr &a : arr) *a.off = a.p ? (uint32_t)((uintptr_t)a.p - lo) : 0u;
  w->n4 = (uint32_t)f;
  w->bytes = (uint32_t)(hi - lo);
  *base = (const char *)lo;
  return 0;
}

// kShift when every array the step kernel touches sits at its canonical slab row (include/usv_hip.h USV_SLAB_*)
// with 2^kShift-byte rows, 2^kShift the next power of two >= 4 n; -1 otherwise (the general window path)
int fixed_slab_shift(const usv_cfg_t &c, const usv_bufs_t &b) {
  int sh = 8;
  while ((1ull << sh) < 4ull * (unsigned long long)b.n) ++sh;
  if (sh < kFixedShiftMin || sh > kFixedShiftMax || !b.px) return -1;
  const char *base = reinterpret_cast<const char *>(b.px);
  const size_t rb = (size_t)1 << sh;
  struct Row {
    const void *p;
    int row;
    bool required;
  };
  const Row rows[] = {
      {b.px, USV_SLAB_STATE, true}, {b.py, USV_SLAB_STATE + 1, true}, {b.yaw, USV_SLAB_STATE + 2, true},
      {b.vx, USV_SLAB_STATE + 3, true}, {b.vy, USV_SLAB_STATE + 4, true}, {b.wz, USV_SLAB_STATE + 5, true},
      {b.fl, USV_SLAB_STATE + 6, true}, {b.fr, USV_SLAB_STATE + 7, true}, {b.mass, USV_SLAB_PARAMS, true},
      {b.com_x, USV_SLAB_PARAMS + 1, true}, {b.com_y, USV_SLAB_PARAMS + 2, true}, {b.com_z, USV_SLAB_PARAMS + 3, true},
      {b.k_drag, USV_SLAB_PARAMS + 4, true}, {b.thr_l, USV_SLAB_PARAMS + 5, true}, {b.thr_r, USV_SLAB_PARAMS + 6, true},
      {b.k_iz, USV_SLAB_PARAMS + 7, true}, {b.lin_damp, USV_SLAB_LIN_DAMP, false},
      {b.quad_damp, USV_SLAB_QUAD_DAMP, false}, {b.tgt_x, USV_SLAB_TGT, true}, {b.tgt_y, USV_SLAB_TGT + 1, true},
      {b.obst, USV_SLAB_OBST, true}, {b.prev_cmd, USV_SLAB_PREV_CMD, true}, {b.prev_dist, USV_SLAB_HIST, true},
      {b.prev_head, USV_SLAB_HIST + 1, true}, {b.prev_pot, USV_SLAB_HIST + 2, true},
      {b.prev_wz, USV_SLAB_HIST + 3, true}, {b.goal_cnt, USV_SLAB_IBUF, true}, {b.progress, USV_SLAB_IBUF + 1, true},
      {b.reset_buf, USV_SLAB_IBUF + 2, true}, {b.done_succ, USV_SLAB_IBUF + 3, true},
      {b.done_coll, USV_SLAB_IBUF + 4, true}, {b.just_reset, USV_SLAB_JUST_RESET, true},
      {c.stats_on ? b.stats : nullptr, USV_SLAB_STATS, c.stats_on != 0}, {b.obs, USV_SLAB_OBS, true},
      {b.rew, USV_SLAB_REW, true}, {b.dones, USV_SLAB_DONES, true}, {b.dist, USV_SLAB_DIST, false},
      {b.dist ? b.env_org : nullptr, USV_SLAB_ENV_ORG, false},
      {c.stale_root ? b.stale : nullptr, USV_SLAB_STALE, c.stale_root != 0}};
  for (const Row &r : rows) {
    if (!r.p) {
      if (r.required) return -1;
      continue;
    }
    if (reinterpret_cast<const char *>(r.p) != base + (size_t)r.row * rb) return -1;
  }
  return sh;
}

// any per-substep disturbance term on (then usv_bufs_t.dist must be set)
bool step_has_dist(const usv_cfg_t &c) { return c.fdist_on || c.tdist_on || c.current_on; }

float enc_centered_scale(float xmin, float xmax, float nominal) {
  double sc = std::fabs((double)xmin - nominal);
  if (std::fabs((double)xmax - nominal) > sc) sc = std::fabs((double)xmax - nominal);
  if (1e-6 > sc) sc = 1e-6;
  return (float)sc;
}
// host restatements of the reference's privileged-observation encoders (USV_Virtual.py:97-151)
float enc_centered_h(float x, float xmin, float xmax, float nominal) {
  const float s = enc_centered_scale(xmin, xmax, nominal);
  const float z = (x - nominal) / s;
  return z < -1.f ? -1.f : (z > 1.f ? 1.f : z);
}
float enc_minmax_h(float x, float xmin, float xmax) {
  if ((double)xmax - (double)xmin <= 1e-6) return 0.f;
  const float z = (x - xmin) / (float)((double)xmax - (double)xmin);
  const float y = 2.0f * z - 1.0f;
  return y < -1.f ? -1.f : (y > 1.f ? 1.f : y);
}

StepK step_constants(const usv_cfg_t &c) {
  StepK k{};
  k.cell = (float)((double)c.map_size / USV_GRID);
  k.inv_r = (float)(1.0 / (double)c.influence_radius);
  k.inv_safe = 1.0f / c.safe_radius;
  {
    const double cell_d = (double)c.map_size / USV_GRID;
    k.gstart = (float)(-(double)c.map_size / 2 + cell_d / 2);
    k.gend = (float)((double)c.map_size / 2 - cell_d / 2);
    k.gstep = (k.gend - k.gstart) / (float)(USV_GRID - 1);
  }
  k.act_rng = (float)((double)c.act_noise_max - (double)c.act_noise_min);
  k.pos_rng = (float)((double)c.pos_noise_max - (double)c.pos_noise_min);
  k.vel_rng = (float)((double)c.vel_noise_max - (double)c.vel_noise_min);
  k.head_rng = (float)((double)c.head_noise_max - (double)c.head_noise_min);
  k.mass_den = (float)(std::fabs((double)c.base_mass) > 1e-6 ? std::fabs((double)c.base_mass) : 1e-6);
  k.inv_mass_den = 1.0f / k.mass_den;
  for (int i = 0; i < 3; ++i) {
    k.com_div[i] = c.com_scale[i] + 1e-6f;
    k.inv_com_div[i] = 1.0f / k.com_div[i];
  }
  const float lo3[3] = {c.kdrag_min, c.thr_min, c.kiz_min}, hi3[3] = {c.kdrag_max, c.thr_max, c.kiz_max};
  for (int j = 0; j < 3; ++j) {
    k.enc_lo[j] = lo3[j];
    if (c.priv_mode == 1) {
      k.enc_r[j] = enc_centered_scale(lo3[j], hi3[j], c.priv_nominal);
      k.enc_ok[j] = 1;
    } else {
      k.enc_r[j] = (float)((double)hi3[j] - (double)lo3[j]);
      k.enc_ok[j] = ((double)hi3[j] - (double)lo3[j]) > 1e-6;
    }
    k.inv_enc_r[j] = k.enc_r[j] != 0.f ? 1.0f / k.enc_r[j] : 0.f;
  }
  k.inv_exp_coeff = c.exp_coeff != 0.f ? 1.0f / c.exp_coeff : 0.f;
  // privileged values of the "base" source: the same for every env
  float v[8];
  v[0] = c.mass_relative ? 0.f : c.base_mass;
  for (int i = 0; i < 3; ++i) v[1 + i] = c.com_scaled ? c.base_com[i] / (c.com_scale[i] + 1e-6f) : c.base_com[i];
  float kdv = 1.f, tl = 1.f, tr = 1.f, kz = 1.f;
  if (c.priv_mode == 2) {
    kdv = 0.5f * (c.kdrag_min + c.kdrag_max);
    tl = tr = c.couple_thr ? (1.0f - 0.5f * c.thr_rand) : 1.0f;
    kz = 0.5f * (c.kiz_min + c.kiz_max);
  }
  if (c.priv_mode == 1) {
    kdv = enc_centered_h(kdv, c.kdrag_min, c.kdrag_max, c.priv_nominal);
    tl = enc_centered_h(tl, c.thr_min, c.thr_max, c.priv_nominal);
    tr = enc_centered_h(tr, c.thr_min, c.thr_max, c.priv_nominal);
    kz = enc_centered_h(kz, c.kiz_min, c.kiz_max, c.priv_nominal);
  } else if (c.priv_mode == 2) {
    kdv = c.priv_drag_on ? enc_minmax_h(kdv, c.kdrag_min, c.kdrag_max) : 0.f;
    tl = c.priv_thr_on ? enc_minmax_h(tl, c.thr_min, c.thr_max) : 0.f;
    tr = c.priv_thr_on ? enc_minmax_h(tr, c.thr_min, c.thr_max) : 0.f;
    kz = c.priv_kiz_on ? enc_minmax_h(kz, c.kiz_min, c.kiz_max) : 0.f;
  }
  v[4] = kdv; v[5] = tl; v[6] = tr; v[7] = kz;
  for (int i = 0; i < 8; ++i) k.priv_base[i] = v[i];
  return k;
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

int usv_reset_part(const usv_cfg_t *cfg, const usv_bufs_t *b, uint64_t seed, uint64_t step, const float *u_inject,
                   int part, void *stream) {
  if (!cfg || !b || b->n <= 0 || part < 0 || part > 2) return 1;
  if (b->scene && (b->n_scenes <= 0 || !b->scene_next || !b->scene_last || cfg->task_kind != USV_TASK_CAPTURE_XY))
    return 1;
  if (cfg->stale_root && !b->stale) return 1;   // the first substep's cached-state inputs have nowhere to go
  hipStream_t s = (hipStream_t)stream;
  const int grid = (b->n + kBlock - 1) / kBlock;
  if (part != 2) {
    // per-step scratch: reset count, field maxima, extras sums
    hipLaunchKernelGGL(k_step_begin, dim3(1), dim3(64), 0, s, *b, cfg->step_inc);
    USV_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_reset, dim3(grid), dim3(kBlock), 0, s, *cfg, *b, seed, step, u_inject);
    USV_CHECK_LAUNCH();
  }
#if USV_RESET_FOLD_KERNEL
  if (part != 1 && cfg->stats_on) {
    hipLaunchKernelGGL(k_extras_fold, dim3(1), dim3(kBlock), 0, s, *cfg, *b, grid);
    USV_CHECK_LAUNCH();
  }
#endif
  return 0;
}

int usv_reset(const usv_cfg_t *cfg, const usv_bufs_t *b, uint64_t seed, uint64_t step, const float *u_inject,
              void *stream) {
  return usv_reset_part(cfg, b, seed, step, u_inject, 0, stream);
}

int usv_env_step_part(const usv_cfg_t *cfg, const usv_bufs_t *b, const float *actions, const float *lut_dev,
                      float action_bias, uint64_t seed, uint64_t step, const float *u_inject, int part,
                      void *stream) {
  if (!cfg || !b || !actions || !lut_dev || b->n <= 0 || part < 0 || part > 3) return 1;
  if (part == 3 && (cfg->task_kind != USV_TASK_CAPTURE_XY || !b->rstash)) return 1;
  if (cfg->stale_root && !b->stale) return 1;   // a reset env's first substep reads usv_reset's cached inputs
  // CaptureXY samples the potential field from its parts (SDF tiles, cost rows, constants)
  if (cfg->task_kind == USV_TASK_CAPTURE_XY && (!b->field || !b->sdf || !b->fnorm)) return 7;
  if (cfg->priv_dim != 4 && cfg->priv_dim != 8) return 3;
  if (cfg->task_kind != USV_TASK_CAPTURE_XY) {
    // GoToPose / TrackXYOVelocity: no potential field, so no split step
    if (part != 0 || !b->tgt_h) return 1;
    if (step_has_dist(*cfg) && !b->dist) return 4;
    if (cfg->task_kind == USV_TASK_TRACK_XYO && !b->task_scratch) return 1;
    const StepK k = step_constants(*cfg);
    const int grid = (b->n + kBlock - 1) / kBlock;
    hipStream_t s = (hipStream_t)stream;
    const bool st = cfg->stats_on != 0, ij = u_inject != nullptr;
    if (cfg->task_kind == USV_TASK_GO_TO_POSE) {
      auto kern = st ? (ij ? k_env_step_task<USV_TASK_GO_TO_POSE, true, true> : k_env_step_task<USV_TASK_GO_TO_POSE, true, false>)
                     : (ij ? k_env_step_task<USV_TASK_GO_TO_POSE, false, true> : k_env_step_task<USV_TASK_GO_TO_POSE, false, false>);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, s, StepCfg{*cfg, k}, *b, actions, lut_dev, action_bias, seed,
                         step, u_inject);
    } else if (cfg->task_kind == USV_TASK_TRACK_XYO) {
      auto kern = st ? (ij ? k_env_step_task<USV_TASK_TRACK_XYO, true, true> : k_env_step_task<USV_TASK_TRACK_XYO, true, false>)
                     : (ij ? k_env_step_task<USV_TASK_TRACK_XYO, false, true> : k_env_step_task<USV_TASK_TRACK_XYO, false, false>);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, s, StepCfg{*cfg, k}, *b, actions, lut_dev, action_bias, seed,
                         step, u_inject);
      USV_CHECK_LAUNCH();
      hipLaunchKernelGGL(st ? k_track_finish<true> : k_track_finish<false>, dim3(grid), dim3(kBlock), 0, s, *cfg, *b,
                         grid);
    } else {
      return 1;
    }
    USV_CHECK_LAUNCH();
    return 0;
  }
  StepWin w{};
  const char *wbase = nullptr;
  const int rc = step_window(*cfg, *b, &wbase, &w);
  if (rc) return rc;
  const StepK k = step_constants(*cfg);
  const int grid = (b->n + kBlock - 1) / kBlock;
  hipStream_t s = (hipStream_t)stream;
  const bool dist = b->dist != nullptr;
  if (step_has_dist(*cfg) && !dist) return 4;   // a disturbance / water current is on: dist is required
  // the production shape (statistics on, in-kernel draws, no disturbance) on the canonical slab: constant offsets
  const int sh = fixed_slab_shift(*cfg, *b);
  if (sh >= 0 && cfg->stats_on && !u_inject && !dist) {
    const char *base = reinterpret_cast<const char *>(b->px);
#define USV_FIXED_CASE(S)                                                                                            \
  case S:                                                                                                            \
    hipLaunchKernelGGL((k_env_step<true, false, false, FixedWin<S>>), dim3(grid), dim3(kBlock), 0, s,                \
                       StepCfg{*cfg, k}, *b, FixedWin<S>{}, base, actions, lut_dev, action_bias, seed, step, u_inject,  \
                       part);                                                                                        \
    break;
    switch (sh) {
      USV_FIXED_CASE(13) USV_FIXED_CASE(14) USV_FIXED_CASE(15) USV_FIXED_CASE(16) USV_FIXED_CASE(17)
      USV_FIXED_CASE(18) USV_FIXED_CASE(19) USV_FIXED_CASE(20) USV_FIXED_CASE(21) USV_FIXED_CASE(22)
      default: return 6;
    }
#undef USV_FIXED_CASE
    USV_CHECK_LAUNCH();
    return 0;
  }
  auto kern = dist ? (cfg->stats_on ? (u_inject ? k_env_step<true, true, true, StepWin> : k_env_step<true, false, true, StepWin>)
                                    : (u_inject ? k_env_step<false, true, true, StepWin> : k_env_step<false, false, true, StepWin>))
                   : (cfg->stats_on ? (u_inject ? k_env_step<true, true, false, StepWin> : k_env_step<true, false, false, StepWin>)
                                    : (u_inject ? k_env_step<false, true, false, StepWin> : k_env_step<false, false, false, StepWin>));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, s, StepCfg{*cfg, k}, *b, w, wbase, actions, lut_dev, action_bias,
                     seed, step, u_inject, part);
  USV_CHECK_LAUNCH();
  return 0;
}

int usv_env_step_late(const usv_cfg_t *cfg, const usv_bufs_t *b, void *stream) {
  if (!cfg || !b || b->n <= 0 || !b->rstash || !b->field || !b->sdf || !b->fnorm ||
      cfg->task_kind != USV_TASK_CAPTURE_XY)
    return 1;
  // one-wave workgroups striding over the device reset count (~1% of the envs per step at the headline size)
  const int grid = (b->n + 63) / 64 < kLateGrid ? (b->n + 63) / 64 : kLateGrid;
  hipLaunchKernelGGL(k_env_reward_late, dim3(grid), dim3(64), 0, (hipStream_t)stream, *cfg, *b);
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

int usv_hydrostatics(const usv_hydro_t *h, int n, const float *quat, const float *root_z, float *volume,
                     float *euler, float *wrench, void *stream) {
  if (!h || !quat || !root_z || !volume || !euler || !wrench || n <= 0) return 1;
  hipLaunchKernelGGL(k_hydrostatics, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, *h, n, quat, root_z,
                     volume, euler, wrench);
  USV_CHECK_LAUNCH();
  return 0;
}

int usv_hip_version(void) { return 1; }

// Every integer #define, enumerator and ABI struct size / field offset of include/usv_hip.h (the generated
// list csrc/usv_layout_gen.h, in header order), folded with its name: see _abi.layout_key_of.
static unsigned long long fnv1a(const char *s) {
  unsigned long long h = 1469598103934665603ull;
  for (; *s; ++s) h = (h ^ (unsigned char)*s) * 1099511628211ull;
  return h;
}
long long usv_hip_layout_key(void) {
  unsigned long long k = 0;
#define USV_LAYOUT_FOLD(expr, name)                                    \
  k = k * 1000003ull + fnv1a(name);                                    \
  k = k * 1000003ull + (unsigned long long)(long long)(expr);
  USV_LAYOUT_ENTRIES(USV_LAYOUT_FOLD)
#undef USV_LAYOUT_FOLD
  return (long long)(k & 0x7fffffffffffffffull);
}

}  // extern "C"
