// Device-side helpers shared by the env and PPO kernels (gfx950 / CDNA4).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/usv_hip.h"

#define USV_PI_F 3.14159265358979323846f
#define USV_2PI_F 6.28318530717958647692f

// ---------------------------------------------------------------------------
// Philox4x32-10 (counter-based RNG; Salmon et al. SC'11).  Every in-kernel
// draw is Philox(key = seed, ctr = {env, step_lo, step_hi, site + i/4})[i%4],
// so a draw depends only on (seed, env, step, site, i): no RNG state in HBM.
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox4x32_10(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// 4 uniforms of block `blk` of a (seed, env, step, site) stream
__device__ __forceinline__ void philox_u4(uint64_t seed, uint32_t env, uint64_t step, uint32_t site_blk,
                                          float out[4]) {
  const u32x4 r = philox4x32_10(u32x4{env, (uint32_t)step, (uint32_t)(step >> 32), site_blk}, (uint32_t)seed,
                                (uint32_t)(seed >> 32));
  out[0] = u01(r.x); out[1] = u01(r.y); out[2] = u01(r.z); out[3] = u01(r.w);
}

// index of texel (r, c) of an env's potential field in the tiled layout (include/usv_hip.h USV_FIELD_STRIDE)
static_assert(USV_FIELD_STRIDE >= USV_FIELD_TROWS * USV_FIELD_TCOLS * USV_FIELD_TH * USV_FIELD_TW &&
              USV_FIELD_STRIDE % 32 == 0, "field stride: every tile, whole 128-B lines");
__host__ __device__ __forceinline__ int field_idx(int r, int c) {
  const unsigned ur = (unsigned)r, uc = (unsigned)c;   // r, c >= 0: constant divisions become multiplies
  return (int)(((ur / USV_FIELD_TH) * USV_FIELD_TCOLS + uc / USV_FIELD_TW) * (USV_FIELD_TH * USV_FIELD_TW) +
               (ur % USV_FIELD_TH) * USV_FIELD_TW + uc % USV_FIELD_TW);
}

__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
// torch's clamp/max/min propagate NaN differently from fminf/fmaxf; inputs here are finite.
__device__ __forceinline__ float maxf(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float minf(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float clampt(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

// torch.norm(v, dim=-1) of a 2-vector == sqrt(fma(y, y, x*x)) (PyTorch CPU reduction)
__device__ __forceinline__ float tnorm2(float x, float y) { return sqrtf(fmaf(y, y, x * x)); }
// x / b given y = RN(1/b): Markstein's correction (q = x*y, r = x - b*q exactly by fma,
// q + r*y).  Equals the IEEE quotient whenever it lies in [2^-90, 2^120] (checked
// exhaustively over every float x for each constant divisor used, and over random
// divisors; below that range r underflows and the result may be 1 ulp off).
__device__ __forceinline__ float div_rn(float x, float b, float y) {
  const float q = x * y;
  const float r = fmaf(-q, b, x);
  return fmaf(r, y, q);
}

// sin and cos of the integrator's angles (yaw, spawn and disturbance phases): this build's own definition (the
// reference's PhysX step has none), restated operation for operation by the C oracle
// (oracle/usv_oracle.c:usv_sincos), so the device and the oracle integrate the same bits.  Reduction by pi/2 in
// three Cody-Waite parts (k * part exact for |k| < 2^13), Cephes' single-precision minimax polynomials on
// [-pi/4, pi/4]; plain IEEE multiplies and adds (the library is built with -ffp-contract=off)
__device__ __forceinline__ void usv_sincos(float x, float *s, float *c) {
  const float k = rintf(x * 0.63661977236758134f);
  float r = x - k * 1.5703125f;
  r = r - k * 4.837512969970703125e-4f;
  r = r - k * 7.54978995489188216e-8f;
  const float z = r * r;
  const float sp = r + r * z * (-1.6666654611e-1f + z * (8.3321608736e-3f + z * -1.9515295891e-4f));
  const float cp = 1.0f - 0.5f * z + z * z * (4.166664568298827e-2f + z * (-1.388731625493765e-3f +
                                                                            z * 2.443315711809948e-5f));
  const int q = (int)k & 3;
  const float sa = (q & 1) ? cp : sp, ca = (q & 1) ? sp : cp;
  *s = (q & 2) ? -sa : sa;
  *c = ((q + 1) & 2) ? -ca : ca;
}
__device__ __forceinline__ float usv_sin(float x) {
  float s, c;
  usv_sincos(x, &s, &c);
  return s;
}
// The rigid body's attitude as the reference reads it back: PhysX's yaw-only quaternion q = (w, 0, 0, z) =
// (cos(yaw/2), 0, 0, sin(yaw/2)) (this build's stand-in for the integrator's pose, usv_sincos of yaw / 2), and
// pytorch3d.transforms.quaternion_to_matrix of it (two_s = 2 / sum(q * q); the reference's drag,
// Hydrodynamics.py:209-217) -- R = [[C, -S, 0], [S, C, 0], [0, 0, 1]] with C = 1 - two_s z^2, S = two_s (z w), the
// x = y = 0 terms exact.  getLocalLinearVelocities (Utils.py:10-14, torch.bmm's CPU order: (r0 vx + r1 vy) + r2 vz,
// no fma) then gives R^T v = (C vx + S vy, -S vx + C vy); the integrator rotates the body-frame wrench with the same
// R (its own definition, the PhysX step's), so one half-angle sincos per substep serves both
struct QuatRot { float C, S, w, z; };
__device__ __forceinline__ QuatRot usv_quat_rot(float yaw) {
  float z, w;
  usv_sincos(yaw * 0.5f, &z, &w);
  // (q * q).sum(-1) of (w, 0, 0, z); torch's 2.0 / t is reciprocal * 2, the same bits as the IEEE quotient.  Round
  // 6 measured two division-free forms of it (a Markstein correction with a fallback branch: +0.75 us per env step;
  // an exact branch-free form on the window s lies in: +0.17 us; profiles/r06/r06e_two_s_ab.txt, r06h_two_s_ab.txt)
  const float two_s = 2.0f / (w * w + z * z);
  return QuatRot{1.0f - two_s * (z * z), two_s * (z * w), w, z};
}
// exp, tanh and atan2 of the observation / reward formulas, by the same rule (oracle/usv_oracle.c restates them):
// Cephes' single-precision reductions and minimax polynomials in plain IEEE multiplies, adds and divisions, the
// power of two by ldexpf (exact).  Within 2 ulp of float64 libm on the ranges the step uses (CPU tests).
__device__ __forceinline__ float usv_exp(float x) {
  if (x != x) return x;
  if (x > 88.72283f) return INFINITY;
  if (x < -103.97208f) return 0.f;
  const float k = rintf(x * 1.44269504088896341f);
  float r = x - k * 0.693359375f;
  r = r - k * -2.12194440e-4f;
  const float z = r * r;
  float p = 1.9875691500e-4f;
  p = p * r + 1.3981999507e-3f;
  p = p * r + 8.3334519073e-3f;
  p = p * r + 4.1665795894e-2f;
  p = p * r + 1.6666665459e-1f;
  p = p * r + 5.0000001201e-1f;
  p = p * z + r + 1.0f;
  return ldexpf(p, (int)k);
}
__device__ __forceinline__ float usv_tanh(float x) {
  const float ax = fabsf(x);
  float y;
  if (ax < 0.625f) {
    const float z = x * x;
    y = ((((-5.70498872745e-3f * z + 2.06390887954e-2f) * z - 5.37397155531e-2f) * z + 1.33314422036e-1f) * z -
         3.33332819422e-1f) * z * x + x;
  } else {
    y = ax > 9.0f ? 1.0f : 1.0f - 2.0f / (usv_exp(ax + ax) + 1.0f);
    y = copysignf(y, x);
  }
  return y;
}
__device__ __forceinline__ float usv_atan2(float y, float x) {
  if (x != x || y != y) return x + y;
  const float ax = fabsf(x), ay = fabsf(y);
  float r;
  if (ax == 0.f && ay == 0.f) {
    r = signbit(x) ? 3.14159265358979323846f : 0.f;
  } else {
    const float a = ay / ax;   // +inf where x = 0
    float t, base, blo;       // base = hi + lo parts of 0, pi / 4, pi / 2
    if (a > 2.414213562373095f) { t = -1.0f / a; base = 1.57079637f; blo = -4.371139e-08f; }
    else if (a > 0.4142135623730950f) { t = (a - 1.0f) / (a + 1.0f); base = 0.785398185f; blo = -2.1855694e-08f; }
    else { t = a; base = 0.f; blo = 0.f; }
    const float z = t * t;
    r = base + (((((8.05374449538e-2f * z - 1.38776856032e-1f) * z + 1.99777106478e-1f) * z - 3.33329491539e-1f) *
                 z * t + t) + blo);
    if (signbit(x)) r = (3.14159274f - r) + -8.742278e-08f;
  }
  return copysignf(r, y);
}
// update_state's heading (USV_Virtual.py:776-786): arctan2(2 (w z + x y), 1 - 2 (y^2 + z^2)) of the read-back
// quaternion (usv_quat_rot's), x = y = 0 terms exact
__device__ __forceinline__ float usv_heading(const QuatRot &q) {
  return usv_atan2(2.0f * (q.w * q.z), 1.0f - 2.0f * (q.z * q.z));
}
// the stand-in's pose from a quaternion set_world_poses receives (w, 0, 0, z): yaw = 2 atan2(z, w)
__device__ __forceinline__ float usv_yaw_of_quat(float w, float z) { return 2.0f * usv_atan2(z, w); }

// sin and cos where the reference itself calls torch.sin / torch.cos on the state path: spawn positions and
// quaternions (static_obs.py:955-961, USV_go_to_pose.py:307-318, USV_track_xyo_velocity.py:217-218, scene replay
// USV_Virtual.py:1447-1450), the constant disturbance direction and the disturbance sinusoids
// (USV_disturbances.py:369-410, 510-530) and the legacy CoM disk (:121-122).  torch's CPU kernels there are MKL
// VML HA (within 0.6 ulp: the correctly rounded value for ~95% of arguments), so this is the double-precision
// value rounded to float: Cody-Waite reduction by pi/2 in three parts (P1, P2 30-bit: k P exact for |k| < 2^23,
// i.e. every float phase below ~1.3e7, the largest env origin x frequency the step forms), fdlibm's kernel
// polynomials.  Plain IEEE double operations (-ffp-contract=off), restated by oracle/usv_oracle.c:usv_sincos_cr,
// so the device and the oracle round the same double.
__host__ __device__ __forceinline__ void usv_sincos_cr(float xf, float *s, float *c) {
  const double x = (double)xf;
  const double k = rint(x * 0x1.45f306dc9c883p-1);
  double r = x - k * 0x1.921fb54p+0;            // P1 = pi/2 to 30 bits
  r = r - k * 0x1.10b46118p-30;               // P2: the next 30 bits
  r = r - k * 0x1.313198a2e037p-61;           // P3: the rest, rounded
  const double z = r * r;
  const double sp = r + (z * r) * (-1.66666666666666324348e-01 +
                                   z * (8.33333333332248946124e-03 +
                                        z * (-1.98412698298579493134e-04 +
                                             z * (2.75573137070700676789e-06 +
                                                  z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)))));
  const double cr = z * (4.16666666666666019037e-02 +
                         z * (-1.38888888888741095749e-03 +
                              z * (2.48015872894767294178e-05 +
                                   z * (-2.75573143513906633035e-07 +
                                        z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
  const double cp = 1.0 - (0.5 * z - z * cr);
  const int q = (int)(long long)k & 3;
  const double sa = (q & 1) ? cp : sp, ca = (q & 1) ? sp : cp;
  *s = (float)((q & 2) ? -sa : sa);
  *c = (float)(((q + 1) & 2) ? -ca : ca);
}
__host__ __device__ __forceinline__ float usv_sin_cr(float x) {
  float s, c;
  usv_sincos_cr(x, &s, &c);
  return s;
}

// cell centre i of the potential field's grid (BatchedMapGPU's torch.linspace of the cell centres,
// d_multi_gemini.py:40-48), or the override table (parity tests)
__device__ __forceinline__ float grid_coord_k(float start, float end, float step, int i) {
  return (i < USV_GRID / 2) ? start + step * (float)i : end - step * (float)(USV_GRID - i - 1);
}
__device__ __forceinline__ float grid_coord(const float *lin, float map_size, int i) {
  if (lin) return lin[i];
  const double cell_d = (double)map_size / USV_GRID;
  const float start = (float)(-(double)map_size / 2 + cell_d / 2);
  const float end = (float)((double)map_size / 2 - cell_d / 2);
  const float step = (end - start) / (float)(USV_GRID - 1);
  return grid_coord_k(start, end, step, i);
}
// compute_occupancy_and_sdf (d_multi_gemini.py:66-104) for one cell, ob(o) -> the centre of obstacle o: min
// over the 16 obstacles of the squared distance (dx*dx rounded, then fma with dy), sqrt, minus the radius --
// k_field_stats' separable SDF forms the same operations per cell, so the bits are the same.  Squared
// distances are >= 0: float order == u32 order (balanced min tree).
template <class Ob>
__device__ __forceinline__ float cell_sdf(Ob ob, float gx, float gy, float radius) {
  uint32_t a[USV_NOBST];
#pragma unroll
  for (int o = 0; o < USV_NOBST; ++o) {
    const float2 p = ob(o);
    const float dx = gx - p.x, dy = gy - p.y;
    a[o] = __float_as_uint(fmaf(dy, dy, dx * dx));
  }
#pragma unroll
  for (int w = USV_NOBST / 2; w >= 1; w >>= 1)
#pragma unroll
    for (int o = 0; o < w; ++o) a[o] = min(a[o], a[o + w]);
  return sqrtf(__uint_as_float(a[0])) - radius;   // sqrt(min) == min(sqrt), bit-exact
}

// ---- the potential field's texel value (BatchedMapGPU.compute_potential_field, d_multi_gemini.py:195-271) ----
// The field is kept as its parts: the raw cost-to-go (usv_bufs_t.field, tiled) and the env's normalisation
// constants (usv_bufs_t.fnorm); the SDF of a texel is recomputed from the env's 16 obstacle centres
// (cell_sdf).  Every reader (the step kernels' bilinear sample, usv_field_view) forms a texel with
// field_value: the operations of the reference's per-env normalisation in its order, so the same bits as
// the materialised field.
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
// usv_bufs_t.fnorm of an env: (gmin, gden, jmn, jden), (inf_val, +-high, 1 / gden, 1 / jden) -- `high` > 0
// always, so its sign carries the batch's any-inside flag (+: some cell of the batch is inside an obstacle)
struct FieldNorm {
  float gmin, gden, jmn, jden, inf_val, high, inv_gden, inv_jden;
  bool any_inside;
};
__device__ __forceinline__ FieldNorm field_norm_of(float4 a, float4 b) {
  return FieldNorm{a.x, a.y, a.z, a.w, b.x, fabsf(b.y), b.z, b.w, b.y > 0.f};
}
// one texel: sv = SDF, g = raw cost (+inf unreachable); cell = map / G, inv_r = 1 / influence radius,
// inv_safe = RN(1 / safe_radius).  The divisions by a per-env or config constant are div_rn with the
// divisor's correctly rounded reciprocal (the IEEE quotient for quotients in [2^-90, 2^120]; 0 stays 0)
__device__ __forceinline__ float field_value(const usv_cfg_t &c, const FieldNorm &k, float sv, float g, float cell,
                                             float inv_r, float inv_safe) {
  const float cv = isinf(g) ? k.inf_val : g;
  const float dte = sv - c.obstacle_radius;
  const float jr = j_raw(c, dte, inv_r);
  const float gm = clampt(div_rn(cv * cell, c.safe_radius, inv_safe), 0.f, 1.f);   // goal_mask
  const float j = (dte < c.influence_radius) ? jr * gm : 0.f;
  const float jv = (k.any_inside && dte <= 0.f) ? k.high : j;
  const float gn = div_rn(cv - k.gmin, k.gden, k.inv_gden);
  const float jn = div_rn(jv - k.jmn, k.jden, k.inv_jden);
  return gn + c.field_alpha * jn;
}

// ---------------------------------------------------------------------------
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
// USV_PLACE_SPLIT 1: the pair tests of a rejection iteration split over the four 16-lane groups (A/B: 0 = every
// group runs all 15)
#ifndef USV_PLACE_SPLIT
#define USV_PLACE_SPLIT 1
#endif
__device__ __forceinline__ float2 place_obstacles(const usv_cfg_t &c, int ee, float sx, float sy, float tx, float ty,
                                                  uint64_t seed, uint64_t step, const float *__restrict__ inj) {
  static_assert(USV_NOBST == 16, "16-lane groups");
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
      const bool vo = ox < 900.f;
#if USV_PLACE_SPLIT
      // the four groups hold the same obstacles, so each checks a quarter of the lower-index ones: group q the
      // obstacles 4q .. 4q + 3 (from its own lanes 16q + 4q + k), and the groups' verdicts meet in one ballot
      // (obstacle o is bad iff bit o of some group is set) -- 4 dependent pair tests per iteration instead of 15
      bool bad = q == 0 && ((ds < c.min_dist_safe) || (dt < c.min_dist_safe));
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int i = 4 * q + k;
        const float xi = __shfl(ox, gbase + i, 64), yi = __shfl(oy, gbase + i, 64);
        const float ddx = xi - ox, ddy = yi - oy;
        if (i < o && vo && (xi < 900.f) && (ddx * ddx + ddy * ddy) < sep2) bad = true;
      }
      const uint64_t bq = __ballot(bad);
      const uint32_t inval = (uint32_t)((bq | (bq >> 16) | (bq >> 32) | (bq >> 48)) & 0xFFFFull);
      bad = ((inval >> o) & 1u) != 0u;
#else
      bool bad = (ds < c.min_dist_safe) || (dt < c.min_dist_safe);
      // the four groups hold the same obstacles, so obstacle i is lane i's value: a scalar read of the lane
      // (v_readlane) instead of a per-lane LDS permute
#pragma unroll
      for (int i = 0; i < USV_NOBST - 1; ++i) {
        const float xi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ox), i));
        const float yi = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(oy), i));
        const float ddx = xi - ox, ddy = yi - oy;
        if (i < o && vo && (xi < 900.f) && (ddx * ddx + ddy * ddy) < sep2) bad = true;
      }
      const uint32_t inval = (uint32_t)((__ballot(bad) >> gbase) & 0xFFFFull);   // same in every group
#endif
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
  (void)q;
  return make_float2(ox, oy);   // obstacle o's centre (every 16-lane group holds the same)
}


__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off, 64));
  return v;
}

// Device NaN probe (the reference's USV_NAN_PROBE fail-fast, USV_Virtual.py:57-95,
// vec_env_rlgames.py:41-80): each lane brings the USV_NAN_* stage bits it saw; the common
// path is one ballot, a wave that saw any ORs them into *flag with one atomic.  Call from
// wave-uniform control flow.
__device__ __forceinline__ void nan_report(int32_t *flag, uint32_t bits) {
  if (__ballot(bits != 0u) == 0ull) return;
  uint32_t m = bits;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m |= (uint32_t)__shfl_xor((int)m, off, 64);
  if ((threadIdx.x & 63) == 0) atomicOr(flag, (int)m);
}
__device__ __forceinline__ uint32_t nonfinite(float x) { return isfinite(x) ? 0u : 1u; }

// float atomic max for non-negative-or-any floats via int ordering
__device__ __forceinline__ void atomic_max_f32(float *addr, float v) {
  if (v >= 0.f) atomicMax((int *)addr, __float_as_int(v));
  else atomicMin((unsigned int *)addr, __float_as_uint(v));
}

// Phase probe (instrumented build only, -DUSV_PHASE_PROBE): thread 0 of each of
// the first 4096 workgroups stamps wall_clock64() (100 MHz) at phase k of the
// last launch of an instrumented kernel; usv_probe_read_<tu>() copies it out.
#ifdef USV_PHASE_PROBE
#define USV_PROBE_DEFINE(tu)                                                           \
  __device__ unsigned long long g_probe_##tu[4096][16];                                \
  extern "C" int usv_probe_read_##tu(void *host_out) {                                 \
    return (int)hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_probe_##tu), sizeof(g_probe_##tu)); \
  }
#define USV_PHASE(tu, k)                                                               \
  do {                                                                                 \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_probe_##tu[blockIdx.x][k] = wall_clock64(); \
  } while (0)
// the same stamp from thread t (another wave's timeline); USV_PHASE_DRAIN first waits for the
// wave's outstanding memory operations (probe build only: it changes the schedule it measures)
#define USV_PHASE_T(tu, k, t)                                                          \
  do {                                                                                 \
    if (threadIdx.x == (t) && blockIdx.x < 4096) g_probe_##tu[blockIdx.x][k] = wall_clock64(); \
  } while (0)
#define USV_PHASE_DRAIN(tu, k, t)                                                      \
  do {                                                                                 \
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");                               \
    USV_PHASE_T(tu, k, t);                                                             \
  } while (0)
#else
#define USV_PROBE_DEFINE(tu)
#define USV_PHASE(tu, k) ((void)0)
#define USV_PHASE_T(tu, k, t) ((void)0)
#define USV_PHASE_DRAIN(tu, k, t) ((void)0)
#endif

#define USV_CHECK_LAUNCH()                                   \
  do {                                                       \
    hipError_t _e = hipGetLastError();                       \
    if (_e != hipSuccess) return 100 + (int)_e;              \
  } while (0)
