/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * Plain-C, scalar, single-threaded restatement of the reference USV CaptureXY
 * env path (loop-Z/omniisaacgymenvs_loop), written op-by-op after the PyTorch
 * code it cites.  It is the parity checker for the HIP kernels and the
 * `cpu_baseline` ("port") leg of bench.py.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline may load it; the product (libusv_hip.so) never
 * links or calls it.
 *
 * Parity pinning: tests/golden/ fixtures (.npz) were produced by importing the reference
 * Python in the build container (tests/golden/make_golden.py) and recording its
 * outputs together with every torch.rand draw it consumed; tests/test_oracle_*.py
 * replay those draws through this file.
 *
 * The rigid-body integrator has NO reference implementation (the reference
 * calls PhysX through Isaac Sim, envs/vec_env_rlgames.py:154-171).  The 3-DoF
 * semi-implicit Euler below is this build's own definition; the
 * forces it integrates are pinned to the reference force model
 * (Hydrodynamics.py:176-245, ThrusterDynamics.py:129-234).
 */
#include <math.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "../include/usv_hip.h"
#include "oracle_philox.h"

#define OPI 3.14159265358979323846

/* OpenMP (bench.py's cpu_baseline build, libusv_oracle_omp.so): every parallel loop is over
 * independent envs / reset slots, the two batch maxima are exact max reductions, so the
 * results are the single-threaded build's bit for bit */
#ifdef _OPENMP
#define OMP_PRAGMA(x) _Pragma(#x)
#define OMP_FOR OMP_PRAGMA(omp parallel for schedule(static))
#define OMP_FOR_DYN OMP_PRAGMA(omp parallel for schedule(dynamic, 1))
#define OMP_REDUCE_MAX(m, f) OMP_PRAGMA(omp parallel for schedule(static) reduction(max : m) reduction(| : f))
#else
#define OMP_FOR
#define OMP_FOR_DYN
#define OMP_REDUCE_MAX(m, f)
#endif
int oracle_threads(void) {
#ifdef _OPENMP
  int t = 1;
  _Pragma("omp parallel") { _Pragma("omp single") t = omp_get_num_threads(); }
  return t;
#else
  return 1;
#endif
}

static inline float clampf_(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
static inline float maxf_(float a, float b) { return a > b ? a : b; }
static inline float minf_(float a, float b) { return a < b ? a : b; }
/* torch.norm(v, dim=-1) of a 2-vector on CPU is sqrt(fma(y, y, x*x)) bit-for-bit
 * (checked on 2M random pairs); sum-of-squares reductions ((e*e).sum(-1)) are
 * plain x*x + y*y. */
static inline float tnorm2(float x, float y) { return sqrtf(fmaf(y, y, x * x)); }

/* sin / cos of the integrator's angles (yaw, spawn and disturbance phases).  The reference's PhysX step has no
 * restatable integrator: this build defines it, and its sin / cos are part of that definition --
 * restated here operation for operation (csrc/usv_device.h:usv_sincos; plain IEEE float multiplies and adds,
 * both sides built with -ffp-contract=off), so the oracle integrates the device's bits.  Reduction by pi/2 in
 * three Cody-Waite parts, Cephes' single-precision minimax polynomials on [-pi/4, pi/4]; the accuracy against
 * libm is a CPU test (tests/test_oracle_golden.py::test_integrator_sincos_accuracy). */
void usv_sincos(float x, float *s, float *c) {
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
void oracle_sincos(const float *x, int n, float *s, float *c) {
  for (int i = 0; i < n; ++i) usv_sincos(x[i], s + i, c + i);
}
static inline float usv_sin(float x) { float s, c; usv_sincos(x, &s, &c); return s; }
static inline float usv_cos(float x) { float s, c; usv_sincos(x, &s, &c); return c; }

/* The attitude the reference reads back (csrc/usv_device.h:usv_quat_rot): the stand-in's yaw-only quaternion
 * q = (w, 0, 0, z) = (cos(yaw/2), 0, 0, sin(yaw/2)) by usv_sincos, pytorch3d.transforms.quaternion_to_matrix of it
 * (two_s = 2 / (q * q).sum(-1); Hydrodynamics.py:209-217): R = [[C, -S, 0], [S, C, 0], [0, 0, 1]] with
 * C = 1 - two_s * (z * z), S = two_s * (z * w).  The drag's R^T v in torch.bmm's CPU order
 * ((r0 vx + r1 vy) + r2 vz, no fma: checked on random batches) is (C vx + S vy, -S vx + C vy); the integrator
 * rotates the body-frame wrench with the same R. */
typedef struct { float C, S, w, z; } quat_rot_t;
static inline quat_rot_t usv_quat_rot(float yaw) {
  float z, w;
  usv_sincos(yaw * 0.5f, &z, &w);
  const float two_s = 2.0f / (w * w + z * z);
  quat_rot_t q = {1.0f - two_s * (z * z), two_s * (z * w), w, z};
  return q;
}
/* update_state's heading (USV_Virtual.py:776-786): arctan2(2 (w z + x y), 1 - 2 (y^2 + z^2)) of that quaternion */
float usv_atan2(float y, float x);
static inline float usv_heading(quat_rot_t q) { return usv_atan2(2.0f * (q.w * q.z), 1.0f - 2.0f * (q.z * q.z)); }
/* the stand-in's pose from a quaternion set_world_poses receives (w, 0, 0, z) */
static inline float usv_yaw_of_quat(float w, float z) { return 2.0f * usv_atan2(z, w); }

/* sin / cos where the reference calls torch.sin / torch.cos on the state path (spawn angle and quaternion, scene
 * yaw, constant-disturbance direction, disturbance sinusoids, legacy CoM disk): torch's CPU kernels there are MKL
 * VML HA (within 0.6 ulp, the correctly rounded value for ~95% of float arguments), so this build rounds a double
 * evaluation (csrc/usv_device.h:usv_sincos_cr, restated operation for operation): Cody-Waite by pi/2 in three
 * parts (P1, P2 of 30 bits, exact k * P for |k| < 2^23), fdlibm's kernel polynomials. */
void usv_sincos_cr(float xf, float *s, float *c) {
  const double x = (double)xf;
  const double k = rint(x * 0x1.45f306dc9c883p-1);
  double r = x - k * 0x1.921fb54p+0;
  r = r - k * 0x1.10b46118p-30;
  r = r - k * 0x1.313198a2e037p-61;
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
static inline float usv_sin_cr(float x) { float s, c; usv_sincos_cr(x, &s, &c); return s; }
void oracle_sincos_cr(const float *x, int n, float *s, float *c) {
  for (int i = 0; i < n; ++i) usv_sincos_cr(x[i], s + i, c + i);
}
/* [n][4] per yaw: C, S (usv_quat_rot), the heading (usv_heading) and the yaw back from (w, z) (usv_yaw_of_quat) */
void oracle_quat(const float *yaw, int n, float *out) {
  for (int i = 0; i < n; ++i) {
    const quat_rot_t q = usv_quat_rot(yaw[i]);
    out[4 * i + 0] = q.C; out[4 * i + 1] = q.S; out[4 * i + 2] = usv_heading(q);
    out[4 * i + 3] = usv_yaw_of_quat(q.w, q.z);
  }
}

/* exp, tanh and atan2 of the observation / reward formulas (the reference's torch.exp / torch.tanh / torch.atan2 in
 * float32), by the same rule as usv_sincos: this build's functions, restated operation for operation from
 * csrc/usv_device.h (Cephes' single-precision reductions and polynomials; the power of two by ldexpf, exact), so the
 * device's observations and rewards are the oracle's bits.  Accuracy against float64 libm: CPU tests. */
float usv_exp(float x) {
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
float usv_tanh(float x) {
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
float usv_atan2(float y, float x) {
  if (x != x || y != y) return x + y;
  const float ax = fabsf(x), ay = fabsf(y);
  float r;
  if (ax == 0.f && ay == 0.f) {
    r = signbit(x) ? 3.14159265358979323846f : 0.f;
  } else {
    const float a = ay / ax;   /* +inf where x = 0 */
    float t, base, blo;       /* base = hi + lo parts of 0, pi / 4, pi / 2 */
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
void oracle_math(const float *x, const float *y, int n, float *e, float *t, float *a) {
  for (int i = 0; i < n; ++i) {
    e[i] = usv_exp(x[i]);
    t[i] = usv_tanh(x[i]);
    a[i] = usv_atan2(y[i], x[i]);
  }
}

/* ------------------------------------------------------------------------ */
/* Philox streams (same mapping as the kernels)                              */
/* ------------------------------------------------------------------------ */
void oracle_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  oracle_philox4x32_10(ctr, key, out);
}

static float philox_u(uint64_t seed, uint32_t env, uint64_t step, uint32_t site, int i) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t ctr[4] = {env, (uint32_t)step, (uint32_t)(step >> 32), site + (uint32_t)(i >> 2)};
  uint32_t out[4];
  oracle_philox4x32_10(ctr, key, out);
  return oracle_u01(out[i & 3]);
}

/* uniforms one env consumes in one step (layout SU_* in usv_hip.h) */
void oracle_step_uniforms(uint64_t seed, uint64_t step, int n, float *u /*[n][USV_NU_STEP]*/) {
  OMP_FOR
  for (int e = 0; e < n; ++e)
    for (int i = 0; i < USV_NU_STEP; ++i) u[(size_t)e * USV_NU_STEP + i] = philox_u(seed, (uint32_t)e, step, 0u, i);
}

/* uniforms of the reset slots (layout RU_* in usv_hip.h) */
void oracle_reset_uniforms(uint64_t seed, uint64_t step, int k, const int32_t *ids, float *u /*[k][USV_NU_RESET]*/) {
  for (int s = 0; s < k; ++s)
    for (int i = 0; i < USV_NU_RESET; ++i)
      u[(size_t)s * USV_NU_RESET + i] = philox_u(seed, (uint32_t)ids[s], step, 0x100u, i);
}

/* ------------------------------------------------------------------------ */
/* Thruster LUT: DynamicsFirstOrder.interpolate_on_field_data                */
/* (ThrusterDynamics.py:152-177) = F.interpolate(mode="linear",               */
/* align_corners=True) of the 21-point table onto 1000 points (fp32).         */
/* ------------------------------------------------------------------------ */
void oracle_lut(const float *table, int n_in, int n_out, float *lut) {
  const float scale = (n_out > 1) ? (float)(n_in - 1) / (float)(n_out - 1) : 0.f;
  for (int i = 0; i < n_out; ++i) {
    const float src = scale * (float)i;
    int i0 = (int)src;
    if (i0 > n_in - 1) i0 = n_in - 1;
    const int off = (i0 < n_in - 1) ? 1 : 0;
    const float l1 = src - (float)i0;
    const float l0 = 1.0f - l1;
    lut[i] = fmaf(l0, table[i0], l1 * table[i0 + off]);   /* torch CPU build contracts to this FMA */
  }
}

/* index used by DynamicsFirstOrder.get_cmd_interpolated (ThrusterDynamics.py:187-191) */
static inline int lut_index(float cmd, int n) {
  float t = (cmd + 1.0f) / 2.0f;
  t = t * (float)(n - 1);
  int idx = (int)rintf(t);        /* torch.round: half to even */
  if (idx < 0) idx = 0;
  if (idx > n - 1) idx = n - 1;
  return idx;
}

/* ------------------------------------------------------------------------ */
/* Env state (SoA, host memory)                                             */
/* ------------------------------------------------------------------------ */
#define USV_ORACLE_NDBG 20
typedef struct oracle_env {
  int n;
  float *px, *py, *yaw, *vx, *vy, *wz, *fl, *fr;
  float *mass, *com_x, *com_y, *com_z, *k_drag, *thr_l, *thr_r, *k_iz, *mass_r;
  float *lin_damp, *quad_damp;      /* [3][n] or NULL */
  float *tgt_x, *tgt_y;
  float *obst;                      /* [16][2][n] */
  float *field;                     /* [n][150*150] */
  float *prev_cmd;                  /* [2][n] */
  float *prev_dist, *prev_head, *prev_pot, *prev_wz;
  int32_t *goal_cnt, *progress, *reset_buf;
  uint8_t *just_reset;
  int32_t *done_succ, *done_coll;
  float *stats;                     /* [28][n] */
  float *obs;                       /* [n][33] */
  float *rew;
  int32_t ctl[USV_CTL_N];
  float extras[USV_NSTAT];
  /* diagnostics of the last step (for parity tests) */
  float *dbg;                       /* [n][USV_ORACLE_NDBG]: u_l, u_r, target_l, target_r, pot (the sample the reward used), danger, total,
                                       pens, shaping, dist_r, align_r, praw (before the dead zone), ppos, ggate, the oracle's
                                       own sample, its sample at pos_in, 1 where prev_pot was replaced by this step's sample
                                       (a reset env or the global None after any reset) */
  float *tmp;                       /* [n][8]: cmd[2], thrust[2], unit[2], target force[2] */
  const float *grid_lin;            /* [150] potential-field cell centres, NULL => linspace formula */
  float *dist;                      /* [USV_NDIST][n] disturbance parameters or NULL */
  const float *env_org;             /* [2][n] env origins (RLTask._env_pos) or NULL */
  float *tgt_h;                     /* [n] GoToPose target heading / TrackXYO target yaw rate */
  double step_f;                    /* USVVirtual.step (+= 1 / horizon_length per calculate_metrics,
                                       USV_Virtual.py:1633): the GoToPose curriculum's clock */
  /* parity harness (tests only): the device's potential samples and post-integration positions.  With
     pot_in the CaptureXY reward uses pot_in[e] as this step's potential sample instead of the oracle's own
     (which is kept in dbg[14]); prev_pot then carries the device's samples from step to step too.  With
     pos_in the oracle also samples its own field at the device's position (+ the same noise) into dbg[15]. */
  const float *pot_in;              /* [n] or NULL */
  const float *pos_in;              /* [2][n] or NULL */
  /* [6][n] (px, py, yaw, vx, vy, wz) or NULL: the reference's cached root_pos / root_quats / root_velocities
     as the first substep after a reset reads them (apply_forces, USV_Virtual.py:1103-1117,
     reads the values of the last update_state, :771-813) -- the pre-reset state, kept by oracle_reset when
     cfg.stale_root is on */
  float *root_cache;
} oracle_env_t;

/* GoToPoseTask spawn curriculum (USV_go_to_pose.py:188-202 kill distance, :266-290 spawn radii): linear in
 * USVVirtual.step between warmup and end, in the reference's Python-float (double) arithmetic */
static double curriculum_lerp(const usv_cfg_t *c, double st, double cur, double fin) {
  if (st < c->cur_warmup) return cur;
  if (st > c->cur_end) return fin;
  const double r = (st - c->cur_warmup) / (c->cur_end - c->cur_warmup);
  return r * (fin - cur) + cur;
}

/* ------------------------------------------------------------------------ */
/* Forces: HydrodynamicsObject.ComputeDampingMatrix/ComputeHydrodynamicsEffects
 * (Hydrodynamics.py:176-245) restricted to the planar DOFs u, v, r; thrusters
 * at the heron.usd lever arms.                           */
/* ------------------------------------------------------------------------ */
static void planar_forces(const usv_cfg_t *c, const oracle_env_t *E, int e, float cy, float sy, float vx, float vy,
                          float wz, float fl, float fr, const float *dist3 /* disturbance fx, fy, tz or NULL */,
                          float *X, float *Y, float *N) {
  /* (cy, sy, vx, vy, wz): the root state apply_forces reads (the current one, or the cached pre-reset one
     in a reset env's first substep); cy, sy = C, S of quaternion_to_matrix (usv_quat_rot) */
  /* getLocalLinearVelocities: R^T v  (Utils.py:10-14) in torch.bmm's order */
  float u = cy * vx + sy * vy;
  float v = -sy * vx + cy * vy;
  const float r = wz;
  if (c->current_on) {   /* relative to the water current (Hydrodynamics.py:224-237): R^T v - R^T flow */
    u = u - (cy * c->flow_vel[0] + sy * c->flow_vel[1]);
    v = v - (-sy * c->flow_vel[0] + cy * c->flow_vel[1]);
  }
  float lin[3], quad[3];
  for (int k = 0; k < 3; ++k) {
    lin[k] = E->lin_damp ? E->lin_damp[k * E->n + e] : c->lin_damp[k];
    quad[k] = E->quad_damp ? E->quad_damp[k * E->n + e] : c->quad_damp[k];
  }
  const float vel[3] = {u, v, r};
  float drag[3];
  for (int k = 0; k < 3; ++k) {
    float D = lin[k] + quad[k] * fabsf(vel[k]);           /* lin_damp + quad_damp (:185-196) */
    D = D * c->scaling_damping;                            /* (:199) */
    if (c->use_drag_scale) D = D * E->k_drag[e];           /* k_drag (:202-203) */
    drag[k] = -D * vel[k];                                 /* (:243) */
  }
  const float comy = E->com_y[e];
  if (dist3) {   /* base force = disturbance + drag (USV_Virtual.py:1118-1125) */
    *X = fl + fr + (dist3[0] + drag[0]);
    *Y = dist3[1] + drag[1];
    *N = -(c->thr_y - comy) * fl + (c->thr_y + comy) * fr + (dist3[2] + drag[2]);
    return;
  }
  *X = fl + fr + drag[0];
  *Y = drag[1];
  *N = -(c->thr_y - comy) * fl + (c->thr_y + comy) * fr + drag[2];
}

/* ForceDisturbance.get_disturbance_forces / TorqueDisturbance.get_torque_disturbance
 * (USV_disturbances.py:386-410, 510-530) at the world root position (root_pos =
 * local + RLTask._env_pos); body-frame base force / yaw torque (is_global=False,
 * USV_Virtual.py:1118-1125). */
static void disturbance(const usv_cfg_t *c, const oracle_env_t *E, int e, float px, float py, float *fx, float *fy,
                        float *tz) {
  const int n = E->n;
  const float *D = E->dist;
  const float wx = px + (E->env_org ? E->env_org[e] : 0.f);
  const float wy = py + (E->env_org ? E->env_org[n + e] : 0.f);
  *fx = D[DI_FCX * n + e];
  *fy = D[DI_FCY * n + e];
  *tz = D[DI_TC * n + e];
  if (c->fsin_on) {
    *fx = *fx + usv_sin_cr(wx * D[DI_FXF * n + e] + D[DI_FXS * n + e]) * D[DI_FAMP * n + e];
    *fy = *fy + usv_sin_cr(wy * D[DI_FYF * n + e] + D[DI_FYS * n + e]) * D[DI_FAMP * n + e];
  }
  if (c->tsin_on) *tz = *tz + usv_sin_cr((wx + wy) * D[DI_TF * n + e] + D[DI_TS * n + e]) * D[DI_TAMP * n + e];
}

/* quat: NULL => the stand-in's quaternion of E->yaw (usv_quat_rot); else [n][4] (w, x, y, z) yaw-only quaternions
 * (x = y = 0) given by the caller -- the reference's own, so the drag is checked bit for bit against it */
void oracle_forces_q(const usv_cfg_t *c, oracle_env_t *E, const float *quat, float *out /*[n][3]*/) {
  for (int e = 0; e < E->n; ++e) {
    float C, S;
    if (quat) {
      const float w = quat[4 * e], z = quat[4 * e + 3];
      const float two_s = 2.0f / (w * w + z * z);
      C = 1.0f - two_s * (z * z);
      S = two_s * (z * w);
    } else {
      const quat_rot_t q = usv_quat_rot(E->yaw[e]);
      C = q.C; S = q.S;
    }
    float X, Y, N;
    planar_forces(c, E, e, C, S, E->vx[e], E->vy[e], E->wz[e], E->fl[e], E->fr[e], NULL, &X, &Y, &N);
    out[e * 3 + 0] = X; out[e * 3 + 1] = Y; out[e * 3 + 2] = N;
  }
}
void oracle_forces(const usv_cfg_t *c, oracle_env_t *E, float *out /*[n][3]*/) { oracle_forces_q(c, E, NULL, out); }

/* Hydrostatic wrench: USVVirtual.update_state volume (USV_Virtual.py:791-798), get_euler_angles
 * (:815-835), HydrostaticsObject.compute_archimedes_metacentric_local (Hydrostatics.py:63-133) */
void oracle_hydrostatics(const usv_hydro_t *h, int n, const float *quat, const float *root_z, float *volume,
                         float *euler, float *wrench) {
  for (int e = 0; e < n; ++e) {
    const float w = quat[4 * e], x = quat[4 * e + 1], y = quat[4 * e + 2], z = quat[4 * e + 3];
    float high = h->zero_height - root_z[e];
    high = high < 0.f ? 0.f : (high > h->zero_height + 20.0f ? h->zero_height + 20.0f : high);
    float vol = high * h->waterplane_area;
    vol = vol < 0.f ? 0.f : (vol > h->max_volume ? h->max_volume : vol);
    const float r00 = 1.0f - 2.0f * (y * y) - 2.0f * (z * z), r10 = 2.0f * x * y + 2.0f * w * z;
    const float r20 = 2.0f * x * z - 2.0f * w * y, r21 = 2.0f * y * z + 2.0f * w * x;
    const float r22 = 1.0f - 2.0f * (x * x) - 2.0f * (y * y);
    const float roll = atan2f(r21, r22), pitch = asinf(-r20), yaw = atan2f(r10, r00);
    const float fz = (-h->water_density * h->gravity) * vol;
    const float tx = (-1.0f * h->metacentric_width) * (sinf(roll) * h->avg_force);
    const float ty = (-1.0f * h->metacentric_length) * (sinf(pitch) * h->avg_force);
    const float two_s = 2.0f / (((w * w + x * x) + y * y) + z * z);
    float *o = wrench + 6 * e;
    o[0] = two_s * (x * z - y * w) * fz;
    o[1] = two_s * (y * z + x * w) * fz;
    o[2] = (1.0f - two_s * (x * x + y * y)) * fz;
    o[3] = tx * h->amplify_torque;
    o[4] = ty * h->amplify_torque;
    o[5] = 0.0f * h->amplify_torque;
    volume[e] = vol;
    euler[3 * e] = roll; euler[3 * e + 1] = pitch; euler[3 * e + 2] = yaw;
  }
}

/* ------------------------------------------------------------------------ */
/* Potential field: BatchedMapGPU (tasks/USV/d_multi_gemini.py:7-271)        */
/* K envs, obstacles [K][16][2], targets [K][2] -> field [K][150][150]       */
/* ------------------------------------------------------------------------ */
static void grid_coords(float *lin /*150*/, float map_size) {
  /* torch.linspace(-map/2 + cell/2, map/2 - cell/2, 150) (:18-20) */
  const double cell_d = (double)map_size / USV_GRID;
  const float start = (float)(-(double)map_size / 2 + cell_d / 2);
  const float end = (float)((double)map_size / 2 - cell_d / 2);
  const float step = (end - start) / (float)(USV_GRID - 1);
  const int half = USV_GRID / 2;
  for (int i = 0; i < USV_GRID; ++i)
    lin[i] = (i < half) ? start + step * (float)i : end - step * (float)(USV_GRID - i - 1);
}

void oracle_grid_lin(float map_size, float *lin) { grid_coords(lin, map_size); }

void oracle_potential_field(const usv_cfg_t *c, int K, const float *obst /*[K][16][2]*/,
                            const float *tgt /*[K][2]*/, float *field /*[K][G2]*/,
                            float *cost_out /*[K][G2] optional*/, const float *grid_lin) {
  const int G = USV_GRID, G2 = USV_GRID2;
  float lin[USV_GRID];
  if (grid_lin) memcpy(lin, grid_lin, sizeof(lin));
  else grid_coords(lin, c->map_size);
  const float cell = (float)((double)c->map_size / G);
  float *sdf = (float *)malloc(sizeof(float) * (size_t)K * G2);
  uint8_t *freec = (uint8_t *)malloc((size_t)K * G2);
  float *cost = (float *)malloc(sizeof(float) * (size_t)K * G2);
  /* compute_occupancy_and_sdf (:66-104) */
  OMP_FOR_DYN
  for (int k = 0; k < K; ++k) {
    for (int i = 0; i < G; ++i)
      for (int j = 0; j < G; ++j) {
        const float gx = lin[j], gy = lin[i];
        float m = INFINITY;
        for (int o = 0; o < USV_NOBST; ++o) {
          const float dx = gx - obst[(k * USV_NOBST + o) * 2 + 0];
          const float dy = gy - obst[(k * USV_NOBST + o) * 2 + 1];
          const float d = tnorm2(dx, dy);
          if (d < m) m = d;
        }
        const float s = m - c->obstacle_radius;
        sdf[(size_t)k * G2 + i * G + j] = s;
        int occ = (s <= 0.f);
        if (i == 0 || i == G - 1 || j == 0 || j == G - 1) occ = 1;
        freec[(size_t)k * G2 + i * G + j] = (uint8_t)(occ ? 0 : 1);  /* is_free = occ < 0.5 (:162) */
      }
  }
  /* compute_cost_field_wavefront (:135-192): Jacobi relaxation, fixed iterations */
  const float diag = 1.414f;
  OMP_FOR_DYN
  for (int k = 0; k < K; ++k) {
    float *nxt = (float *)malloc(sizeof(float) * (size_t)G2);
    float *C = cost + (size_t)k * G2;
    const uint8_t *F = freec + (size_t)k * G2;
    for (int q = 0; q < G2; ++q) C[q] = INFINITY;
    const float half_map = (float)((double)c->map_size / 2);
    const float tx = (tgt[k * 2 + 0] + half_map) / cell;
    const float ty = (tgt[k * 2 + 1] + half_map) / cell;
    long ix = (long)tx, iy = (long)ty;       /* .long() truncates */
    if (ix < 0) ix = 0;
    if (ix > G - 1) ix = G - 1;
    if (iy < 0) iy = 0;
    if (iy > G - 1) iy = G - 1;
    C[iy * G + ix] = 0.f;
    for (int it = 0; it < c->field_iters; ++it) {
      int changed = 0;
      for (int i = 0; i < G; ++i)
        for (int j = 0; j < G; ++j) {
          float m = C[i * G + j];
          for (int di = -1; di <= 1; ++di)
            for (int dj = -1; dj <= 1; ++dj) {
              if (!di && !dj) continue;
              const int ii = i + di, jj = j + dj;
              if (ii < 0 || ii >= G || jj < 0 || jj >= G) continue;
              const float cand = C[ii * G + jj] + ((di && dj) ? diag : 1.0f);
              if (cand < m) m = cand;
            }
          const float nv = F[i * G + j] ? m : INFINITY;
          if (nv != C[i * G + j]) changed = 1;
          nxt[i * G + j] = nv;
        }
      memcpy(C, nxt, sizeof(float) * G2);
      if (!changed) break;   /* a Jacobi fixed point stays fixed: exact early exit */
    }
    free(nxt);
  }
  if (cost_out) memcpy(cost_out, cost, sizeof(float) * (size_t)K * G2);
  /* compute_potential_field (:194-271) */
  float max_val = -INFINITY;
  int any_finite = 0;
  OMP_REDUCE_MAX(max_val, any_finite)
  for (size_t q = 0; q < (size_t)K * G2; ++q)
    if (isfinite(cost[q])) { any_finite = 1; if (cost[q] > max_val) max_val = cost[q]; }
  if (!any_finite) max_val = 100.0f;
  const float inf_val = max_val * 1.5f;
  float *J = (float *)malloc(sizeof(float) * (size_t)K * G2);
  float jmax = -INFINITY;
  int any_inside = 0;
  const float inv_r = (float)(1.0 / (double)c->influence_radius);
  OMP_REDUCE_MAX(jmax, any_inside)
  for (int k = 0; k < K; ++k)
    for (int q = 0; q < G2; ++q) {
      const size_t p = (size_t)k * G2 + q;
      const float cv = isinf(cost[p]) ? inf_val : cost[p];
      const float dte = sdf[p] - c->obstacle_radius;
      const float dist_goal = cv * cell;
      const float rmask = clampf_(dist_goal / c->safe_radius, 0.f, 1.f);
      float j = 0.f;
      if (dte < c->influence_radius) {
        const float d = maxf_(dte, 1e-3f);
        const float t = 1.0f / d - inv_r;
        j = c->eta * (t * t) * rmask;
      }
      J[p] = j;
      if (j > jmax) jmax = j;
      if (dte <= 0.f) any_inside = 1;
    }
  if (any_inside) {
    const float high = (jmax > 1e-6f) ? jmax * 10.0f : 100.0f;
    for (int k = 0; k < K; ++k)
      for (int q = 0; q < G2; ++q) {
        const size_t p = (size_t)k * G2 + q;
        if (sdf[p] - c->obstacle_radius <= 0.f) J[p] = high;
      }
  }
  OMP_FOR_DYN
  for (int k = 0; k < K; ++k) {
    float gmin = INFINITY, gmax = -INFINITY, jmn = INFINITY, jmx = -INFINITY;
    for (int q = 0; q < G2; ++q) {
      const size_t p = (size_t)k * G2 + q;
      const float cv = isinf(cost[p]) ? inf_val : cost[p];
      gmin = minf_(gmin, cv); gmax = maxf_(gmax, cv);
      jmn = minf_(jmn, J[p]); jmx = maxf_(jmx, J[p]);
    }
    const float gden = (gmax - gmin) + 1e-6f;
    const float jden = (jmx - jmn) + 1e-6f;
    for (int q = 0; q < G2; ++q) {
      const size_t p = (size_t)k * G2 + q;
      const float cv = isinf(cost[p]) ? inf_val : cost[p];
      const float gn = (cv - gmin) / gden;
      const float jn = (J[p] - jmn) / jden;
      field[p] = gn + c->field_alpha * jn;
    }
  }
  free(sdf); free(freec); free(cost); free(J);
}

/* ------------------------------------------------------------------------ */
/* grid_sample(field, 2*pos/map, bilinear, align_corners=False, border)      */
/* (USV_capture_xy_static_obs.py:302-326)                                    */
/* ------------------------------------------------------------------------ */
static float sample_field(const float *F, float map_size, float x, float y) {
  /* PyTorch CPU grid_sampler_2d, bilinear/border/align_corners=False
   * (aten/src/ATen/native/cpu/GridSamplerKernel.cpp: ComputeLocation::unnormalize
   * = (g + 1) * (size / 2) - 0.5, clip to [0, size-1]; weights from floor).
   * The CPU build contracts the unnormalise and the corner sum into FMAs;
   * this form reproduces torch's result bit-for-bit (tests/test_oracle_golden.py). */
  const int G = USV_GRID;
  const float gx = 2.0f * x / map_size, gy = 2.0f * y / map_size;
  const float half = (float)G / 2.0f;
  float ix = fmaf(gx + 1.f, half, -0.5f);
  float iy = fmaf(gy + 1.f, half, -0.5f);
  ix = minf_((float)(G - 1), maxf_(ix, 0.f));
  iy = minf_((float)(G - 1), maxf_(iy, 0.f));
  const float xw = floorf(ix), yn = floorf(iy);
  const float w = ix - xw, e = 1.f - w;
  const float nn = iy - yn, ss = 1.f - nn;
  const float nw = ss * e, ne = ss * w, sw = nn * e, se = nn * w;
  const int i0 = (int)xw, j0 = (int)yn, i1 = i0 + 1, j1 = j0 + 1;
  const float v_nw = (i0 >= 0 && i0 < G && j0 >= 0 && j0 < G) ? F[j0 * G + i0] : 0.f;
  const float v_ne = (i1 >= 0 && i1 < G && j0 >= 0 && j0 < G) ? F[j0 * G + i1] : 0.f;
  const float v_sw = (i0 >= 0 && i0 < G && j1 >= 0 && j1 < G) ? F[j1 * G + i0] : 0.f;
  const float v_se = (i1 >= 0 && i1 < G && j1 >= 0 && j1 < G) ? F[j1 * G + i1] : 0.f;
  return fmaf(v_se, se, fmaf(v_sw, sw, fmaf(v_ne, ne, v_nw * nw)));
}

float oracle_sample_field(const float *F, float map_size, float x, float y) { return sample_field(F, map_size, x, y); }

/* ------------------------------------------------------------------------ */
/* Penalties.compute_penalty closed forms (USV_task_rewards.py:440-523)      */
/* ------------------------------------------------------------------------ */
static float pen_scalar(int kind, float k, float x0, float cc, float x) {
  switch (kind) {
    case PEN_DEADZONE: return -maxf_(fabsf(x) - x0, 0.f) * k + cc;
    case PEN_EXPABS: return (usv_exp(x0 * fabsf(x)) - 1.0f) * k + cc;
    default: return 0.f;
  }
}

/* priv-tail encoders (USV_Virtual.py:97-151) */
static float enc_centered(float x, float xmin, float xmax, float nominal) {
  double s = fabs((double)xmin - nominal);
  if (fabs((double)xmax - nominal) > s) s = fabs((double)xmax - nominal);
  if (1e-6 > s) s = 1e-6;
  return clampf_((x - nominal) / (float)s, -1.f, 1.f);
}
static float enc_minmax(float x, float xmin, float xmax) {
  if ((double)xmax - (double)xmin <= 1e-6) return 0.f;
  const float z = (x - xmin) / (float)((double)xmax - (double)xmin);
  return clampf_(2.0f * z - 1.0f, -1.f, 1.f);
}

/* ------------------------------------------------------------------------ */
/* Reset path: USVVirtual.reset_idx (USV_Virtual.py:1502-1618)               */
/* ids: compacted reset list (reset_buf.nonzero(), :1045); u: [k][NU_RESET]. */
/* ------------------------------------------------------------------------ */
static int g_skip_field = 0;
void oracle_set_skip_field(int on) { g_skip_field = on; }

void oracle_reset_scene(const usv_cfg_t *c, oracle_env_t *E, int k, const int32_t *ids, const float *U,
                        const float *rows);
void oracle_reset(const usv_cfg_t *c, oracle_env_t *E, int k, const int32_t *ids, const float *U) {
  oracle_reset_scene(c, E, k, ids, U, NULL);
}

/* rows: NULL, or [k][USV_SCENE_STRIDE] replay scenes of the reset slots (scene replay) */
void oracle_reset_scene(const usv_cfg_t *c, oracle_env_t *E, int k, const int32_t *ids, const float *U,
                        const float *rows) {
  const int n = E->n;
  if (k <= 0) return;
  float *obst_k = (float *)malloc(sizeof(float) * (size_t)k * USV_NOBST * 2);
  float *tgt_k = (float *)malloc(sizeof(float) * (size_t)k * 2);
  float *fld_k = (float *)malloc(sizeof(float) * (size_t)k * USV_GRID2);
  /* extras: episode sums of the envs being reset, BEFORE they are cleared (:1591-1612);
   * success/collision come from get_episode_outcomes (:1508-1514, static_obs.py:708-713) */
  double acc[USV_NSTAT];
  memset(acc, 0, sizeof(acc));
  for (int s = 0; s < k; ++s) {
    const int e = ids[s];
    for (int q = 0; q < USV_NSTAT; ++q) {
      float v = E->stats[q * n + e];
      if (q == ST_SUCCESS) v = (float)E->done_succ[e];
      if (q == ST_COLLISION) v = (float)E->done_coll[e];
      acc[q] += v;
    }
  }
  for (int q = 0; q < USV_NSTAT; ++q) {
    float m = (float)(acc[q] / k);
    if (q != ST_SUCCESS && q != ST_COLLISION) m = m / (float)c->max_episode_length;
    E->extras[q] = isnan(m) ? 0.f : m;
  }
  E->ctl[USV_CTL_POT_VALID] = 0;  /* CaptureXYTask.reset: prev_potential = None (:773) */
  OMP_FOR_DYN
  for (int s = 0; s < k; ++s) {
    const int e = ids[s];
    const float *u = U + (size_t)s * USV_NU_RESET;
    /* the cached root state keeps the pre-reset pose until the next update_state */
    if (c->stale_root && E->root_cache) {
      float *rc = E->root_cache;
      rc[0 * n + e] = E->px[e]; rc[1 * n + e] = E->py[e]; rc[2 * n + e] = E->yaw[e];
      rc[3 * n + e] = E->vx[e]; rc[4 * n + e] = E->vy[e]; rc[5 * n + e] = E->wz[e];
    }
    /* CaptureXYTask.reset (static_obs.py:767-778) */
    E->goal_cnt[e] = 0; E->done_succ[e] = 0; E->done_coll[e] = 0;
    E->just_reset[e] = 1;
    /* MassDistributionDisturbances.randomize_masses (USV_disturbances.py:127-150) */
    if (c->mass_dr_on) {
      E->mass[e] = u[RU_MASS] * (float)((double)c->mass_max - (double)c->mass_min) + c->mass_min;
    } else {
      E->mass[e] = u[RU_MASS] * 0.0f + c->base_mass;
    }
    if (c->mass_dr_on && c->com_mode == 1) {         /* _randomize_com box (:98-103) */
      float cm[3];
      for (int a = 0; a < 3; ++a) cm[a] = c->base_com[a] + (u[RU_COM + a] * 2.0f - 1.0f) * c->com_disp[a];
      E->com_x[e] = cm[0]; E->com_y[e] = cm[1]; E->com_z[e] = cm[2];
    } else if (c->mass_dr_on && c->com_mode == 2 && c->com_legacy_r > 0.f) {  /* legacy disk (:112-124) */
      const float r = u[RU_COM] * c->com_legacy_r;
      const float th = u[RU_COM + 1] * (float)OPI * 2.0f;
      float sth, cth;
      usv_sincos_cr(th, &sth, &cth);
      E->com_x[e] = c->base_com[0] + cth * r;
      E->com_y[e] = c->base_com[1] + sth * r;
      E->com_z[e] = c->base_com[2];
    } else {
      E->com_x[e] = c->base_com[0]; E->com_y[e] = c->base_com[1]; E->com_z[e] = c->base_com[2];
    }
    /* independent yaw-inertia randomisation (USV_Virtual.py:193-240), skipped when coupled */
    if (c->indep_kiz_on && !c->couple_kiz) {
      const float uu = u[RU_KIZ];
      E->k_iz[e] = c->kiz_log ? expf(logf(c->kiz_min) + uu * (logf(c->kiz_max) - logf(c->kiz_min)))
                              : c->kiz_min + uu * (c->kiz_max - c->kiz_min);
    }
    /* HydrodynamicsObject.reset_coefficients (Hydrodynamics.py:136-174) */
    if (c->drag_rand_on && E->lin_damp) {
      for (int a = 0; a < 3; ++a) {
        const int dof = (a == 2) ? 5 : a;  (void)dof;
        E->lin_damp[a * n + e] = c->lin_damp[a] + (u[RU_DRAG + a] * 2.0f - 1.0f) * c->lin_rand[a];
        E->quad_damp[a * n + e] = c->quad_damp[a] + (u[RU_DRAG + 6 + a] * 2.0f - 1.0f) * c->quad_rand[a];
      }
    }
    if (c->indep_kdrag_on) {
      const float uu = u[RU_KDRAG];
      E->k_drag[e] = c->kdrag_log ? expf(logf(c->kdrag_min) + uu * (logf(c->kdrag_max) - logf(c->kdrag_min)))
                                  : c->kdrag_min + uu * (c->kdrag_max - c->kdrag_min);
    }
    /* DynamicsFirstOrder.reset_thruster_randomization (ThrusterDynamics.py:112-127) */
    if (c->indep_thr_on) {
      if (c->thr_separate) {
        E->thr_l[e] = u[RU_THR] * 2.0f * c->left_rand + (1.0f - c->left_rand);
        E->thr_r[e] = u[RU_THR + 1] * 2.0f * c->right_rand + (1.0f - c->right_rand);
      } else {
        const float m = u[RU_THR] * 2.0f * c->thr_rand + (1.0f - c->thr_rand);
        E->thr_l[e] = m; E->thr_r[e] = m;
      }
    }
    /* ForceDisturbance.generate_force / TorqueDisturbance.generate_torque
     * (USV_disturbances.py:327-508, reset_idx:1517-1518) */
    if (E->dist) {
      float *D = E->dist;
      if (c->fdist_on && c->fsin_on) {
        const float fr_ = (float)((double)c->ffreq_max - (double)c->ffreq_min);
        const float sr_ = (float)((double)c->fshift_max - (double)c->fshift_min);
        D[DI_FXF * n + e] = u[RU_FSIN] * fr_ + c->ffreq_min;
        D[DI_FYF * n + e] = u[RU_FSIN + 1] * fr_ + c->ffreq_min;
        D[DI_FXS * n + e] = u[RU_FSIN + 2] * sr_ + c->fshift_min;
        D[DI_FYS * n + e] = u[RU_FSIN + 3] * sr_ + c->fshift_min;
        D[DI_FAMP * n + e] = u[RU_FSIN + 4] * (float)((double)c->fsin_max - (double)c->fsin_min) + c->fsin_min;
      }
      if (c->fdist_on && c->fconst_on) {
        const float rr = u[RU_FCONST] * (float)((double)c->fconst_max - (double)c->fconst_min) + c->fconst_min;
        const float tt = u[RU_FCONST + 1] * (float)OPI * 2.0f;
        float st, ct;
        usv_sincos_cr(tt, &st, &ct);
        if (c->inj_trig) { ct = u[RU_TRIG + 4]; st = u[RU_TRIG + 5]; }   /* the reference's recorded values */
        D[DI_FCX * n + e] = ct * rr;
        D[DI_FCY * n + e] = st * rr;
      }
      if (c->tdist_on && c->tsin_on) {
        D[DI_TF * n + e] = u[RU_TSIN] * (float)((double)c->tfreq_max - (double)c->tfreq_min) + c->tfreq_min;
        D[DI_TS * n + e] = u[RU_TSIN + 1] * (float)((double)c->tshift_max - (double)c->tshift_min) + c->tshift_min;
        D[DI_TAMP * n + e] = u[RU_TSIN + 2] * (float)((double)c->tsin_max - (double)c->tsin_min) + c->tsin_min;
      }
      if (c->tdist_on && c->tconst_on) {
        float rr = u[RU_TCONST] * (float)((double)c->tconst_max - (double)c->tconst_min) + c->tconst_min;
        if (u[RU_TCONST + 1] > 0.5f) rr = rr * -1.0f;
        D[DI_TC * n + e] = rr;
      }
    }
    /* _apply_mass_driven_coupling (USV_Virtual.py:988-1040) */
    if (c->couple_drag || c->couple_thr || c->couple_kiz) {
      const double denom = ((double)c->mass_max - (double)c->base_mass) > 1e-6 ? ((double)c->mass_max - (double)c->base_mass) : 1e-6;
      float r = (E->mass[e] - c->base_mass) / (float)denom;
      r = clampf_(r, 0.f, 1.f);
      E->mass_r[e] = r;
      if (c->couple_drag) E->k_drag[e] = c->kdrag_min + r * (float)((double)c->kdrag_max - (double)c->kdrag_min);
      if (c->couple_thr) {
        float s_thr = 1.0f - r * c->thr_rand;
        s_thr = clampf_(s_thr, (float)(1.0 - (double)c->thr_rand), 1.0f);
        E->thr_l[e] = s_thr; E->thr_r[e] = s_thr;
      }
      if (c->couple_kiz) E->k_iz[e] = c->kiz_min + r * (float)((double)c->kiz_max - (double)c->kiz_min);
    }
    /* CaptureXYTask.get_spawns (static_obs.py:936-1060).  The field and the
     * obstacle box use the target of the PREVIOUS episode: get_goals runs later
     * in set_targets (USV_Virtual.py:1618). */
    const float rmin = c->spawn_rmin, rmax = c->spawn_rmax;
    /* the spawn heading reaches the stand-in as the quaternion (cos(yaw0 / 2), 0, 0, sin(yaw0 / 2))
       (static_obs.py:959-961), which set_world_poses turns into its yaw; c->inj_trig: the parity harness's
       recorded torch.cos / torch.sin values (RU_TRIG) instead of usv_sincos_cr */
    float qz0, qw0;
    usv_sincos_cr(u[RU_YAW] * (float)OPI * 0.5f, &qz0, &qw0);
    if (c->inj_trig) { qw0 = u[RU_TRIG + 2]; qz0 = u[RU_TRIG + 3]; }
    const float yaw0 = usv_yaw_of_quat(qw0, qz0);
    float cth = 0.f, sth = 0.f;
    if (c->task_kind != USV_TASK_TRACK_XYO) {
      usv_sincos_cr(u[RU_SPAWN_TH] * 2.0f * (float)OPI, &sth, &cth);
      if (c->inj_trig) { cth = u[RU_TRIG]; sth = u[RU_TRIG + 1]; }
    }
    float sx, sy;
    if (c->task_kind == USV_TASK_GO_TO_POSE) {
      /* GoToPoseTask.get_spawns (USV_go_to_pose.py:256-319): disk around the previous target, radii from the
         curriculum at the reset's USVVirtual.step when it is on (:266-290) */
      double dmax = rmax, dmin = rmin;
      if (c->curriculum_on) {
        dmax = curriculum_lerp(c, E->step_f, c->cur_max_dist, c->max_spawn_d);
        dmin = curriculum_lerp(c, E->step_f, c->cur_min_dist, c->min_spawn_d);
      }
      const float r = u[RU_SPAWN_R] * (float)(dmax - dmin) + (float)dmin;
      sx = r * cth + E->tgt_x[e];
      sy = r * sth + E->tgt_y[e];
      E->prev_dist[e] = 0.f;   /* GoToPoseTask.reset: prev_position_dist = 0 (:227) */
    } else if (c->task_kind == USV_TASK_TRACK_XYO) {
      sx = 0.f; sy = 0.f;      /* TrackXYOVelocityTask.get_spawns (:203-219): heading only */
    } else {
      const float r = u[RU_SPAWN_R] * (rmax - rmin) + rmin;
      sx = r * cth; sy = r * sth;
    }
    if (c->task_kind != USV_TASK_CAPTURE_XY) {
      E->px[e] = sx; E->py[e] = sy; E->yaw[e] = yaw0;
      E->vx[e] = u[RU_VX] * 3.0f - 1.5f;
      E->vy[e] = u[RU_VY] * 3.0f - 1.5f;
      E->wz[e] = 0.f;
      E->reset_buf[e] = 0; E->progress[e] = 0;
      E->prev_cmd[0 * n + e] = 0.f; E->prev_cmd[1 * n + e] = 0.f;
      for (int q = 0; q < USV_NSTAT; ++q) E->stats[q * n + e] = 0.f;
      if (c->task_kind == USV_TASK_GO_TO_POSE) {   /* get_goals (USV_go_to_pose.py:229-254) */
        const float g = c->goal_random_position;
        E->tgt_x[e] = u[RU_GOAL + 0] * g * 2.0f - g;
        E->tgt_y[e] = u[RU_GOAL + 1] * g * 2.0f - g;
        E->tgt_h[e] = u[RU_GOAL_H] * (float)OPI * 2.0f;
      } else {                                     /* get_goals (USV_track_xyo_velocity.py:178-199) */
        const float gl = c->tk_goal_rand[0], ga = c->tk_goal_rand[1];
        E->tgt_x[e] = u[RU_GOAL + 0] * gl * 2.0f - gl;
        E->tgt_y[e] = u[RU_GOAL + 1] * gl * 2.0f - gl;
        E->tgt_h[e] = u[RU_GOAL_H] * ga * 2.0f - ga;
      }
      continue;
    }
    if (rows) {
      /* scene replay (USVVirtual._scene_replay_apply, USV_Virtual.py:1395-1457; CaptureXYTask.apply_scene
       * static_obs.py:785-863): pose / velocity / goal / obstacles from the scene row; the field uses
       * the NEW goal; no spawn, velocity or goal draws; set_targets is not called */
      const float *sc = rows + (size_t)s * USV_SCENE_STRIDE;
      for (int o = 0; o < USV_NOBST; ++o)
        for (int a = 0; a < 2; ++a) {
          const float v = sc[USV_SC_OBST + 2 * o + a];
          E->obst[(o * 2 + a) * n + e] = v;
          obst_k[(s * USV_NOBST + o) * 2 + a] = v;
        }
      E->tgt_x[e] = sc[USV_SC_GOAL]; E->tgt_y[e] = sc[USV_SC_GOAL + 1];
      tgt_k[s * 2 + 0] = sc[USV_SC_GOAL]; tgt_k[s * 2 + 1] = sc[USV_SC_GOAL + 1];
      E->px[e] = sc[USV_SC_START]; E->py[e] = sc[USV_SC_START + 1];
      {  /* the yaw-only quaternion of the start yaw (USV_Virtual.py:1447-1450) through set_world_poses */
        float hz, hw;
        usv_sincos_cr(0.5f * sc[USV_SC_YAW], &hz, &hw);
        if (c->inj_trig) { hw = u[RU_TRIG + 2]; hz = u[RU_TRIG + 3]; }
        E->yaw[e] = usv_yaw_of_quat(hw, hz);
      }
      E->vx[e] = sc[USV_SC_VEL]; E->vy[e] = sc[USV_SC_VEL + 1];
      E->wz[e] = 0.f;
      E->reset_buf[e] = 0; E->progress[e] = 0;
      E->prev_cmd[0 * n + e] = 0.f; E->prev_cmd[1 * n + e] = 0.f;
      for (int q = 0; q < USV_NSTAT; ++q) E->stats[q * n + e] = 0.f;
      continue;
    }
    const float tx = E->tgt_x[e], ty = E->tgt_y[e];
    float oc[USV_NOBST][2];
    const float mn[2] = {tx - c->obst_box, ty - c->obst_box};
    const float mx[2] = {tx + c->obst_box, ty + c->obst_box};
    for (int o = 0; o < USV_NOBST; ++o)
      for (int a = 0; a < 2; ++a) oc[o][a] = u[RU_OBST + o * 2 + a] * (mx[a] - mn[a]) + mn[a];
    const float sep2 = c->min_obs_sep * c->min_obs_sep;
    for (int it = 0; it < USV_SPAWN_ITERS; ++it) {
      int inval[USV_NOBST], any = 0;
      for (int o = 0; o < USV_NOBST; ++o) {
        const float ds = tnorm2(oc[o][0] - sx, oc[o][1] - sy);
        const float dt = tnorm2(oc[o][0] - tx, oc[o][1] - ty);
        inval[o] = (ds < c->min_dist_safe) || (dt < c->min_dist_safe);
      }
      for (int j = 0; j < USV_NOBST; ++j)
        for (int i = 0; i < j; ++i) {
          const int vi = oc[i][0] < 900.f, vj = oc[j][0] < 900.f;
          const float dx = oc[i][0] - oc[j][0], dy = oc[i][1] - oc[j][1];
          if (vi && vj && (dx * dx + dy * dy) < sep2) inval[j] = 1;
        }
      for (int o = 0; o < USV_NOBST; ++o) any |= inval[o];
      if (!any) break;
      const float *rs = u + RU_RESAMPLE + it * USV_NOBST * 2;
      for (int o = 0; o < USV_NOBST; ++o)
        if (inval[o])
          for (int a = 0; a < 2; ++a) oc[o][a] = rs[o * 2 + a] * (mx[a] - mn[a]) + mn[a];
    }
    {
      int inval[USV_NOBST];
      for (int o = 0; o < USV_NOBST; ++o) {
        const float ds = tnorm2(oc[o][0] - sx, oc[o][1] - sy);
        const float dt = tnorm2(oc[o][0] - tx, oc[o][1] - ty);
        inval[o] = (ds < c->min_dist_safe) || (dt < c->min_dist_safe);
      }
      for (int j = 0; j < USV_NOBST; ++j)
        for (int i = 0; i < j; ++i) {
          const int vi = oc[i][0] < 900.f, vj = oc[j][0] < 900.f;
          const float dx = oc[i][0] - oc[j][0], dy = oc[i][1] - oc[j][1];
          if (vi && vj && (dx * dx + dy * dy) < sep2) inval[j] = 1;
        }
      for (int o = 0; o < USV_NOBST; ++o)
        if (inval[o]) { oc[o][0] = 999.0f; oc[o][1] = 999.0f; }    /* limbo (:1042-1048) */
    }
    for (int o = 0; o < USV_NOBST; ++o) {
      E->obst[(o * 2 + 0) * n + e] = oc[o][0];
      E->obst[(o * 2 + 1) * n + e] = oc[o][1];
      obst_k[(s * USV_NOBST + o) * 2 + 0] = oc[o][0];
      obst_k[(s * USV_NOBST + o) * 2 + 1] = oc[o][1];
    }
    tgt_k[s * 2 + 0] = tx; tgt_k[s * 2 + 1] = ty;
    /* pose and velocities (USV_Virtual.py:1541-1572) */
    E->px[e] = sx; E->py[e] = sy; E->yaw[e] = yaw0;
    E->vx[e] = u[RU_VX] * 3.0f - 1.5f;
    E->vy[e] = u[RU_VY] * 3.0f - 1.5f;
    E->wz[e] = 0.f;
    /* bookkeeping (:1574-1579) */
    E->reset_buf[e] = 0; E->progress[e] = 0;
    E->prev_cmd[0 * n + e] = 0.f; E->prev_cmd[1 * n + e] = 0.f;
    for (int q = 0; q < USV_NSTAT; ++q) E->stats[q * n + e] = 0.f;
    E->stats[ST_SUCCESS * n + e] = 0.f; E->stats[ST_COLLISION * n + e] = 0.f;
    /* set_targets -> get_goals (static_obs.py:913-930) */
    const float g = c->goal_random_position;
    E->tgt_x[e] = u[RU_GOAL + 0] * g * 2.0f - g;
    E->tgt_y[e] = u[RU_GOAL + 1] * g * 2.0f - g;
  }
  /* potential field of the reset batch (static_obs.py:1054-1057); skipped when a test supplies the fields
     itself (oracle_set_skip_field: the full-size check copies the device's fields into E->field) */
  if (c->task_kind == USV_TASK_CAPTURE_XY && !g_skip_field) {
    oracle_potential_field(c, k, obst_k, tgt_k, fld_k, NULL, E->grid_lin);
    for (int s = 0; s < k; ++s)
      memcpy(E->field + (size_t)ids[s] * USV_GRID2, fld_k + (size_t)s * USV_GRID2, sizeof(float) * USV_GRID2);
  }
  free(obst_k); free(tgt_k); free(fld_k);
}

void oracle_step_pre(const usv_cfg_t *c, oracle_env_t *E, const float *actions, const float *lut,
                     float action_bias, const float *U);
void oracle_step_physics(const usv_cfg_t *c, oracle_env_t *E);
void oracle_step_post(const usv_cfg_t *c, oracle_env_t *E, const float *U);

/* ------------------------------------------------------------------------ */
/* One control step (VecEnvRLGames.step, envs/vec_env_rlgames.py:120-217)    */
/* actions: [n][2] policy output; U: [n][NU_STEP] uniforms.                  */
/* The reset part of pre_physics_step must be run first (oracle_reset).      */
/* ------------------------------------------------------------------------ */
void oracle_step(const usv_cfg_t *c, oracle_env_t *E, const float *actions, const float *lut /*[2][1000]*/,
                 float action_bias, const float *U) {
  oracle_step_pre(c, E, actions, lut, action_bias, U);
  oracle_step_physics(c, E);
  oracle_step_post(c, E, U);
}

void oracle_step_pre(const usv_cfg_t *c, oracle_env_t *E, const float *actions, const float *lut,
                     float action_bias, const float *U) {
  const int n = E->n;
  OMP_FOR
  for (int e = 0; e < n; ++e) {
    const float *u = U + (size_t)e * USV_NU_STEP;
    const int was_reset = E->just_reset[e];
    float *dbg = E->dbg ? E->dbg + (size_t)e * USV_ORACLE_NDBG : NULL;
    float *tmp = E->tmp + (size_t)e * 8;
    /* ---- VecEnvRLGames.step: clamp actions (:136-140) ---- */
    float cmd[2], thrust[2], uu[2], unit[2], tgt[2];
    for (int a = 0; a < 2; ++a) cmd[a] = clampf_(actions[e * 2 + a], -c->clip_actions, c->clip_actions);
    /* ---- USVVirtual.pre_physics_step (USV_Virtual.py:1050-1099) ---- */
    for (int a = 0; a < 2; ++a) {
      E->prev_cmd[a * n + e] = was_reset ? 0.f : cmd[a];                 /* :1064-1066 */
      float t = cmd[a];
      if (action_bias != 0.f) t = t + action_bias;                        /* :1071-1075 */
      if (c->act_noise_on) t = t + (u[SU_ACT + a] * (float)((double)c->act_noise_max - (double)c->act_noise_min) + c->act_noise_min);
      t = clampf_(t, -1.f, 1.f);                                          /* :1082 */
      thrust[a] = t;
      float v = c->affine_thrust ? 0.5f * (t + 1.0f) : clampf_(t, 0.f, 1.f);
      v = clampf_(v, 0.f, 1.f);
      unit[a] = v;                                                        /* thrust_cmds_unit :1095 */
      uu[a] = was_reset ? 0.f : v;                                        /* :1097 */
    }
    /* set_target_force -> get_cmd_interpolated (ThrusterDynamics.py:179-219) */
    for (int a = 0; a < 2; ++a) {
      const int idx = lut_index(uu[a], USV_LUT_N);
      float f = lut[a * USV_LUT_N + idx];
      if (c->use_thr_mult) f = f * (a == 0 ? E->thr_l[e] : E->thr_r[e]);
      tgt[a] = f;
    }
    if (dbg) { dbg[0] = uu[0]; dbg[1] = uu[1]; dbg[2] = tgt[0]; dbg[3] = tgt[1]; }
    tmp[0] = cmd[0]; tmp[1] = cmd[1]; tmp[2] = thrust[0]; tmp[3] = thrust[1];
    tmp[4] = unit[0]; tmp[5] = unit[1]; tmp[6] = tgt[0]; tmp[7] = tgt[1];
  }
}

void oracle_step_physics(const usv_cfg_t *c, oracle_env_t *E) {
  const float PI_F = (float)OPI, TWO_PI_F = (float)(2.0 * OPI);
  const int n = E->n;
  OMP_FOR
  for (int e = 0; e < E->n; ++e) {
    const float *tmp = E->tmp + (size_t)e * 8;
    const float tgt[2] = {tmp[6], tmp[7]};
    /* ---- 10 physics substeps (:154-171): forces then integration ---- */
    const float m = E->mass[e];
    const float izz = c->izz0 * E->k_iz[e];
    for (int s = 0; s < c->substeps; ++s) {
      /* DynamicsFirstOrder.update (ThrusterDynamics.py:132-136) */
      E->fl[e] = E->fl[e] * c->thr_alpha + (1.0f - c->thr_alpha) * tgt[0];
      E->fr[e] = E->fr[e] * c->thr_alpha + (1.0f - c->thr_alpha) * tgt[1];
      /* the read-back attitude R = quaternion_to_matrix(q(yaw)) (usv_quat_rot) */
      const quat_rot_t qr = usv_quat_rot(E->yaw[e]);
      const float cy = qr.C, sy = qr.S;
      /* apply_forces reads the cached root state: the pre-reset one in a reset env's first substep (C.1) */
      const int cached = s == 0 && c->stale_root && E->just_reset[e] && E->root_cache;
      const float *rc = E->root_cache;
      const float hpx = cached ? rc[0 * n + e] : E->px[e], hpy = cached ? rc[1 * n + e] : E->py[e];
      const quat_rot_t qc = usv_quat_rot(cached ? rc[2 * n + e] : E->yaw[e]);
      const float hcy = qc.C, hsy = qc.S;
      const float hvx = cached ? rc[3 * n + e] : E->vx[e], hvy = cached ? rc[4 * n + e] : E->vy[e];
      const float hwz = cached ? rc[5 * n + e] : E->wz[e];
      float X, Y, N, d3[3];
      if (E->dist) disturbance(c, E, e, hpx, hpy, &d3[0], &d3[1], &d3[2]);
      planar_forces(c, E, e, hcy, hsy, hvx, hvy, hwz, E->fl[e], E->fr[e], E->dist ? d3 : NULL, &X, &Y, &N);
      /* PhysX applies the body-frame wrench in the body's CURRENT frame (is_global=False) */
      /* build's 3-DoF semi-implicit Euler (no reference: PhysX) */
      const float ax = (cy * X - sy * Y) / m;
      const float ay = (sy * X + cy * Y) / m;
      const float aw = N / izz;
      E->vx[e] = E->vx[e] + ax * c->dt;
      E->vy[e] = E->vy[e] + ay * c->dt;
      E->wz[e] = E->wz[e] + aw * c->dt;
      E->px[e] = E->px[e] + E->vx[e] * c->dt;
      E->py[e] = E->py[e] + E->vy[e] * c->dt;
      float yw = E->yaw[e] + E->wz[e] * c->dt;
      if (yw > PI_F) yw -= TWO_PI_F;
      else if (yw <= -PI_F) yw += TWO_PI_F;
      E->yaw[e] = yw;
    }
  }
}

/* privileged tail (USV_Virtual.py:840-976; MDD.get_masses USV_disturbances.py:153-194) */
static void priv_tail(const usv_cfg_t *c, const oracle_env_t *E, int e, float *obs) {
  float mass_o, com_o[3];
  const float comv[3] = {E->com_x[e], E->com_y[e], E->com_z[e]};
  if (c->masscom_base) {
    mass_o = c->mass_relative ? 0.f : c->base_mass;
    for (int a = 0; a < 3; ++a) com_o[a] = c->com_scaled ? c->base_com[a] / (c->com_scale[a] + 1e-6f) : c->base_com[a];
  } else {
    const float denom = (float)(fabs((double)c->base_mass) > 1e-6 ? fabs((double)c->base_mass) : 1e-6);
    mass_o = c->mass_relative ? (E->mass[e] - c->base_mass) / denom : E->mass[e];
    for (int a = 0; a < 3; ++a) com_o[a] = c->com_scaled ? comv[a] / (c->com_scale[a] + 1e-6f) : comv[a];
  }
  float *pt = obs + USV_NOBS_BASE;   /* priv_dim = 4: columns 29..32 stay 0 (input padding) */
  pt[0] = mass_o; pt[1] = com_o[0]; pt[2] = com_o[1]; pt[3] = com_o[2];
  if (c->priv_dim == 8) {
    float kd, tl, tr, kz;
    if (c->masscom_base) {
      if (c->priv_mode == 2) {
        kd = 0.5f * (c->kdrag_min + c->kdrag_max);
        tl = tr = c->couple_thr ? (1.0f - 0.5f * c->thr_rand) : 1.0f;
        kz = 0.5f * (c->kiz_min + c->kiz_max);
      } else { kd = tl = tr = kz = 1.0f; }
    } else {
      kd = E->k_drag[e];
      tl = E->thr_l[e]; tr = E->thr_r[e];
      kz = E->k_iz[e];
    }
    if (c->priv_mode == 1) {
      kd = enc_centered(kd, c->kdrag_min, c->kdrag_max, c->priv_nominal);
      tl = enc_centered(tl, c->thr_min, c->thr_max, c->priv_nominal);
      tr = enc_centered(tr, c->thr_min, c->thr_max, c->priv_nominal);
      kz = enc_centered(kz, c->kiz_min, c->kiz_max, c->priv_nominal);
    } else if (c->priv_mode == 2) {
      kd = c->priv_drag_on ? enc_minmax(kd, c->kdrag_min, c->kdrag_max) : 0.f;
      tl = c->priv_thr_on ? enc_minmax(tl, c->thr_min, c->thr_max) : 0.f;
      tr = c->priv_thr_on ? enc_minmax(tr, c->thr_min, c->thr_max) : 0.f;
      kz = c->priv_kiz_on ? enc_minmax(kz, c->kiz_min, c->kiz_max) : 0.f;
    }
    pt[4] = kd; pt[5] = tl; pt[6] = tr; pt[7] = kz;
  }
}

static void oracle_step_post_task(const usv_cfg_t *c, oracle_env_t *E, const float *U);

static void oracle_step_post_impl(const usv_cfg_t *c, oracle_env_t *E, const float *U);
void oracle_step_post(const usv_cfg_t *c, oracle_env_t *E, const float *U) {
  oracle_step_post_impl(c, E, U);
  E->step_f += c->step_inc;   /* calculate_metrics: USVVirtual.step += 1 / horizon_length (USV_Virtual.py:1633) */
}
static void oracle_step_post_impl(const usv_cfg_t *c, oracle_env_t *E, const float *U) {
  if (c->task_kind != USV_TASK_CAPTURE_XY) { oracle_step_post_task(c, E, U); return; }
  const int n = E->n;
  const int any_reset_none = (E->ctl[USV_CTL_POT_VALID] == 0);
  const int pen_valid = E->ctl[USV_CTL_PEN_VALID];
  const int rew_valid = E->ctl[USV_CTL_REW_VALID];
  const float PI_F = (float)OPI, TWO_PI_F = (float)(2.0 * OPI);
  OMP_FOR
  for (int e = 0; e < n; ++e) {
    const float *u = U + (size_t)e * USV_NU_STEP;
    const int was_reset = E->just_reset[e];
    float *dbg = E->dbg ? E->dbg + (size_t)e * USV_ORACLE_NDBG : NULL;
    const float *tmp = E->tmp + (size_t)e * 8;
    const float cmd[2] = {tmp[0], tmp[1]}, thrust[2] = {tmp[2], tmp[3]}, unit[2] = {tmp[4], tmp[5]};
    /* ---- post_physics_step (rl_task.py:283-303) ---- */
    E->progress[e] += 1;
    /* update_state (USV_Virtual.py:771-813) with the noise of the last call */
    float px = E->px[e], py = E->py[e];
    if (c->pos_noise_on) {
      const float rng = (float)((double)c->pos_noise_max - (double)c->pos_noise_min);
      px = px + (u[SU_PX] * rng + c->pos_noise_min);
      py = py + (u[SU_PX + 1] * rng + c->pos_noise_min);
    }
    float vxn = E->vx[e], vyn = E->vy[e], wzn = E->wz[e];
    if (c->vel_noise_on) {
      const float rng = (float)((double)c->vel_noise_max - (double)c->vel_noise_min);
      vxn = vxn + (u[SU_VX] * rng + c->vel_noise_min);
      vyn = vyn + (u[SU_VY] * rng + c->vel_noise_min);
      wzn = wzn + (u[SU_WZ] * rng + c->vel_noise_min);
    }
    float yawn = usv_heading(usv_quat_rot(E->yaw[e]));   /* update_state's heading (USV_Virtual.py:776-786) */
    if (c->head_noise_on) {
      const float rng = (float)((double)c->head_noise_max - (double)c->head_noise_min);
      yawn = yawn + (u[SU_HEAD] * rng + c->head_noise_min);
    }
    const float hc = usv_cos(yawn), hs = usv_sin(yawn);
    /* ---- get_observations -> CaptureXYTask.get_state_observations (static_obs.py:193-299) ---- */
    float obs[USV_NOBS];
    memset(obs, 0, sizeof(obs));
    const float ex = E->tgt_x[e] - px, ey = E->tgt_y[e] - py;
    const float theta = usv_atan2(hs, hc);
    const float beta = usv_atan2(ey, ex);
    const float alpha = fmodf((beta - theta) + PI_F, TWO_PI_F) - PI_F;
    const float herr = fabsf(alpha);
    const float dist = sqrtf(ex * ex + ey * ey);       /* compute_reward :338 */
    const float dist_n = tnorm2(ex, ey);                /* task_data[2] :224 */
    float od[USV_NOBST], orx[USV_NOBST], ory[USV_NOBST];
    float min_od = INFINITY;
    for (int o = 0; o < USV_NOBST; ++o) {
      orx[o] = E->obst[(o * 2 + 0) * n + e] - px;
      ory[o] = E->obst[(o * 2 + 1) * n + e] - py;
      od[o] = tnorm2(orx[o], ory[o]);
      if (od[o] < min_od) min_od = od[o];
    }
    /* torch.topk(k=5, largest=False): ascending, ties keep lower index first */
    int used[USV_NOBST] = {0}, sel[USV_NCLOSE];
    for (int q = 0; q < USV_NCLOSE; ++q) {
      int best = -1;
      for (int o = 0; o < USV_NOBST; ++o)
        if (!used[o] && (best < 0 || od[o] < od[best])) best = o;
      used[best] = 1; sel[q] = best;
    }
    const float ct = usv_cos(theta), st = usv_sin(theta);
    float task[5 + 3 * USV_NCLOSE];
    memset(task, 0, sizeof(task));
    task[0] = usv_cos(alpha); task[1] = usv_sin(alpha); task[2] = dist_n;
    for (int q = 0; q < USV_NCLOSE; ++q) {
      const int o = sel[q];
      const float bx = orx[o] * ct + ory[o] * st;
      const float by = -orx[o] * st + ory[o] * ct;
      const float nf = sqrtf(bx * bx + by * by + 1e-6f);
      task[5 + q * 3 + 0] = od[o] - c->obstacle_radius;
      task[5 + q * 3 + 1] = -bx / nf;
      task[5 + q * 3 + 2] = -by / nf;
    }
    /* Core.update_observation_tensor (USV_core.py:55-125) */
    if (c->obs_local) {
      obs[0] = hc * vxn + hs * vyn;
      obs[1] = -hs * vxn + hc * vyn;
    } else {
      obs[0] = vxn; obs[1] = vyn;
    }
    obs[2] = wzn;
    for (int q = 0; q < 5 + 3 * USV_NCLOSE; ++q) obs[3 + q] = task[q];
    const int pa = USV_NOBS_BASE - 2;
    obs[pa + 0] = E->prev_cmd[0 * n + e];
    obs[pa + 1] = E->prev_cmd[1 * n + e];
    priv_tail(c, E, e, obs);
    /* ---- calculate_metrics -> CaptureXYTask.compute_reward (static_obs.py:335-657) ---- */
    const float bover = maxf_(dist - c->kill_dist, 0.f);
    const float bx_ = minf_(bover / 0.25f, 20.0f);
    const float boundary_pen = -expm1f(bx_) * c->boundary_cost;
    const int gir = dist < c->position_tolerance;
    E->goal_cnt[e] = E->goal_cnt[e] * gir + gir;
    /* CaptureXYReward.compute_reward (USV_task_rewards.py:44-80) */
    const float prev_err = rew_valid ? E->prev_dist[e] : dist;
    float dist_r;
    if (c->reward_mode == 0) dist_r = c->position_scale * (prev_err - dist);
    else if (c->reward_mode == 1) dist_r = c->position_scale * (prev_err * prev_err - dist * dist);
    else dist_r = c->position_scale * (usv_exp(-dist / c->exp_coeff) - usv_exp(-prev_err / c->exp_coeff));
    const float h2 = herr * herr;
    float align_r = c->align_la1 * (usv_exp(c->align_la2 * (h2 * h2)) + usv_exp(c->align_la3 * h2));
    if (was_reset) dist_r = 0.f;                                          /* :374 */
    const float prev_dist = was_reset ? dist : (rew_valid ? E->prev_dist[e] : dist);  /* :361-380 */
    float pot = sample_field(E->field + (size_t)e * USV_GRID2, c->map_size, px, py);
    if (dbg) dbg[14] = pot;
    if (E->pos_in && dbg) {   /* the oracle's field at the device's integrated position, same noise as above */
      float qx = E->pos_in[e], qy = E->pos_in[n + e];
      if (c->pos_noise_on) {
        const float rng = (float)((double)c->pos_noise_max - (double)c->pos_noise_min);
        qx = qx + (u[SU_PX] * rng + c->pos_noise_min);
        qy = qy + (u[SU_PX + 1] * rng + c->pos_noise_min);
      }
      dbg[15] = sample_field(E->field + (size_t)e * USV_GRID2, c->map_size, qx, qy);
    }
    if (E->pot_in) pot = E->pot_in[e];
    const float pn = clampf_(pot, 0.f, 1.f);
    const float xs = clampf_((pn - 0.6f) / (0.3f + 1e-6f), 0.f, 1.f);
    const float danger = xs * xs * (3.0f - 2.0f * xs);
    align_r = align_r * maxf_(0.3f, 1.0f - danger);
    dist_r = dist_r * maxf_(0.6f, 1.0f - danger * 0.5f);
    const float g = clampf_(usv_cos(herr), 0.f, 1.f);
    dist_r = minf_(dist_r, 0.f) + g * maxf_(dist_r, 0.f);
    float prev_h = (rew_valid && !was_reset) ? E->prev_head[e] : herr;
    float hi = clampf_(prev_h - herr, -0.4f, 0.4f);
    const float hi_r = hi * 0.05f;
    E->prev_head[e] = herr;
    const float prev_pot = (any_reset_none || was_reset) ? pot : E->prev_pot[e];
    float praw = (prev_pot - pot) * 100.0f;
    const float praw_in = praw;   /* before the dead zone (dbg[11]: the tests' discontinuity margins) */
    if (fabsf(praw) < 0.01f) praw = 0.f;
    const float pa1 = 2.0f * usv_tanh(praw / (2.0f + 1e-6f));
    const float gdx = ex / (dist + 1e-6f), gdy = ey / (dist + 1e-6f);
    const float vtow = vxn * gdx + vyn * gdy;
    const float vtp = maxf_(vtow, 0.f);
    const float dd = prev_dist - dist;
    const float ddp = maxf_(dd, 0.f);
    const float gv = clampf_((vtp - 0.02f) / ((0.15f - 0.02f) + 1e-6f), 0.f, 1.f);
    const float gd = clampf_(ddp / (0.01f + 1e-6f), 0.f, 1.f);
    const float gprog = maxf_(gv, gd);
    const float ggate = gprog * g;
    const float ppos = maxf_(pa1, 0.f), pneg = minf_(pa1, 0.f);
    const float gate_pos = (ppos < 0.5f) ? 1.0f : ggate;
    const float shaping = gate_pos * ppos + pneg;
    const int worsening = shaping < -0.05f;
    const int turning = fabsf(wzn) > 0.2f;
    const float vfwd = vxn * hc + vyn * hs;
    const float sf = clampf_((fabsf(vfwd) - 0.15f) / ((0.60f - 0.15f) + 1e-6f), 0.f, 1.f);
    const float turn_haz = (float)(worsening && turning) * (-10.0f) * (g * g) * sf;
    E->prev_pot[e] = pot;
    const float speed_r = (1.0f - usv_exp(-vtp / (0.8f + 1e-6f))) * 0.05f;
    float sgn = (alpha > 0.f) ? 1.f : ((alpha < 0.f) ? -1.f : 0.f);
    const float tang = (herr > 1.0f) ? sgn * 1.0f : sgn * 0.2f;
    const float dw = wzn - tang;
    const float ang_r = usv_exp(-(dw * dw) / 0.2f) * 0.03f;
    float coll = 0.f;
    for (int o = 0; o < USV_NOBST; ++o) coll += (float)(od[o] < c->collision_threshold) * (-10.0f) * 10.0f;
    const float goal_r = ((float)E->goal_cnt[e] * c->goal_reward) * 5.0f;
    E->prev_dist[e] = dist;
    const float total = dist_r * 0.5f + align_r * 0.5f + shaping * 2.0f + turn_haz + goal_r + c->time_reward +
                        coll + speed_r + ang_r + hi_r;
    /* ---- Penalties.compute_penalty (USV_task_rewards.py:440-523) ---- */
    const float pact0 = c->pen_use_u ? unit[0] : cmd[0];
    const float pact1 = c->pen_use_u ? unit[1] : cmd[1];
    float p_lin = 0.f, p_ang = 0.f, p_angv = 0.f, p_en = 0.f;
    if (c->pen_lin_kind == PEN_NORM) p_lin = -tnorm2(vxn, vyn) * c->pen_lin_k + c->pen_lin_c;
    if (c->pen_ang_kind) p_ang = pen_scalar(c->pen_ang_kind, c->pen_ang_k, c->pen_ang_x0, c->pen_ang_c, wzn);
    if (c->pen_angv_kind) {
      const float prev_w = pen_valid ? E->prev_wz[e] : wzn;
      p_angv = pen_scalar(c->pen_angv_kind, c->pen_angv_k, c->pen_angv_x0, c->pen_angv_c, wzn - prev_w);
    }
    if (c->pen_en_kind == PEN_SUM) p_en = -(pact0 + pact1) * c->pen_en_k + c->pen_en_c;
    else if (c->pen_en_kind == PEN_SUMSQ) p_en = -(pact0 * pact0 + pact1 * pact1) * c->pen_en_k + c->pen_en_c;
    E->prev_wz[e] = wzn;
    const float pens = p_lin + p_ang + p_angv + p_en;
    E->rew[e] = total + pens;
    /* ---- is_done -> CaptureXYTask.update_kills (static_obs.py:661-706) ---- */
    const int dkill = dist > c->kill_dist;
    const int ckill = min_od < c->collision_threshold;
    const int skill = E->goal_cnt[e] >= c->kill_after_n;
    const int die = dkill || ckill || skill;
    if (die) { E->done_coll[e] = ckill; E->done_succ[e] = skill && !ckill; }
    const int tout = E->progress[e] >= c->max_episode_length - 1;
    E->reset_buf[e] = c->fixed_horizon_eval ? tout : (tout ? 1 : die);
    /* ---- episode_sums (static_obs.py:720-765, Penalties.update_statistics, USV_Virtual.py:1187-1221) ---- */
    if (c->stats_on) {
      float *S = E->stats;
#define ADDS(k, v) S[(k) * n + e] += (v)
      ADDS(ST_TOTAL_REWARD, total); ADDS(ST_DISTANCE_REWARD, dist_r); ADDS(ST_ALIGNMENT_REWARD, align_r);
      ADDS(ST_HEADING_IMPROVE_REWARD, hi_r); ADDS(ST_POTENTIAL_SHAPING_REWARD, shaping);
      ADDS(ST_SPEED_REWARD, speed_r); ADDS(ST_ANGULAR_REWARD, ang_r); ADDS(ST_TURN_HAZARD_PENALTY, turn_haz);
      ADDS(ST_GOAL_REWARD, goal_r); ADDS(ST_TIME_REWARD, c->time_reward); ADDS(ST_COLLISION_REWARD, coll);
      ADDS(ST_DANGER_MEAN, danger); ADDS(ST_DANGER_HI_RATE, (float)(danger > 0.5f)); ADDS(ST_G_GATE_MEAN, gate_pos);
      ADDS(ST_POSITION_ERROR, dist); ADDS(ST_BOUNDARY_PENALTY, boundary_pen);
      if (c->pen_ang_kind) ADDS(ST_ANGULAR_VEL_PENALTY, p_ang);
      if (c->pen_angv_kind) ADDS(ST_ANGULAR_VEL_VARIATION_PENALTY, p_angv);
      if (c->pen_en_kind) ADDS(ST_ENERGY_PENALTY, p_en);
      ADDS(ST_NORMED_LINEAR_VEL, tnorm2(vxn, vyn));
      ADDS(ST_NORMED_ANGULAR_VEL, fabsf(wzn));
      ADDS(ST_CMD_NEG_RATE, ((float)(thrust[0] < 0.f) + (float)(thrust[1] < 0.f)) / 2.0f);
      ADDS(ST_U_MEAN, (unit[0] + unit[1]) / 2.0f);
      ADDS(ST_U_LOW_RATE, ((float)(unit[0] < 0.05f) + (float)(unit[1] < 0.05f)) / 2.0f);
      ADDS(ST_U_SUM, unit[0] + unit[1]);
#undef ADDS
    }
    if (dbg) { dbg[4] = pot; dbg[5] = danger; dbg[6] = total; dbg[7] = pens; dbg[8] = shaping; dbg[9] = dist_r; dbg[10] = align_r;
               dbg[11] = praw_in; dbg[12] = ppos; dbg[13] = ggate; dbg[16] = (float)(any_reset_none || was_reset); }
    /* ---- _process_data: clamp obs (vec_env_rlgames.py:85-95) ---- */
    for (int q = 0; q < USV_NOBS; ++q) E->obs[(size_t)e * USV_NOBS + q] = clampf_(obs[q], -c->clip_obs, c->clip_obs);
    E->just_reset[e] = 0;
  }
  E->ctl[USV_CTL_POT_VALID] = 1;
  E->ctl[USV_CTL_PEN_VALID] = 1;
  E->ctl[USV_CTL_REW_VALID] = 1;
}

/* ------------------------------------------------------------------------ */
/* GoToPose / TrackXYOVelocity post-physics step:               */
/* GoToPoseTask.get_state_observations/compute_reward/update_kills           */
/* (tasks/USV/USV_go_to_pose.py:89-209), GoToPoseReward (USV_task_rewards.py: */
/* 160-233); TrackXYOVelocityTask (USV_track_xyo_velocity.py:75-166),         */
/* TrackXYOVelocityReward (USV_task_rewards.py:328-393).  Glue as calculate_   */
/* metrics / is_done do for every task (USV_Virtual.py:1223-1237,1628-1652);  */
/* the task_data block is Core's 20 columns (unwritten ones 0).              */
/* ------------------------------------------------------------------------ */
static float task_term(int mode, float x, float coeff) {
  if (mode == 0) return 1.0f / (1.0f + x);
  if (mode == 1) return 1.0f / (1.0f + x * x);
  return usv_exp(-x / coeff);
}

/* torch.square(ang_err).sum(-1) over ALL envs (USV_track_xyo_velocity.py:121-123): the sum in the order the device
 * forms it (the reference's reduction order is torch's, unspecified), so the two agree bit for bit -- per 64-env wave
 * a butterfly (partners 32, 16, .., 1 apart), per 256-env block the four wave sums in order, then thread t of one
 * 256-thread block adds blocks t, t + 256, .. in order and a halving tree folds the 256 thread sums
 * (csrc/usv_env.hip: k_env_step_task's wave_sum / block partial, k_track_finish). */
static float track_ang_sum(const float *sq, int n) {
  const int nblk = (n + 255) / 256;
  float *part = (float *)calloc((size_t)nblk, sizeof(float));
  for (int blk = 0; blk < nblk; ++blk) {
    float sblk = 0.f;
    for (int w = 0; w < 4; ++w) {
      float v[64];
      for (int l = 0; l < 64; ++l) {
        const int e = blk * 256 + w * 64 + l;
        v[l] = e < n ? sq[e] : 0.f;
      }
      for (int off = 32; off > 0; off >>= 1) {
        float nv[64];
        for (int l = 0; l < 64; ++l) nv[l] = v[l] + v[l ^ off];
        memcpy(v, nv, sizeof(v));
      }
      sblk += v[0];
    }
    part[blk] = sblk;
  }
  float red[256];
  for (int t = 0; t < 256; ++t) {
    float acc = 0.f;
    for (int i = t; i < nblk; i += 256) acc += part[i];
    red[t] = acc;
  }
  for (int w = 128; w > 0; w >>= 1)
    for (int t = 0; t < w; ++t) red[t] += red[t + w];
  free(part);
  return red[0];
}

static void oracle_step_post_task(const usv_cfg_t *c, oracle_env_t *E, const float *U) {
  const int n = E->n;
  const int pen_valid = E->ctl[USV_CTL_PEN_VALID];
  const float PI_F = (float)OPI, TWO_PI_F = (float)(2.0 * OPI);
  const int track = c->task_kind == USV_TASK_TRACK_XYO;
  /* TrackXYOVelocity: torch.square(ang_err).sum(-1) of a 1-D tensor sums over ALL envs (:121-123) */
  float *ang_sq_e = (float *)calloc((size_t)n, sizeof(float));
  float *lin_r = (float *)malloc(sizeof(float) * (size_t)n), *pen_v = (float *)malloc(sizeof(float) * (size_t)n);
  int *lin_ok = (int *)malloc(sizeof(int) * (size_t)n), *pkill = (int *)malloc(sizeof(int) * (size_t)n);
  for (int e = 0; e < n; ++e) {
    const float *u = U + (size_t)e * USV_NU_STEP;
    const float *tmp = E->tmp + (size_t)e * 8;
    const float cmd[2] = {tmp[0], tmp[1]}, thrust[2] = {tmp[2], tmp[3]}, unit[2] = {tmp[4], tmp[5]};
    E->progress[e] += 1;
    float px = E->px[e], py = E->py[e];
    if (c->pos_noise_on) {
      const float rng = (float)((double)c->pos_noise_max - (double)c->pos_noise_min);
      px = px + (u[SU_PX] * rng + c->pos_noise_min);
      py = py + (u[SU_PX + 1] * rng + c->pos_noise_min);
    }
    float vxn = E->vx[e], vyn = E->vy[e], wzn = E->wz[e];
    if (c->vel_noise_on) {
      const float rng = (float)((double)c->vel_noise_max - (double)c->vel_noise_min);
      vxn = vxn + (u[SU_VX] * rng + c->vel_noise_min);
      vyn = vyn + (u[SU_VY] * rng + c->vel_noise_min);
      wzn = wzn + (u[SU_WZ] * rng + c->vel_noise_min);
    }
    float yawn = usv_heading(usv_quat_rot(E->yaw[e]));   /* update_state's heading (USV_Virtual.py:776-786) */
    if (c->head_noise_on) {
      const float rng = (float)((double)c->head_noise_max - (double)c->head_noise_min);
      yawn = yawn + (u[SU_HEAD] * rng + c->head_noise_min);
    }
    const float hc = usv_cos(yawn), hs = usv_sin(yawn);
    float obs[USV_NOBS];
    memset(obs, 0, sizeof(obs));
    if (c->obs_local) {
      obs[0] = hc * vxn + hs * vyn;
      obs[1] = -hs * vxn + hc * vyn;
    } else {
      obs[0] = vxn; obs[1] = vyn;
    }
    obs[2] = wzn;
    const int pa = USV_NOBS_BASE - 2;
    obs[pa + 0] = E->prev_cmd[0 * n + e];
    obs[pa + 1] = E->prev_cmd[1 * n + e];
    priv_tail(c, E, e, obs);
    /* Penalties.compute_penalty (USV_task_rewards.py:440-523) */
    const float pact0 = c->pen_use_u ? unit[0] : cmd[0];
    const float pact1 = c->pen_use_u ? unit[1] : cmd[1];
    float p_lin = 0.f, p_ang = 0.f, p_angv = 0.f, p_en = 0.f;
    if (c->pen_lin_kind == PEN_NORM) p_lin = -tnorm2(vxn, vyn) * c->pen_lin_k + c->pen_lin_c;
    if (c->pen_ang_kind) p_ang = pen_scalar(c->pen_ang_kind, c->pen_ang_k, c->pen_ang_x0, c->pen_ang_c, wzn);
    if (c->pen_angv_kind) {
      const float prev_w = pen_valid ? E->prev_wz[e] : wzn;
      p_angv = pen_scalar(c->pen_angv_kind, c->pen_angv_k, c->pen_angv_x0, c->pen_angv_c, wzn - prev_w);
    }
    if (c->pen_en_kind == PEN_SUM) p_en = -(pact0 + pact1) * c->pen_en_k + c->pen_en_c;
    else if (c->pen_en_kind == PEN_SUMSQ) p_en = -(pact0 * pact0 + pact1 * pact1) * c->pen_en_k + c->pen_en_c;
    E->prev_wz[e] = wzn;
    const float pens = p_lin + p_ang + p_angv + p_en;
    float t_add[4] = {0.f, 0.f, 0.f, 0.f};
    if (!track) {
      /* GoToPoseTask.get_state_observations (:89-130) */
      const float ex = E->tgt_x[e] - px, ey = E->tgt_y[e] - py;
      const float theta = usv_atan2(hs, hc);
      const float beta = usv_atan2(ey, ex);
      const float alpha = fmodf((beta - theta) + PI_F, TWO_PI_F) - PI_F;
      const float hraw = fmodf((E->tgt_h[e] - theta) + PI_F, TWO_PI_F) - PI_F;
      const float herr = usv_atan2(usv_sin(hraw), usv_cos(hraw));
      obs[3] = usv_cos(alpha); obs[4] = usv_sin(alpha); obs[5] = tnorm2(ex, ey);
      obs[6] = usv_cos(herr); obs[7] = usv_sin(herr);
      /* compute_reward (:134-181) */
      const float pdist = sqrtf(ex * ex + ey * ey);
      const float hdist = fabsf(herr);
      const float prog = 2.0f * clampf_(E->prev_dist[e] - pdist, -2.0f, 2.0f);
      E->prev_dist[e] = pdist;
      const float speed = tnorm2(vxn, vyn);
      const int gir = (pdist < c->position_tolerance) && (speed < 0.1f);
      E->goal_cnt[e] = E->goal_cnt[e] * gir + gir;
      const float hw = 1.0f - 1.0f / (1.0f + usv_exp(-c->sig_gain * (pdist - 2.0f)));
      const float pos_r = c->tk_scale[0] * task_term(c->tk_mode[0], pdist, c->tk_coeff[0]);
      const float head_r = hw * c->tk_scale[1] * task_term(c->tk_mode[1], hdist, c->tk_coeff[1]);
      const float act_pen = -0.05f * (fabsf(cmd[0]) + fabsf(cmd[1]));
      const float overall = pos_r + head_r + prog + 2.0f * (float)gir + act_pen;
      E->rew[e] = overall + pens;
      /* update_kills (:183-209), with the step after this calculate_metrics */
      const float kd = c->curriculum_on ? (float)curriculum_lerp(c, E->step_f + c->step_inc, c->cur_kill_dist,
                                                                 c->kill_dist_d)
                                        : c->kill_dist;
      const int die = (pdist > kd) || (E->goal_cnt[e] >= c->kill_after_n);
      const int tout = E->progress[e] >= c->max_episode_length - 1;
      E->reset_buf[e] = c->fixed_horizon_eval ? tout : (tout ? 1 : die);
      t_add[0] = pos_r; t_add[1] = head_r; t_add[2] = pdist; t_add[3] = speed;   /* update_statistics (:211-219) */
    } else {
      /* TrackXYOVelocityTask.get_state_observations (:75-101) */
      const float lex = E->tgt_x[e] - vxn, ley = E->tgt_y[e] - vyn, aerr = E->tgt_h[e] - wzn;
      obs[3] = lex; obs[4] = ley; obs[5] = aerr;
      const float pos_d = sqrtf(px * px + py * py);
      const float lin_d = sqrtf(lex * lex + ley * ley);
      ang_sq_e[e] = aerr * aerr;
      lin_r[e] = task_term(c->tk_mode[0], lin_d, c->tk_coeff[0]) * c->tk_scale[0];
      lin_ok[e] = lin_d < c->tk_tol[0];
      pkill[e] = pos_d > c->kill_dist;
      pen_v[e] = pens;
      t_add[0] = lin_r[e]; t_add[1] = lin_d;
    }
    if (c->stats_on) {
      float *S = E->stats;
#define ADDS(k, v) S[(k) * n + e] += (v)
      ADDS(0, t_add[0]); ADDS(1, t_add[1]);
      if (!track) { ADDS(2, t_add[2]); ADDS(3, t_add[3]); }
      if (c->pen_ang_kind) ADDS(ST_ANGULAR_VEL_PENALTY, p_ang);
      if (c->pen_angv_kind) ADDS(ST_ANGULAR_VEL_VARIATION_PENALTY, p_angv);
      if (c->pen_en_kind) ADDS(ST_ENERGY_PENALTY, p_en);
      ADDS(ST_NORMED_LINEAR_VEL, tnorm2(vxn, vyn));
      ADDS(ST_NORMED_ANGULAR_VEL, fabsf(wzn));
      ADDS(ST_CMD_NEG_RATE, ((float)(thrust[0] < 0.f) + (float)(thrust[1] < 0.f)) / 2.0f);
      ADDS(ST_U_MEAN, (unit[0] + unit[1]) / 2.0f);
      ADDS(ST_U_LOW_RATE, ((float)(unit[0] < 0.05f) + (float)(unit[1] < 0.05f)) / 2.0f);
      ADDS(ST_U_SUM, unit[0] + unit[1]);
#undef ADDS
    }
    for (int q = 0; q < USV_NOBS; ++q) E->obs[(size_t)e * USV_NOBS + q] = clampf_(obs[q], -c->clip_obs, c->clip_obs);
    E->just_reset[e] = 0;
  }
  if (track) {   /* TrackXYOVelocityTask.compute_reward / update_kills (:103-166) with the all-env angular distance */
    const float ang_d = sqrtf(track_ang_sum(ang_sq_e, n));
    const int ang_ok = ang_d < c->tk_tol[1];
    const float ang_r = task_term(c->tk_mode[1], ang_d, c->tk_coeff[1]) * c->tk_scale[1];
    for (int e = 0; e < n; ++e) {
      const int gir = lin_ok[e] * ang_ok;
      E->goal_cnt[e] = E->goal_cnt[e] * gir + gir;
      E->rew[e] = (lin_r[e] + ang_r) + pen_v[e];
      const int die = pkill[e] || (E->goal_cnt[e] > c->kill_after_n);
      const int tout = E->progress[e] >= c->max_episode_length - 1;
      E->reset_buf[e] = c->fixed_horizon_eval ? tout : (tout ? 1 : die);
      if (c->stats_on) {
        E->stats[2 * n + e] += ang_r;
        E->stats[3 * n + e] += ang_d;
      }
    }
  }
  free(lin_r); free(pen_v); free(lin_ok); free(pkill); free(ang_sq_e);
  E->ctl[USV_CTL_POT_VALID] = 1;
  E->ctl[USV_CTL_PEN_VALID] = 1;
  E->ctl[USV_CTL_REW_VALID] = 1;
}

/* compaction: reset_buf.nonzero() (USV_Virtual.py:1045) */
int oracle_compact(const oracle_env_t *E, int32_t *ids) {
  int k = 0;
  for (int e = 0; e < E->n; ++e)
    if (E->reset_buf[e]) ids[k++] = e;
  return k;
}
