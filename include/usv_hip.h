/*
 * usv_hip.h -- C ABI of libusv_hip.so, the MI355X (gfx950) hot path of the
 * USV CaptureXY environment + rl_games PPO trainer.
 *
 * The reference (loop-Z/omniisaacgymenvs_loop) is pure Python/PyTorch; it has
 * no FFI.  Each entry point below replaces one reference call chain; the
 * reference file:line it stands in for is cited next to it.  A maintainer binds
 * these from Python with ctypes; the in-tree host package
 * omniisaacgymenvs_loop_amd/_capi.py is exactly that binding.
 *
 * Conventions
 *   - every pointer is a DEVICE pointer owned by the caller (torch tensors),
 *     except `const usv_cfg_t*` / `const ppo_cfg_t*` which are host structs
 *     passed by value into the kernels;
 *   - every call is asynchronous on the given hipStream_t (passed as void*),
 *     performs no allocation and no host synchronisation (graph-capturable);
 *   - return value: 0 = launched, nonzero = argument error (the Python side
 *     raises RuntimeError, mirroring the reference's exception-based errors,
 *     e.g. tasks/USV_Virtual.py:91-95).
 *   - env state is struct-of-arrays: field f of env e lives at f[e].
 */
#ifndef USV_HIP_H
#define USV_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define USV_NOBS        33   /* obs row: 3 + (5 + 5*3) + 2 + priv_dim (tasks/USV/USV_core.py:46), priv_dim <= 8 */
#define USV_NOBS_BASE   25   /* columns before the privileged tail; a priv_dim = 4 row is the reference's
                                29 columns followed by 4 zero columns (the policy's padded input) */
#define USV_NOBST       16   /* obstacles per env                 (USV_capture_xy_static_obs.py:70) */
#define USV_NCLOSE       5   /* closest obstacles in obs          (USV_core.py:33) */
#define USV_GRID       150   /* potential-field grid              (USV_capture_xy_static_obs.py:30) */
#define USV_GRID2    (USV_GRID * USV_GRID)
/* the potential field in HBM (usv_bufs_t.field, .sdf): per env USV_FIELD_STRIDE floats of 10 x 10-texel tiles
 * (400 B, row-major inside), tiles row-major over the 150 x 150 grid: texel (row r, column c) at
 * ((r / 10) * USV_FIELD_TCOLS + c / 10) * 100 + (r % 10) * 10 + c % 10.  The tiles are the potential-field
 * sweep kernel's per-thread tiles, so that kernel stores its cells as immediate offsets of one base; the env
 * step's bilinear potential sample (a 2 x 2 texel block, 48 B inside a tile) touches ~1.6 lines instead of the
 * >= 2 of row-major rows.  The stride is padded to whole 128-B lines. */
#define USV_FIELD_TH    10
#define USV_FIELD_TW    10
#define USV_FIELD_TROWS  ((USV_GRID + USV_FIELD_TH - 1) / USV_FIELD_TH)
#define USV_FIELD_TCOLS  ((USV_GRID + USV_FIELD_TW - 1) / USV_FIELD_TW)
#define USV_FIELD_STRIDE 22528   /* 15 x 15 tiles x 100 texels = 22,500, padded to whole 128-B lines */
#define USV_LUT_N     1000   /* thruster LUT points               (TEST yaml dynamics.thrusters) */
#define USV_NSTAT       28   /* episode_sums keys                 (USV_Virtual.py:586-601) */
#define USV_SPAWN_ITERS 20   /* obstacle rejection iterations     (static_obs.py:980) */
/* Layout of the uniform draws of one reset slot (device [K][USV_NU_RESET]
 * when injected; otherwise Philox4x32-10(key=seed, ctr={env, step_lo, step_hi,
 * 0x100 + i/4})[i%4]).  Every torch.rand call of the reference reset path has
 * one slot range here (tests/golden/make_golden.py records them by call site). */
#define RU_MASS       0     /* MassDistributionDisturbances.randomize_masses:137 */
#define RU_COM        1     /* _randomize_com:98-124 (3)                         */
#define RU_KIZ        4     /* USVVirtual._sample_k_iz:164                        */
#define RU_KDRAG      5     /* HydrodynamicsObject._sample_k_drag:129             */
#define RU_THR        6     /* DynamicsFirstOrder.reset_thruster_randomization (2)*/
#define RU_DRAG       8     /* HydrodynamicsObject.reset_coefficients (6 lin, 6 quad) */
#define RU_SPAWN_R   20     /* CaptureXYTask.get_spawns:952                       */
#define RU_SPAWN_TH  21     /* :953 */
#define RU_YAW       22     /* :959 */
#define RU_OBST      23     /* :977 (16 x 2) */
#define RU_RESAMPLE  55     /* :1020, one 16x2 block per rejection iteration (20) */
#define RU_VX       695     /* USVVirtual.reset_idx:1561 */
#define RU_VY       696     /* :1564 */
#define RU_GOAL     697     /* CaptureXYTask.get_goals:924 (2) */
#define RU_FSIN     699     /* ForceDisturbance.generate_force:342-362 (x_freq, y_freq, x_shift, y_shift, amp) */
#define RU_FCONST   704     /* :369-374 (r, theta) */
#define RU_TSIN     706     /* TorqueDisturbance.generate_torque:484-494 (freq, shift, amp) */
#define RU_TCONST   709     /* :500-506 (r, sign draw) */
#define RU_GOAL_H   711     /* GoToPoseTask.get_goals:248 heading / TrackXYOVelocityTask.get_goals:193 angular velocity */
/* parity tests only (usv_cfg_t.inj_trig with injected uniforms): the reference's own torch.cos / torch.sin values on
 * the reset's state path -- cos, sin of the spawn angle (static_obs.py:955-956, USV_go_to_pose.py:307-310), cos, sin
 * of half the spawn / scene yaw (the quaternion, static_obs.py:960-961, USV_Virtual.py:1449-1450), cos, sin of the
 * constant disturbance's direction (USV_disturbances.py:369-374).  Never drawn. */
#define RU_TRIG     712
#define USV_NU_RESET 718
/* Layout of the uniform draws of one env step (device [n][USV_NU_STEP] when
 * injected; otherwise Philox(ctr={env, step_lo, step_hi, i/4})[i%4]).
 * Only the draws of the LAST update_state of the step reach obs/reward
 * (USV_Virtual.py:785-787 via post_physics_step -> get_observations:838). */
#define SU_VX   0   /* NoisyObservations.add_noise_on_vel, column 0 */
#define SU_VY   1   /* column 1 */
#define SU_WZ   2   /* column 5 */
#define SU_HEAD 3   /* add_noise_on_heading */
#define SU_PX   4   /* add_noise_on_pos (2) */
#define SU_ACT  6   /* NoisyActions.add_noise_on_act (2) */
#define USV_NU_STEP 8

/* episode_sums key order (dict insertion order of the reference) */
enum usv_stat_key {
  ST_TOTAL_REWARD = 0, ST_DISTANCE_REWARD, ST_ALIGNMENT_REWARD, ST_HEADING_IMPROVE_REWARD,
  ST_POTENTIAL_SHAPING_REWARD, ST_SPEED_REWARD, ST_ANGULAR_REWARD, ST_TURN_HAZARD_PENALTY,
  ST_GOAL_REWARD, ST_COLLISION_REWARD, ST_TIME_REWARD, ST_SUCCESS, ST_COLLISION,
  ST_POSITION_ERROR, ST_BOUNDARY_PENALTY, ST_DANGER_MEAN, ST_DANGER_HI_RATE, ST_G_GATE_MEAN,
  ST_G_SAFE_MEAN, ST_ANGULAR_VEL_PENALTY, ST_ANGULAR_VEL_VARIATION_PENALTY, ST_ENERGY_PENALTY,
  ST_NORMED_LINEAR_VEL, ST_NORMED_ANGULAR_VEL, ST_CMD_NEG_RATE, ST_U_MEAN, ST_U_LOW_RATE, ST_U_SUM
};

/* penalty function kinds (the eval'd lambda strings of USV_task_rewards.py:429-438,
 * TEST yaml :262-291, parsed host-side into one of these closed forms) */
enum usv_pen_kind {
  PEN_OFF = 0,
  PEN_DEADZONE = 1,   /* -k * max(|x| - x0, 0) + c                      */
  PEN_SUM = 2,        /* -k * sum(x) + c        (energy on u)            */
  PEN_SUMSQ = 3,      /* -k * sum(x^2) + c                               */
  PEN_NORM = 4,       /* -k * ||x|| + c         (linear velocity)        */
  PEN_EXPABS = 5      /* k * (exp(x0 * |x|) - 1) + c                     */
};

/* All constants of the env step / reset path.  Built host-side from the task
 * yaml (omniisaacgymenvs_loop_amd/tasks/usv_config.py). */
typedef struct usv_cfg {
  /* ---- integration (sim.dt, controlFrequencyInv, dynamics.*) ---- */
  float dt;                 /* 0.02 */
  int   substeps;           /* 10 */
  float thr_alpha;          /* exp(-dt/tau), ThrusterDynamics.py:132 */
  float thr_y;              /* thruster lateral lever arm (heron.usd) 0.37765 */
  float izz0;               /* base_link Izz (heron.usd) 8.061 */
  float lin_damp[3];        /* effective linear damping u, v, r (Hydrodynamics.py:185-192) */
  float quad_damp[3];       /* quadratic damping + offset, u, v, r */
  float scaling_damping;
  int   use_drag_scale;     /* multiply damping by k_drag (Hydrodynamics.py:202) */
  int   use_thr_mult;       /* apply thruster multiplier (ThrusterDynamics.py:200) */
  int   thr_separate;       /* separate L/R multipliers */
  /* ---- actions (USV_Virtual.py:1042-1101) ---- */
  float clip_actions;       /* 1.0 */
  int   affine_thrust;      /* u = 0.5(a+1) else clamp(a,0,1) */
  int   act_noise_on;  float act_noise_min, act_noise_max;
  /* ---- observation noise (USV_disturbances.py:533-601) ---- */
  int   pos_noise_on;  float pos_noise_min, pos_noise_max;
  int   vel_noise_on;  float vel_noise_min, vel_noise_max;
  int   head_noise_on; float head_noise_min, head_noise_max;
  /* ---- observation layout ---- */
  int   obs_local;          /* observation_frame == "local" */
  int   priv_dim;           /* 4 or 8 */
  float clip_obs;           /* 12 */
  int   masscom_base;       /* masscom_obs_source == "base" */
  int   mass_relative;      /* mass_obs_mode == "relative" */
  float base_mass;
  int   com_scaled;         /* com_obs_mode == "scaled" */
  float com_scale[3];       /* box_length, box_width, max(zero_height,1) */
  float base_com[3];
  int   priv_mode;          /* 0 raw, 1 centered, 2 minmax */
  float priv_nominal;
  int   priv_drag_on, priv_thr_on, priv_kiz_on;
  float kdrag_min, kdrag_max, thr_min, thr_max, kiz_min, kiz_max;
  /* ---- task (CaptureXYParameters, TEST yaml task_parameters) ---- */
  float position_tolerance;
  int   kill_after_n;
  float kill_dist, boundary_cost, goal_reward, time_reward;
  float collision_threshold;   /* 1.2 (static_obs.py:105) */
  float obstacle_radius;       /* 0.5 */
  int   max_episode_length;    /* 200 */
  int   fixed_horizon_eval;
  /* ---- CaptureXYReward (USV_task_rewards.py:20-80) ---- */
  int   reward_mode;           /* 0 linear, 1 square, 2 exponential */
  float position_scale, exp_coeff, align_la1, align_la2, align_la3;
  /* ---- Penalties (USV_task_rewards.py:440-523) ---- */
  int   pen_lin_kind;  float pen_lin_k,  pen_lin_x0,  pen_lin_c;
  int   pen_ang_kind;  float pen_ang_k,  pen_ang_x0,  pen_ang_c;
  int   pen_angv_kind; float pen_angv_k, pen_angv_x0, pen_angv_c;
  int   pen_en_kind;   float pen_en_k,   pen_en_x0,   pen_en_c;
  int   pen_actv_kind; float pen_actv_k, pen_actv_x0, pen_actv_c;
  int   pen_use_u;           /* penalties_use_thrust_u */
  /* ---- potential field (d_multi_gemini.py) ---- */
  float map_size;            /* 30 */
  int   field_iters;         /* 225 */
  float influence_radius, eta, safe_radius, field_alpha;
  /* ---- reset / domain randomisation ---- */
  int   mass_dr_on;  float mass_min, mass_max;
  int   com_mode;            /* 0 base, 1 xyz box, 2 legacy disk */
  float com_disp[3];  float com_legacy_r;
  int   couple_drag, couple_thr, couple_kiz;
  int   indep_kdrag_on, kdrag_log;
  int   indep_thr_on;  float thr_rand, left_rand, right_rand;
  int   indep_kiz_on, kiz_log;
  int   drag_rand_on; float lin_rand[3], quad_rand[3];
  float spawn_rmin, spawn_rmax, goal_random_position;
  float obst_box, min_dist_safe, min_obs_sep;
  float init_vel;            /* 1.5 */
  int   stats_on;            /* accumulate episode_sums */
  /* initial action bias (USV_Virtual.py:1070-1077): added to the command for the
   * first act_bias_steps pre_physics_step calls; used in device-clock mode */
  float act_bias;
  int   act_bias_steps;
  /* ---- force / torque disturbances (USV_disturbances.py:268-530, TEST yaml
   * disturbances.forces/torques) and water current (Hydrodynamics.py:224-237) ---- */
  int   fdist_on, fconst_on, fsin_on;
  float fconst_min, fconst_max, fsin_min, fsin_max, ffreq_min, ffreq_max, fshift_min, fshift_max;
  int   tdist_on, tconst_on, tsin_on;
  float tconst_min, tconst_max, tsin_min, tsin_max, tfreq_min, tfreq_max, tshift_min, tshift_max;
  int   current_on;
  float flow_vel[2];        /* world-frame water velocity x, y */
  /* ---- task selection (USV_task_factory.py:58-64) and the GoToPose /
   * TrackXYOVelocity parameters (USV_task_parameters.py:74-148,
   * USV_task_rewards.py:160-393).  Index 0 = position / linear velocity term,
   * 1 = heading / angular velocity term. ---- */
  int   task_kind;          /* USV_TASK_* */
  int   tk_mode[2];         /* 0 linear, 1 square, 2 exponential */
  float tk_coeff[2];        /* *_exponential_reward_coeff */
  float tk_scale[2];        /* position_scale/heading_scale, linear_scale/angular_scale */
  float tk_tol[2];          /* TrackXYO lin_vel_tolerance, ang_vel_tolerance */
  float tk_goal_rand[2];    /* TrackXYO goal_random_linear_velocity, goal_random_angular_velocity */
  float sig_gain;           /* GoToPoseReward.sig_gain */
  /* ---- device NaN probe (USV_Virtual.py:57-95, vec_env_rlgames.py:41-80, env USV_NAN_PROBE):
   * the step kernels OR the USV_NAN_* stage bits of any non-finite clamped action, state,
   * reward or observation into ctl[USV_CTL_NAN_FLAG]; the host raises after the epoch ---- */
  int   nan_probe;
  /* ---- GoToPose spawn curriculum (GoToPoseTask.get_spawns / update_kills, USV_go_to_pose.py:183-209,
   * 256-300; GoToPoseParameters.spawn_curriculum*, USV_task_parameters.py:107-113): the spawn disk and the kill
   * distance move linearly from the curriculum values to the task's as the reference's USVVirtual.step (a
   * Python float += 1 / horizon_length per calculate_metrics, USV_Virtual.py:1633) goes from warmup to end;
   * get_spawns sees the value at the step's reset, update_kills the value after its calculate_metrics
   * (usv_bufs_t.clock[4..5]).  Doubles: the reference's Python floats. ---- */
  int   curriculum_on;
  int   pad_curriculum;
  double step_inc;          /* 1 / horizon_length (the increment of USVVirtual.step) */
  double cur_min_dist, cur_max_dist, cur_kill_dist, cur_warmup, cur_end;
  double min_spawn_d, max_spawn_d, kill_dist_d;   /* the task's min_spawn_dist, max_spawn_dist, kill_dist */
  /* ---- the first substep after a reset computes the drag and the disturbances from the
   * reference's CACHED root state, which still holds the pre-reset pose and velocity (apply_forces reads
   * root_pos / root_quats / root_velocities, USV_Virtual.py:1103-1117, refreshed only by update_state,
   * :771-813, which runs after each world step, vec_env_rlgames.py:154-171).  usv_reset keeps those inputs
   * in usv_bufs_t.stale; 0 = the first substep uses the new state instead. ---- */
  int   stale_root;
  /* parity tests: with injected reset uniforms, take the spawn / disturbance-direction sin and cos from the
   * RU_TRIG slots (the reference's recorded CPU values) instead of usv_sincos_cr; 0 in training */
  int   inj_trig;
} usv_cfg_t;

/* stage bits of ctl[USV_CTL_NAN_FLAG] / ppo_cfg_t.nan_flag (the reference's probe names) */
#define USV_NAN_ACTIONS  1   /* actions(clamped)           vec_env_rlgames.py:143 */
#define USV_NAN_STATE    2   /* state.position/orientation/velocities  USV_Virtual.py:810-813 */
#define USV_NAN_REWARD   4   /* reward.rew_buf             USV_Virtual.py:1642-1648 */
#define USV_NAN_OBS      8   /* obs(post_physics_step)     vec_env_rlgames.py:187-192 */
#define USV_NAN_POLICY  16   /* policy mu / value of the rollout (get_action_values) */
#define USV_NAN_EXTRAS  32   /* extras["episode"][key] NaN before masking   USV_Virtual.py:1601-1605 */

#define USV_TASK_CAPTURE_XY   0
#define USV_TASK_GO_TO_POSE   1
#define USV_TASK_TRACK_XYO    2
/* per-env scratch rows of the two-phase TrackXYOVelocity step (usv_bufs_t.task_scratch) */
#define USV_TS_LIN_REW 0
#define USV_TS_PEN     1
#define USV_TS_LIN_OK  2
#define USV_TS_POS_KILL 3
#define USV_TS_ROWS    4

/* per-env disturbance parameters (rows of usv_bufs_t.dist, drawn at reset) */
enum usv_dist_row {
  DI_FCX = 0, DI_FCY,                          /* disturbance_forces_const x, y */
  DI_FXF, DI_FYF, DI_FXS, DI_FYS, DI_FAMP,     /* _force_{x,y}_freq, _force_{x,y}_shift, _force_amp */
  DI_TC, DI_TF, DI_TS, DI_TAMP,                /* disturbance_torques_const z, _torque_freq/shift/amp */
  USV_NDIST
};

/* Device buffers of the env (SoA).  All arrays have n entries unless noted. */
typedef struct usv_bufs {
  int n;
  int pad0;
  /* planar rigid-body state (local frame) */
  float *px, *py, *yaw, *vx, *vy, *wz;
  float *fl, *fr;                  /* thruster first-order lag state (ThrusterDynamics.py:133) */
  /* per-episode parameters */
  float *mass, *com_x, *com_y, *com_z, *k_drag, *thr_l, *thr_r, *k_iz, *mass_r;
  float *lin_damp, *quad_damp;     /* [3][n] only when cfg.drag_rand_on, else NULL */
  /* task */
  float *tgt_x, *tgt_y;
  float *obst;                     /* [16][2][n]  obstacle centres, local frame */
  float *field;                    /* [n][USV_FIELD_STRIDE] raw cost-to-go of the potential field's grid (tiled, see
                                      USV_FIELD_STRIDE; +inf unreachable): a field texel = field_value(SDF from the
                                      env's obstacles, this cost, .fnorm) -- the field is never materialised */
  /* history */
  float *prev_cmd;                 /* [2][n] raw policy command (obs 23:25) */
  float *prev_dist, *prev_head, *prev_pot, *prev_wz;
  int32_t *goal_cnt, *progress, *reset_buf;
  uint8_t *just_reset;
  int32_t *done_succ, *done_coll;
  float *stats;                    /* [USV_NSTAT][n] episode sums */
  /* outputs */
  float *obs;                      /* [n][33] clamped observation */
  float *rew;                      /* [n] */
  int64_t *dones;                  /* [n] reset_buf copy as int64 (rl_games API) */
  /* control block (device) */
  int32_t *ctl;                    /* [USV_CTL_N] see USV_CTL_* */
  int32_t *reset_ids;              /* [n] compacted reset list */
  float   *fscratch;               /* [16] float reductions (max_val, jmax, J max finite / infinite) */
  float   *extras;                 /* [USV_NSTAT] extras["episode"] (persistent) */
  float   *extras_acc;             /* [ceil(n/256)][USV_NSTAT] reset-kernel per-workgroup sums (scratch) */
  float   *field_old_tgt;          /* [2][n] target used by the field of each reset env */
  float   *slot_stats;             /* [n][USV_FIELD_SLOT_STATS] per-reset-slot field statistics (scratch) */
  float   *sdf;                    /* [n][USV_FIELD_STRIDE] raw cost-to-go of each env's field as the sweeps leave it,
                                      row-major [150][150] (+inf unreachable): k_field_stats tiles it into .field */
  const float *grid_lin;           /* [150] cell centres of the field grid */
  float   *dist;                   /* [USV_NDIST][n] disturbance parameters; NULL when no disturbance is on */
  const float *env_org;            /* [2][n] world x, y of each env's origin (RLTask._env_pos); NULL = 0 */
  float   *tgt_h;                  /* [n] GoToPose target heading / TrackXYO target angular velocity (tgt_x/y:
                                      target position / target linear velocity); NULL for CaptureXY */
  float   *task_scratch;           /* TrackXYO: [USV_TS_ROWS][n] + [ceil(n/256)] partial sums; else NULL */
  /* scene replay (USVVirtual._scene_replay_*, USV_Virtual.py:1329-1457): NULL scene = random spawns */
  const float *scene;              /* [n_scenes][USV_SCENE_STRIDE] (USV_SC_* layout) */
  int32_t *scene_next;             /* [n] next scene index of each env (starts at scene_replay.start_index) */
  int32_t *scene_last;             /* [n] scene index applied at the env's last reset */
  int32_t n_scenes, scene_cycle;
  /* device step clock (nullable): [0] next step index, [1] next bias-call count,
   * [2] current step, [3] current bias-call count, [4] / [5] the bits of the double
   * USVVirtual.step at the current step's reset / after its calculate_metrics (cfg.step_inc
   * per step, USV_CLOCK_WORDS words, zero-initialised).  When set, usv_reset advances
   * it and the step / bias arguments of usv_reset / usv_env_step are ignored, so
   * a captured HIP graph replays consecutive steps. */
  uint64_t *clock;
  /* usv_env_step_part(.., 3) -> usv_env_step_late: the potential-independent reward terms and the sample
     position of the envs reset this step ([USV_RSTASH_ROWS][n]); NULL unless the overlapped step is used */
  float *rstash;
  /* [n][USV_FNORM] per-env normalisation constants of the potential field (usv_potential_field writes them
     for the reset envs): cost min, cost range + 1e-6, J min, J range + 1e-6, the batch's inf_val, the
     batch's inside value `high` (> 0; negated when no cell of the batch is inside an obstacle),
     RN(1 / cost range), RN(1 / J range) */
  float *fnorm;
  /* [USV_STALE_ROWS][n] the hydrodynamic / disturbance inputs of a reset env's first substep (cfg.stale_root):
     usv_reset writes them from the pre-reset state before it spawns the env -- the water-relative body
     velocity R(yaw)^T (v - flow) (Hydrodynamics.py:207-245), the yaw rate, and the local position at which
     the disturbance sinusoids are evaluated (USV_disturbances.py:386-410, 510-530) */
  float *stale;
} usv_bufs_t;
#define USV_STALE_UB 0
#define USV_STALE_VB 1
#define USV_STALE_RB 2
#define USV_STALE_PX 3
#define USV_STALE_PY 4
#define USV_STALE_ROWS 5
#define USV_FNORM 8
#define USV_RSTASH_ROWS 14
#define USV_CLOCK_WORDS 6

/* one replay scene (scripts/build_usv_scenes.py:566-577 keys; obstacles padded to
 * 16 with limbo (999, 999) past obstacles_count as CaptureXYTask.apply_scene does,
 * static_obs.py:829-842) */
#define USV_SC_OBST      0    /* 16 x (x, y) */
#define USV_SC_START    32    /* start_pos x, y */
#define USV_SC_YAW      34    /* start_yaw */
#define USV_SC_VEL      35    /* start_vel x, y */
#define USV_SC_GOAL     37    /* goal_pos x, y */
#define USV_SCENE_STRIDE 40

#define USV_FIELD_SLOT_STATS 192   /* 16 + 12 per 30-row band (5 bands), obstacles at 160 (32) */

/* control words */
#define USV_CTL_RESET_COUNT 0
#define USV_CTL_POT_VALID   1   /* 0 => prev_potential is None (static_obs.py:448,773) */
#define USV_CTL_PEN_VALID   2   /* 0 => Penalties.prev_state is None (USV_task_rewards.py:450) */
#define USV_CTL_REW_VALID   3   /* 0 => CaptureXYReward.prev_position_error is None */
#define USV_CTL_NAN_FLAG    4   /* device NaN probe (replaces USV_NAN_PROBE host syncs) */
#define USV_CTL_ANY_INSIDE  5   /* potential field: any cell inside an obstacle in the batch */
#define USV_CTL_ANY_FINITE  6   /* potential field: any finite cost in the batch */
#define USV_CTL_OBST_DONE   7   /* completion counter of the obstacle kernel (extras finalisation) */
#define USV_CTL_STEPPED     8   /* set by every env step; usv_reset promotes it to the 3 flags above */
#define USV_CTL_PLACE       9   /* set by usv_reset: usv_potential_field places the reset envs' obstacles */
#define USV_CTL_H_SEED_LO  10   /* usv_reset -> usv_potential_field: Philox key and step of the */
#define USV_CTL_H_SEED_HI  11   /*   obstacle draws, and the injected-uniform buffer (or 0)      */
#define USV_CTL_H_STEP_LO  12
#define USV_CTL_H_STEP_HI  13
#define USV_CTL_H_INJ_LO   14
#define USV_CTL_H_INJ_HI   15
#define USV_CTL_SCENE_ERR  16   /* scene replay: an index fell outside [0, n_scenes) with cycle off */
#define USV_CTL_BATCH_DONE 17   /* completion counter of the potential-field batch fold (keep 0) */
#define USV_CTL_FIELD_EXACT 18  /* count of reset envs whose cost field took the reference's 225 literal sweeps */
#define USV_CTL_N           20

/* ------------------------------------------------------------------------ */
/* Env entry points                                                          */
/* ------------------------------------------------------------------------ */

/* Build the 1000-point thruster LUT from the 21-point tables.
 * Replaces DynamicsFirstOrder.interpolate_on_field_data, ThrusterDynamics.py:152-177.
 * lut: device [2][USV_LUT_N]. */
int usv_build_lut(const float *table_l21, const float *table_r21, int n_table,
                  float *lut_dev, void *stream);

/* Reset path, part 1: compact reset_buf into reset_ids/ctl[RESET_COUNT],
 * reduce episode extras, sample domain randomisation, spawn + obstacle
 * rejection sampling, initial velocities, new goals.
 * Replaces USVVirtual.pre_physics_step:1045-1048 -> reset_idx:1502-1618
 * (MassDistributionDisturbances.randomize_masses, _apply_mass_driven_coupling,
 *  CaptureXYTask.reset/get_spawns/get_goals).
 * u_inject: NULL => in-kernel Philox(seed, step); else device [n][USV_NU_RESET]
 * uniforms per reset slot (parity tests). */
int usv_reset(const usv_cfg_t *cfg, const usv_bufs_t *b, uint64_t seed,
              uint64_t step, const float *u_inject, void *stream);
/* usv_reset in two parts (the overlapped step, tasks/usv_virtual.py): part 1 = the step clock / scratch reset,
 * the reset kernel (compaction, DR, spawns, goals, the per-workgroup episode-extras partials); part 2 = the
 * fold of those partials into b->extras (in workgroup order).  Part 1 then part 2 == usv_reset; part 2 must run
 * before the next part 1 (which rewrites the partials).  Same Python-side API as usv_reset, no reference analogue
 * beyond it. */
int usv_reset_part(const usv_cfg_t *cfg, const usv_bufs_t *b, uint64_t seed, uint64_t step,
                   const float *u_inject, int part, void *stream);

/* Reset path, part 2: per-reset-env potential field (occupancy/SDF,
 * 8-neighbour wavefront cost-to-go, repulsion, batch-global normalisation).
 * Replaces BatchedMapGPU.compute_occupancy_and_sdf / compute_cost_field_wavefront /
 * compute_potential_field, tasks/USV/d_multi_gemini.py:66-271 (called from
 * USV_capture_xy_static_obs.py:1054-1057). */
int usv_potential_field(const usv_cfg_t *cfg, const usv_bufs_t *b, void *stream);
/* The potential fields of envs env_ids[0..count) materialised row-major into out [count][150][150] (what
 * BatchedMapGPU returns per env; the step kernels sample the field from its parts, never from this). */
int usv_field_view(const usv_cfg_t *cfg, const usv_bufs_t *b, const int32_t *env_ids, int count, float *out,
                   void *stream);

/* One control step for all envs: action mapping, thruster LUT + lag,
 * 10 substeps of 3-DoF hydrodynamics + semi-implicit Euler, state readback
 * with observation noise, observation, reward, penalties, kills, stats.
 * Replaces VecEnvRLGames.step (envs/vec_env_rlgames.py:120-217):
 *   USVVirtual.pre_physics_step:1050-1101, apply_forces:1103-1133 + PhysX
 *   World.step (x10), post_physics_step -> get_observations:837-986,
 *   calculate_metrics:1628-1652, is_done:1223-1237, _process_data:82-112.
 * actions: device [n][2]; action_bias: initial_action_bias if the global
 * counter is below initial_action_bias_steps else 0 (USV_Virtual.py:1071-1077).
 * u_inject: NULL => Philox, else device [n][USV_NU_STEP]. */
int usv_env_step(const usv_cfg_t *cfg, const usv_bufs_t *b, const float *actions,
                 const float *lut_dev, float action_bias, uint64_t seed,
                 uint64_t step, const float *u_inject, void *stream);

/* The canonical env slab (tasks/usv_virtual.py allocates it): every per-env array of usv_bufs_t the step kernel
 * touches at base + USV_SLAB_<X> * row_bytes, row_bytes = the next power of two >= 4 n (>= 256).  When the
 * pointers follow this layout (and 4 n <= 2^22) usv_env_step runs a variant whose array offsets are compile-time
 * constants (no per-array scalar registers live across the kernel); any other layout takes the general path. */
#define USV_SLAB_STATE     0    /* px, py, yaw, vx, vy, wz, fl, fr (8 rows) */
#define USV_SLAB_PARAMS    8    /* mass, com_x, com_y, com_z, k_drag, thr_l, thr_r, k_iz, mass_r (9) */
#define USV_SLAB_LIN_DAMP 17    /* 3 rows, then quad_damp 3 rows */
#define USV_SLAB_QUAD_DAMP 20
#define USV_SLAB_TGT      23    /* tgt_x, tgt_y */
#define USV_SLAB_OBST     25    /* 32 rows */
#define USV_SLAB_PREV_CMD 57    /* 2 */
#define USV_SLAB_HIST     59    /* prev_dist, prev_head, prev_pot, prev_wz */
#define USV_SLAB_IBUF     63    /* goal_cnt, progress, reset_buf, done_succ, done_coll (i32) */
#define USV_SLAB_JUST_RESET 68  /* u8 [n] */
#define USV_SLAB_STATS    69    /* USV_NSTAT rows */
#define USV_SLAB_OBS      97    /* [n][USV_NOBS] */
#define USV_SLAB_REW     130
#define USV_SLAB_DONES   131    /* i64 [n]: 2 rows */
#define USV_SLAB_FIELD_OLD_TGT 133
#define USV_SLAB_RESET_IDS 135
#define USV_SLAB_DIST    136    /* USV_NDIST rows */
#define USV_SLAB_ENV_ORG 147    /* 2 */
#define USV_SLAB_TGT_H   149
#define USV_SLAB_STALE   150    /* USV_STALE_ROWS rows */
#define USV_SLAB_ROWS    155

/* usv_env_step split in two so the non-reset envs can run while the reset envs'
 * potential fields are built: part 1 = envs not reset this step (needs only
 * usv_reset to have run), part 2 = the envs reset this step (after
 * usv_potential_field); part 0 = all (== usv_env_step).  Parts 1 and 2 together
 * produce exactly part 0's results. */
int usv_env_step_part(const usv_cfg_t *cfg, const usv_bufs_t *b, const float *actions,
                      const float *lut_dev, float action_bias, uint64_t seed, uint64_t step,
                      const float *u_inject, int part, void *stream);

/* The overlapped step (the reset envs' fields build on a second stream while every env steps): part 3 of
 * usv_env_step_part runs the whole step for every env except the potential-dependent reward of the envs
 * reset this step (their fields do not exist yet), which it stashes in b->rstash; after the fields,
 * usv_env_step_late finishes it (field sample, reward_tail, reward, prev_pot, the reward episode sums).
 * The observations, dones and state of part 3 are final, so the next policy step can run beside the field
 * kernels.  Stream order: usv_reset -> usv_field_stage(1) -> {part 3 || usv_field_stage(2)} -> late.
 * Together they produce exactly part 0's results (usv_potential_field + usv_env_step). */
int usv_env_step_late(const usv_cfg_t *cfg, const usv_bufs_t *b, void *stream);
/* usv_potential_field in two stages: 1 = the reset envs' obstacle placement (k_field_place: the step
 * kernels read the new obstacles), 2 = the cost-to-go sweeps, SDF statistics, batch fold and the fields;
 * stage 2 is also available as its two halves 3 (sweeps, exactness fallback, statistics) then 4 (batch fold,
 * normalisation constants), so a caller can order other work after the statistics */
int usv_field_stage(const usv_cfg_t *cfg, const usv_bufs_t *b, int stage, void *stream);

/* Planar force/moment model only (no integration), for parity with
 * HydrodynamicsObject.ComputeHydrodynamicsEffects (Hydrodynamics.py:207-245)
 * and the thruster lever arms.  out: [n][3] body X, Y, N. */
int usv_forces(const usv_cfg_t *cfg, const usv_bufs_t *b, float *out, void *stream);

/* Hydrostatics constants (task yaml dynamics.hydrostatics + sim.gravity), USV_Virtual.py:441-456,
 * 724-736: metacentric width / length = box_width / 2, box_length / 2; max_volume =
 * box_width * box_length * (heron_zero_height + 20). */
typedef struct usv_hydro {
  float water_density;
  float gravity;              /* sim.gravity[2] (-9.81) */
  float metacentric_width;
  float metacentric_length;
  float avg_force;            /* average_hydrostatics_force_value (275) */
  float amplify_torque;
  float waterplane_area;
  float zero_height;          /* heron_zero_height */
  float max_volume;
} usv_hydro_t;

/* 6-DoF hydrostatic wrench of the hull (buoyancy + metacentric restoring torques), body frame:
 * submerged volume from the root height (USVVirtual.update_state, USV_Virtual.py:791-798), euler
 * angles (get_euler_angles :815-835), HydrostaticsObject.compute_archimedes_metacentric_local
 * (Hydrostatics.py:63-133; force rotated by R^T, torque not rotated, x amplify_torque).
 * quat [n][4] (w, x, y, z), root_z [n] -> volume [n], euler [n][3], wrench [n][6].
 * On the planar model (roll = pitch = 0) the surge, sway and yaw components are exactly 0, which is
 * why usv_env_step does not add them (tests/test_env_gpu.py::test_hydrostatics_vs_reference). */
int usv_hydrostatics(const usv_hydro_t *h, int n, const float *quat, const float *root_z, float *volume,
                     float *euler, float *wrench, void *stream);

/* ------------------------------------------------------------------------ */
/* PPO entry points (rl_games a2c_continuous / a2c_common)                   */
/* ------------------------------------------------------------------------ */

#define PPO_NIN   33
#define PPO_NH    128
#define PPO_NA    2
/* flat parameter order = model.parameters() order of the reference:
 * sigma[2], W1[128][33], b1[128], W2[128][128], b2[128], Wv[1][128], bv[1],
 * Wmu[2][128], bmu[2]  (network_builder.py:1480-1575)  => 21253 floats */
#define PPO_NPARAM 21253
#define PPO_OFF_SIGMA 0
#define PPO_OFF_W1    2
#define PPO_OFF_B1    (PPO_OFF_W1 + PPO_NH * PPO_NIN)
#define PPO_OFF_W2    (PPO_OFF_B1 + PPO_NH)
#define PPO_OFF_B2    (PPO_OFF_W2 + PPO_NH * PPO_NH)
#define PPO_OFF_WV    (PPO_OFF_B2 + PPO_NH)
#define PPO_OFF_BV    (PPO_OFF_WV + PPO_NH)
#define PPO_OFF_WMU   (PPO_OFF_BV + 1)
#define PPO_OFF_BMU   (PPO_OFF_WMU + PPO_NA * PPO_NH)

typedef struct ppo_cfg {
  int   horizon;            /* 16 */
  int   n_envs;             /* num_actors per rank */
  int   minibatch;          /* 8192 */
  int   normalize_input, normalize_value, normalize_advantage;
  float gamma, tau;         /* 0.99, 0.95 */
  float e_clip;             /* 0.2 */
  float critic_coef;        /* 0.5 */
  float entropy_coef;       /* 0 */
  float bounds_loss_coef;   /* 1e-4 */
  int   clip_value;
  int   truncate_grads;  float grad_norm;
  float adam_b1, adam_b2, adam_eps, weight_decay;
  int   lr_adaptive;  float kl_threshold, lr_min, lr_max;
  float reward_scale, reward_shift;
  float rms_eps;            /* 1e-5 */
  int   bf16_gemm;          /* 0: fp32 (the reference); 1: bf16 operands / fp32 accumulation for the
                               128x128 products (layer 2, dW2, dh1) of the training step
                               (ppo_minibatch_*; the reference's autocast covers calc_gradients only,
                               a2c_continuous.py:121): the rollout kernels stay fp32 -- BASELINE configs[2] */
  int   nan_probe;          /* 1: ppo_policy_step ORs USV_NAN_POLICY into *nan_flag on a non-finite mu / value */
  int32_t *nan_flag;        /* device int (nullable) */
} ppo_cfg_t;

/* Rollout: obs RMS normalise (eval) -> MLP -> mu, value (denormalised),
 * Normal sample, neglogp; writes rollout slot t of the env-major experience
 * buffer. Replaces A2CBase.get_action_values (a2c_common.py:385-405) +
 * ModelA2CContinuousLogStd.forward (models.py:366-401) +
 * ExperienceBuffer.update_data (experience.py:392-398).
 * params: [PPO_NPARAM]; obs_rms: double [2][33] (mean, var), non-NULL (read also when
 * normalize_input = 0; the same for ppo_value / ppo_minibatch_grad / _fused); val_rms double [2];
 * buffers of the experience store are env-major [n][H][...].
 * eps_inject: NULL => Philox normal draws, else device [n][2] N(0,1) draws.
 * step_dev (nullable): device counter holding the rollout's first step; slot t draws
 * with step *step_dev + t instead of `step` (graph replay).  ppo_store_reward of the
 * last slot advances it by the horizon. */
int ppo_policy_step(const ppo_cfg_t *cfg, const float *params, const double *obs_rms,
                    const double *val_rms, const float *obs, int t,
                    float *exp_obs, float *exp_act, float *exp_nlp, float *exp_val,
                    float *exp_mu, float *exp_sigma, uint8_t *exp_done,
                    const int64_t *dones_prev, float *actions_out,
                    uint64_t seed, uint64_t step, const uint64_t *step_dev,
                    const float *eps_inject, void *stream);

/* Value of the last observation (A2CBase.get_values, a2c_common.py:407-430). */
int ppo_value(const ppo_cfg_t *cfg, const float *params, const double *obs_rms,
              const double *val_rms, const float *obs, float *values, void *stream);

/* Store rewards of slot t shaped by DefaultRewardsShaper (tr_helpers.py:33-43)
 * and accumulate the episode meters (a2c_common.py:738-759).
 * meter: device [ppo_meter_floats(n_envs, H)]: [H][4] per-step sums (reward of done envs,
 * shaped reward, length, count), complete after slot H - 1 (a fixed-order fold of the
 * per-workgroup partials that follow them: deterministic, no float atomics).
 * step_dev (nullable): advanced by the horizon when t == horizon - 1. */
int ppo_store_reward(const ppo_cfg_t *cfg, const float *rew, const int64_t *dones, int t,
                     float *exp_rew, float *cur_rew, float *cur_shaped, float *cur_len,
                     float *meter, uint64_t *step_dev, void *stream);

/* GAE (A2CBase.discount_values a2c_common.py:525-540) + returns (:763) +
 * value RMS train/normalise (prepare_dataset a2c_common.py:1257-1290) +
 * advantage normalisation.  work: device scratch >= 64 doubles + 4*n*H floats. */
int ppo_prepare(const ppo_cfg_t *cfg, const float *params, const double *obs_rms,
                double *val_rms, const float *last_obs, const int64_t *last_dones,
                const uint8_t *exp_done, float *exp_val, const float *exp_rew,
                float *exp_ret, float *exp_adv, double *work, void *stream);

/* One PPO minibatch: [obs RMS update (mini-epoch 0)], forward, losses,
 * backward, [grad all-reduce happens between the two halves on multi-GPU],
 * grad-norm clip, Adam, KL, adaptive LR, mu/sigma write-back.
 * Replaces A2CAgent.calc_gradients (a2c_continuous.py:78-196),
 * trancate_gradients_and_step (a2c_common.py:308-330),
 * PPODataset.update_mu_sigma (datasets.py:25-29),
 * AdaptiveScheduler.update (schedulers.py:26-32).
 * Split in two so the flat gradient can be all-reduced in between:
 *   ppo_minibatch_grad  -> grad[PPO_NPARAM] (+ kl sum in grad[PPO_NPARAM])
 *   ppo_minibatch_apply -> clip + Adam + lr update.
 * opt: device floats [2][8], two slots of [0]=lr [1]=step [2]=last kl [3]=last grad norm
 *      [4..7] unused; ppo_minibatch_apply reads slot opt_slot (0 or 1) and writes the
 *      next values to the other slot (callers alternate; no in-kernel completion counter);
 * m, v: [PPO_NPARAM].  minibatch must be a multiple of 32 (one 512-thread workgroup per 32 rows).
 * grad must be 16-byte aligned.  losses (nullable) receives the minibatch means
 * (a_loss, c_loss, entropy, b_loss, kl) of this rank; kl_out (nullable) the KL
 * the LR schedule used (after the all-reduce), as kls[] of the reference log.
 * grad has ppo_grad_floats() entries: [0, NPARAM) gradient, [NPARAM] kl, then
 * the reduce kernel's per-workgroup squared norms; norm_from_partials = 1 (only
 * when grad was NOT all-reduced) takes the clip norm from those. */
int ppo_minibatch_grad(const ppo_cfg_t *cfg, const float *params, double *obs_rms,
                       const double *val_rms, int update_obs_rms, int mb_index,
                       const float *exp_obs, const float *exp_act, const float *exp_nlp,
                       const float *exp_val, const float *exp_ret, const float *exp_adv,
                       float *exp_mu, float *exp_sigma, float *grad, float *losses,
                       float *partials, double *work, void *stream);
/* RunningMeanStd.train of mini-epoch 0 for the whole epoch at once (it depends only on the
 * rollout's observations): merges the rows / minibatch minibatches of exp_obs in order into
 * obs_rms (final state) and writes the running (mean[33], var[33]) after merge k to
 * rms_seq[k * 66]; minibatch k of mini-epoch 0 then calls ppo_minibatch_grad with
 * obs_rms = rms_seq + 66 k and update_obs_rms = 0 (same normalisation as update_obs_rms = 1).
 * rms_seq: ppo_rms_seq_doubles(cfg, rows) doubles (the tail is scratch). */
int ppo_obs_rms_epoch(const ppo_cfg_t *cfg, const float *exp_obs, int rows, double *obs_rms, double *rms_seq,
                      void *stream);
int ppo_rms_seq_doubles(const ppo_cfg_t *cfg, int rows);
int ppo_minibatch_apply(const ppo_cfg_t *cfg, float *params, float *grad, float *adam_m,
                        float *adam_v, float *opt, int opt_slot, float grad_scale,
                        float *kl_out, int norm_from_partials, void *stream);

/* The single-GPU minibatch chain in two launches per minibatch instead of three (the same
 * training step as ppo_minibatch_grad + ppo_minibatch_apply(norm_from_partials = 1), bit for
 * bit).  The parameters and Adam moments live in two banks; minibatch seq (0-based position in
 * the update's chain: mini-epoch x num_minibatches + minibatch) trains on bank seq % 2, and its
 * reduce kernel takes the Adam step with clip coefficient 1 into bank (seq + 1) % 2.  The clip
 * norm needs the whole gradient, so the next launch (minibatch seq + 1's gradient kernel, or
 * ppo_minibatch_finish after the last minibatch) checks it: when clipping was due it redoes
 * the step from bank seq % 2 and writes the result over bank (seq + 1) % 2.  The optimiser
 * scalars advance as with ppo_minibatch_apply (slot seq % 2 -> (seq + 1) % 2); kl_prev_out
 * receives minibatch seq - 1's KL (seq > 0), ppo_minibatch_finish's kl_out the last one's.
 * After a chain of count minibatches the state is in bank count % 2 (the caller copies it
 * back to bank 0 when count is odd).  Not for several ranks (the gradient is all-reduced
 * between the reduction and the step there: ppo_minibatch_grad / ppo_minibatch_apply).
 * Status 4: a bank pointer is NULL or params[i] is not 16-byte aligned. */
typedef struct ppo_adam_banks {
  float *params[2];
  float *m[2];
  float *v[2];
  float *opt;                          /* [2][8], as ppo_minibatch_apply */
} ppo_adam_banks_t;
int ppo_minibatch_fused(const ppo_cfg_t *cfg, const ppo_adam_banks_t *banks, int seq, double *obs_rms,
                        int update_obs_rms, int mb_index, const float *exp_obs, const float *exp_act,
                        const float *exp_nlp, const float *exp_val, const float *exp_ret, const float *exp_adv,
                        float *exp_mu, float *exp_sigma, float *grad, float *losses, float *partials, double *work,
                        float *kl_prev_out, void *stream);
int ppo_minibatch_finish(const ppo_cfg_t *cfg, const ppo_adam_banks_t *banks, int count, const float *grad,
                         float *kl_out, void *stream);

/* ------------------------------------------------------------------------
 * Several ranks (one process per GPU, a2c_common.py:87-101): the same two-launch chain with the
 * gradient all-reduce (trancate_gradients_and_step's flat SUM / rank_size, a2c_common.py:308-323, and the
 * legacy schedule's KL SUM / rank_size, :1218-1222) done INSIDE the reduction kernel as a one-shot
 * exchange over xGMI peer memory: the workgroup that owns a 128-slot chunk stores its rank's chunk into
 * every rank's receive buffer (IPC-mapped), raises one flag per receiver, waits for every sender's flag of
 * its chunk, sums the senders in rank order (deterministic, the same result on every rank), divides by
 * the rank count and takes the speculative Adam step as ppo_minibatch_fused does.  No collective library,
 * nothing for the host to launch between the kernels: the whole update stays one HIP graph.
 * Replaces A2CBase.trancate_gradients_and_step's dist.all_reduce (a2c_common.py:308-323).
 * ------------------------------------------------------------------------ */
#define PPO_DP_MAX 8
typedef struct ppo_dp {
  int rank, world;              /* this rank, number of ranks (<= PPO_DP_MAX) */
  void *peer[PPO_DP_MAX];       /* receive buffer of rank r mapped into this process (peer[rank] = own);
                                   each ppo_dp_buffer_bytes(), zeroed, from ppo_dp_alloc */
  uint32_t *clock;              /* this rank's device minibatch counter (advanced by the gradient kernel) */
  int32_t *err;                 /* device word: bit 0 set when a peer's chunk did not arrive within timeout_ms */
  int timeout_ms;
  int pad;
} ppo_dp_t;
/* bytes of one rank's receive buffer: [2 parities][PPO_DP_MAX senders][slots] floats + arrival flags */
long long ppo_dp_buffer_bytes(void);
/* allocate (uncached device memory, else hipMalloc) + zero one receive buffer; ipc_handle (64 bytes,
   hipIpcMemHandle_t) for the other ranks */
int ppo_dp_alloc(void **dptr, void *ipc_handle);
/* start-up check of the exchange on every rank at once (each rank launches it after the handles went
   around): `rounds` exchanges with keys key0.. of payloads naming (sender, round, slot), every received
   value compared; sets bit 0 of *dp->err when a flag did not arrive within timeout_ms, bit 1 when a
   payload arrived wrong or stale.  Afterwards the ranks agree, reset *dp->err and set *dp->clock to
   key0 + rounds - 1 (the flags' last key), or fall back to collectives. */
int ppo_dp_selftest(const ppo_dp_t *dp, unsigned key0, int rounds, int timeout_ms, void *stream);
/* map another rank's receive buffer (hipIpcOpenMemHandle, lazy peer access) / unmap / free our own */
int ppo_dp_open(const void *ipc_handle, void **dptr);
int ppo_dp_close(void *dptr);
int ppo_dp_free(void *dptr);
int ppo_minibatch_fused_dp(const ppo_cfg_t *cfg, const ppo_adam_banks_t *banks, const ppo_dp_t *dp, int seq,
                           double *obs_rms, int update_obs_rms, int mb_index, const float *exp_obs,
                           const float *exp_act, const float *exp_nlp, const float *exp_val, const float *exp_ret,
                           const float *exp_adv, float *exp_mu, float *exp_sigma, float *grad, float *losses,
                           float *partials, double *work, float *kl_prev_out, void *stream);

/* Several ranks WITHOUT the peer exchange (its set-up or start-up test failed, or USV_DP_EXCHANGE=collective): the
 * RCCL fallback, still two launches per minibatch.  The caller SUM-all-reduces grad[0, PPO_NPARAM] (gradient + KL,
 * a2c_common.py:308-323, 1218-1222) in stream order after each ppo_minibatch_coll; minibatch seq's gradient kernel
 * then takes minibatch seq - 1's clip + Adam + LR step itself in every workgroup (the all-reduced gradient x
 * grad_scale = 1 / world, ppo_minibatch_apply's norm of it) from bank (seq - 1) % 2 into bank seq % 2 and trains on
 * the result; ppo_minibatch_coll_finish takes the last minibatch's step.  Same bits as ppo_minibatch_grad +
 * all-reduce + ppo_minibatch_apply(grad_scale, norm_from_partials = 0) per minibatch; banks / opt / kl outputs as
 * ppo_minibatch_fused (state in bank count % 2).  Graph-capturable with the collectives (nccl). */
int ppo_minibatch_coll(const ppo_cfg_t *cfg, const ppo_adam_banks_t *banks, int seq, float grad_scale,
                       double *obs_rms, int update_obs_rms, int mb_index, const float *exp_obs, const float *exp_act,
                       const float *exp_nlp, const float *exp_val, const float *exp_ret, const float *exp_adv,
                       float *exp_mu, float *exp_sigma, float *grad, float *losses, float *partials, double *work,
                       float *kl_prev_out, void *stream);
int ppo_minibatch_coll_finish(const ppo_cfg_t *cfg, const ppo_adam_banks_t *banks, int count, const float *grad,
                              float grad_scale, float *kl_out, void *stream);

/* size (floats) of the per-block partial-gradient scratch of ppo_minibatch_grad (16-byte aligned): one row per
 * 32-row workgroup, chunk-major ([128-slot chunk][workgroup][128]) for the reduction's contiguous reads, then the
 * group fold's rows and control words (after the larger of the two row layouts); <= 0 when minibatch is not a
 * positive multiple of 32 or the buffer would pass 2^31 floats -- the minibatch entry points return 2 then */
int ppo_partials_floats(int minibatch);
/* size (floats) of the grad buffer of ppo_minibatch_grad / ppo_minibatch_apply */
int ppo_grad_floats(void);
/* size (floats) of the meter buffer of ppo_store_reward */
int ppo_meter_floats(int n_envs, int horizon);
/* ------------------------------------------------------------------------
 * loopz trainer (the reference's default trainer, scripts/rlgames_train.py:273-328 with
 * algo/ppo/{ppo,storage,module}.py): MLPEncode actor / critic (mass encoder 8-64-16-8, main
 * MLP (obs_dim - 8 + 8)-128-128-{2 tanh, 1}, LeakyReLU 0.01), tanh-squashed diagonal
 * Gaussian, time-major rollout storage [T][N], GAE, in-order minibatches, clip_grad_norm_ +
 * Adam.  Flat parameters (optimizer order): actor net | std[2] | critic net, each net
 * mass_encoder.{0,2,4}.{weight,bias} then action_mlp.{0,2,4}.{weight,bias}.
 * ------------------------------------------------------------------------ */
#define LZ_MASS 8
#define LZ_LAT  8
#define LZ_E1   64
#define LZ_E2   16
#define LZ_NH   128
#define LZ_NA   2
#define LZ_MAX_OBS 36
typedef struct lz_cfg {
  int   n_envs;
  int   horizon;             /* num_transitions_per_env: floor(max_time / control_dt) */
  int   obs_dim;             /* 33 (priv_dim 8) or 29 (priv_dim 4); <= LZ_MAX_OBS */
  int   mini_batches;        /* 4 */
  int   epochs;              /* num_learning_epochs 4 */
  int   use_clipped_value_loss;
  float gamma, lam;          /* 0.997, 0.95 */
  float clip;                /* clip_param 0.2 */
  float value_loss_coef;     /* 0.5 */
  float entropy_coef;        /* 0.0 */
  float max_grad_norm;       /* 0.5 */
  float lr, adam_b1, adam_b2, adam_eps;
  float min_std;             /* enforce_minimum_std 0.05 */
  float action_scale[LZ_NA]; /* clipActions */
  /* imitation term of PPO._train_step (ppo.py:253-286, flat_expert + update_rl_coeff :97-100): loss +=
   * mean_rows((1 - rl_coeff) * sum_a (expert_a - action_mean_a)^2); expert_act [T][N][2] (storage-row order)
   * holds flat_expert.evaluate of the stored observations (the expert is frozen: once per update), NULL = no
   * expert (the trainer's flat_expert = None, rlgames_train.py:92) */
  float im_coef;             /* 1 - rl_coeff */
  const float *expert_act;
} lz_cfg_t;

/* size (floats) of the flat loopz parameter vector (actor | std | critic) for obs_dim */
int lz_nparam(int obs_dim);
/* rollout step t: actor forward + squashed-Gaussian sample (u = mu + std eps, a = tanh(u) scale,
 * log_prob of module.py:555-583) and critic forward on obs [N][obs_dim] (nan_to_num'd, as
 * storage.add_transitions does); writes actions_out [N][2] and the storage rows
 * st_obs[t], st_act[t], st_logp[t], st_val[t].  eps_inject [N][2] (nullable): the N(0,1) draws;
 * otherwise Philox(seed, env, step, site 0x300). */
int lz_act(const lz_cfg_t *cfg, const float *params, const float *obs, int t, float *st_obs, float *st_act,
           float *st_logp, float *st_val, float *actions_out, uint64_t seed, uint64_t step,
           const float *eps_inject, void *stream);
/* critic forward only: values [N] (ppo.update's last_values) */
int lz_value(const lz_cfg_t *cfg, const float *params, const float *obs, float *values, void *stream);
/* storage.add_transitions' rewards / dones at step t (nan_to_num on the reward) */
int lz_store(const lz_cfg_t *cfg, const float *rew, const int64_t *dones, int t, float *st_rew, uint8_t *st_done,
             void *stream);
/* RolloutStorage.compute_returns (storage.py:92-121): returns, normalised advantages [T][N].
 * work: >= 8 + 4 * ceil(N / 256) doubles of device scratch. */
int lz_returns(const lz_cfg_t *cfg, const float *last_values, const float *st_rew, const uint8_t *st_done,
               const float *st_val, float *st_ret, float *st_adv, double *work, void *stream);
/* One PPO minibatch of _train_step (ppo.py:242-305): actor and critic gradients of rows
 * [mb * M, (mb + 1) * M) of the time-major batch (M = N T / mini_batches), fixed-order
 * reduction into grad (lz_grad_floats()), then clip_grad_norm_ + Adam, skipped when the loss
 * is not finite.  opt: [2][8] floats, slot opt_slot read, the other written ([0] lr, [1] step,
 * [2] value loss, [3] surrogate loss, [4] total norm, [5] 1 if the step was applied).
 * partials: lz_partials_floats(cfg) floats. */
int lz_minibatch(const lz_cfg_t *cfg, float *params, float *adam_m, float *adam_v, float *opt, int opt_slot, int mb,
                 const float *st_obs, const float *st_act, const float *st_logp, const float *st_val,
                 const float *st_ret, const float *st_adv, float *partials, float *grad, void *stream);
/* lz_minibatch with the rows of the minibatch given: rows (device [M], M = N T / mini_batches) are indices
 * into the flattened [T * N] storage -- the 'shuffle' sampler's minibatch (storage.py:123-134,
 * BatchSampler(SubsetRandomSampler(range(N T)), M, drop_last=True), the reference PPO's default sampling,
 * ppo.py:52-53); rows = NULL is lz_minibatch's in-order minibatch mb. */
int lz_minibatch_rows(const lz_cfg_t *cfg, float *params, float *adam_m, float *adam_v, float *opt, int opt_slot,
                      int mb, const float *st_obs, const float *st_act, const float *st_logp, const float *st_val,
                      const float *st_ret, const float *st_adv, const int32_t *rows, float *partials, float *grad,
                      void *stream);
/* enforce_minimum_std (module.py:649-659): std = max(finite(std) ? std : min_std, min_std) */
int lz_enforce_min_std(const lz_cfg_t *cfg, float *params, void *stream);
int lz_partials_floats(const lz_cfg_t *cfg);
int lz_grad_floats(int obs_dim);

/* library version */
int usv_hip_version(void);
/* the layout this library was compiled with: every object-like integer #define of this header (except the
 * include guard), every enumerator, and sizeof / offsetof of every field of every struct above, in header order,
 * each folded with its name: k = k * 1000003 + fnv1a(name), k = k * 1000003 + value (mod 2^64, top bit cleared).
 * A binding that allocates from this header compares it with the same fold of its own parse before its first
 * call (omniisaacgymenvs_loop_amd/_abi.py layout_entries), so a library built from another layout fails loudly
 * instead of addressing past a buffer */
long long usv_hip_layout_key(void);

#ifdef __cplusplus
}
#endif
#endif /* USV_HIP_H */
