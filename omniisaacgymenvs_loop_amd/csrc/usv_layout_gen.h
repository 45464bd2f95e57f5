/* generated from include/usv_hip.h by omniisaacgymenvs_loop_amd/_abi.py (gen_layout_header): do not edit.
 * X(expression, "name") for every entry of usv_hip_layout_key() in fold order. */
#define USV_LAYOUT_ENTRIES(X) \
  X(USV_NOBS, "USV_NOBS") \
  X(USV_NOBS_BASE, "USV_NOBS_BASE") \
  X(USV_NOBST, "USV_NOBST") \
  X(USV_NCLOSE, "USV_NCLOSE") \
  X(USV_GRID, "USV_GRID") \
  X(USV_GRID2, "USV_GRID2") \
  X(USV_FIELD_TH, "USV_FIELD_TH") \
  X(USV_FIELD_TW, "USV_FIELD_TW") \
  X(USV_FIELD_TROWS, "USV_FIELD_TROWS") \
  X(USV_FIELD_TCOLS, "USV_FIELD_TCOLS") \
  X(USV_FIELD_STRIDE, "USV_FIELD_STRIDE") \
  X(USV_LUT_N, "USV_LUT_N") \
  X(USV_NSTAT, "USV_NSTAT") \
  X(USV_SPAWN_ITERS, "USV_SPAWN_ITERS") \
  X(RU_MASS, "RU_MASS") \
  X(RU_COM, "RU_COM") \
  X(RU_KIZ, "RU_KIZ") \
  X(RU_KDRAG, "RU_KDRAG") \
  X(RU_THR, "RU_THR") \
  X(RU_DRAG, "RU_DRAG") \
  X(RU_SPAWN_R, "RU_SPAWN_R") \
  X(RU_SPAWN_TH, "RU_SPAWN_TH") \
  X(RU_YAW, "RU_YAW") \
  X(RU_OBST, "RU_OBST") \
  X(RU_RESAMPLE, "RU_RESAMPLE") \
  X(RU_VX, "RU_VX") \
  X(RU_VY, "RU_VY") \
  X(RU_GOAL, "RU_GOAL") \
  X(RU_FSIN, "RU_FSIN") \
  X(RU_FCONST, "RU_FCONST") \
  X(RU_TSIN, "RU_TSIN") \
  X(RU_TCONST, "RU_TCONST") \
  X(RU_GOAL_H, "RU_GOAL_H") \
  X(RU_TRIG, "RU_TRIG") \
  X(USV_NU_RESET, "USV_NU_RESET") \
  X(SU_VX, "SU_VX") \
  X(SU_VY, "SU_VY") \
  X(SU_WZ, "SU_WZ") \
  X(SU_HEAD, "SU_HEAD") \
  X(SU_PX, "SU_PX") \
  X(SU_ACT, "SU_ACT") \
  X(USV_NU_STEP, "USV_NU_STEP") \
  X(USV_NAN_ACTIONS, "USV_NAN_ACTIONS") \
  X(USV_NAN_STATE, "USV_NAN_STATE") \
  X(USV_NAN_REWARD, "USV_NAN_REWARD") \
  X(USV_NAN_OBS, "USV_NAN_OBS") \
  X(USV_NAN_POLICY, "USV_NAN_POLICY") \
  X(USV_NAN_EXTRAS, "USV_NAN_EXTRAS") \
  X(USV_TASK_CAPTURE_XY, "USV_TASK_CAPTURE_XY") \
  X(USV_TASK_GO_TO_POSE, "USV_TASK_GO_TO_POSE") \
  X(USV_TASK_TRACK_XYO, "USV_TASK_TRACK_XYO") \
  X(USV_TS_LIN_REW, "USV_TS_LIN_REW") \
  X(USV_TS_PEN, "USV_TS_PEN") \
  X(USV_TS_LIN_OK, "USV_TS_LIN_OK") \
  X(USV_TS_POS_KILL, "USV_TS_POS_KILL") \
  X(USV_TS_ROWS, "USV_TS_ROWS") \
  X(USV_STALE_UB, "USV_STALE_UB") \
  X(USV_STALE_VB, "USV_STALE_VB") \
  X(USV_STALE_RB, "USV_STALE_RB") \
  X(USV_STALE_PX, "USV_STALE_PX") \
  X(USV_STALE_PY, "USV_STALE_PY") \
  X(USV_STALE_ROWS, "USV_STALE_ROWS") \
  X(USV_FNORM, "USV_FNORM") \
  X(USV_RSTASH_ROWS, "USV_RSTASH_ROWS") \
  X(USV_CLOCK_WORDS, "USV_CLOCK_WORDS") \
  X(USV_SC_OBST, "USV_SC_OBST") \
  X(USV_SC_START, "USV_SC_START") \
  X(USV_SC_YAW, "USV_SC_YAW") \
  X(USV_SC_VEL, "USV_SC_VEL") \
  X(USV_SC_GOAL, "USV_SC_GOAL") \
  X(USV_SCENE_STRIDE, "USV_SCENE_STRIDE") \
  X(USV_FIELD_SLOT_STATS, "USV_FIELD_SLOT_STATS") \
  X(USV_CTL_RESET_COUNT, "USV_CTL_RESET_COUNT") \
  X(USV_CTL_POT_VALID, "USV_CTL_POT_VALID") \
  X(USV_CTL_PEN_VALID, "USV_CTL_PEN_VALID") \
  X(USV_CTL_REW_VALID, "USV_CTL_REW_VALID") \
  X(USV_CTL_NAN_FLAG, "USV_CTL_NAN_FLAG") \
  X(USV_CTL_ANY_INSIDE, "USV_CTL_ANY_INSIDE") \
  X(USV_CTL_ANY_FINITE, "USV_CTL_ANY_FINITE") \
  X(USV_CTL_OBST_DONE, "USV_CTL_OBST_DONE") \
  X(USV_CTL_STEPPED, "USV_CTL_STEPPED") \
  X(USV_CTL_PLACE, "USV_CTL_PLACE") \
  X(USV_CTL_H_SEED_LO, "USV_CTL_H_SEED_LO") \
  X(USV_CTL_H_SEED_HI, "USV_CTL_H_SEED_HI") \
  X(USV_CTL_H_STEP_LO, "USV_CTL_H_STEP_LO") \
  X(USV_CTL_H_STEP_HI, "USV_CTL_H_STEP_HI") \
  X(USV_CTL_H_INJ_LO, "USV_CTL_H_INJ_LO") \
  X(USV_CTL_H_INJ_HI, "USV_CTL_H_INJ_HI") \
  X(USV_CTL_SCENE_ERR, "USV_CTL_SCENE_ERR") \
  X(USV_CTL_BATCH_DONE, "USV_CTL_BATCH_DONE") \
  X(USV_CTL_FIELD_EXACT, "USV_CTL_FIELD_EXACT") \
  X(USV_CTL_N, "USV_CTL_N") \
  X(USV_SLAB_STATE, "USV_SLAB_STATE") \
  X(USV_SLAB_PARAMS, "USV_SLAB_PARAMS") \
  X(USV_SLAB_LIN_DAMP, "USV_SLAB_LIN_DAMP") \
  X(USV_SLAB_QUAD_DAMP, "USV_SLAB_QUAD_DAMP") \
  X(USV_SLAB_TGT, "USV_SLAB_TGT") \
  X(USV_SLAB_OBST, "USV_SLAB_OBST") \
  X(USV_SLAB_PREV_CMD, "USV_SLAB_PREV_CMD") \
  X(USV_SLAB_HIST, "USV_SLAB_HIST") \
  X(USV_SLAB_IBUF, "USV_SLAB_IBUF") \
  X(USV_SLAB_JUST_RESET, "USV_SLAB_JUST_RESET") \
  X(USV_SLAB_STATS, "USV_SLAB_STATS") \
  X(USV_SLAB_OBS, "USV_SLAB_OBS") \
  X(USV_SLAB_REW, "USV_SLAB_REW") \
  X(USV_SLAB_DONES, "USV_SLAB_DONES") \
  X(USV_SLAB_FIELD_OLD_TGT, "USV_SLAB_FIELD_OLD_TGT") \
  X(USV_SLAB_RESET_IDS, "USV_SLAB_RESET_IDS") \
  X(USV_SLAB_DIST, "USV_SLAB_DIST") \
  X(USV_SLAB_ENV_ORG, "USV_SLAB_ENV_ORG") \
  X(USV_SLAB_TGT_H, "USV_SLAB_TGT_H") \
  X(USV_SLAB_STALE, "USV_SLAB_STALE") \
  X(USV_SLAB_ROWS, "USV_SLAB_ROWS") \
  X(PPO_NIN, "PPO_NIN") \
  X(PPO_NH, "PPO_NH") \
  X(PPO_NA, "PPO_NA") \
  X(PPO_NPARAM, "PPO_NPARAM") \
  X(PPO_OFF_SIGMA, "PPO_OFF_SIGMA") \
  X(PPO_OFF_W1, "PPO_OFF_W1") \
  X(PPO_OFF_B1, "PPO_OFF_B1") \
  X(PPO_OFF_W2, "PPO_OFF_W2") \
  X(PPO_OFF_B2, "PPO_OFF_B2") \
  X(PPO_OFF_WV, "PPO_OFF_WV") \
  X(PPO_OFF_BV, "PPO_OFF_BV") \
  X(PPO_OFF_WMU, "PPO_OFF_WMU") \
  X(PPO_OFF_BMU, "PPO_OFF_BMU") \
  X(PPO_DP_MAX, "PPO_DP_MAX") \
  X(LZ_MASS, "LZ_MASS") \
  X(LZ_LAT, "LZ_LAT") \
  X(LZ_E1, "LZ_E1") \
  X(LZ_E2, "LZ_E2") \
  X(LZ_NH, "LZ_NH") \
  X(LZ_NA, "LZ_NA") \
  X(LZ_MAX_OBS, "LZ_MAX_OBS") \
  X(ST_TOTAL_REWARD, "ST_TOTAL_REWARD") \
  X(ST_DISTANCE_REWARD, "ST_DISTANCE_REWARD") \
  X(ST_ALIGNMENT_REWARD, "ST_ALIGNMENT_REWARD") \
  X(ST_HEADING_IMPROVE_REWARD, "ST_HEADING_IMPROVE_REWARD") \
  X(ST_POTENTIAL_SHAPING_REWARD, "ST_POTENTIAL_SHAPING_REWARD") \
  X(ST_SPEED_REWARD, "ST_SPEED_REWARD") \
  X(ST_ANGULAR_REWARD, "ST_ANGULAR_REWARD") \
  X(ST_TURN_HAZARD_PENALTY, "ST_TURN_HAZARD_PENALTY") \
  X(ST_GOAL_REWARD, "ST_GOAL_REWARD") \
  X(ST_COLLISION_REWARD, "ST_COLLISION_REWARD") \
  X(ST_TIME_REWARD, "ST_TIME_REWARD") \
  X(ST_SUCCESS, "ST_SUCCESS") \
  X(ST_COLLISION, "ST_COLLISION") \
  X(ST_POSITION_ERROR, "ST_POSITION_ERROR") \
  X(ST_BOUNDARY_PENALTY, "ST_BOUNDARY_PENALTY") \
  X(ST_DANGER_MEAN, "ST_DANGER_MEAN") \
  X(ST_DANGER_HI_RATE, "ST_DANGER_HI_RATE") \
  X(ST_G_GATE_MEAN, "ST_G_GATE_MEAN") \
  X(ST_G_SAFE_MEAN, "ST_G_SAFE_MEAN") \
  X(ST_ANGULAR_VEL_PENALTY, "ST_ANGULAR_VEL_PENALTY") \
  X(ST_ANGULAR_VEL_VARIATION_PENALTY, "ST_ANGULAR_VEL_VARIATION_PENALTY") \
  X(ST_ENERGY_PENALTY, "ST_ENERGY_PENALTY") \
  X(ST_NORMED_LINEAR_VEL, "ST_NORMED_LINEAR_VEL") \
  X(ST_NORMED_ANGULAR_VEL, "ST_NORMED_ANGULAR_VEL") \
  X(ST_CMD_NEG_RATE, "ST_CMD_NEG_RATE") \
  X(ST_U_MEAN, "ST_U_MEAN") \
  X(ST_U_LOW_RATE, "ST_U_LOW_RATE") \
  X(ST_U_SUM, "ST_U_SUM") \
  X(PEN_OFF, "PEN_OFF") \
  X(PEN_DEADZONE, "PEN_DEADZONE") \
  X(PEN_SUM, "PEN_SUM") \
  X(PEN_SUMSQ, "PEN_SUMSQ") \
  X(PEN_NORM, "PEN_NORM") \
  X(PEN_EXPABS, "PEN_EXPABS") \
  X(DI_FCX, "DI_FCX") \
  X(DI_FCY, "DI_FCY") \
  X(DI_FXF, "DI_FXF") \
  X(DI_FYF, "DI_FYF") \
  X(DI_FXS, "DI_FXS") \
  X(DI_FYS, "DI_FYS") \
  X(DI_FAMP, "DI_FAMP") \
  X(DI_TC, "DI_TC") \
  X(DI_TF, "DI_TF") \
  X(DI_TS, "DI_TS") \
  X(DI_TAMP, "DI_TAMP") \
  X(USV_NDIST, "USV_NDIST") \
  X(sizeof(usv_cfg_t), "sizeof usv_cfg") \
  X(offsetof(usv_cfg_t, dt), "usv_cfg.dt") \
  X(offsetof(usv_cfg_t, substeps), "usv_cfg.substeps") \
  X(offsetof(usv_cfg_t, thr_alpha), "usv_cfg.thr_alpha") \
  X(offsetof(usv_cfg_t, thr_y), "usv_cfg.thr_y") \
  X(offsetof(usv_cfg_t, izz0), "usv_cfg.izz0") \
  X(offsetof(usv_cfg_t, lin_damp), "usv_cfg.lin_damp") \
  X(offsetof(usv_cfg_t, quad_damp), "usv_cfg.quad_damp") \
  X(offsetof(usv_cfg_t, scaling_damping), "usv_cfg.scaling_damping") \
  X(offsetof(usv_cfg_t, use_drag_scale), "usv_cfg.use_drag_scale") \
  X(offsetof(usv_cfg_t, use_thr_mult), "usv_cfg.use_thr_mult") \
  X(offsetof(usv_cfg_t, thr_separate), "usv_cfg.thr_separate") \
  X(offsetof(usv_cfg_t, clip_actions), "usv_cfg.clip_actions") \
  X(offsetof(usv_cfg_t, affine_thrust), "usv_cfg.affine_thrust") \
  X(offsetof(usv_cfg_t, act_noise_on), "usv_cfg.act_noise_on") \
  X(offsetof(usv_cfg_t, act_noise_min), "usv_cfg.act_noise_min") \
  X(offsetof(usv_cfg_t, act_noise_max), "usv_cfg.act_noise_max") \
  X(offsetof(usv_cfg_t, pos_noise_on), "usv_cfg.pos_noise_on") \
  X(offsetof(usv_cfg_t, pos_noise_min), "usv_cfg.pos_noise_min") \
  X(offsetof(usv_cfg_t, pos_noise_max), "usv_cfg.pos_noise_max") \
  X(offsetof(usv_cfg_t, vel_noise_on), "usv_cfg.vel_noise_on") \
  X(offsetof(usv_cfg_t, vel_noise_min), "usv_cfg.vel_noise_min") \
  X(offsetof(usv_cfg_t, vel_noise_max), "usv_cfg.vel_noise_max") \
  X(offsetof(usv_cfg_t, head_noise_on), "usv_cfg.head_noise_on") \
  X(offsetof(usv_cfg_t, head_noise_min), "usv_cfg.head_noise_min") \
  X(offsetof(usv_cfg_t, head_noise_max), "usv_cfg.head_noise_max") \
  X(offsetof(usv_cfg_t, obs_local), "usv_cfg.obs_local") \
  X(offsetof(usv_cfg_t, priv_dim), "usv_cfg.priv_dim") \
  X(offsetof(usv_cfg_t, clip_obs), "usv_cfg.clip_obs") \
  X(offsetof(usv_cfg_t, masscom_base), "usv_cfg.masscom_base") \
  X(offsetof(usv_cfg_t, mass_relative), "usv_cfg.mass_relative") \
  X(offsetof(usv_cfg_t, base_mass), "usv_cfg.base_mass") \
  X(offsetof(usv_cfg_t, com_scaled), "usv_cfg.com_scaled") \
  X(offsetof(usv_cfg_t, com_scale), "usv_cfg.com_scale") \
  X(offsetof(usv_cfg_t, base_com), "usv_cfg.base_com") \
  X(offsetof(usv_cfg_t, priv_mode), "usv_cfg.priv_mode") \
  X(offsetof(usv_cfg_t, priv_nominal), "usv_cfg.priv_nominal") \
  X(offsetof(usv_cfg_t, priv_drag_on), "usv_cfg.priv_drag_on") \
  X(offsetof(usv_cfg_t, priv_thr_on), "usv_cfg.priv_thr_on") \
  X(offsetof(usv_cfg_t, priv_kiz_on), "usv_cfg.priv_kiz_on") \
  X(offsetof(usv_cfg_t, kdrag_min), "usv_cfg.kdrag_min") \
  X(offsetof(usv_cfg_t, kdrag_max), "usv_cfg.kdrag_max") \
  X(offsetof(usv_cfg_t, thr_min), "usv_cfg.thr_min") \
  X(offsetof(usv_cfg_t, thr_max), "usv_cfg.thr_max") \
  X(offsetof(usv_cfg_t, kiz_min), "usv_cfg.kiz_min") \
  X(offsetof(usv_cfg_t, kiz_max), "usv_cfg.kiz_max") \
  X(offsetof(usv_cfg_t, position_tolerance), "usv_cfg.position_tolerance") \
  X(offsetof(usv_cfg_t, kill_after_n), "usv_cfg.kill_after_n") \
  X(offsetof(usv_cfg_t, kill_dist), "usv_cfg.kill_dist") \
  X(offsetof(usv_cfg_t, boundary_cost), "usv_cfg.boundary_cost") \
  X(offsetof(usv_cfg_t, goal_reward), "usv_cfg.goal_reward") \
  X(offsetof(usv_cfg_t, time_reward), "usv_cfg.time_reward") \
  X(offsetof(usv_cfg_t, collision_threshold), "usv_cfg.collision_threshold") \
  X(offsetof(usv_cfg_t, obstacle_radius), "usv_cfg.obstacle_radius") \
  X(offsetof(usv_cfg_t, max_episode_length), "usv_cfg.max_episode_length") \
  X(offsetof(usv_cfg_t, fixed_horizon_eval), "usv_cfg.fixed_horizon_eval") \
  X(offsetof(usv_cfg_t, reward_mode), "usv_cfg.reward_mode") \
  X(offsetof(usv_cfg_t, position_scale), "usv_cfg.position_scale") \
  X(offsetof(usv_cfg_t, exp_coeff), "usv_cfg.exp_coeff") \
  X(offsetof(usv_cfg_t, align_la1), "usv_cfg.align_la1") \
  X(offsetof(usv_cfg_t, align_la2), "usv_cfg.align_la2") \
  X(offsetof(usv_cfg_t, align_la3), "usv_cfg.align_la3") \
  X(offsetof(usv_cfg_t, pen_lin_kind), "usv_cfg.pen_lin_kind") \
  X(offsetof(usv_cfg_t, pen_lin_k), "usv_cfg.pen_lin_k") \
  X(offsetof(usv_cfg_t, pen_lin_x0), "usv_cfg.pen_lin_x0") \
  X(offsetof(usv_cfg_t, pen_lin_c), "usv_cfg.pen_lin_c") \
  X(offsetof(usv_cfg_t, pen_ang_kind), "usv_cfg.pen_ang_kind") \
  X(offsetof(usv_cfg_t, pen_ang_k), "usv_cfg.pen_ang_k") \
  X(offsetof(usv_cfg_t, pen_ang_x0), "usv_cfg.pen_ang_x0") \
  X(offsetof(usv_cfg_t, pen_ang_c), "usv_cfg.pen_ang_c") \
  X(offsetof(usv_cfg_t, pen_angv_kind), "usv_cfg.pen_angv_kind") \
  X(offsetof(usv_cfg_t, pen_angv_k), "usv_cfg.pen_angv_k") \
  X(offsetof(usv_cfg_t, pen_angv_x0), "usv_cfg.pen_angv_x0") \
  X(offsetof(usv_cfg_t, pen_angv_c), "usv_cfg.pen_angv_c") \
  X(offsetof(usv_cfg_t, pen_en_kind), "usv_cfg.pen_en_kind") \
  X(offsetof(usv_cfg_t, pen_en_k), "usv_cfg.pen_en_k") \
  X(offsetof(usv_cfg_t, pen_en_x0), "usv_cfg.pen_en_x0") \
  X(offsetof(usv_cfg_t, pen_en_c), "usv_cfg.pen_en_c") \
  X(offsetof(usv_cfg_t, pen_actv_kind), "usv_cfg.pen_actv_kind") \
  X(offsetof(usv_cfg_t, pen_actv_k), "usv_cfg.pen_actv_k") \
  X(offsetof(usv_cfg_t, pen_actv_x0), "usv_cfg.pen_actv_x0") \
  X(offsetof(usv_cfg_t, pen_actv_c), "usv_cfg.pen_actv_c") \
  X(offsetof(usv_cfg_t, pen_use_u), "usv_cfg.pen_use_u") \
  X(offsetof(usv_cfg_t, map_size), "usv_cfg.map_size") \
  X(offsetof(usv_cfg_t, field_iters), "usv_cfg.field_iters") \
  X(offsetof(usv_cfg_t, influence_radius), "usv_cfg.influence_radius") \
  X(offsetof(usv_cfg_t, eta), "usv_cfg.eta") \
  X(offsetof(usv_cfg_t, safe_radius), "usv_cfg.safe_radius") \
  X(offsetof(usv_cfg_t, field_alpha), "usv_cfg.field_alpha") \
  X(offsetof(usv_cfg_t, mass_dr_on), "usv_cfg.mass_dr_on") \
  X(offsetof(usv_cfg_t, mass_min), "usv_cfg.mass_min") \
  X(offsetof(usv_cfg_t, mass_max), "usv_cfg.mass_max") \
  X(offsetof(usv_cfg_t, com_mode), "usv_cfg.com_mode") \
  X(offsetof(usv_cfg_t, com_disp), "usv_cfg.com_disp") \
  X(offsetof(usv_cfg_t, com_legacy_r), "usv_cfg.com_legacy_r") \
  X(offsetof(usv_cfg_t, couple_drag), "usv_cfg.couple_drag") \
  X(offsetof(usv_cfg_t, couple_thr), "usv_cfg.couple_thr") \
  X(offsetof(usv_cfg_t, couple_kiz), "usv_cfg.couple_kiz") \
  X(offsetof(usv_cfg_t, indep_kdrag_on), "usv_cfg.indep_kdrag_on") \
  X(offsetof(usv_cfg_t, kdrag_log), "usv_cfg.kdrag_log") \
  X(offsetof(usv_cfg_t, indep_thr_on), "usv_cfg.indep_thr_on") \
  X(offsetof(usv_cfg_t, thr_rand), "usv_cfg.thr_rand") \
  X(offsetof(usv_cfg_t, left_rand), "usv_cfg.left_rand") \
  X(offsetof(usv_cfg_t, right_rand), "usv_cfg.right_rand") \
  X(offsetof(usv_cfg_t, indep_kiz_on), "usv_cfg.indep_kiz_on") \
  X(offsetof(usv_cfg_t, kiz_log), "usv_cfg.kiz_log") \
  X(offsetof(usv_cfg_t, drag_rand_on), "usv_cfg.drag_rand_on") \
  X(offsetof(usv_cfg_t, lin_rand), "usv_cfg.lin_rand") \
  X(offsetof(usv_cfg_t, quad_rand), "usv_cfg.quad_rand") \
  X(offsetof(usv_cfg_t, spawn_rmin), "usv_cfg.spawn_rmin") \
  X(offsetof(usv_cfg_t, spawn_rmax), "usv_cfg.spawn_rmax") \
  X(offsetof(usv_cfg_t, goal_random_position), "usv_cfg.goal_random_position") \
  X(offsetof(usv_cfg_t, obst_box), "usv_cfg.obst_box") \
  X(offsetof(usv_cfg_t, min_dist_safe), "usv_cfg.min_dist_safe") \
  X(offsetof(usv_cfg_t, min_obs_sep), "usv_cfg.min_obs_sep") \
  X(offsetof(usv_cfg_t, init_vel), "usv_cfg.init_vel") \
  X(offsetof(usv_cfg_t, stats_on), "usv_cfg.stats_on") \
  X(offsetof(usv_cfg_t, act_bias), "usv_cfg.act_bias") \
  X(offsetof(usv_cfg_t, act_bias_steps), "usv_cfg.act_bias_steps") \
  X(offsetof(usv_cfg_t, fdist_on), "usv_cfg.fdist_on") \
  X(offsetof(usv_cfg_t, fconst_on), "usv_cfg.fconst_on") \
  X(offsetof(usv_cfg_t, fsin_on), "usv_cfg.fsin_on") \
  X(offsetof(usv_cfg_t, fconst_min), "usv_cfg.fconst_min") \
  X(offsetof(usv_cfg_t, fconst_max), "usv_cfg.fconst_max") \
  X(offsetof(usv_cfg_t, fsin_min), "usv_cfg.fsin_min") \
  X(offsetof(usv_cfg_t, fsin_max), "usv_cfg.fsin_max") \
  X(offsetof(usv_cfg_t, ffreq_min), "usv_cfg.ffreq_min") \
  X(offsetof(usv_cfg_t, ffreq_max), "usv_cfg.ffreq_max") \
  X(offsetof(usv_cfg_t, fshift_min), "usv_cfg.fshift_min") \
  X(offsetof(usv_cfg_t, fshift_max), "usv_cfg.fshift_max") \
  X(offsetof(usv_cfg_t, tdist_on), "usv_cfg.tdist_on") \
  X(offsetof(usv_cfg_t, tconst_on), "usv_cfg.tconst_on") \
  X(offsetof(usv_cfg_t, tsin_on), "usv_cfg.tsin_on") \
  X(offsetof(usv_cfg_t, tconst_min), "usv_cfg.tconst_min") \
  X(offsetof(usv_cfg_t, tconst_max), "usv_cfg.tconst_max") \
  X(offsetof(usv_cfg_t, tsin_min), "usv_cfg.tsin_min") \
  X(offsetof(usv_cfg_t, tsin_max), "usv_cfg.tsin_max") \
  X(offsetof(usv_cfg_t, tfreq_min), "usv_cfg.tfreq_min") \
  X(offsetof(usv_cfg_t, tfreq_max), "usv_cfg.tfreq_max") \
  X(offsetof(usv_cfg_t, tshift_min), "usv_cfg.tshift_min") \
  X(offsetof(usv_cfg_t, tshift_max), "usv_cfg.tshift_max") \
  X(offsetof(usv_cfg_t, current_on), "usv_cfg.current_on") \
  X(offsetof(usv_cfg_t, flow_vel), "usv_cfg.flow_vel") \
  X(offsetof(usv_cfg_t, task_kind), "usv_cfg.task_kind") \
  X(offsetof(usv_cfg_t, tk_mode), "usv_cfg.tk_mode") \
  X(offsetof(usv_cfg_t, tk_coeff), "usv_cfg.tk_coeff") \
  X(offsetof(usv_cfg_t, tk_scale), "usv_cfg.tk_scale") \
  X(offsetof(usv_cfg_t, tk_tol), "usv_cfg.tk_tol") \
  X(offsetof(usv_cfg_t, tk_goal_rand), "usv_cfg.tk_goal_rand") \
  X(offsetof(usv_cfg_t, sig_gain), "usv_cfg.sig_gain") \
  X(offsetof(usv_cfg_t, nan_probe), "usv_cfg.nan_probe") \
  X(offsetof(usv_cfg_t, curriculum_on), "usv_cfg.curriculum_on") \
  X(offsetof(usv_cfg_t, pad_curriculum), "usv_cfg.pad_curriculum") \
  X(offsetof(usv_cfg_t, step_inc), "usv_cfg.step_inc") \
  X(offsetof(usv_cfg_t, cur_min_dist), "usv_cfg.cur_min_dist") \
  X(offsetof(usv_cfg_t, cur_max_dist), "usv_cfg.cur_max_dist") \
  X(offsetof(usv_cfg_t, cur_kill_dist), "usv_cfg.cur_kill_dist") \
  X(offsetof(usv_cfg_t, cur_warmup), "usv_cfg.cur_warmup") \
  X(offsetof(usv_cfg_t, cur_end), "usv_cfg.cur_end") \
  X(offsetof(usv_cfg_t, min_spawn_d), "usv_cfg.min_spawn_d") \
  X(offsetof(usv_cfg_t, max_spawn_d), "usv_cfg.max_spawn_d") \
  X(offsetof(usv_cfg_t, kill_dist_d), "usv_cfg.kill_dist_d") \
  X(offsetof(usv_cfg_t, stale_root), "usv_cfg.stale_root") \
  X(offsetof(usv_cfg_t, inj_trig), "usv_cfg.inj_trig") \
  X(sizeof(usv_bufs_t), "sizeof usv_bufs") \
  X(offsetof(usv_bufs_t, n), "usv_bufs.n") \
  X(offsetof(usv_bufs_t, pad0), "usv_bufs.pad0") \
  X(offsetof(usv_bufs_t, px), "usv_bufs.px") \
  X(offsetof(usv_bufs_t, py), "usv_bufs.py") \
  X(offsetof(usv_bufs_t, yaw), "usv_bufs.yaw") \
  X(offsetof(usv_bufs_t, vx), "usv_bufs.vx") \
  X(offsetof(usv_bufs_t, vy), "usv_bufs.vy") \
  X(offsetof(usv_bufs_t, wz), "usv_bufs.wz") \
  X(offsetof(usv_bufs_t, fl), "usv_bufs.fl") \
  X(offsetof(usv_bufs_t, fr), "usv_bufs.fr") \
  X(offsetof(usv_bufs_t, mass), "usv_bufs.mass") \
  X(offsetof(usv_bufs_t, com_x), "usv_bufs.com_x") \
  X(offsetof(usv_bufs_t, com_y), "usv_bufs.com_y") \
  X(offsetof(usv_bufs_t, com_z), "usv_bufs.com_z") \
  X(offsetof(usv_bufs_t, k_drag), "usv_bufs.k_drag") \
  X(offsetof(usv_bufs_t, thr_l), "usv_bufs.thr_l") \
  X(offsetof(usv_bufs_t, thr_r), "usv_bufs.thr_r") \
  X(offsetof(usv_bufs_t, k_iz), "usv_bufs.k_iz") \
  X(offsetof(usv_bufs_t, mass_r), "usv_bufs.mass_r") \
  X(offsetof(usv_bufs_t, lin_damp), "usv_bufs.lin_damp") \
  X(offsetof(usv_bufs_t, quad_damp), "usv_bufs.quad_damp") \
  X(offsetof(usv_bufs_t, tgt_x), "usv_bufs.tgt_x") \
  X(offsetof(usv_bufs_t, tgt_y), "usv_bufs.tgt_y") \
  X(offsetof(usv_bufs_t, obst), "usv_bufs.obst") \
  X(offsetof(usv_bufs_t, field), "usv_bufs.field") \
  X(offsetof(usv_bufs_t, prev_cmd), "usv_bufs.prev_cmd") \
  X(offsetof(usv_bufs_t, prev_dist), "usv_bufs.prev_dist") \
  X(offsetof(usv_bufs_t, prev_head), "usv_bufs.prev_head") \
  X(offsetof(usv_bufs_t, prev_pot), "usv_bufs.prev_pot") \
  X(offsetof(usv_bufs_t, prev_wz), "usv_bufs.prev_wz") \
  X(offsetof(usv_bufs_t, goal_cnt), "usv_bufs.goal_cnt") \
  X(offsetof(usv_bufs_t, progress), "usv_bufs.progress") \
  X(offsetof(usv_bufs_t, reset_buf), "usv_bufs.reset_buf") \
  X(offsetof(usv_bufs_t, just_reset), "usv_bufs.just_reset") \
  X(offsetof(usv_bufs_t, done_succ), "usv_bufs.done_succ") \
  X(offsetof(usv_bufs_t, done_coll), "usv_bufs.done_coll") \
  X(offsetof(usv_bufs_t, stats), "usv_bufs.stats") \
  X(offsetof(usv_bufs_t, obs), "usv_bufs.obs") \
  X(offsetof(usv_bufs_t, rew), "usv_bufs.rew") \
  X(offsetof(usv_bufs_t, dones), "usv_bufs.dones") \
  X(offsetof(usv_bufs_t, ctl), "usv_bufs.ctl") \
  X(offsetof(usv_bufs_t, reset_ids), "usv_bufs.reset_ids") \
  X(offsetof(usv_bufs_t, fscratch), "usv_bufs.fscratch") \
  X(offsetof(usv_bufs_t, extras), "usv_bufs.extras") \
  X(offsetof(usv_bufs_t, extras_acc), "usv_bufs.extras_acc") \
  X(offsetof(usv_bufs_t, field_old_tgt), "usv_bufs.field_old_tgt") \
  X(offsetof(usv_bufs_t, slot_stats), "usv_bufs.slot_stats") \
  X(offsetof(usv_bufs_t, sdf), "usv_bufs.sdf") \
  X(offsetof(usv_bufs_t, grid_lin), "usv_bufs.grid_lin") \
  X(offsetof(usv_bufs_t, dist), "usv_bufs.dist") \
  X(offsetof(usv_bufs_t, env_org), "usv_bufs.env_org") \
  X(offsetof(usv_bufs_t, tgt_h), "usv_bufs.tgt_h") \
  X(offsetof(usv_bufs_t, task_scratch), "usv_bufs.task_scratch") \
  X(offsetof(usv_bufs_t, scene), "usv_bufs.scene") \
  X(offsetof(usv_bufs_t, scene_next), "usv_bufs.scene_next") \
  X(offsetof(usv_bufs_t, scene_last), "usv_bufs.scene_last") \
  X(offsetof(usv_bufs_t, n_scenes), "usv_bufs.n_scenes") \
  X(offsetof(usv_bufs_t, scene_cycle), "usv_bufs.scene_cycle") \
  X(offsetof(usv_bufs_t, clock), "usv_bufs.clock") \
  X(offsetof(usv_bufs_t, rstash), "usv_bufs.rstash") \
  X(offsetof(usv_bufs_t, fnorm), "usv_bufs.fnorm") \
  X(offsetof(usv_bufs_t, stale), "usv_bufs.stale") \
  X(sizeof(usv_hydro_t), "sizeof usv_hydro") \
  X(offsetof(usv_hydro_t, water_density), "usv_hydro.water_density") \
  X(offsetof(usv_hydro_t, gravity), "usv_hydro.gravity") \
  X(offsetof(usv_hydro_t, metacentric_width), "usv_hydro.metacentric_width") \
  X(offsetof(usv_hydro_t, metacentric_length), "usv_hydro.metacentric_length") \
  X(offsetof(usv_hydro_t, avg_force), "usv_hydro.avg_force") \
  X(offsetof(usv_hydro_t, amplify_torque), "usv_hydro.amplify_torque") \
  X(offsetof(usv_hydro_t, waterplane_area), "usv_hydro.waterplane_area") \
  X(offsetof(usv_hydro_t, zero_height), "usv_hydro.zero_height") \
  X(offsetof(usv_hydro_t, max_volume), "usv_hydro.max_volume") \
  X(sizeof(ppo_cfg_t), "sizeof ppo_cfg") \
  X(offsetof(ppo_cfg_t, horizon), "ppo_cfg.horizon") \
  X(offsetof(ppo_cfg_t, n_envs), "ppo_cfg.n_envs") \
  X(offsetof(ppo_cfg_t, minibatch), "ppo_cfg.minibatch") \
  X(offsetof(ppo_cfg_t, normalize_input), "ppo_cfg.normalize_input") \
  X(offsetof(ppo_cfg_t, normalize_value), "ppo_cfg.normalize_value") \
  X(offsetof(ppo_cfg_t, normalize_advantage), "ppo_cfg.normalize_advantage") \
  X(offsetof(ppo_cfg_t, gamma), "ppo_cfg.gamma") \
  X(offsetof(ppo_cfg_t, tau), "ppo_cfg.tau") \
  X(offsetof(ppo_cfg_t, e_clip), "ppo_cfg.e_clip") \
  X(offsetof(ppo_cfg_t, critic_coef), "ppo_cfg.critic_coef") \
  X(offsetof(ppo_cfg_t, entropy_coef), "ppo_cfg.entropy_coef") \
  X(offsetof(ppo_cfg_t, bounds_loss_coef), "ppo_cfg.bounds_loss_coef") \
  X(offsetof(ppo_cfg_t, clip_value), "ppo_cfg.clip_value") \
  X(offsetof(ppo_cfg_t, truncate_grads), "ppo_cfg.truncate_grads") \
  X(offsetof(ppo_cfg_t, grad_norm), "ppo_cfg.grad_norm") \
  X(offsetof(ppo_cfg_t, adam_b1), "ppo_cfg.adam_b1") \
  X(offsetof(ppo_cfg_t, adam_b2), "ppo_cfg.adam_b2") \
  X(offsetof(ppo_cfg_t, adam_eps), "ppo_cfg.adam_eps") \
  X(offsetof(ppo_cfg_t, weight_decay), "ppo_cfg.weight_decay") \
  X(offsetof(ppo_cfg_t, lr_adaptive), "ppo_cfg.lr_adaptive") \
  X(offsetof(ppo_cfg_t, kl_threshold), "ppo_cfg.kl_threshold") \
  X(offsetof(ppo_cfg_t, lr_min), "ppo_cfg.lr_min") \
  X(offsetof(ppo_cfg_t, lr_max), "ppo_cfg.lr_max") \
  X(offsetof(ppo_cfg_t, reward_scale), "ppo_cfg.reward_scale") \
  X(offsetof(ppo_cfg_t, reward_shift), "ppo_cfg.reward_shift") \
  X(offsetof(ppo_cfg_t, rms_eps), "ppo_cfg.rms_eps") \
  X(offsetof(ppo_cfg_t, bf16_gemm), "ppo_cfg.bf16_gemm") \
  X(offsetof(ppo_cfg_t, nan_probe), "ppo_cfg.nan_probe") \
  X(offsetof(ppo_cfg_t, nan_flag), "ppo_cfg.nan_flag") \
  X(sizeof(ppo_adam_banks_t), "sizeof ppo_adam_banks") \
  X(offsetof(ppo_adam_banks_t, params), "ppo_adam_banks.params") \
  X(offsetof(ppo_adam_banks_t, m), "ppo_adam_banks.m") \
  X(offsetof(ppo_adam_banks_t, v), "ppo_adam_banks.v") \
  X(offsetof(ppo_adam_banks_t, opt), "ppo_adam_banks.opt") \
  X(sizeof(ppo_dp_t), "sizeof ppo_dp") \
  X(offsetof(ppo_dp_t, rank), "ppo_dp.rank") \
  X(offsetof(ppo_dp_t, world), "ppo_dp.world") \
  X(offsetof(ppo_dp_t, peer), "ppo_dp.peer") \
  X(offsetof(ppo_dp_t, clock), "ppo_dp.clock") \
  X(offsetof(ppo_dp_t, err), "ppo_dp.err") \
  X(offsetof(ppo_dp_t, timeout_ms), "ppo_dp.timeout_ms") \
  X(offsetof(ppo_dp_t, pad), "ppo_dp.pad") \
  X(sizeof(lz_cfg_t), "sizeof lz_cfg") \
  X(offsetof(lz_cfg_t, n_envs), "lz_cfg.n_envs") \
  X(offsetof(lz_cfg_t, horizon), "lz_cfg.horizon") \
  X(offsetof(lz_cfg_t, obs_dim), "lz_cfg.obs_dim") \
  X(offsetof(lz_cfg_t, mini_batches), "lz_cfg.mini_batches") \
  X(offsetof(lz_cfg_t, epochs), "lz_cfg.epochs") \
  X(offsetof(lz_cfg_t, use_clipped_value_loss), "lz_cfg.use_clipped_value_loss") \
  X(offsetof(lz_cfg_t, gamma), "lz_cfg.gamma") \
  X(offsetof(lz_cfg_t, lam), "lz_cfg.lam") \
  X(offsetof(lz_cfg_t, clip), "lz_cfg.clip") \
  X(offsetof(lz_cfg_t, value_loss_coef), "lz_cfg.value_loss_coef") \
  X(offsetof(lz_cfg_t, entropy_coef), "lz_cfg.entropy_coef") \
  X(offsetof(lz_cfg_t, max_grad_norm), "lz_cfg.max_grad_norm") \
  X(offsetof(lz_cfg_t, lr), "lz_cfg.lr") \
  X(offsetof(lz_cfg_t, adam_b1), "lz_cfg.adam_b1") \
  X(offsetof(lz_cfg_t, adam_b2), "lz_cfg.adam_b2") \
  X(offsetof(lz_cfg_t, adam_eps), "lz_cfg.adam_eps") \
  X(offsetof(lz_cfg_t, min_std), "lz_cfg.min_std") \
  X(offsetof(lz_cfg_t, action_scale), "lz_cfg.action_scale") \
  X(offsetof(lz_cfg_t, im_coef), "lz_cfg.im_coef") \
  X(offsetof(lz_cfg_t, expert_act), "lz_cfg.expert_act") \

