"""Task-yaml -> usv_cfg_t (the constant block every env kernel receives).

Accepts the reference's task config dict unchanged (the keys of
cfg/task/USV/IROS2024/USV_Virtual_CaptureXY_SysID-TEST.yaml and siblings) and
resolves every flag the reference resolves at construction time:

* USVVirtual.__init__ (tasks/USV_Virtual.py:295-648): action processing,
  mass-driven coupling activation, privileged-tail encoding ranges;
* HydrodynamicsObject / DynamicsFirstOrder constructors
  (envs/USV/Hydrodynamics.py:6-117, envs/USV/ThrusterDynamics.py:33-110);
* Penalties.__post_init__ (tasks/USV/USV_task_rewards.py:429-438): the
  penalty lambdas are *strings eval'd* by the reference; here they are parsed
  into a closed set of forms (usv_pen_kind) and anything else is rejected.
"""
from __future__ import annotations

import math
import os
import re
from typing import Any, Dict

import numpy as np

from .._abi import PEN, UsvCfg, UsvHydro

# heron.usd rigid-body constants (decoded offline)
HERON_THRUSTER_Y = 0.37765
HERON_THRUSTER_X = -0.5006
HERON_IZZ = 8.061

# CaptureXYParameters / CaptureXYReward defaults (USV_task_parameters.py:16-52,
# USV_task_rewards.py:20-32)
_TASK_DEFAULTS = dict(position_tolerance=0.1, kill_after_n_steps_in_tolerance=1, goal_random_position=0.0,
                      max_spawn_dist=11.0, min_spawn_dist=0.5, kill_dist=20.0, boundary_cost=25.0,
                      goal_reward=100.0, time_reward=-0.1)
_REWARD_DEFAULTS = dict(reward_mode="exponential", position_scale=1.5, exponential_reward_coeff=0.25,
                        align_la1=0.04, align_la2=-10.0, align_la3=-0.1)
_PEN_DEFAULTS = dict(
    penalize_linear_velocities=False, penalize_linear_velocities_fn="lambda x,step: -torch.norm(x, dim=-1)*c1 + c2",
    penalize_linear_velocities_c1=0.01, penalize_linear_velocities_c2=0.0,
    penalize_angular_velocities=False, penalize_angular_velocities_fn="lambda x,step : -torch.abs(x)*c1 + c2",
    penalize_angular_velocities_c1=0.01, penalize_angular_velocities_c2=0.0,
    penalize_angular_velocities_variation=False,
    penalize_angular_velocities_variation_fn="lambda x,step: torch.exp(c1 * torch.abs(x)) - 1.0",
    penalize_angular_velocities_variation_c1=-0.033,
    penalize_energy=False, penalize_energy_fn="lambda x,step : -torch.sum(x**2)*c1 + c2",
    penalize_energy_c1=0.01, penalize_energy_c2=0.0,
    penalize_action_variation=False, penalize_action_variation_fn="lambda x,step: torch.exp(c1 * torch.abs(x)) - 1.0",
    penalize_action_variation_c1=-0.033,
)

_NUM = r"([-+]?(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?|c1|c2)"


def parse_penalty_fn(src: str, consts: Dict[str, float]):
    """Map a reference penalty lambda string to (kind, k, x0, c).

    The reference eval()s these strings (USV_task_rewards.py:432-438); only the
    closed forms below are accepted, everything else raises ValueError.
    """
    s = re.sub(r"\s+", "", src)
    body = s.split(":", 1)[1] if s.startswith("lambda") else s

    def num(tok):
        if tok in ("c1", "c2"):
            return float(consts[tok])
        return float(tok)

    pats = [
        # -torch.clamp(torch.abs(x)-X0,min=0.0)*K [+C]
        (rf"^-torch\.clamp\(torch\.abs\(x\)-{_NUM},min=0(?:\.0)?\)\*{_NUM}(?:\+{_NUM})?$",
         lambda m: (PEN["PEN_DEADZONE"], num(m[1]), num(m[0]), num(m[2]) if m[2] else 0.0)),
        # -torch.abs(x)*K [+C]
        (rf"^-torch\.abs\(x\)\*{_NUM}(?:\+{_NUM})?$",
         lambda m: (PEN["PEN_DEADZONE"], num(m[0]), 0.0, num(m[1]) if m[1] else 0.0)),
        # -torch.sum(x,dim=-1)*K [+C]
        (rf"^-torch\.sum\(x(?:,dim=-1)?\)\*{_NUM}(?:\+{_NUM})?$",
         lambda m: (PEN["PEN_SUM"], num(m[0]), 0.0, num(m[1]) if m[1] else 0.0)),
        # -torch.sum(x**2[,dim=-1])*K [+C]
        (rf"^-torch\.sum\(x\*\*2(?:,dim=-1)?\)\*{_NUM}(?:\+{_NUM})?$",
         lambda m: (PEN["PEN_SUMSQ"], num(m[0]), 0.0, num(m[1]) if m[1] else 0.0)),
        # -torch.norm(x,dim=-1)*K [+C]
        (rf"^-torch\.norm\(x,dim=-1\)\*{_NUM}(?:\+{_NUM})?$",
         lambda m: (PEN["PEN_NORM"], num(m[0]), 0.0, num(m[1]) if m[1] else 0.0)),
        # (torch.exp(C1*torch.abs(x))-1.0)*K   or  torch.exp(C1*torch.abs(x))-1.0
        (rf"^\(torch\.exp\({_NUM}\*torch\.abs\(x\)\)-1(?:\.0)?\)\*{_NUM}$",
         lambda m: (PEN["PEN_EXPABS"], num(m[1]), num(m[0]), 0.0)),
        (rf"^torch\.exp\({_NUM}\*torch\.abs\(x\)\)-1(?:\.0)?$",
         lambda m: (PEN["PEN_EXPABS"], 1.0, num(m[0]), 0.0)),
    ]
    for pat, mk in pats:
        m = re.match(pat, body)
        if m:
            return mk(m.groups())
    raise ValueError(f"unsupported penalty function string: {src!r}")


def _f32(x) -> float:
    return float(np.float32(x))


def build_usv_cfg(task_cfg: Dict[str, Any]) -> UsvCfg:
    """Resolve the task config into the kernel constant block."""
    env = task_cfg["env"]
    dyn = task_cfg["dynamics"]
    dist = env["disturbances"]
    c = UsvCfg()

    # ---- integration ----
    dt = float(task_cfg["sim"]["dt"])
    c.dt = dt
    c.substeps = int(env.get("controlFrequencyInv", 10))
    tau = float(dyn["thrusters"]["timeConstant"])
    # alpha = torch.exp(torch.tensor(-dt/tau)) in fp32 (ThrusterDynamics.py:132);
    # -dt/tau is formed in double from the yaml values, then rounded once.
    c.thr_alpha = float(np.exp(np.float32(-dt / tau), dtype=np.float32))
    c.thr_y = HERON_THRUSTER_Y
    c.izz0 = HERON_IZZ
    hd = dyn["hydrodynamics"]
    lin, quad = hd["linear_damping"], hd["quadratic_damping"]
    fwd = hd["linear_damping_forward_speed"]
    for k, dof in enumerate((0, 1, 5)):  # u, v, r
        # lin + offset - (fwd + offset_fwd) (Hydrodynamics.py:185-192), in fp32
        l = np.float32(lin[dof]) + np.float32(hd["offset_linear_damping"])
        l = l - (np.float32(fwd[dof]) + np.float32(hd["offset_lin_forward_damping_speed"]))
        c.lin_damp[k] = float(np.float32(l))
        c.quad_damp[k] = float(np.float32(quad[dof]) + np.float32(hd["offset_nonlin_damping"]))
    c.scaling_damping = hd["scaling_damping"]

    # ---- domain randomisation / coupling flags (USV_Virtual.py:361-528) ----
    mass = dist["mass"]
    drag = dist.get("drag", {}) or {}
    thr = dist.get("thruster", {}) or {}
    inertia = dist.get("inertia", {}) or {}
    coupling = ((dist.get("coupling", {}) or {}).get("mass_driven", {}) or {})
    mass_dr = bool(mass.get("add_mass_disturbances", False))
    coupled = bool(coupling.get("enabled", False)) and mass_dr
    targets = coupling.get("targets", ["drag_scale", "thruster", "yaw_inertia"]) or []
    if isinstance(targets, str):
        targets = [targets]
    c.couple_drag = int(coupled and "drag_scale" in targets)
    c.couple_thr = int(coupled and "thruster" in targets)
    c.couple_kiz = int(coupled and "yaw_inertia" in targets)
    c.indep_kdrag_on = int(bool(drag.get("use_drag_scale_randomization", False)))
    c.kdrag_log = int(str(drag.get("k_drag_sample_space", "linear")) == "log")
    c.indep_thr_on = int(bool(thr.get("use_thruster_randomization", False)) or bool(c.couple_thr))
    c.thr_separate = int(bool(thr.get("use_separate_randomization", False)) and not c.couple_thr)
    c.thr_rand = float(thr.get("thruster_rand", 0.0))
    c.left_rand = float(thr.get("left_rand", 0.0))
    c.right_rand = float(thr.get("right_rand", 0.0))
    c.indep_kiz_on = int(bool(inertia.get("use_yaw_inertia_randomization", False)))
    c.kiz_log = int(str(inertia.get("k_Iz_sample_space", "linear")) == "log")
    c.use_drag_scale = int(bool(c.indep_kdrag_on) or bool(c.couple_drag))
    c.use_thr_mult = int(bool(c.indep_thr_on))
    c.drag_rand_on = int(bool(drag.get("use_drag_randomization", False)))
    for k, dof in enumerate((0, 1, 5)):
        key = "uvwpqr"[dof]
        c.lin_rand[k] = float(drag.get(f"{key}_linear_rand", 0.0)) * lin[dof]
        c.quad_rand[k] = float(drag.get(f"{key}_quad_rand", 0.0)) * quad[dof]

    c.mass_dr_on = int(mass_dr)
    c.base_mass = float(mass.get("base_mass", mass.get("min_mass", 0.0)))
    c.mass_min = float(mass.get("min_mass", c.base_mass))
    c.mass_max = float(mass.get("max_mass", c.base_mass))
    base_com = [float(v) for v in mass.get("base_com", [0.0, 0.0, 0.0])]
    for a in range(3):
        c.base_com[a] = base_com[a]
    if mass.get("com_displacement_xyz", None) is not None:
        c.com_mode = 1
        for a in range(3):
            c.com_disp[a] = float(mass["com_displacement_xyz"][a])
    elif float(mass.get("CoM_max_displacement", 0.0) or 0.0) > 0.0:
        c.com_mode = 2
        c.com_legacy_r = float(mass["CoM_max_displacement"])
    else:
        c.com_mode = 0

    # ---- actions ----
    ap = env.get("action_processing", {}) or {}
    c.clip_actions = float(env.get("clipActions", 1.0))
    c.affine_thrust = int(bool(ap.get("use_affine_thrust_mapping", True)))
    an = dist["actions"]
    c.act_noise_on = int(bool(an["add_noise_on_act"]))
    c.act_noise_min, c.act_noise_max = an["min_action_noise"], an["max_action_noise"]
    on = dist["observations"]
    c.pos_noise_on = int(bool(on["add_noise_on_pos"]))
    c.pos_noise_min, c.pos_noise_max = on["position_noise_min"], on["position_noise_max"]
    c.vel_noise_on = int(bool(on["add_noise_on_vel"]))
    c.vel_noise_min, c.vel_noise_max = on["velocity_noise_min"], on["velocity_noise_max"]
    c.head_noise_on = int(bool(on["add_noise_on_heading"]))
    c.head_noise_min, c.head_noise_max = on["heading_noise_min"], on["heading_noise_max"]

    # ---- observation ----
    frame = env.get("observation_frame", "local")
    if frame not in ("local", "global"):
        raise ValueError(f"observation_frame must be local/global, got {frame}")
    c.obs_local = int(frame == "local")
    c.priv_dim = int(env.get("priv_dim", env.get("mass_dim", 4)))
    if c.priv_dim not in (4, 8):
        raise ValueError(f"Unsupported priv_dim/mass_dim={c.priv_dim}. Supported: 4 or 8.")
    clip_obs = env.get("clipObservations", {"state": 12.0})
    c.clip_obs = float(clip_obs["state"] if isinstance(clip_obs, dict) else clip_obs)
    src = str(mass.get("masscom_obs_source", "sim"))
    if src not in ("sim", "base"):
        raise ValueError(f"mass.masscom_obs_source must be 'sim' or 'base', got {src}")
    c.masscom_base = int(src == "base")
    mom = mass.get("mass_obs_mode", "raw")
    if mom not in ("raw", "relative"):
        raise ValueError(f"Unknown mass_obs_mode: {mom}")
    c.mass_relative = int(mom == "relative")
    com_mode = mass.get("com_obs_mode", "raw")
    if com_mode not in ("raw", "scaled"):
        raise ValueError(f"Unknown com_obs_mode: {com_mode}")
    c.com_scaled = int(com_mode == "scaled")
    hs = dyn["hydrostatics"]
    scale = mass.get("com_obs_scale", None)
    if c.com_scaled and scale is None:
        scale = [float(hs["box_length"]), float(hs["box_width"]), float(max(hs["heron_zero_height"], 1.0))]
    if scale is not None:
        for a in range(3):
            c.com_scale[a] = float(scale[a])
    pp = env.get("privileged_params", {}) or {}
    mode = str(pp.get("mode", "raw"))
    if mode not in ("raw", "centered", "minmax"):
        raise ValueError(f"env.privileged_params.mode must be 'raw', 'centered' or 'minmax', got {mode}")
    c.priv_mode = {"raw": 0, "centered": 1, "minmax": 2}[mode]
    c.priv_nominal = float(pp.get("nominal", 1.0))
    c.kdrag_min, c.kdrag_max = float(drag.get("k_drag_min", 1.0)), float(drag.get("k_drag_max", 1.0))
    c.kiz_min, c.kiz_max = float(inertia.get("k_Iz_min", 1.0)), float(inertia.get("k_Iz_max", 1.0))
    c.thr_min = 1.0 - c.thr_rand
    c.thr_max = 1.0 if c.couple_thr else 1.0 + c.thr_rand
    c.priv_drag_on = int(bool(drag.get("use_drag_scale_randomization", False)) or bool(c.couple_drag))
    c.priv_thr_on = int(bool(thr.get("use_thruster_randomization", False)) or bool(c.couple_thr))
    c.priv_kiz_on = int(bool(inertia.get("use_yaw_inertia_randomization", False)) or bool(c.couple_kiz))

    # ---- task / reward ----
    name = env["task_parameters"].get("name", "CaptureXY")
    if name not in TASK_KINDS:
        raise ValueError(f"task {name!r}: this kernel set implements {sorted(TASK_KINDS)}")
    c.task_kind = TASK_KINDS[name]
    tp = dict(_TASK_DEFAULTS)
    tp.update(env["task_parameters"] if name == "CaptureXY" else _pose_task_cfg(c, name, env))
    c.position_tolerance = tp["position_tolerance"]
    c.kill_after_n = int(tp["kill_after_n_steps_in_tolerance"])
    c.kill_dist, c.boundary_cost = tp["kill_dist"], tp["boundary_cost"]
    c.goal_reward, c.time_reward = tp["goal_reward"], tp["time_reward"]
    c.goal_random_position = tp["goal_random_position"]
    c.spawn_rmin, c.spawn_rmax = tp["min_spawn_dist"], tp["max_spawn_dist"]
    rp = dict(_REWARD_DEFAULTS)
    if name == "CaptureXY":
        rp.update(env["reward_parameters"])
    rm = rp["reward_mode"].lower()
    if rm not in ("linear", "square", "exponential"):
        raise ValueError("Linear, Square and Exponential are the only currently supported mode.")
    c.reward_mode = {"linear": 0, "square": 1, "exponential": 2}[rm]
    c.position_scale, c.exp_coeff = rp["position_scale"], rp["exponential_reward_coeff"]
    c.align_la1, c.align_la2, c.align_la3 = rp["align_la1"], rp["align_la2"], rp["align_la3"]
    c.collision_threshold = 1.2
    c.obstacle_radius = 0.5
    c.max_episode_length = int(env["maxEpisodeLength"])
    c.fixed_horizon_eval = int(bool(env.get("fixed_horizon_eval", env.get("fixedHorizonEval", False))))

    # ---- penalties ----
    pen = dict(_PEN_DEFAULTS)
    pen.update(env["penalties_parameters"])
    for tag, key in (("lin", "linear_velocities"), ("ang", "angular_velocities"),
                     ("angv", "angular_velocities_variation"), ("en", "energy"), ("actv", "action_variation")):
        if bool(pen[f"penalize_{key}"]):
            consts = {"c1": pen.get(f"penalize_{key}_c1", 0.0), "c2": pen.get(f"penalize_{key}_c2", 0.0)}
            kind, k, x0, cc = parse_penalty_fn(pen[f"penalize_{key}_fn"], consts)
        else:
            kind, k, x0, cc = 0, 0.0, 0.0, 0.0
        setattr(c, f"pen_{tag}_kind", kind)
        setattr(c, f"pen_{tag}_k", k)
        setattr(c, f"pen_{tag}_x0", x0)
        setattr(c, f"pen_{tag}_c", cc)
    if c.pen_lin_kind not in (0, PEN["PEN_NORM"]):
        raise ValueError("linear-velocity penalty must be the norm form")
    if c.pen_en_kind not in (0, PEN["PEN_SUM"], PEN["PEN_SUMSQ"]):
        raise ValueError("energy penalty must be a sum form")
    if c.pen_actv_kind != 0:
        raise NotImplementedError("penalize_action_variation is not on the CaptureXY hot path")
    c.pen_use_u = int(bool(ap.get("penalties_use_thrust_u", True)))

    # ---- potential field (d_multi_gemini.py / static_obs.py:30-32) ----
    c.map_size = 30.0
    c.field_iters = int(150 * 1.5)
    c.influence_radius, c.eta, c.safe_radius, c.field_alpha = 0.7, 20.0, 3.0, 0.5
    # ---- spawn (static_obs.py:974-983) ----
    c.obst_box, c.min_dist_safe, c.min_obs_sep = 12.0, 3.0, 2.5
    c.init_vel = 1.5
    c.stats_on = 1
    c.act_bias, c.act_bias_steps = action_bias_cfg(task_cfg)
    if bool((env.get("scene_replay", {}) or {}).get("enabled", False)) and c.task_kind != 0:
        # only CaptureXYTask implements apply_scene (USV_Virtual.py:1427-1428 raises AttributeError)
        raise AttributeError("Inner task does not implement apply_scene(); cannot use scene_replay")
    # ---- disturbances (ForceDisturbance / TorqueDisturbance.__init__, USV_disturbances.py:268-298,
    # 412-440) and water current (USVVirtual.__init__ -> ComputeHydrodynamicsEffects) ----
    fd = dist.get("forces", {}) or {}
    c.fdist_on = int(bool(fd.get("use_force_disturbance", False)))
    c.fconst_on = int(bool(fd.get("use_constant_force", False)))
    c.fsin_on = int(bool(fd.get("use_sinusoidal_force", False)))
    for k, key in (("fconst_min", "force_const_min"), ("fconst_max", "force_const_max"),
                   ("fsin_min", "force_sin_min"), ("fsin_max", "force_sin_max"),
                   ("ffreq_min", "force_min_freq"), ("ffreq_max", "force_max_freq"),
                   ("fshift_min", "force_min_shift"), ("fshift_max", "force_max_shift")):
        v = float(fd.get(key, 0.0))
        if k in ("fconst_min", "fconst_max", "fsin_min", "fsin_max"):
            v = math.sqrt(v ** 2 / 2)   # per-axis magnitude (USV_disturbances.py:281-288)
        setattr(c, k, v)
    td = dist.get("torques", {}) or {}
    c.tdist_on = int(bool(td.get("use_torque_disturbance", False)))
    c.tconst_on = int(bool(td.get("use_constant_torque", False)))
    c.tsin_on = int(bool(td.get("use_sinusoidal_torque", False)))
    for k, key in (("tconst_min", "torque_const_min"), ("tconst_max", "torque_const_max"),
                   ("tsin_min", "torque_sin_min"), ("tsin_max", "torque_sin_max"),
                   ("tfreq_min", "torque_min_freq"), ("tfreq_max", "torque_max_freq"),
                   ("tshift_min", "torque_min_shift"), ("tshift_max", "torque_max_shift")):
        setattr(c, k, float(td.get(key, 0.0)))
    wc = env.get("water_current", {}) or {}
    c.current_on = int(bool(wc.get("use_water_current", False)))
    flow = list(wc.get("flow_velocity", [0.0, 0.0, 0.0]) or [0.0, 0.0, 0.0])
    c.flow_vel[0], c.flow_vel[1] = float(flow[0]), float(flow[1])
    # the reference's fail-fast probe toggle (USV_Virtual.py:57-59): on unless USV_NAN_PROBE=0
    c.nan_probe = nan_probe_enabled()
    c.step_inc = 1 / int(env.get("horizon_length", 16))   # USVVirtual.step += 1 / horizon_length (:1633)
    # the first substep after a reset sees the cached pre-reset root state, as the reference's
    # apply_forces does (USV_Virtual.py:1103-1117).  Not a reference yaml key: this build's switch, on by default
    c.stale_root = int(bool(env.get("stale_root_after_reset", True)))
    return c


def nan_probe_enabled() -> int:
    """USV_NAN_PROBE (USV_Virtual.py:57-59, vec_env_rlgames.py:41-43): default on, "0" disables."""
    return int(os.getenv("USV_NAN_PROBE", "1") != "0")


NAN_STAGES = (("actions(clamped)", "USV_NAN_ACTIONS"), ("state", "USV_NAN_STATE"), ("reward.rew_buf", "USV_NAN_REWARD"),
              ("obs(post_physics_step)", "USV_NAN_OBS"), ("policy mu/value (get_action_values)", "USV_NAN_POLICY"),
              ("episode extra is NaN before masking", "USV_NAN_EXTRAS"))


def raise_nan_flag(bits: int, where: str) -> None:
    """The reference's RuntimeError of _raise_if_nonfinite (USV_Virtual.py:91-95) for a device flag word."""
    if not bits:
        return
    from .._abi import DEFINES
    names = [name for name, key in NAN_STAGES if bits & DEFINES[key]]
    raise RuntimeError(f"[USV_NAN_PROBE] non-finite detected: {', '.join(names)} ({where}; flag bits {bits:#x}; "
                       f"set USV_NAN_PROBE=0 to disable)")


TASK_KINDS = {"CaptureXY": 0, "GoToPose": 1, "TrackXYOVelocity": 2}   # USV_TASK_* (include/usv_hip.h)
_MODES = {"linear": 0, "square": 1, "exponential": 2}
# GoToPoseParameters / TrackXYOVelocityParameters and their reward dataclasses
# (USV_task_parameters.py:74-148, USV_task_rewards.py:160-393)
# GoToPoseParameters (USV_task_parameters.py:95-113), its own curriculum defaults (not GoToXYParameters' :70-76)
_POSE_DEFAULTS = dict(position_tolerance=0.01, heading_tolerance=0.025, kill_after_n_steps_in_tolerance=500,
                      goal_random_position=0.0, max_spawn_dist=3.0, min_spawn_dist=0.5, kill_dist=10.0,
                      spawn_curriculum=False, spawn_curriculum_min_dist=0.5, spawn_curriculum_max_dist=2.5,
                      spawn_curriculum_kill_dist=3.0, spawn_curriculum_mode="linear", spawn_curriculum_warmup=250,
                      spawn_curriculum_end=750)
_POSE_REWARD = dict(position_reward_mode="exponential", heading_reward_mode="exponential",
                    position_exponential_reward_coeff=0.25, heading_exponential_reward_coeff=0.25,
                    position_scale=1.0, heading_scale=5.0, sig_gain=3.0)
_TRACK_DEFAULTS = dict(lin_vel_tolerance=0.01, ang_vel_tolerance=0.025, kill_after_n_steps_in_tolerance=50,
                       goal_random_linear_velocity=0.75, goal_random_angular_velocity=1.0, kill_dist=500.0)
_TRACK_REWARD = dict(linear_reward_mode="exponential", angular_reward_mode="exponential",
                     linear_exponential_reward_coeff=0.25, angular_exponential_reward_coeff=0.25,
                     linear_scale=1.0, angular_scale=1.0)


def _mode(v: str) -> int:
    m = str(v).lower()
    if m not in _MODES:
        raise ValueError("Linear, Square and Exponential are the only currently supported mode.")
    return _MODES[m]


def _pose_task_cfg(c: UsvCfg, name: str, env: Dict[str, Any]) -> Dict[str, Any]:
    """GoToPose / TrackXYOVelocity constants; the task's own parameter defaults
    replace CaptureXY's (env.task_parameters / env.reward_parameters override)."""
    if name == "GoToPose":
        tp = dict(_POSE_DEFAULTS)
        tp.update(env["task_parameters"])
        rp = dict(_POSE_REWARD)
        rp.update(env.get("reward_parameters", {}) or {})
        if bool(tp.get("spawn_curriculum", False)):
            # GoToPoseParameters (USV_task_parameters.py:107-128): linear mode only, as the reference asserts
            if str(tp["spawn_curriculum_mode"]).lower() != "linear":
                raise AssertionError("Linear is the only currently supported mode.")
            c.curriculum_on = 1
            c.cur_min_dist = float(tp["spawn_curriculum_min_dist"])
            c.cur_max_dist = float(tp["spawn_curriculum_max_dist"])
            c.cur_kill_dist = float(tp["spawn_curriculum_kill_dist"])
            c.cur_warmup = float(int(tp["spawn_curriculum_warmup"]))
            c.cur_end = float(int(tp["spawn_curriculum_end"]))
            c.min_spawn_d, c.max_spawn_d = float(tp["min_spawn_dist"]), float(tp["max_spawn_dist"])
            c.kill_dist_d = float(tp["kill_dist"])
        c.tk_mode[0], c.tk_mode[1] = _mode(rp["position_reward_mode"]), _mode(rp["heading_reward_mode"])
        c.tk_coeff[0] = rp["position_exponential_reward_coeff"]
        c.tk_coeff[1] = rp["heading_exponential_reward_coeff"]
        c.tk_scale[0], c.tk_scale[1] = rp["position_scale"], rp["heading_scale"]
        c.sig_gain = rp["sig_gain"]
    else:
        tp = dict(_TRACK_DEFAULTS)
        tp.update(env["task_parameters"])
        rp = dict(_TRACK_REWARD)
        rp.update(env.get("reward_parameters", {}) or {})
        c.tk_mode[0], c.tk_mode[1] = _mode(rp["linear_reward_mode"]), _mode(rp["angular_reward_mode"])
        c.tk_coeff[0] = rp["linear_exponential_reward_coeff"]
        c.tk_coeff[1] = rp["angular_exponential_reward_coeff"]
        c.tk_scale[0], c.tk_scale[1] = rp["linear_scale"], rp["angular_scale"]
        c.tk_tol[0], c.tk_tol[1] = tp["lin_vel_tolerance"], tp["ang_vel_tolerance"]
        c.tk_goal_rand[0] = tp["goal_random_linear_velocity"]
        c.tk_goal_rand[1] = tp["goal_random_angular_velocity"]
        tp.setdefault("position_tolerance", 0.0)   # read by the common parser, unused by this task
    return tp


def build_hydro_cfg(task_cfg: Dict[str, Any]) -> UsvHydro:
    """dynamics.hydrostatics + sim.gravity as USVVirtual reads them (USV_Virtual.py:441-456, 724-736)."""
    hs = task_cfg["dynamics"]["hydrostatics"]
    h = UsvHydro()
    h.water_density = float(hs["water_density"])
    h.gravity = float(task_cfg.get("sim", {}).get("gravity", [0.0, 0.0, -9.81])[2])
    h.metacentric_width = float(hs["box_width"]) / 2
    h.metacentric_length = float(hs["box_length"]) / 2
    h.avg_force = float(hs["average_hydrostatics_force_value"])
    h.amplify_torque = float(hs["amplify_torque"])
    h.waterplane_area = float(hs["waterplane_area"])
    h.zero_height = float(hs["heron_zero_height"])
    h.max_volume = float(hs["box_width"]) * float(hs["box_length"]) * (float(hs["heron_zero_height"]) + 20)
    return h


def stat_names(c: UsvCfg):
    """(extras["episode"] key, episode-sum slot) pairs in the reference's dict order:
    task.create_stats, Penalties.get_stats_name, success/collision, state statistics
    (USV_Virtual.py:584-601).  CaptureXY keeps the fixed 28-key layout of _abi.STAT_NAMES."""
    from .._abi import STAT_KEYS_ENUM as S, STAT_NAMES
    if c.task_kind == 0:
        return list(zip(STAT_NAMES, range(len(STAT_NAMES))))
    task = (["position_reward", "position_error", "heading_reward", "heading_error"] if c.task_kind == 1 else
            ["linear_velocity_reward", "linear_velocity_error", "angular_velocity_reward", "angular_velocity_error"])
    slot = ({"position_reward": 0, "heading_reward": 1, "position_error": 2, "heading_error": 3} if c.task_kind == 1
            else {k: i for i, k in enumerate(task)})
    out = [(k, slot[k]) for k in task]
    if c.pen_ang_kind:
        out.append(("angular_vel_penalty", S["ST_ANGULAR_VEL_PENALTY"]))
    if c.pen_angv_kind:
        out.append(("angular_vel_variation_penalty", S["ST_ANGULAR_VEL_VARIATION_PENALTY"]))
    if c.pen_en_kind:
        out.append(("energy_penalty", S["ST_ENERGY_PENALTY"]))
    for k in ("success", "collision", "normed_linear_vel", "normed_angular_vel", "cmd_neg_rate", "u_mean",
              "u_low_rate", "u_sum"):
        out.append((k, S["ST_" + k.upper()]))
    return out


def has_disturbance(c: UsvCfg) -> bool:
    """Any per-substep disturbance term on (the kernels then need usv_bufs_t.dist)."""
    return bool(c.fdist_on or c.tdist_on or c.current_on)


def env_origins(num_envs: int, spacing: float = 50.0, per_row: int = 8) -> np.ndarray:
    """RLTask._env_pos when the stage has no env translate (USV_Virtual.py:1670-1696):
    x = (i % per_row) * spacing, y = (i // per_row) * spacing ([2][n] float32)."""
    i = np.arange(num_envs)
    return np.stack([(i % per_row) * spacing, (i // per_row) * spacing]).astype(np.float32)


def action_bias_cfg(task_cfg: Dict[str, Any]):
    ap = task_cfg["env"].get("action_processing", {}) or {}
    return float(ap.get("initial_action_bias", 0.0)), int(ap.get("initial_action_bias_steps", 0))


def thruster_tables(task_cfg: Dict[str, Any]):
    it = task_cfg["dynamics"]["thrusters"]["interpolation"]
    n = int(it["numberOfPointsForInterpolation"])
    if n != 1000:
        raise ValueError("numberOfPointsForInterpolation must be 1000")
    return (np.asarray(it["interpolationPointsFromRealDataLeft"], np.float32),
            np.asarray(it["interpolationPointsFromRealDataRight"], np.float32))


def load_yaml(path: str) -> Dict[str, Any]:
    import yaml
    with open(path, "r", encoding="utf-8") as f:
        return yaml.safe_load(f)
