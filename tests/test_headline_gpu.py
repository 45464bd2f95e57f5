"""Parity at the headline size (131,072 envs per GPU: BASELINE configs[4]'s 2^20 envs over 8 GPUs) for the
code paths that only run above the sizes of the other parity tests:

* the rollout kernels' persistent multi-tile loop (8 tiles per workgroup at 131,072 envs in the register-weight
  form, 16 in the LDS-staged one: next-tile obs prefetch, next-tile normal draws by wave 0), with injected draws and
  with the in-kernel Philox + Box-Muller sampler (models.py:372-386 Normal.sample), and ppo_value;
* GAE + prepare_dataset over 131,072 x 16 rows (k_gae's 512 block partials, the k_prepare_finalize fold);
* the potential field for ~1,300 resets in both launch shapes (3 rounds of the 512-workgroup sweep grid,
  grid-stride statistics / final kernels, the 64-workgroup batch-max fold) and with in-step obstacle
  placement over 8,192 resets (k_field_place's grid stride);
* the episode-meter fold over several reward workgroups.

Checkers: the numpy PPO oracle (oracle/ppo_oracle.py) and the C env oracle (oracle/usv_oracle.c, OpenMP
build), both pinned to the reference's fixtures by the CPU tests.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle as O
from oracle import ppo_oracle as PO
from omniisaacgymenvs_loop_amd.tasks.usv_config import load_yaml
from tests import errtab as ET
from tests.test_env_gpu import _oracle_for, _run_field, _task, _vs_oracle, device_samples, oracle_step
from tests.test_oracle_golden import TEST_YAML
from tests.test_ppo_gpu import _agent

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HEAD = 131072          # envs per GPU of BASELINE configs[4]
H = 16


def _rand_agent(n, rng, mini_epochs=1, minibatch=8192):
    """Agent with random weights incl. biases / log-sigma and non-trivial obs / value statistics."""
    ag = _agent(n, minibatch, mini_epochs)
    P = PO.unflatten(ag.model_params.cpu().numpy())
    for k in ("b1", "b2", "bv", "bmu"):
        P[k] = rng.normal(0, 0.1, P[k].shape).astype(np.float32)
    P["sigma"] = np.array([-0.3, 0.2], np.float32)
    ag.model_params.copy_(torch.tensor(PO.flatten(P), device=DEV))
    om, ov = rng.normal(0, 0.5, 33), rng.uniform(0.5, 3.0, 33)
    ag.obs_rms[:33] = torch.tensor(om, dtype=torch.float64)
    ag.obs_rms[33:66] = torch.tensor(ov, dtype=torch.float64)
    ag.val_rms[:2] = torch.tensor([0.3, 2.5], dtype=torch.float64)
    return ag, P, PO.RMS(om, ov, 1.0), PO.RMS(np.array([0.3]), np.array([2.5]), 1.0)


@pytest.mark.parametrize("inject", [True, False], ids=["eps_inject", "philox"])
def test_policy_step_headline_multi_tile(inject):
    """k_policy_step at 131,072 envs (512 workgroups x 8 tiles) vs the oracle forward: actions, mu, sigma,
    neglogp, denormalised value, raw obs rows and done flags of rollout slot t, the clamped env actions.
    philox: the in-kernel sampler (site 0x200, step from the device clock as in graph replay) vs its
    restatement PO.policy_normals."""
    from omniisaacgymenvs_loop_amd import _capi as c
    rng = np.random.default_rng(11)
    N, t, seed = HEAD, 5, 1234
    ag, P, orms, vrms = _rand_agent(N, rng)
    obs = rng.normal(0, 2, (N, 33)).astype(np.float32)
    dprev = (rng.random(N) < 0.1).astype(np.int64)
    step0 = 2 ** 33 + 11
    step_dev = torch.tensor([step0], device=DEV, dtype=torch.int64)
    z = rng.normal(0, 1, (N, 2)).astype(np.float32) if inject else PO.policy_normals(seed, step0 + t, N)
    eps = torch.tensor(z, device=DEV) if inject else None
    c.call("ppo_policy_step", c.byref(ag.cfg), c.ptr(ag.model_params), c.ptr(ag.obs_rms), c.ptr(ag.val_rms),
           c.ptr(torch.tensor(obs, device=DEV)), t, c.ptr(ag.exp_obs), c.ptr(ag.exp_act), c.ptr(ag.exp_nlp),
           c.ptr(ag.exp_val), c.ptr(ag.exp_mu), c.ptr(ag.exp_sigma), c.ptr(ag.exp_done),
           c.ptr(torch.tensor(dprev, device=DEV)), c.ptr(ag.actions), seed, 0, c.ptr(step_dev), c.ptr(eps),
           c.stream_ptr())
    torch.cuda.synchronize()
    _, _, mu, v = PO.forward(P, orms.norm(obs))
    v = vrms.denorm(v)[:, 0]
    logstd = mu * 0 + P["sigma"]
    sigma = np.exp(logstd).astype(np.float32)
    act = (mu + sigma * z).astype(np.float32)
    nlp = PO.neglogp(act, mu, sigma, logstd)
    sl = np.arange(N) * H + t
    g = lambda x: x.cpu().numpy()[sl]
    tn = f"headline_policy_{'inj' if inject else 'philox'}"
    np.testing.assert_array_equal(g(ag.exp_obs), obs)
    np.testing.assert_array_equal(g(ag.exp_done), dprev.astype(np.uint8))
    ET.check(tn, "mu", g(ag.exp_mu), mu, 1e-5, 1e-5, ["mu0", "mu1"])
    ET.check(tn, "sigma", g(ag.exp_sigma), sigma, 1e-5, 1e-5, ["s0", "s1"])
    ET.check(tn, "value", g(ag.exp_val), v, 1e-5, 1e-5)
    ET.check(tn, "action", g(ag.exp_act), act, 1e-5, 1e-5, ["a0", "a1"])
    ET.check(tn, "neglogp", g(ag.exp_nlp), nlp, 1e-5, 1e-5)
    ET.check(tn, "env_action", ag.actions.cpu().numpy(), np.clip(act, -1, 1), 1e-5, 1e-5, ["a0", "a1"])
    # the other slots of the experience rows are untouched
    other = np.arange(N) * H + (t + 1)
    assert float(np.abs(ag.exp_act.cpu().numpy()[other]).max()) == 0.0


@pytest.mark.parametrize("n,grid_cap,inject", [(HEAD, 0, False), (HEAD, 0, True), (4128, 7, False), (100, 0, True)])
def test_policy_step_register_weights_bit_identical(monkeypatch, n, grid_cap, inject):
    """The register-weight policy kernel (k_policy_step<true>: W1 / W2 as the waves' matrix-core operands in VGPRs,
    41 KB of LDS, two workgroups per CU) equals the LDS-staged one (USV_POLICY_RW=0) bit for bit: every experience
    array and the env actions, at the headline size (512 workgroups, 8 tiles each), over a capped grid (4,128 rows on 7
    workgroups: 19 tiles each, a ragged last tile) and for one partial tile."""
    from omniisaacgymenvs_loop_amd import _capi as c
    rng = np.random.default_rng(21)
    ag, _, _, _ = _rand_agent(n, rng, minibatch=8192 if n % 512 == 0 else 16 * n)
    obs = torch.tensor(rng.normal(0, 2, (n, 33)).astype(np.float32), device=DEV)
    dprev = torch.tensor((rng.random(n) < 0.1).astype(np.int64), device=DEV)
    eps = torch.tensor(rng.normal(0, 1, (n, 2)).astype(np.float32), device=DEV) if inject else None
    step_dev = torch.tensor([2 ** 33 + 5], device=DEV, dtype=torch.int64)
    monkeypatch.setenv("USV_POLICY_GRID", str(grid_cap))
    out = {}
    for rw in ("0", "1"):
        monkeypatch.setenv("USV_POLICY_RW", rw)
        for a in (ag.exp_obs, ag.exp_act, ag.exp_nlp, ag.exp_val, ag.exp_mu, ag.exp_sigma, ag.exp_done, ag.actions):
            a.fill_(7)
        for t in (0, 3):
            c.call("ppo_policy_step", c.byref(ag.cfg), c.ptr(ag.model_params), c.ptr(ag.obs_rms), c.ptr(ag.val_rms),
                   c.ptr(obs), t, c.ptr(ag.exp_obs), c.ptr(ag.exp_act), c.ptr(ag.exp_nlp), c.ptr(ag.exp_val),
                   c.ptr(ag.exp_mu), c.ptr(ag.exp_sigma), c.ptr(ag.exp_done), c.ptr(dprev), c.ptr(ag.actions), 99, 0,
                   c.ptr(step_dev), c.ptr(eps), c.stream_ptr())
        torch.cuda.synchronize()
        out[rw] = [x.cpu().numpy().copy() for x in (ag.exp_obs, ag.exp_act, ag.exp_nlp, ag.exp_val, ag.exp_mu,
                                                     ag.exp_sigma, ag.exp_done, ag.actions)]
    for k, (a, b) in enumerate(zip(out["0"], out["1"])):
        np.testing.assert_array_equal(a.view(np.uint8), b.view(np.uint8), err_msg=str(k))


@pytest.mark.parametrize("n", [HEAD, 4128, 100])
def test_value_register_weights_bit_identical(monkeypatch, n):
    """ppo_value's register-weight kernel (k_value<true>) equals the LDS-staged one (USV_POLICY_RW=0) bit for bit."""
    from omniisaacgymenvs_loop_amd import _capi as c
    rng = np.random.default_rng(22)
    ag, _, _, _ = _rand_agent(n, rng, minibatch=8192 if n % 512 == 0 else 16 * n)
    obs = torch.tensor(rng.normal(0, 2, (n, 33)).astype(np.float32), device=DEV)
    out = {}
    for rw in ("0", "1"):
        monkeypatch.setenv("USV_POLICY_RW", rw)
        v = torch.full((n,), 7.0, device=DEV)
        c.call("ppo_value", c.byref(ag.cfg), c.ptr(ag.model_params), c.ptr(ag.obs_rms), c.ptr(ag.val_rms), c.ptr(obs),
               c.ptr(v), c.stream_ptr())
        torch.cuda.synchronize()
        out[rw] = v.cpu().numpy()
    np.testing.assert_array_equal(out["0"].view(np.uint32), out["1"].view(np.uint32))


def test_value_headline_multi_tile():
    """k_value (ppo_value) at 131,072 envs vs the oracle's denormalised value."""
    from omniisaacgymenvs_loop_amd import _capi as c
    rng = np.random.default_rng(12)
    ag, P, orms, vrms = _rand_agent(HEAD, rng)
    obs = rng.normal(0, 2, (HEAD, 33)).astype(np.float32)
    out = torch.zeros(HEAD, device=DEV)
    c.call("ppo_value", c.byref(ag.cfg), c.ptr(ag.model_params), c.ptr(ag.obs_rms), c.ptr(ag.val_rms),
           c.ptr(torch.tensor(obs, device=DEV)), c.ptr(out), c.stream_ptr())
    torch.cuda.synchronize()
    _, _, _, v = PO.forward(P, orms.norm(obs))
    ET.check("headline_value", "value", out.cpu().numpy(), vrms.denorm(v)[:, 0], 1e-5, 1e-5)


def test_prepare_headline_multi_block():
    """ppo_prepare over 131,072 x 16 rows: GAE (a2c_common.py:525-540), returns, the value RMS trained on the
    values then the returns, normalised values / returns, normalised advantages (:1257-1290) -- the 512-block
    fp64 partials and their fold -- vs PO.prepare_dataset."""
    rng = np.random.default_rng(13)
    N = HEAD
    ag, P, orms, vrms = _rand_agent(N, rng)
    values = rng.normal(0.5, 1.0, (H, N)).astype(np.float32)
    rewards = rng.normal(0.0, 0.2, (H, N)).astype(np.float32)
    dones = (rng.random((H, N)) < 0.05).astype(np.uint8)
    last_obs = rng.normal(0, 2, (N, 33)).astype(np.float32)
    last_dones = (rng.random(N) < 0.05).astype(np.int64)
    flat = lambda a: torch.tensor(np.ascontiguousarray(np.swapaxes(a, 0, 1).reshape(N * H)), device=DEV)
    ag.exp_val.copy_(flat(values))
    ag.exp_rew.copy_(flat(rewards))
    ag.exp_done.copy_(flat(dones))
    ag.obs = {"obs": {"state": torch.tensor(last_obs, device=DEV)}}
    ag.dones = torch.tensor(last_dones, device=DEV)
    ag.prepare_dataset()
    torch.cuda.synchronize()
    assert ag.normalize_input
    _, _, _, lv = PO.forward(P, orms.norm(last_obs))
    lv = (vrms.denorm(lv) if ag.normalize_value else lv)[:, 0]
    vn, rn, an = PO.prepare_dataset(values, rewards, dones, lv, last_dones, PO.PPOConfig(), vrms,
                                    ag.normalize_value, ag.normalize_advantage)
    tn = "headline_prepare"
    ET.check(tn, "values", ag.exp_val.cpu().numpy(), vn, 1e-5, 1e-5)
    ET.check(tn, "returns", ag.exp_ret.cpu().numpy(), rn, 1e-5, 1e-5)
    ET.check(tn, "advantages", ag.exp_adv.cpu().numpy(), an, 1e-5, 1e-5)
    vr = ag.val_rms.cpu().numpy()
    np.testing.assert_allclose(vr[:2], [vrms.mean[0], vrms.var[0]], rtol=1e-7)   # fp64 one-pass vs two-pass
    assert vr[2] == vrms.count


def test_gae_vector_form_bit_identical(monkeypatch):
    """k_gae<16> (an env's 16 rows loaded and stored as 16-byte vectors) equals the runtime-horizon loop
    (USV_GAE_VEC=0) bit for bit at 131,072 x 16 rows: normalised values, returns, advantages and the value RMS."""
    rng = np.random.default_rng(14)
    N = HEAD
    ag, _, _, _ = _rand_agent(N, rng)
    val0 = torch.tensor(rng.normal(0.5, 1.0, N * H).astype(np.float32), device=DEV)
    ag.exp_rew.copy_(torch.tensor(rng.normal(0.0, 0.2, N * H).astype(np.float32), device=DEV))
    ag.exp_done.copy_(torch.tensor((rng.random(N * H) < 0.05).astype(np.uint8), device=DEV))
    ag.obs = {"obs": {"state": torch.tensor(rng.normal(0, 2, (N, 33)).astype(np.float32), device=DEV)}}
    ag.dones = torch.tensor((rng.random(N) < 0.05).astype(np.int64), device=DEV)
    rms0 = ag.val_rms.clone()
    out = {}
    for vec in ("1", "0"):
        monkeypatch.setenv("USV_GAE_VEC", vec)
        ag.exp_val.copy_(val0)
        ag.val_rms.copy_(rms0)
        ag.prepare_dataset()
        torch.cuda.synchronize()
        out[vec] = [x.cpu().numpy().copy() for x in (ag.exp_val, ag.exp_ret, ag.exp_adv, ag.val_rms)]
    for a, b in zip(out["1"], out["0"]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("pack", ["0", "1"])
def test_potential_field_1300_resets_vs_oracle(pack, monkeypatch):
    """~1,300 reset envs (the headline size's steady-state reset count) at 4,096 envs, whose launch geometry
    equals 131,072 envs' (512 sweep workgroups -> 3 rounds, 4,096 statistics / final workgroups -> grid
    stride, 64-workgroup batch-max fold): bit-exact against the oracle (d_multi_gemini.py:66-271)."""
    monkeypatch.setenv("USV_FIELD_PACK", pack)
    task = _task(load_yaml(TEST_YAML), 4096)
    rng = np.random.default_rng(21)
    K = 1300
    obst = (rng.uniform(0, 1, (K, 16, 2)) * 24 - 12).astype(np.float32)
    obst[0, :3] = [[0.3, 0.1], [1.2, -0.4], [-0.9, 0.8]]     # crowd the target
    obst[1, :] = 999.0                                         # empty map
    obst[2, 5:] = 999.0                                        # leftovers in limbo
    tgt = rng.uniform(-3, 3, (K, 2)).astype(np.float32)
    tgt[3] = obst[3, 0]                                        # occupied target cell
    ids = rng.choice(4096, K, replace=False).astype(np.int32)
    f = _run_field(task, ids, obst, tgt)
    ref = O.potential_field(task.cfg, obst, tgt)
    np.testing.assert_array_equal(f, ref)


def test_philox_placement_8192_resets_vs_oracle(monkeypatch):
    """The large-batch reset path at 8,192 envs, all reset on the first step: k_field_place's grid stride
    (1,024 workgroups x 4 waves < 8,192 reset envs), 16 rounds of the packed sweep grid and the batch fold,
    with in-kernel Philox draws vs the oracle: obstacles and every field bit-exact, then two more steps
    (obs / reward / dones as in test_env_gpu's Philox tests)."""
    monkeypatch.setenv("USV_FIELD_PACK", "1")
    task_cfg = load_yaml(TEST_YAML)
    n = 8192
    task = _task(task_cfg, n)
    E = _oracle_for(task.cfg, n, task_cfg)
    rng = np.random.default_rng(22)
    dp = np.zeros(n)
    for t in range(3):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        bias = task.current_action_bias()
        obs, rew, dones = task.env_step(torch.tensor(a, device=DEV))
        ids = oracle_step(task, E, a, bias, t)
        if t == 0:
            assert len(ids) == n
            np.testing.assert_array_equal(task.obst.cpu().numpy().reshape(16, 2, n), E.obst)
            np.testing.assert_array_equal(task.field_rowmajor().cpu().numpy(), E.field)
        dp = _vs_oracle("headline_philox_8192", task, E, obs, rew, dones, t, dp)


def test_meter_fold_multi_workgroup():
    """ppo_store_reward over 4 reward workgroups (1,024 envs): shaped rewards into the experience rows, the
    per-slot meter sums folded in workgroup order (a2c_common.py:721-759, tr_helpers.py:33-43), and the
    AverageMeter replay, vs a numpy restatement of the per-env episode bookkeeping."""
    from omniisaacgymenvs_loop_amd import _capi as c
    from omniisaacgymenvs_loop_amd.rl_games.a2c_continuous import AverageMeter
    N = 1024
    ag = _agent(N, 8192)
    rng = np.random.default_rng(14)
    rew = rng.uniform(0.2, 2.0, (H, N)).astype(np.float32)   # positive: the sums have no cancellation
    dn = (rng.random((H, N)) < 0.15).astype(np.int64)
    ag.meter_buf.zero_()
    cr, cs, cl = (np.zeros(N, np.float32) for _ in range(3))
    sums = np.zeros((H, 4))
    ends = []
    scale, shift = ag.cfg.reward_scale, ag.cfg.reward_shift
    for t in range(H):
        r_t, d_t = torch.tensor(rew[t], device=DEV), torch.tensor(dn[t], device=DEV)
        c.call("ppo_store_reward", c.byref(ag.cfg), c.ptr(r_t), c.ptr(d_t), t, c.ptr(ag.exp_rew), c.ptr(ag.cur_rew),
               c.ptr(ag.cur_shaped), c.ptr(ag.cur_len), c.ptr(ag.meter_buf), None, c.stream_ptr())
        torch.cuda.synchronize()
        shaped = ((rew[t] + np.float32(shift)) * np.float32(scale)).astype(np.float32)
        cr, cs, cl = cr + rew[t], cs + shaped, cl + np.float32(1)
        d = dn[t] != 0
        sums[t] = [cr[d].sum(dtype=np.float64), cs[d].sum(dtype=np.float64), cl[d].sum(dtype=np.float64), d.sum()]
        ends.append((cr[d].copy(), cl[d].copy()))
        cr, cs, cl = cr * ~d, cs * ~d, cl * ~d
    np.testing.assert_array_equal(ag.exp_rew.cpu().numpy().reshape(N, H), ((rew + np.float32(shift)) *
                                                                           np.float32(scale)).T)
    ET.check("headline_meters", "sums", ag.meter.cpu().numpy(), sums, 1e-5, 1e-5, ["rew", "shaped", "len", "cnt"])
    ag._replay_meters()
    ref = AverageMeter(ag.games_to_track)
    for t in range(H):
        cnt = int(sums[t, 3])
        if cnt:
            ref.update_stats(sums[t, 0] / cnt, cnt)
    assert ag.game_rewards.current_size == ref.current_size
    ET.check("headline_meters", "game_rewards", ag.game_rewards.get_mean(), ref.get_mean(), 1e-5, 1e-5)


def _detile(t):
    """[k][USV_FIELD_STRIDE] tiled raw cost (include/usv_hip.h: 10 x 10 tiles, row-major inside and over the
    15 x 15 tiles) -> [k][150 * 150] row-major."""
    k = t.shape[0]
    return t[:, :22500].reshape(k, 15, 15, 10, 10).transpose(0, 1, 3, 2, 4).reshape(k, 22500)


def test_full_size_131072_step_vs_oracle():
    """BASELINE configs[4]'s per-GPU size through the constant-shift step kernel (FixedWin<19>: every slab row
    at base + (row << 19)) and the reset path of 131,072 envs in one batch, against the C oracle on the same
    Philox draws: every env reset on the first step -- DR parameters, spawns and obstacles bit-exact for all
    131,072 envs, the raw cost-to-go of 64 sampled envs bit-exact against the oracle's wavefront, the batch's
    inf_val equal to 1.5 x the largest finite cost over all 131,072 fields -- then three steps with the state
    bit-exact, obs at 1e-5, dones exact, the potential samples against the oracle's field at the device's positions and
    the reward at 1e-5 against the oracle fed those samples (test_env_gpu._vs_oracle).
    The oracle's reset skips its own 131,072 fields (oracle_set_skip_field: hours of CPU) and steps on the
    device's fields, whose texels are checked above and at 8,192 resets in
    test_philox_placement_8192_resets_vs_oracle; later resets (few envs) build their fields in the oracle."""
    task_cfg = load_yaml(TEST_YAML)
    n = HEAD
    task = _task(task_cfg, n)
    E = _oracle_for(task.cfg, n, task_cfg)
    rng = np.random.default_rng(31)
    dp = np.zeros(n)
    for t in range(4):
        a = rng.uniform(-1, 1, (n, 2)).astype(np.float32)
        bias = task.current_action_bias()
        obs, rew, dones = task.env_step(torch.tensor(a, device=DEV))
        if t == 0:
            ids = E.compact()
            assert len(ids) == n
            O.lib().oracle_set_skip_field(1)
            try:
                E.reset(ids, O.reset_uniforms(task.seed, 0, ids))
            finally:
                O.lib().oracle_set_skip_field(0)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(task.obst.cpu().numpy().reshape(16, 2, n), E.obst)
            for j, k in enumerate(("mass", "com_x", "com_y", "com_z", "k_drag", "thr_l", "thr_r", "k_iz", "mass_r")):
                np.testing.assert_array_equal(task.params[j].cpu().numpy(), getattr(E, k), err_msg=k)
            # fields: raw cost of a sample vs the oracle's wavefront, the batch constant, then the device's
            # materialised fields become the oracle's
            smp = np.sort(rng.choice(n, 64, replace=False))
            obst_s = task.obst[:, smp].cpu().numpy().reshape(16, 2, 64).transpose(2, 0, 1).copy()
            tgt_s = task.field_old_tgt[:, smp].cpu().numpy().T.copy()
            _, cost_ref = O.potential_field(task.cfg, obst_s, tgt_s, want_cost=True)
            np.testing.assert_array_equal(_detile(task.field[smp].cpu().numpy()), cost_ref)
            raw = task.field[:, :22500]
            fin_max = torch.where(torch.isfinite(raw), raw, torch.full_like(raw, -1.0)).max()
            inf_val = (fin_max * 1.5).item()
            assert torch.all(task.fnorm[:, 4] == inf_val), "batch inf_val != 1.5 x max finite cost"
            for c0 in range(0, n, 16384):
                idx = torch.arange(c0, min(c0 + 16384, n), device=DEV)
                E.field[c0:c0 + len(idx)] = task.field_rowmajor(idx).cpu().numpy()
            E.set_device_samples(*device_samples(task))
            E.step(a, bias, O.step_uniforms(task.seed, 0, n))
        else:
            oracle_step(task, E, a, bias, t)
        dp = _vs_oracle("full_size_131072", task, E, obs, rew, dones, t, dp)
        st = task.state.cpu().numpy()
        for j, k in enumerate(("px", "py", "yaw", "vx", "vy", "wz", "fl", "fr")):
            ET.check("full_size_131072", f"state_{k}", st[j][:, None], getattr(E, k)[:, None], 0.0, 0.0,
                     [k], f"{k} t={t}")
