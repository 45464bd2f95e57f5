"""HIP PPO kernels (via A2CAgent + the C ABI) vs the reference rl_games fixture
(tests/golden/ppo_epoch.npz) and the numpy oracle (oracle/ppo_oracle.py)."""
import copy
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import ppo_oracle as PO
from tests import errtab as ET
from tests.test_ppo_oracle import _params

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeVecEnv:
    def __init__(self, n):
        from omniisaacgymenvs_loop_amd.utils.spaces import Box, DictSpace
        self.n = n
        self.info = {"action_space": Box(np.array([-1, -1], np.float32), np.array([1, 1], np.float32)),
                     "observation_space": DictSpace({"state": Box(-np.inf, np.inf, (33,))})}

    def get_env_info(self):
        return self.info

    def set_train_info(self, *a, **k):
        pass

    def get_env_state(self):
        return None

    def set_env_state(self, s):
        pass


def _agent(n, minibatch, mini_epochs=8):
    import yaml
    from omniisaacgymenvs_loop_amd.rl_games.a2c_continuous import A2CAgent
    with open(os.path.join(ROOT, "omniisaacgymenvs_loop_amd/cfg/train/USV/USV_PPOcontinuous_MLP.yaml")) as f:
        params = yaml.safe_load(f)["params"]
    params["config"].update(num_actors=n, minibatch_size=minibatch, mini_epochs=mini_epochs, device=DEV,
                            vec_env=FakeVecEnv(n), train_dir="/tmp/ppo_gpu_runs")
    return A2CAgent("run", params)


def _flat_params(P):
    return torch.tensor(PO.flatten(P), device=DEV)


def _swap(a):  # [H, N, ...] -> [N*H, ...] (swap_and_flatten01)
    return np.ascontiguousarray(np.swapaxes(a, 0, 1).reshape(a.shape[0] * a.shape[1], *a.shape[2:]))


@pytest.fixture(scope="module")
def ppo(golden):
    return golden("ppo_epoch.npz")


def test_policy_kernel_vs_reference_rollout(ppo):
    from omniisaacgymenvs_loop_amd import _capi as c
    H, N = ppo["exp_rewards"].shape[:2]
    ag = _agent(N, 128)
    ag.model_params.copy_(_flat_params(_params(ppo, "init")))
    for t in range(H):
        obs = torch.tensor(ppo["env_obs"][t], device=DEV)
        eps = (ppo["exp_actions"][t] - ppo["exp_mus"][t]) / ppo["exp_sigmas"][t]
        dones_prev = torch.tensor(ppo["exp_dones"][t].astype(np.int64), device=DEV)
        c.call("ppo_policy_step", c.byref(ag.cfg), c.ptr(ag.model_params), c.ptr(ag.obs_rms), c.ptr(ag.val_rms),
               c.ptr(obs), t, c.ptr(ag.exp_obs), c.ptr(ag.exp_act), c.ptr(ag.exp_nlp), c.ptr(ag.exp_val),
               c.ptr(ag.exp_mu), c.ptr(ag.exp_sigma), c.ptr(ag.exp_done), c.ptr(dones_prev), c.ptr(ag.actions),
               1, t, None, c.ptr(torch.tensor(eps, device=DEV)), c.stream_ptr())
        torch.cuda.synchronize()
        np.testing.assert_allclose(ag.actions.cpu().numpy(), np.clip(ppo["exp_actions"][t], -1, 1), atol=2e-6)
    rows = lambda x: x.cpu().numpy()
    np.testing.assert_array_equal(rows(ag.exp_obs), _swap(ppo["exp_obses"]))
    tn = "ppo_rollout"
    ET.check(tn, "mu", rows(ag.exp_mu), _swap(ppo["exp_mus"]), 1e-5, 1e-5, ["mu0", "mu1"])
    ET.check(tn, "sigma", rows(ag.exp_sigma), _swap(ppo["exp_sigmas"]), 1e-5, 1e-5, ["s0", "s1"])
    ET.check(tn, "value", rows(ag.exp_val), _swap(ppo["exp_values"])[:, 0], 1e-5, 1e-5)
    ET.check(tn, "neglogp", rows(ag.exp_nlp), _swap(ppo["exp_neglogpacs"]), 1e-5, 1e-5)
    np.testing.assert_array_equal(rows(ag.exp_done), _swap(ppo["exp_dones"]))


def _load_rollout(ag, ppo):
    H, N = ppo["exp_rewards"].shape[:2]
    T = lambda a, **k: torch.tensor(np.ascontiguousarray(a), device=DEV, **k)
    ag.exp_val.copy_(T(_swap(ppo["exp_values"])[:, 0]))
    ag.exp_rew.copy_(T(_swap(ppo["exp_rewards"])[:, 0]))
    ag.exp_done.copy_(T(_swap(ppo["exp_dones"])))
    ag.obs = {"obs": {"state": T(ppo["env_obs"][H])}}
    ag.dones = T(ppo["env_dones"][H - 1].astype(np.int64))


def test_prepare_kernel_vs_reference(ppo):
    H, N = ppo["exp_rewards"].shape[:2]
    ag = _agent(N, 128)
    ag.model_params.copy_(_flat_params(_params(ppo, "init")))
    _load_rollout(ag, ppo)
    ag.prepare_dataset()
    torch.cuda.synchronize()
    tn = "ppo_prepare"
    ET.check(tn, "values", ag.exp_val.cpu().numpy(), ppo["ds_old_values"][:, 0], 1e-5, 1e-5)
    ET.check(tn, "returns", ag.exp_ret.cpu().numpy(), ppo["ds_returns"][:, 0], 1e-5, 1e-5)
    ET.check(tn, "advantages", ag.exp_adv.cpu().numpy(), ppo["ds_advantages"], 1e-5, 1e-5)
    vr = ag.val_rms.cpu().numpy()
    np.testing.assert_allclose(vr[0], ppo["final_value_mean_std__running_mean"][0], rtol=1e-6)
    np.testing.assert_allclose(vr[1], ppo["final_value_mean_std__running_var"][0], rtol=1e-6)
    assert vr[2] == float(ppo["final_value_mean_std__count"])


def _load_dataset(ag, ppo):
    ag.model_params.copy_(_flat_params(_params(ppo, "init")))
    T = lambda a: torch.tensor(np.ascontiguousarray(a), device=DEV)
    ag.exp_obs.copy_(T(ppo["ds_obs_state"]))
    ag.exp_act.copy_(T(ppo["ds_actions"]))
    ag.exp_nlp.copy_(T(ppo["ds_old_logp_actions"]))
    ag.exp_val.copy_(T(ppo["ds_old_values"][:, 0]))
    ag.exp_ret.copy_(T(ppo["ds_returns"][:, 0]))
    ag.exp_adv.copy_(T(ppo["ds_advantages"]))
    ag.exp_mu.copy_(T(ppo["batch_mus"]))
    ag.exp_sigma.copy_(T(ppo["batch_sigmas"]))


def _run_update(ppo, monkeypatch, fused, minibatch, mini_epochs, grad_norm=None, bf16=False):
    monkeypatch.setenv("USV_PPO_FUSED", "1" if fused else "0")
    H, N = ppo["exp_rewards"].shape[:2]
    ag = _agent(N, minibatch, mini_epochs)
    ag.cfg.bf16_gemm = int(bf16)
    if grad_norm is not None:
        ag.cfg.truncate_grads, ag.cfg.grad_norm = 1, grad_norm
    _load_dataset(ag, ppo)
    ag.update_epoch_minibatches()
    torch.cuda.synchronize()
    return {k: getattr(ag, k).cpu().numpy().copy()
            for k in ("model_params", "adam_m", "adam_v", "opt", "kls", "loss_log", "obs_rms")}


@pytest.mark.parametrize("mb_div,mini_epochs,bf16,fold", [(4, 8, False, "0"), (1, 3, False, "0"), (4, 8, True, "0"),
                                                         (4, 8, False, "1")])
def test_fused_chain_matches_split_path(ppo, monkeypatch, mb_div, mini_epochs, bf16, fold):
    """ppo_minibatch_fused / ppo_minibatch_finish (Adam step speculated inside the reduction, checked by
    the next launch) vs ppo_minibatch_grad + ppo_minibatch_apply: bit-identical parameters, moments,
    optimiser scalars, KLs and losses -- without clipping, with clipping at every step (the redo path),
    with clipping at some steps, for an odd chain (state copied back from bank 1), in the bf16 GEMM mode and
    with the XCD-group fold of the partial rows (USV_PPO_FOLD=1, off by default)."""
    monkeypatch.setenv("USV_PPO_FOLD", fold)
    H, N = ppo["exp_rewards"].shape[:2]
    mb = N * H // mb_div
    ref = _run_update(ppo, monkeypatch, False, mb, mini_epochs, bf16=bf16)
    last_norm = float(ref["opt"][3])   # the last minibatch's gradient norm: some steps above, some below
    assert last_norm > 0
    for gn in (None, 1e-4, last_norm):
        a = ref if gn is None else _run_update(ppo, monkeypatch, False, mb, mini_epochs, gn, bf16)
        b = _run_update(ppo, monkeypatch, True, mb, mini_epochs, gn, bf16)
        for k in a:
            np.testing.assert_array_equal(a[k], b[k], err_msg=f"{k} grad_norm={gn}")
        if gn == 1e-4:
            assert not np.array_equal(a["model_params"], ref["model_params"])   # clipping happened


def test_minibatch_epoch_vs_reference(ppo):
    """32 optimizer steps: per-minibatch KL / losses, adaptive LR, obs RMS and final weights."""
    H, N = ppo["exp_rewards"].shape[:2]
    ag = _agent(N, int(ppo["hyper"][2]))
    _load_dataset(ag, ppo)
    ag.update_epoch_minibatches()
    torch.cuda.synchronize()
    tn = "ppo_epoch"
    ET.check(tn, "kl", ag.kls.cpu().numpy(), ppo["kl"], 1e-5, 1e-5)
    ET.check(tn, "losses", ag.loss_log[:, :4].cpu().numpy(), ppo["losses"], 1e-5, 1e-5, ["a", "c", "ent", "b"])
    np.testing.assert_allclose(float(ag.opt[0]), ppo["lr_seq"][-1], rtol=1e-6)
    orms = ag.obs_rms.cpu().numpy()
    np.testing.assert_allclose(orms[:33], ppo["final_running_mean_std__running_mean_std__state__running_mean"],
                               rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(orms[33:66], ppo["final_running_mean_std__running_mean_std__state__running_var"],
                               rtol=1e-6)
    Pf = PO.unflatten(ag.model_params.cpu().numpy())
    for k, v in _params(ppo, "final").items():
        ET.check(tn, "weights", Pf[k], v, 1e-5, 1e-5, None, k)
        ET.record(tn, f"w:{k}", Pf[k], v)


@pytest.mark.parametrize("entropy_coef,bf16,rows", [(0.0, False, 8192), (0.01, False, 8192), (0.0, True, 8192),
                                                    (0.0, False, 65536)])
def test_minibatch_gradient_vs_oracle_full_size(entropy_coef, bf16, rows):
    """One 8192-row minibatch (BASELINE minibatch_size) vs the numpy oracle's gradient (with and without
    the entropy bonus of a2c_continuous.py:159); bf16: the bf16 GEMM mode (mixed_precision, BASELINE
    configs[2]) vs the oracle with the same bf16 operand rounding (1e-5 of the largest component) and,
    recorded, vs fp32.  65,536 rows: a minibatch of horizon_length x num_envs (the reference yaml's suggestion),
    2,048 gradient workgroups whose chunk-major partial rows need more than the row-major footprint."""
    N, H = rows // 16, 16
    ag = _agent(N, rows, mini_epochs=1)
    ag.cfg.entropy_coef = entropy_coef
    ag.cfg.bf16_gemm = int(bf16)
    rng = np.random.default_rng(0)
    B = N * H
    obs = rng.normal(0, 2, (B, 33)).astype(np.float32)
    act = rng.normal(0, 1, (B, 2)).astype(np.float32)
    P = PO.unflatten(ag.model_params.cpu().numpy())
    xn = PO.RMS.zeros(33)
    xn.update(obs)
    _, _, mu0, _ = PO.forward(P, xn.norm(obs))
    sig0 = np.ones_like(mu0)
    nlp0 = PO.neglogp(act, mu0, sig0, np.zeros_like(mu0)) + rng.normal(0, 0.05, B).astype(np.float32)
    val = rng.normal(0, 1, B).astype(np.float32)
    ret = (val + rng.normal(0, 0.5, B)).astype(np.float32)
    adv = rng.normal(0, 1, B).astype(np.float32)
    T = lambda a: torch.tensor(np.ascontiguousarray(a), device=DEV)
    for name, arr in (("exp_obs", obs), ("exp_act", act), ("exp_nlp", nlp0), ("exp_val", val), ("exp_ret", ret),
                      ("exp_adv", adv), ("exp_mu", mu0 + 0.01), ("exp_sigma", sig0)):
        getattr(ag, name).copy_(T(arr))
    from omniisaacgymenvs_loop_amd import _capi as c
    c.call("ppo_minibatch_grad", c.byref(ag.cfg), c.ptr(ag.model_params), c.ptr(ag.obs_rms), c.ptr(ag.val_rms), 1,
           0, c.ptr(ag.exp_obs), c.ptr(ag.exp_act), c.ptr(ag.exp_nlp), c.ptr(ag.exp_val), c.ptr(ag.exp_ret),
           c.ptr(ag.exp_adv), c.ptr(ag.exp_mu), c.ptr(ag.exp_sigma), c.ptr(ag.grad), c.ptr(ag.losses),
           c.ptr(ag.partials), c.ptr(ag.work), c.stream_ptr())
    torch.cuda.synchronize()
    orms = PO.RMS.zeros(33)
    orms.update(obs)
    np.testing.assert_allclose(ag.obs_rms.cpu().numpy()[:33], orms.mean, rtol=1e-6, atol=1e-9)
    g_ref, losses, kl, _, _ = PO.minibatch_grad(P, orms.norm(obs), act, nlp0, val, ret, adv, mu0 + 0.01, sig0,
                                                PO.PPOConfig(minibatch=rows, entropy_coef=entropy_coef), lowp=bf16)
    g = ag.grad.cpu().numpy()[:PO.NPARAM]
    scale = np.abs(g_ref).max()
    tn = f"ppo_grad_full_ent{entropy_coef}" + ("_bf16" if bf16 else "") + ("" if rows == 8192 else f"_{rows}")
    if bf16:   # the bf16 mode's distance from the fp32 gradient (documented, not asserted)
        g32, _, _, _, _ = PO.minibatch_grad(P, orms.norm(obs), act, nlp0, val, ret, adv, mu0 + 0.01, sig0,
                                            PO.PPOConfig(minibatch=rows, entropy_coef=entropy_coef))
        ET.record(tn, "grad/max vs fp32", g / scale, g32 / scale)
    # 8192-row sums in different orders: each component within 1e-5 of the largest one.  bf16 mode: 5e-5 --
    # an operand whose fp32 value differs from the oracle's in the last bit can round to the neighbouring
    # bf16 value (a 2^-8 step) when it sits at a rounding midpoint; ~0.5% of the components see one
    ET.check(tn, "grad/max", g / scale, g_ref / scale, 0, 5e-5 if bf16 else 1e-5)
    ET.check(tn, "losses", ag.losses.cpu().numpy()[:4], losses, 1e-5, 1e-5, ["a", "c", "ent", "b"])
    ET.check(tn, "kl", float(ag.grad[PO.NPARAM]), kl, 1e-5, 1e-5)


def test_bf16_mode_leaves_rollout_kernels_fp32():
    """mixed_precision maps to bf16 GEMM operands in the training step only: the reference's autocast covers
    calc_gradients (a2c_continuous.py:121) while get_action_values / get_values run in fp32 under no_grad
    (a2c_common.py:385-430).  ppo_value and ppo_policy_step with bf16_gemm = 1 are bit-identical to bf16_gemm = 0
    and equal the fp32 oracle forward at 1e-5."""
    from omniisaacgymenvs_loop_amd import _capi as c
    N = 4096
    rng = np.random.default_rng(2)
    obs = torch.tensor(rng.normal(0, 1.5, (N, 33)).astype(np.float32), device=DEV)
    eps = torch.tensor(rng.normal(0, 1, (N, 2)).astype(np.float32), device=DEV)
    outs = []
    for bf in (0, 1):
        ag = _agent(N, 8192, mini_epochs=1)
        ag.cfg.bf16_gemm = bf
        v = torch.zeros(N, device=DEV)
        c.call("ppo_value", c.byref(ag.cfg), c.ptr(ag.model_params), c.ptr(ag.obs_rms), c.ptr(ag.val_rms), c.ptr(obs),
               c.ptr(v), c.stream_ptr())
        c.call("ppo_policy_step", c.byref(ag.cfg), c.ptr(ag.model_params), c.ptr(ag.obs_rms), c.ptr(ag.val_rms),
               c.ptr(obs), 0, c.ptr(ag.exp_obs), c.ptr(ag.exp_act), c.ptr(ag.exp_nlp), c.ptr(ag.exp_val),
               c.ptr(ag.exp_mu), c.ptr(ag.exp_sigma), c.ptr(ag.exp_done), c.ptr(ag.dones), c.ptr(ag.actions),
               1, 0, None, c.ptr(eps), c.stream_ptr())
        torch.cuda.synchronize()
        outs.append([v.cpu().numpy(), ag.exp_mu.cpu().numpy(), ag.exp_nlp.cpu().numpy(), ag.actions.cpu().numpy()])
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)
    P = PO.unflatten(ag.model_params.cpu().numpy())
    _, _, mu, v32 = PO.forward(P, PO.RMS.zeros(33).norm(obs.cpu().numpy()))
    if ag.normalize_value:   # the kernels return denormalised values (val_rms = (0, 1, count 1))
        v32 = PO.RMS.zeros(1).denorm(v32)
    ET.check("ppo_value_bf16mode", "value", outs[1][0], v32[:, 0], 1e-5, 1e-5)
    ET.check("ppo_value_bf16mode", "mu", outs[1][1][::16], mu, 1e-5, 1e-5, ["mu0", "mu1"])


def test_checkpoint_roundtrip(tmp_path):
    from omniisaacgymenvs_loop_amd.rl_games import checkpoint as ck
    ag = _agent(64, 128)
    ag.model_params.add_(0.25)
    ag.obs_rms[:33] = 3.0
    ag.epoch_num, ag.frame = 7, 1024
    ag.save(str(tmp_path / "ck"))
    sd = torch.load(str(tmp_path / "ck.pth"), weights_only=True)
    assert list(sd.keys()) == ["model", "epoch", "optimizer", "frame", "last_mean_rewards", "env_state"]
    assert list(sd["model"].keys())[:6] == ["value_mean_std.running_mean", "value_mean_std.running_var",
                                            "value_mean_std.count",
                                            "running_mean_std.running_mean_std.state.running_mean",
                                            "running_mean_std.running_mean_std.state.running_var",
                                            "running_mean_std.running_mean_std.state.count"]
    assert sd["model"]["a2c_network.actor_mlp.2.weight"].shape == (128, 128)
    ag2 = _agent(64, 128)
    ag2.restore(str(tmp_path / "ck.pth"))
    assert torch.equal(ag2.model_params, ag.model_params)
    assert torch.equal(ag2.obs_rms, ag.obs_rms)
    assert ag2.epoch_num == 7 and ag2.frame == 1024



def test_reward_shaper_and_meters_vs_reference(ppo):
    """DefaultRewardsShaper x0.01 (tr_helpers.py:33-43) into the experience buffer and the
    episode meters (a2c_common.py:738-759, AverageMeter torch_ext.py:281-307) replayed from the reference
    epoch's env rewards / dones: game_rewards mean and size as the reference left them."""
    from omniisaacgymenvs_loop_amd import _capi as c
    H, N = ppo["exp_rewards"].shape[:2]
    ag = _agent(N, 128)
    T = lambda a: torch.tensor(np.ascontiguousarray(a), device=DEV)
    ag.meter.zero_()
    for t in range(H):
        rew, dones = T(ppo["env_rew"][t]), T(ppo["env_dones"][t])     # alive until the launch has run
        c.call("ppo_store_reward", c.byref(ag.cfg), c.ptr(rew), c.ptr(dones), t, c.ptr(ag.exp_rew), c.ptr(ag.cur_rew),
               c.ptr(ag.cur_shaped), c.ptr(ag.cur_len), c.ptr(ag.meter_buf), None, c.stream_ptr())
        torch.cuda.synchronize()
    torch.cuda.synchronize()
    ET.check("ppo_meters", "exp_rew", ag.exp_rew.cpu().numpy(), _swap(ppo["exp_rewards"])[:, 0], 1e-5, 1e-5)
    ag._replay_meters()
    assert ag.game_rewards.current_size == int(ppo["game_rewards_size"])
    ET.check("ppo_meters", "game_rewards", np.float32(ag.game_rewards.get_mean()), ppo["game_rewards_mean"][0],
             1e-5, 1e-5)


class _Env13(FakeVecEnv):
    """The 13-dim observation space of the Aug-11 task the 811 checkpoint was trained on."""

    def __init__(self, n):
        super().__init__(n)
        from omniisaacgymenvs_loop_amd.utils.spaces import Box, DictSpace
        self.info["observation_space"] = DictSpace({"state": Box(-np.inf, np.inf, (13,))})


def test_reference_checkpoint_player_forward(golden, tmp_path):
    """The reference's 811 checkpoint (13-input net, zero-padded to the kernels' 33 inputs) restored by
    PpoPlayerContinuous (players.py:107-182) through torch.load(weights_only=True): the HIP forward equals the
    reference ModelA2CContinuousLogStd's mus / sigmas / denormalised values / neglogp on the same inputs, and the
    deterministic action is clamp(mu) (players.py:139-150)."""
    import yaml
    from omniisaacgymenvs_loop_amd import _capi as c
    from omniisaacgymenvs_loop_amd.rl_games.players import PpoPlayerContinuous
    from tests.test_checkpoint_cpu import ckpt811_dict
    d = golden("ckpt811.npz")
    n = d["obs"].shape[0]
    torch.save(ckpt811_dict(d), str(tmp_path / "811.pth"))
    with open(os.path.join(ROOT, "omniisaacgymenvs_loop_amd/cfg/train/USV/USV_PPOcontinuous_MLP.yaml")) as f:
        params = yaml.safe_load(f)["params"]
    params["config"].update(num_actors=n, device=DEV, vec_env=_Env13(n))
    pl = PpoPlayerContinuous(params)
    assert pl.obs_dim == 13
    pl.restore(str(tmp_path / "811.pth"))
    obs = torch.tensor(d["obs"], device=DEV)
    act = pl.get_action(obs, is_deterministic=True)
    torch.cuda.synchronize()
    tn = "ckpt811_player"
    mus = pl._scratch["mu"].cpu().numpy()
    ET.check(tn, "mu", mus, d["mus"], 1e-5, 1e-5, ["mu0", "mu1"])
    ET.check(tn, "sigma", pl._scratch["sigma"].cpu().numpy(), d["sigmas"], 1e-5, 1e-5, ["s0", "s1"])
    ET.check(tn, "value", pl._scratch["val"].cpu().numpy(), d["values"][:, 0], 1e-5, 1e-5)
    np.testing.assert_array_equal(act.cpu().numpy(), np.clip(mus, -1, 1))
    # the reference's sampled actions replayed through the same kernel: its neglogp
    eps = torch.tensor((d["actions"] - d["mus"]) / d["sigmas"], device=DEV)
    obs_pad = torch.zeros((n, 33), device=DEV)
    obs_pad[:, :13] = obs
    sc = pl._scratch
    c.call("ppo_policy_step", c.byref(pl.cfg), c.ptr(pl.model_params), c.ptr(pl.obs_rms), c.ptr(pl.val_rms),
           c.ptr(obs_pad), 0, c.ptr(sc["obs"]), c.ptr(sc["act"]), c.ptr(sc["nlp"]), c.ptr(sc["val"]), c.ptr(sc["mu"]),
           c.ptr(sc["sigma"]), c.ptr(pl._done8), c.ptr(pl._dones), c.ptr(pl._actions), 0, 0, None, c.ptr(eps),
           c.stream_ptr())
    torch.cuda.synchronize()
    ET.check(tn, "action", sc["act"].cpu().numpy(), d["actions"], 1e-5, 1e-5, ["a0", "a1"])
    ET.check(tn, "neglogp", sc["nlp"].cpu().numpy(), d["neglogpacs"], 1e-5, 1e-5)


def test_player_runs_the_usv_task(tmp_path):
    """test=True path: a trained-then-saved checkpoint restored into PpoPlayerContinuous plays the USV task
    (common/player.py:319-423) through VecEnvRLGames; finished games are counted and rewards are finite."""
    from omniisaacgymenvs_loop_amd.rl_games.players import PpoPlayerContinuous
    from tests.test_train_gpu import _agent_env
    env, task, ag = _agent_env(256, 2048, True, seed=3)
    ag.obs = ag.env_reset()
    for _ in range(2):
        ag.train_epoch()
    ag.save(str(tmp_path / "ck"))
    params = copy.deepcopy({k: v for k, v in ag.params.items() if k != "config"})
    params["config"] = {k: v for k, v in ag.config.items() if k != "vec_env"}
    params["config"]["vec_env"] = env
    params["player"] = {"deterministic": True, "games_num": 64, "max_steps": 400}
    pl = PpoPlayerContinuous(params)
    pl.restore(str(tmp_path / "ck.pth"))
    torch.testing.assert_close(pl.model_params, ag.model_params, rtol=0, atol=0)
    mean_reward = pl.run()
    assert np.isfinite(mean_reward)


@pytest.mark.parametrize("minibatch", [8192, 1024, 256])
def test_group_fold_matches_raw_row_path_and_oracle(minibatch, monkeypatch):
    """The XCD-group fold of the partial rows (ppo.hip FOLD_G; 8 groups of nblk / 8 = 32, 4 or 1 workgroups):
    folded in the gradient kernel (USV_PPO_FOLD=1; off by default, see ppo.hip fold_env), or every member arriving without folding so
    the reduction sums the raw rows in the fold's order (USV_PPO_FOLD=2): bit-identical gradients, losses and
    KL, twice in a row (the monotonic arrival counters carry the launch generation); without the fold
    (USV_PPO_FOLD=0, the reduction's 16-group order) the same gradient within 1e-6 of its largest component,
    and the oracle's within 1e-5."""
    from omniisaacgymenvs_loop_amd import _capi as c
    N, H = minibatch // 16, 16
    ag = _agent(N, minibatch, mini_epochs=1)
    rng = np.random.default_rng(5)
    B = N * H
    obs = rng.normal(0, 2, (B, 33)).astype(np.float32)
    act = rng.normal(0, 1, (B, 2)).astype(np.float32)
    P = PO.unflatten(ag.model_params.cpu().numpy())
    xn = PO.RMS.zeros(33)
    xn.update(obs)
    _, _, mu0, _ = PO.forward(P, xn.norm(obs))
    sig0 = np.ones_like(mu0)
    nlp0 = PO.neglogp(act, mu0, sig0, np.zeros_like(mu0)) + rng.normal(0, 0.05, B).astype(np.float32)
    val = rng.normal(0, 1, B).astype(np.float32)
    ret = (val + rng.normal(0, 0.5, B)).astype(np.float32)
    adv = rng.normal(0, 1, B).astype(np.float32)
    T = lambda a: torch.tensor(np.ascontiguousarray(a), device=DEV)
    for name, arr in (("exp_obs", obs), ("exp_act", act), ("exp_nlp", nlp0), ("exp_val", val), ("exp_ret", ret),
                      ("exp_adv", adv), ("exp_mu", mu0 + 0.01), ("exp_sigma", sig0)):
        getattr(ag, name).copy_(T(arr))
    orms = ag.obs_rms.clone()
    mu_in, sig_in = ag.exp_mu.clone(), ag.exp_sigma.clone()

    def grad(mode):
        # the gradient kernel writes each row's new mu / sigma back (rl_games' dataset.update_mu_sigma), so every
        # call starts from the same experience
        monkeypatch.setenv("USV_PPO_FOLD", mode)
        ag.obs_rms.copy_(orms)
        ag.exp_mu.copy_(mu_in)
        ag.exp_sigma.copy_(sig_in)
        c.call("ppo_minibatch_grad", c.byref(ag.cfg), c.ptr(ag.model_params), c.ptr(ag.obs_rms), c.ptr(ag.val_rms),
               1, 0, c.ptr(ag.exp_obs), c.ptr(ag.exp_act), c.ptr(ag.exp_nlp), c.ptr(ag.exp_val), c.ptr(ag.exp_ret),
               c.ptr(ag.exp_adv), c.ptr(ag.exp_mu), c.ptr(ag.exp_sigma), c.ptr(ag.grad), c.ptr(ag.losses),
               c.ptr(ag.partials), c.ptr(ag.work), c.stream_ptr())
        torch.cuda.synchronize()
        return ag.grad[:PO.NPARAM + 1].cpu().numpy().copy(), ag.losses.cpu().numpy()[:5].copy()

    g1, l1 = grad("1")
    g2, l2 = grad("2")
    g1b, _ = grad("1")
    g0, _ = grad("0")
    np.testing.assert_array_equal(g1, g2)
    np.testing.assert_array_equal(l1, l2)
    np.testing.assert_array_equal(g1, g1b)
    scale = np.abs(g0[:PO.NPARAM]).max()
    ET.check(f"group_fold_{minibatch}", "fold vs unfolded", g1[:PO.NPARAM] / scale, g0[:PO.NPARAM] / scale, 0, 1e-6)
    o = PO.RMS.zeros(33)
    o.update(obs)
    g_ref, _, _, _, _ = PO.minibatch_grad(P, o.norm(obs), act, nlp0, val, ret, adv, mu0 + 0.01, sig0,
                                          PO.PPOConfig(minibatch=minibatch))
    ET.check(f"group_fold_{minibatch}", "grad/max", g1[:PO.NPARAM] / scale, g_ref / scale, 0, 1e-5)
