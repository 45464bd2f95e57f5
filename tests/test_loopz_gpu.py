"""The loopz trainer's HIP path (csrc/loopz.hip through the C ABI) against the reference's own
PPO class (tests/golden/loopz_update.npz) and the oracle (oracle/loopz_oracle.py)."""
import numpy as np
import pytest
import torch

from oracle import loopz_oracle as L
from omniisaacgymenvs_loop_amd.loopz import PPO, Actor, Critic, MLPEncode_wrap, SquashedGaussianDiagonalCovariance

from tests import errtab as ET

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
OBS = 33


_Leaky, _Tanh = torch.nn.LeakyReLU, torch.nn.Tanh   # the activation constructors the reference passes


def _build(n, T, d=None, seed=0, sampling="in_order", flat_expert=None):
    kw = dict(speed_dim=3, mass_dim=8, mass_latent_dim=8, mass_encoder_shape=(64, 16))
    actor = Actor(MLPEncode_wrap([128, 128], _Leaky, OBS, 2, _Tanh, False, seed=seed, **kw),
                  SquashedGaussianDiagonalCovariance(2, 0.3, action_scale=1.0), DEV)
    critic = Critic(MLPEncode_wrap([128, 128], _Leaky, OBS, 1, seed=seed + 1, **kw), DEV)
    if d is not None:
        sd = lambda net: {k.split("/", 2)[2]: torch.tensor(d[k]) for k in d if k.startswith(f"init/{net}/")}
        actor.architecture.load_state_dict(sd("actor"))
        actor.distribution.load_state_dict(sd("dist"))
        critic.architecture.load_state_dict(sd("critic"))
    return PPO(actor, critic, n, T, 4, 4, gamma=0.997, lam=0.95, device=DEV, mini_batch_sampling=sampling,
               learning_rate=5e-4, log_dir="/tmp/loopz_test", flat_expert=flat_expert)


def _params(d, tag):
    sd = lambda net: {k.split("/", 2)[2]: d[k] for k in d if k.startswith(f"{tag}/{net}/")}
    return L.from_state_dicts(sd("actor"), sd("dist"), sd("critic"), OBS)


def _rollout(ppo, d):
    T = d["rew"].shape[0]
    for t in range(T):
        a = ppo.observe_device(torch.tensor(d["obs"][t], device=DEV), torch.tensor(d["eps"][t], device=DEV))
        ET.check("loopz_rollout", "actions", a.cpu().numpy(), d["actions"][t], 1e-5, 1e-5, ["a0", "a1"])
        ppo.step_device(torch.tensor(d["rew"][t]), torch.tensor(d["done"][t].astype(np.int64)))
    st = ppo.storage
    ET.check("loopz_rollout", "logp", st.actions_log_prob.cpu().numpy(), d["logp"], 1e-5, 1e-5)
    ET.check("loopz_rollout", "values", st.values.cpu().numpy(), d["values"], 1e-5, 1e-5)


def test_rollout_and_update_vs_reference(golden):
    d = golden("loopz_update.npz")
    T, n = d["rew"].shape
    ppo = _build(n, T, d)
    np.testing.assert_array_equal(ppo.params.cpu().numpy(), _params(d, "init"))
    _rollout(ppo, d)
    ppo.update(actor_obs=None, value_obs=torch.tensor(d["obs"][T]), log_this_iteration=False, update=0)
    st = ppo.storage
    ET.check("loopz_update", "returns", st.returns.cpu().numpy(), d["returns"], 1e-5, 1e-5)
    ET.check("loopz_update", "advantages", st.advantages.cpu().numpy(), d["advantages"], 1e-5, 1e-5)
    assert ppo.adam_step() == int(d["adam_step"]) == 16
    got, want, p0 = ppo.params.cpu().numpy(), _params(d, "after"), _params(d, "init")
    # 16 Adam steps of lr 5e-4: parameters at 1e-5 relative to their size (absolute 1e-6)
    ET.check("loopz_update", "params", got, want, 1e-5, 1e-6)
    ET.record("loopz_update", "param_delta", got - p0, want - p0)
    np.testing.assert_allclose(ppo.mean_value_loss, float(d["loss_value"]), rtol=1e-5)
    np.testing.assert_allclose(ppo.mean_surrogate_loss, float(d["loss_surrogate"]), rtol=1e-4, atol=1e-6)
    ppo.actor.distribution.enforce_minimum_std(0.05)
    np.testing.assert_allclose(ppo.actor.distribution.std.cpu().numpy(), d["std_enforced"], rtol=1e-6)
    # state dicts come back in the reference's key set and shapes
    sd = ppo.actor.architecture.state_dict()
    ref_keys = {k.split("/", 2)[2] for k in d if k.startswith("after/actor/")}
    assert set(sd) == ref_keys
    osd = ppo.optimizer_state_dict()
    for i in range(len(osd["param_groups"][0]["params"])):
        ref = d[f"adam_m_{i}"]   # gradient moments: 1e-5 of the tensor's largest entry
        np.testing.assert_allclose(osd["state"][i]["exp_avg"].numpy(), ref, rtol=1e-4, atol=1e-5 * np.abs(ref).max())


def test_shuffle_update_vs_reference(golden):
    """mini_batch_sampling='shuffle' (ppo.py:52-53, storage.py:123-134): the reference's recorded
    BatchSampler(SubsetRandomSampler) minibatches replayed through lz_minibatch_rows."""
    d = golden("loopz_update_shuffle.npz")
    T, n = d["rew"].shape
    ppo = _build(n, T, d, sampling="shuffle")
    _rollout(ppo, d)
    ppo.inject_batches(d["batches"])
    ppo.update(actor_obs=None, value_obs=torch.tensor(d["obs"][T]), log_this_iteration=False, update=0)
    assert ppo.adam_step() == 16
    got, want = ppo.params.cpu().numpy(), _params(d, "after")
    ET.check("loopz_update_shuffle", "params", got, want, 1e-5, 1e-6)
    np.testing.assert_allclose(ppo.mean_value_loss, float(d["loss_value"]), rtol=1e-5)
    np.testing.assert_allclose(ppo.mean_surrogate_loss, float(d["loss_surrogate"]), rtol=1e-4, atol=1e-6)


def test_shuffle_rows_are_per_epoch_permutations():
    n, T = 37, 24
    ppo = _build(n, T, seed=2, sampling="shuffle")
    rows = ppo._shuffle_rows().cpu().numpy()
    M = n * T // 4
    assert rows.shape == (16, M)
    for e in range(4):
        ep = rows[4 * e:4 * e + 4].reshape(-1)
        assert len(np.unique(ep)) == 4 * M and ep.min() >= 0 and ep.max() < n * T
    assert not np.array_equal(rows[:4], rows[4:8])


@pytest.mark.parametrize("n,T,rows_shuffled", [(512, 600, False), (37, 24, False), (512, 600, True), (37, 24, True)])
def test_minibatch_vs_oracle(n, T, rows_shuffled):
    """One full-size minibatch (76800 rows at the loopz default of 512 envs x 600 steps; and a ragged
    size), in order or of shuffled rows, through lz_minibatch_rows against the oracle's gradient + clip + Adam."""
    rng = np.random.default_rng(3)
    ppo = _build(n, T, seed=5)
    st = ppo.storage
    obs = rng.uniform(-2.5, 2.5, (T, n, OBS)).astype(np.float32)
    obs[..., 25:] = rng.uniform(-1, 1, (T, n, 8))
    act = np.tanh(rng.normal(0, 1, (T, n, 2))).astype(np.float32)
    data = {"obs": obs, "actions": act, "logp": rng.normal(-1, 0.5, (T, n)).astype(np.float32),
            "values": rng.normal(0, 1, (T, n)).astype(np.float32), "returns": rng.normal(0, 1.5, (T, n)).astype(np.float32),
            "advantages": rng.normal(0, 1, (T, n)).astype(np.float32)}
    for k, buf in (("obs", st.actor_obs), ("actions", st.actions), ("logp", st.actions_log_prob), ("values", st.values),
                   ("returns", st.returns), ("advantages", st.advantages)):
        buf.copy_(torch.tensor(data[k]))
    p0 = ppo.params.cpu().numpy()
    mb = 1
    B = n * T
    M = B // 4
    # in order at full size; the ragged case takes a shuffled minibatch (random rows of the T N storage)
    sl = slice(mb * M, (mb + 1) * M) if rows_shuffled is False else rng.permutation(B)[:M]
    rows = None if rows_shuffled is False else torch.tensor(sl, dtype=torch.int32, device=DEV)
    from omniisaacgymenvs_loop_amd import _capi
    _capi.call("lz_minibatch_rows", _capi.byref(ppo.cfg), _capi.ptr(ppo.params), _capi.ptr(ppo.adam_m),
               _capi.ptr(ppo.adam_v), _capi.ptr(ppo.opt), 0, mb, _capi.ptr(st.actor_obs), _capi.ptr(st.actions),
               _capi.ptr(st.actions_log_prob), _capi.ptr(st.values), _capi.ptr(st.returns), _capi.ptr(st.advantages),
               _capi.ptr(rows), _capi.ptr(ppo.partials), _capi.ptr(ppo.grad), _capi.stream_ptr())
    torch.cuda.synchronize()
    flat = {k: v.reshape((B,) + v.shape[2:]) for k, v in data.items()}
    G, vl, sl_loss, loss = L.minibatch_grad(L.unflatten(p0, OBS), flat["obs"][sl], flat["actions"][sl],
                                            flat["logp"][sl], flat["values"][sl], flat["returns"][sl],
                                            flat["advantages"][sl], np.float32(1.0), L.Config())
    g_ref = L.flatten(G, OBS)
    np_ = ppo.nparam
    g = ppo.grad[:np_].cpu().numpy()
    scale = float(np.abs(g_ref).max())
    ET.check(f"loopz_grad_{n}x{T}{'s' if rows_shuffled else ''}", "grad/max", g / scale, g_ref / scale, 1e-5, 1e-5)
    gc, _ = L.clip_grad(G, OBS, 0.5)
    adam = L.Adam.zeros(np_)
    want = adam.apply(p0, gc, L.Config())
    # Adam's first step is ~lr * sign(g): where |g| is within the gradient tolerance of 0 the step
    # itself is ill-conditioned, so the 1e-6 parameter check covers |g| > 1e-3 max|g| (recorded in full)
    got = ppo.params.cpu().numpy()
    ET.record(f"loopz_grad_{n}x{T}{'s' if rows_shuffled else ''}", "params(all)", got, want)
    well = np.abs(g_ref) > 1e-3 * scale
    ET.check(f"loopz_grad_{n}x{T}{'s' if rows_shuffled else ''}", "params", got[well], want[well], 1e-5, 1e-6)
    assert np.abs(got - want).max() <= 2.0 * L.Config().lr + 1e-6
    np.testing.assert_allclose(float(ppo.opt[8 + 2].item()), vl, rtol=1e-5)


def test_nonfinite_loss_skips_the_step():
    n, T = 32, 8
    ppo = _build(n, T, seed=9)
    st = ppo.storage
    st.actor_obs.uniform_(-1, 1)
    st.advantages.fill_(float("nan"))
    p0 = ppo.params.clone()
    from omniisaacgymenvs_loop_amd import _capi
    _capi.call("lz_minibatch", _capi.byref(ppo.cfg), _capi.ptr(ppo.params), _capi.ptr(ppo.adam_m),
               _capi.ptr(ppo.adam_v), _capi.ptr(ppo.opt), 0, 0, _capi.ptr(st.actor_obs), _capi.ptr(st.actions),
               _capi.ptr(st.actions_log_prob), _capi.ptr(st.values), _capi.ptr(st.returns), _capi.ptr(st.advantages),
               _capi.ptr(ppo.partials), _capi.ptr(ppo.grad), _capi.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(ppo.params, p0)
    assert float(ppo.opt[8 + 1].item()) == 0.0 and float(ppo.opt[8 + 5].item()) == 0.0


def test_loopz_trainer_runs_on_the_usv_task(tmp_path, monkeypatch):
    """scripts/loopz_train.py's loop on the USV env (64 envs, 16 transitions per update), two updates,
    then a resume from the written full_0.pt checkpoint (reference key set)."""
    from omniisaacgymenvs_loop_amd.scripts import loopz_train as LT
    monkeypatch.chdir(tmp_path)
    cfg = LT.build_config({"num_envs": 64, "seed": 3, "train": "USV/USV_MLP"})
    cfg = LT.merge_loopz_overrides(cfg, LT.os.path.join(LT.os.path.dirname(LT.os.path.dirname(LT.os.path.abspath(LT.__file__))), "cfg"))
    cfg["environment"]["max_time"] = 0.16
    cfg["environment"]["eval_every_n"] = 1
    hist, ppo = LT.train(cfg, max_updates=1, log=lambda *a: None)
    assert len(hist) == 2 and all(np.isfinite(h["average_ll_reward"]) for h in hist)
    assert ppo.adam_step() == 2 * 16
    assert np.all(np.isfinite(ppo.params.cpu().numpy()))
    ck = tmp_path / "runs" / "USV" / "nn" / "full_1.pt"
    sd = torch.load(ck, map_location="cpu", weights_only=True)
    assert set(sd) == {"actor_architecture_state_dict", "actor_distribution_state_dict", "critic_architecture_state_dict",
                       "optimizer_state_dict", "update"} and sd["update"] == 1
    assert "architecture.mass_encoder.0.weight" in sd["actor_architecture_state_dict"]
    env, actor, critic, ppo2, _ = LT.build(cfg)
    assert LT.load_full(str(ck), actor, critic, ppo2) == 2
    p_saved = np.concatenate([v.numpy().reshape(-1) for v in sd["actor_architecture_state_dict"].values()])
    np.testing.assert_array_equal(actor.architecture.flat().numpy(), p_saved)


class _Expert:
    """The fixture's frozen expert (tests/golden/make_golden.py ScriptedExpert): tanh(obs @ w)."""

    def __init__(self, w):
        self.w = torch.tensor(w, device=DEV)

    def evaluate(self, obs):
        return torch.tanh(obs @ self.w)


def test_imitation_update_vs_reference(golden):
    """PPO(flat_expert=...) + update_rl_coeff(0.3) (ppo.py:93-100, 253-286): the expert's actions on the stored
    observations feed the gradient kernel's (1 - rl_coeff) * sum_a (expert_a - action_mean_a)^2 term.  Against
    the reference run (loopz_update_expert.npz) with the oracle test's tolerance (clip_grad_norm_ is active at
    every step), and against the oracle (same gradient kernel inputs) at 1e-5."""
    d = golden("loopz_update_expert.npz")
    T, n = d["rew"].shape
    ppo = _build(n, T, d, flat_expert=_Expert(d["expert_w"]))
    ppo.update_rl_coeff(0.3)
    _rollout(ppo, d)
    ppo.update(actor_obs=None, value_obs=torch.tensor(d["obs"][T]), log_this_iteration=False, update=0)
    np.testing.assert_allclose(ppo._expert_act.cpu().numpy(), d["expert_act"], rtol=1e-5, atol=1e-6)
    assert ppo.adam_step() == 16
    got, want, p0 = ppo.params.cpu().numpy(), _params(d, "after"), _params(d, "init")
    a, b = got - p0, want - p0
    bad = ~np.isclose(a, b, rtol=1e-3, atol=2e-7)
    ET.record("loopz_update_expert", "param_delta", a, b)
    assert bad.mean() < 2e-3 and np.abs(a - b).max() < 3e-4, (int(bad.sum()), float(np.abs(a - b).max()))
    np.testing.assert_allclose(ppo.mean_value_loss, float(d["loss_value"]), rtol=1e-5)
    np.testing.assert_allclose(ppo.mean_surrogate_loss, float(d["loss_surrogate"]), rtol=5e-4)
    # the same update on the oracle from the same rollout buffers: the kernels' arithmetic, tight
    data = {k: d[k] for k in ("obs", "actions", "logp", "values", "returns", "advantages")}
    data["obs"] = data["obs"][:-1]
    pv, _, _ = L.train_step(p0, L.Adam.zeros(len(p0)), data, np.float32(1.0),
                            L.Config(im_coef=float(np.float32(0.7))), expert=d["expert_act"])
    bad_o = ~np.isclose(got - p0, pv - p0, rtol=1e-3, atol=2e-7)
    assert bad_o.mean() < 2e-3, int(bad_o.sum())


def test_imitation_gradient_vs_oracle_each_step(golden):
    """The imitation update on identical inputs at every step: the 16 minibatch gradients of the fixture's rollout
    (loopz_update_expert.npz, in-order minibatches, (1 - rl_coeff) = 0.7 with the frozen expert's actions on the
    stored observations) from the oracle's parameters before each step, against the oracle's gradient at 1e-5 of
    its largest component (test_minibatch_vs_oracle's bar) -- no drift carried from step to step, no outliers
    allowed.  The oracle then takes the clipped Adam step and both continue from its parameters."""
    d = golden("loopz_update_expert.npz")
    T, n = d["rew"].shape
    ppo = _build(n, T, d, flat_expert=_Expert(d["expert_w"]))
    ppo.update_rl_coeff(0.3)
    st = ppo.storage
    data = {"obs": d["obs"][:T], "actions": d["actions"], "logp": d["logp"], "values": d["values"],
            "returns": d["returns"], "advantages": d["advantages"]}
    for k, buf in (("obs", st.actor_obs), ("actions", st.actions), ("logp", st.actions_log_prob), ("values", st.values),
                   ("returns", st.returns), ("advantages", st.advantages)):
        buf.copy_(torch.tensor(np.ascontiguousarray(data[k]).reshape(buf.shape)))
    ppo._bind_expert()
    ex = ppo._expert_act.cpu().numpy().reshape(-1, 2)       # the kernel's expert actions, fed to the oracle too
    np.testing.assert_allclose(ex, np.asarray(d["expert_act"]).reshape(-1, 2), rtol=1e-5, atol=1e-6)
    cfg = L.Config(im_coef=float(np.float32(0.7)))
    assert float(ppo.cfg.im_coef) == cfg.im_coef
    flat = {k: np.asarray(v, np.float32).reshape((T * n,) + np.asarray(v).shape[2:]) for k, v in data.items()}
    M = T * n // 4
    pv = _params(d, "init")
    adam = L.Adam.zeros(len(pv))
    from omniisaacgymenvs_loop_amd import _capi
    np_ = ppo.nparam
    for k in range(16):
        i = k % 4
        sl = slice(i * M, (i + 1) * M)
        ppo.params.copy_(torch.tensor(pv, device=DEV))
        _capi.call("lz_minibatch", _capi.byref(ppo.cfg), _capi.ptr(ppo.params), _capi.ptr(ppo.adam_m),
                   _capi.ptr(ppo.adam_v), _capi.ptr(ppo.opt), 0, i, _capi.ptr(st.actor_obs), _capi.ptr(st.actions),
                   _capi.ptr(st.actions_log_prob), _capi.ptr(st.values), _capi.ptr(st.returns),
                   _capi.ptr(st.advantages), _capi.ptr(ppo.partials), _capi.ptr(ppo.grad), _capi.stream_ptr())
        torch.cuda.synchronize()
        G, _, _, _ = L.minibatch_grad(L.unflatten(pv, OBS), flat["obs"][sl], flat["actions"][sl], flat["logp"][sl],
                                      flat["values"][sl], flat["returns"][sl], flat["advantages"][sl], np.float32(1.0),
                                      cfg, ex[sl])
        g_ref = L.flatten(G, OBS)
        scale = float(np.abs(g_ref).max())
        ET.check("loopz_expert_grad_per_step", "grad/max", ppo.grad[:np_].cpu().numpy() / scale, g_ref / scale,
                 1e-5, 1e-5, err_msg=f"step {k}")
        gc, _ = L.clip_grad(G, OBS, cfg.max_grad_norm)
        pv = adam.apply(pv, gc, cfg)
