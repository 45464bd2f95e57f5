"""The loopz PPO oracle (oracle/loopz_oracle.py) against the reference's own PPO class
(tests/golden/loopz_update.npz, recorded by tests/golden/make_golden.py::gen_loopz): rollout
actions / log-probs / values, GAE returns and normalised advantages, and one update (4 epochs x 4
in-order minibatches, clip 0.5, Adam 5e-4) of every actor / critic parameter and the Adam state."""
import numpy as np

from oracle import loopz_oracle as L

OBS = 33


def _params(d, tag):
    sd = lambda net: {k.split("/", 2)[2]: d[k] for k in d if k.startswith(f"{tag}/{net}/")}
    return L.from_state_dicts(sd("actor"), sd("dist"), sd("critic"), OBS)


def test_rollout_matches_reference(golden):
    d = golden("loopz_update.npz")
    p = L.unflatten(_params(d, "init"), OBS)
    T = d["rew"].shape[0]
    for t in range(T):
        a, lp, _ = L.sample(p, d["obs"][t], d["eps"][t], np.float32(1.0))
        np.testing.assert_allclose(a, d["actions"][t], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(lp, d["logp"][t], rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(L.value(p, d["obs"][t]), d["values"][t], rtol=1e-5, atol=1e-5)


def test_gae_matches_reference(golden):
    d = golden("loopz_update.npz")
    p = L.unflatten(_params(d, "init"), OBS)
    last = L.value(p, d["obs"][-1])
    ret, adv = L.compute_returns(d["rew"], d["values"], d["done"], last)
    np.testing.assert_allclose(ret, d["returns"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(adv, d["advantages"], rtol=1e-5, atol=1e-5)


def test_update_matches_reference(golden):
    d = golden("loopz_update.npz")
    pv0 = _params(d, "init")
    data = {k: d[k] for k in ("obs", "actions", "logp", "values", "returns", "advantages")}
    data["obs"] = data["obs"][:-1]
    adam = L.Adam.zeros(len(pv0))
    pv, vl, sl = L.train_step(pv0, adam, data, np.float32(1.0), L.Config())
    want = _params(d, "after")
    assert adam.step == int(d["adam_step"]) == 16
    np.testing.assert_allclose(vl, float(d["loss_value"]), rtol=1e-5)
    np.testing.assert_allclose(sl, float(d["loss_surrogate"]), rtol=1e-4, atol=1e-7)
    # parameter deltas (lr 5e-4 per step) at 1e-5 of their size: absolute 1e-7 on the weights
    np.testing.assert_allclose(pv - pv0, want - pv0, rtol=1e-3, atol=2e-7)
    lay, _ = L.layout(OBS)
    for i, (k, s, o) in enumerate(lay):
        n = int(np.prod(s))
        np.testing.assert_allclose(adam.m[o:o + n], d[f"adam_m_{i}"].reshape(-1), rtol=1e-3, atol=1e-7, err_msg=k)
        np.testing.assert_allclose(adam.v[o:o + n], d[f"adam_v_{i}"].reshape(-1), rtol=1e-3, atol=1e-10, err_msg=k)
    std = L.enforce_minimum_std(pv, OBS)[[o for k, _, o in lay if k == "std"][0]:][:2]
    np.testing.assert_allclose(std, d["std_enforced"], rtol=1e-6)


def test_shuffle_update_matches_reference(golden):
    """mini_batch_sampling='shuffle' (the reference PPO's default, ppo.py:52-53; storage.py:123-134): the same
    rollout updated over the recorded BatchSampler(SubsetRandomSampler) minibatches."""
    d = golden("loopz_update_shuffle.npz")
    pv0 = _params(d, "init")
    data = {k: d[k] for k in ("obs", "actions", "logp", "values", "returns", "advantages")}
    data["obs"] = data["obs"][:-1]
    adam = L.Adam.zeros(len(pv0))
    assert d["batches"].shape == (16, d["rew"].size // 4)
    pv, vl, sl = L.train_step(pv0, adam, data, np.float32(1.0), L.Config(), batches=d["batches"])
    want = _params(d, "after")
    np.testing.assert_allclose(vl, float(d["loss_value"]), rtol=1e-5)
    np.testing.assert_allclose(sl, float(d["loss_surrogate"]), rtol=1e-4, atol=1e-7)
    np.testing.assert_allclose(pv - pv0, want - pv0, rtol=1e-3, atol=2e-7)
    # the shuffled minibatches really differ from the in-order ones
    assert not np.array_equal(np.sort(d["batches"][0]), np.arange(d["batches"].shape[1]))


def test_imitation_update_matches_reference(golden):
    """PPO(flat_expert=...) with update_rl_coeff(0.3) (ppo.py:93-100, 253-286): the loss gains
    mean((1 - rl_coeff) * sum_a (expert_a - action_mean_a)^2) over each minibatch; the fixture's expert is a
    fixed map of the observation, recorded with its actions on the stored observations."""
    d = golden("loopz_update_expert.npz")
    assert float(d["rl_coeff"]) == 0.3
    obs = d["obs"][:-1].reshape(-1, OBS)
    np.testing.assert_allclose(d["expert_act"], np.tanh(obs @ d["expert_w"]), rtol=1e-5, atol=1e-6)
    pv0 = _params(d, "init")
    data = {k: d[k] for k in ("obs", "actions", "logp", "values", "returns", "advantages")}
    data["obs"] = data["obs"][:-1]
    adam = L.Adam.zeros(len(pv0))
    cfg = L.Config(im_coef=float(np.float32(1 - 0.3)))
    pv, vl, sl = L.train_step(pv0, adam, data, np.float32(1.0), cfg, expert=d["expert_act"])
    want = _params(d, "after")
    np.testing.assert_allclose(vl, float(d["loss_value"]), rtol=1e-5)
    np.testing.assert_allclose(sl, float(d["loss_surrogate"]), rtol=5e-4)
    # the imitation gradient is large enough to engage clip_grad_norm_ (0.5) at every step, and the summation
    # order of 96-row sums differs from torch's: 16 Adam steps leave ~0.1% of the weights beyond the tight
    # tolerance of the other updates (51 of 45,621 here, each within 3e-4 of lr 5e-4 x 16 steps); the imitation
    # term's own head (mlp4) agrees to 1e-6
    a, b = pv - pv0, want - pv0
    bad = ~np.isclose(a, b, rtol=1e-3, atol=2e-7)
    assert bad.mean() < 2e-3 and np.abs(a - b).max() < 3e-4, (int(bad.sum()), float(np.abs(a - b).max()))
    # the imitation term moved the actor: without it the update lands elsewhere
    pv_rl, _, _ = L.train_step(pv0, L.Adam.zeros(len(pv0)), data, np.float32(1.0), L.Config())
    assert np.abs((pv_rl - pv0) - (want - pv0)).max() > 1e-2
