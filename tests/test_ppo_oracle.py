"""numpy PPO oracle (oracle/ppo_oracle.py) vs the reference rl_games A2CAgent.

Fixture tests/golden/ppo_epoch.npz: one full train_epoch of the reference
(N=32 envs, horizon 16, minibatch 128 -> 4 minibatches x 8 mini-epochs) driven
by a scripted env, with the initial/final weights, the rollout buffers, the
GAE returns, the prepared dataset, the per-minibatch losses/KL and the LR
sequence of the adaptive schedule.
"""
import numpy as np
import pytest

from oracle import ppo_oracle as PO


def _params(g, prefix):
    return {k: g[f"{prefix}_{v.replace('.', '__')}"] for k, v in PO.STATE_KEYS.items()}


def _rms(g, prefix, key):
    base = f"{prefix}_{key}"
    return PO.RMS(g[f"{base}__running_mean"].astype(np.float64), g[f"{base}__running_var"].astype(np.float64),
                  float(g[f"{base}__count"]))


@pytest.fixture(scope="module")
def ppo(golden):
    return golden("ppo_epoch.npz")


def test_rollout_forward(ppo):
    P = _params(ppo, "init")
    H = ppo["exp_obses"].shape[0]
    orms = PO.RMS.zeros(33)
    vrms = PO.RMS.zeros(1)
    for t in range(H):
        obs = ppo["exp_obses"][t]
        np.testing.assert_array_equal(obs, ppo["env_obs"][t])
        _, _, mu, v = PO.forward(P, orms.norm(obs))
        np.testing.assert_allclose(mu, ppo["exp_mus"][t], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(vrms.denorm(v), ppo["exp_values"][t], rtol=1e-5, atol=1e-6)
        sigma = np.exp(mu * 0 + P["sigma"])
        np.testing.assert_allclose(sigma, ppo["exp_sigmas"][t], rtol=1e-6)
        nlp = PO.neglogp(ppo["exp_actions"][t], mu, sigma, mu * 0 + P["sigma"])
        np.testing.assert_allclose(nlp, ppo["exp_neglogpacs"][t], rtol=1e-5, atol=1e-5)
        # env received clamp(-1, 1) of the sampled actions (a2c_common.py:1134-1144)
        np.testing.assert_array_equal(ppo["env_actions"][t], np.clip(ppo["exp_actions"][t], -1, 1))


def test_gae_and_prepare(ppo):
    P = _params(ppo, "init")
    cfg = PO.PPOConfig(minibatch=int(ppo["hyper"][2]))
    H, N = ppo["exp_rewards"].shape[:2]
    last_obs = ppo["env_obs"][H]
    _, _, _, last_v = PO.forward(P, PO.RMS.zeros(33).norm(last_obs))
    last_v = PO.RMS.zeros(1).denorm(last_v)
    fd = ppo["env_dones"][H - 1].astype(np.float32)
    mb_fd = ppo["exp_dones"].astype(np.float32)
    advs = PO.discount_values(cfg.gamma, cfg.tau, fd, last_v, mb_fd, ppo["exp_values"], ppo["exp_rewards"])
    returns = advs + ppo["exp_values"]
    flat = lambda a: np.swapaxes(a, 0, 1).reshape(N * H, *a.shape[2:])
    np.testing.assert_allclose(flat(returns), ppo["batch_returns"], rtol=1e-5, atol=1e-5)
    # prepare_dataset: value RMS trained on values then returns, advantage normalisation
    values, rets = flat(ppo["exp_values"]), flat(returns)
    adv = (rets - values).sum(1)
    vrms = PO.RMS.zeros(1)
    vrms.update(values)
    vn = vrms.norm(values)
    vrms.update(rets)
    rn = vrms.norm(rets)
    an = (adv - adv.mean()) / (adv.std(ddof=1) + 1e-8)
    np.testing.assert_allclose(vn, ppo["ds_old_values"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(rn, ppo["ds_returns"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(an, ppo["ds_advantages"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(vrms.mean, ppo["final_value_mean_std__running_mean"], rtol=1e-6)
    np.testing.assert_allclose(vrms.var, ppo["final_value_mean_std__running_var"], rtol=1e-6)


def test_minibatch_update_epoch(ppo):
    """8 mini-epochs x 4 minibatches: losses, KL, adaptive LR, final weights, obs RMS."""
    P = _params(ppo, "init")
    cfg = PO.PPOConfig(minibatch=int(ppo["hyper"][2]))
    ds = {"obs": ppo["ds_obs_state"] if "ds_obs_state" in ppo else ppo["ds_obs"],
          "actions": ppo["ds_actions"], "old_logp": ppo["ds_old_logp_actions"], "old_values": ppo["ds_old_values"][:, 0],
          "returns": ppo["ds_returns"][:, 0], "advantages": ppo["ds_advantages"],
          "mu": ppo["batch_mus"], "sigma": ppo["batch_sigmas"]}
    orms = PO.RMS.zeros(33)
    Pf, lr, log = PO.train_epoch_update(P, PO.Adam.zeros(), 1e-4, orms, ds, cfg)
    np.testing.assert_allclose(log["kl"], ppo["kl"], rtol=2e-3, atol=1e-7)
    np.testing.assert_allclose(np.array(log["losses"]), ppo["losses"], rtol=2e-3, atol=1e-6)
    np.testing.assert_allclose(log["lr"], ppo["lr_seq"], rtol=1e-12)
    ref_obs = _rms(ppo, "final", "running_mean_std__running_mean_std__state")
    np.testing.assert_allclose(orms.mean, ref_obs.mean, rtol=1e-6, atol=1e-9)
    np.testing.assert_allclose(orms.var, ref_obs.var, rtol=1e-6)
    assert orms.count == ref_obs.count
    Pr = _params(ppo, "final")
    for k in Pr:
        np.testing.assert_allclose(Pf[k], Pr[k], rtol=0, atol=2e-5, err_msg=k)


def test_vectorised_philox_matches_c_oracle():
    """PO.philox4x32_10 (numpy, the checker of the rollout kernel's in-kernel normals) == the C oracle's
    Philox (itself pinned by the Random123 known-answer vectors in test_oracle_golden.py)."""
    from oracle import oracle as O
    rng = np.random.default_rng(0)
    ctr = rng.integers(0, 2 ** 32, (64, 4), dtype=np.uint64)
    key = rng.integers(0, 2 ** 32, (64, 2), dtype=np.uint64)
    for c, k in zip(ctr, key):
        want = O.philox(c.astype(np.uint32), k.astype(np.uint32))
        got = PO.philox4x32_10(tuple(int(x) for x in c), (int(k[0]), int(k[1])))
        assert [int(x) for x in got] == [int(x) for x in want]
    z = PO.policy_normals(42, 2 ** 33 + 7, 200_000)
    assert abs(float(z.mean())) < 0.01 and abs(float(z.std()) - 1) < 0.01


def test_prepare_dataset_helper_vs_reference(ppo):
    """PO.prepare_dataset (the headline-size checker of ppo_prepare) reproduces the reference's prepared dataset."""
    P = _params(ppo, "init")
    cfg = PO.PPOConfig(minibatch=int(ppo["hyper"][2]))
    H, N = ppo["exp_rewards"].shape[:2]
    _, _, _, last_v = PO.forward(P, PO.RMS.zeros(33).norm(ppo["env_obs"][H]))
    last_v = PO.RMS.zeros(1).denorm(last_v)[:, 0]
    vrms = PO.RMS.zeros(1)
    vn, rn, an = PO.prepare_dataset(ppo["exp_values"][:, :, 0], ppo["exp_rewards"][:, :, 0], ppo["exp_dones"],
                                    last_v, ppo["env_dones"][H - 1], cfg, vrms)
    np.testing.assert_allclose(vn, ppo["ds_old_values"][:, 0], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(rn, ppo["ds_returns"][:, 0], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(an, ppo["ds_advantages"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(vrms.var, ppo["final_value_mean_std__running_var"], rtol=1e-6)
