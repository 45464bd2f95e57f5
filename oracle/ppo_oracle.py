"""ORACLE / TEST INFRASTRUCTURE ONLY.

numpy restatement of the rl_games PPO path the reference uses for
train=USV/USV_PPOcontinuous_MLP (a2c_continuous + actor_critic_mlp_dict +
continuous_a2c_logstd), with explicit backprop.  Checker for the HIP PPO
kernels (omniisaacgymenvs_loop_amd/csrc/ppo.hip) and pinned against
tests/golden/ppo_epoch.npz, recorded from the reference A2CAgent.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

NIN, NH, NA = 33, 128, 2
LOG2PI = np.float32(0.5 * math.log(2.0 * math.pi) * 2)   # models.py:400
F = np.float32

# flat parameter order = model.parameters() order (network_builder.py:1480-1575)
SHAPES = [("sigma", (NA,)), ("W1", (NH, NIN)), ("b1", (NH,)), ("W2", (NH, NH)), ("b2", (NH,)),
          ("Wv", (1, NH)), ("bv", (1,)), ("Wmu", (NA, NH)), ("bmu", (NA,))]
STATE_KEYS = {"sigma": "a2c_network.sigma", "W1": "a2c_network.actor_mlp.0.weight",
              "b1": "a2c_network.actor_mlp.0.bias", "W2": "a2c_network.actor_mlp.2.weight",
              "b2": "a2c_network.actor_mlp.2.bias", "Wv": "a2c_network.value.weight",
              "bv": "a2c_network.value.bias", "Wmu": "a2c_network.mu.weight", "bmu": "a2c_network.mu.bias"}
NPARAM = sum(int(np.prod(s)) for _, s in SHAPES)


def flatten(p: dict) -> np.ndarray:
    return np.concatenate([np.asarray(p[k], F).reshape(-1) for k, _ in SHAPES])


def unflatten(v: np.ndarray) -> dict:
    out, o = {}, 0
    for k, s in SHAPES:
        m = int(np.prod(s))
        out[k] = v[o:o + m].reshape(s).astype(F)
        o += m
    return out


@dataclass
class RMS:
    """RunningMeanStd (running_mean_std.py:44-118), fp64 stats, count init 1."""
    mean: np.ndarray
    var: np.ndarray
    count: float = 1.0
    eps: float = 1e-5

    @classmethod
    def zeros(cls, n):
        return cls(np.zeros(n, np.float64), np.ones(n, np.float64), 1.0)

    def update(self, x: np.ndarray):
        x = np.asarray(x, np.float64).reshape(len(x), -1)
        bm = x.mean(0)
        bv = x.var(0, ddof=1)
        bc = x.shape[0]
        delta = bm - self.mean
        tot = self.count + bc
        self.mean = self.mean + delta * bc / tot
        M2 = self.var * self.count + bv * bc + delta ** 2 * self.count * bc / tot
        self.var = M2 / tot
        self.count = tot

    def norm(self, x):
        y = (np.asarray(x, F) - self.mean.astype(F)) / np.sqrt(self.var.astype(F) + F(self.eps))
        return np.clip(y, F(-5), F(5)).astype(F)

    def denorm(self, x):
        y = np.clip(np.asarray(x, F), F(-5), F(5))
        return (np.sqrt(self.var.astype(F) + F(self.eps)) * y + self.mean.astype(F)).astype(F)


def bf16(a: np.ndarray) -> np.ndarray:
    """fp32 -> bf16 (round to nearest even) -> fp32: the operand rounding of the bf16 GEMM mode
    (ppo_cfg_t.bf16_gemm: the 128x128 products -- layer 2, dW2, dh1 -- take bf16 operands with fp32
    accumulation on v_mfma_f32_32x32x16_bf16; everything else stays fp32)."""
    u = np.ascontiguousarray(a, np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    out = r.astype(np.uint32).view(np.float32)
    return np.where(np.isnan(a), a, out).astype(F)


def _mm(a, b, lowp):
    return (bf16(a) @ bf16(b)).astype(F) if lowp else (a @ b).astype(F)


def forward(P: dict, x: np.ndarray, lowp: bool = False):
    z1 = x @ P["W1"].T + P["b1"]
    h1 = np.tanh(z1).astype(F)
    z2 = _mm(h1, P["W2"].T, lowp) + P["b2"]
    h2 = np.tanh(z2).astype(F)
    mu = (h2 @ P["Wmu"].T + P["bmu"]).astype(F)
    v = (h2 @ P["Wv"].T + P["bv"]).astype(F)
    return h1, h2, mu, v


def neglogp(x, mu, sigma, logstd):
    return (F(0.5) * (((x - mu) / sigma) ** 2).sum(-1) + LOG2PI + logstd.sum(-1)).astype(F)


def discount_values(gamma, tau, fdones, last_values, mb_fdones, mb_values, mb_rewards):
    """A2CBase.discount_values (a2c_common.py:525-540); arrays [H, N(,1)]."""
    H = mb_rewards.shape[0]
    lastgaelam = 0
    mb_advs = np.zeros_like(mb_rewards)
    for t in reversed(range(H)):
        if t == H - 1:
            nnt = F(1.0) - fdones
            nv = last_values
        else:
            nnt = F(1.0) - mb_fdones[t + 1]
            nv = mb_values[t + 1]
        nnt = nnt[:, None]
        delta = mb_rewards[t] + F(gamma) * nv * nnt - mb_values[t]
        mb_advs[t] = lastgaelam = delta + F(gamma) * F(tau) * nnt * lastgaelam
    return mb_advs.astype(F)


@dataclass
class PPOConfig:
    e_clip: float = 0.2
    critic_coef: float = 0.5
    entropy_coef: float = 0.0
    bounds_loss_coef: float = 1e-4
    clip_value: bool = True
    grad_norm: float = 1.0
    truncate_grads: bool = True
    kl_threshold: float = 0.016
    gamma: float = 0.99
    tau: float = 0.95
    mini_epochs: int = 8
    minibatch: int = 8192
    b1: float = 0.9
    b2: float = 0.999
    eps: float = 1e-8


@dataclass
class Adam:
    m: np.ndarray
    v: np.ndarray
    step: int = 0

    @classmethod
    def zeros(cls):
        return cls(np.zeros(NPARAM, F), np.zeros(NPARAM, F), 0)

    def apply(self, p: np.ndarray, g: np.ndarray, lr: float, cfg: PPOConfig):
        self.step += 1
        self.m = (self.m + F(1 - cfg.b1) * (g - self.m)).astype(F)
        self.v = (self.v * F(cfg.b2) + F(1 - cfg.b2) * g * g).astype(F)
        bc1 = 1 - cfg.b1 ** self.step
        bc2 = 1 - cfg.b2 ** self.step
        step_size = lr / bc1
        denom = np.sqrt(self.v) / F(math.sqrt(bc2)) + F(cfg.eps)
        return (p - F(step_size) * (self.m / denom)).astype(F)


def minibatch_grad(P: dict, xn, act, old_nlp, old_val, ret, adv, old_mu, old_sigma, cfg: PPOConfig,
                   lowp: bool = False):
    """Forward + losses + explicit backward of A2CAgent.calc_gradients (a2c_continuous.py:78-196);
    lowp: the bf16 GEMM mode's operand rounding (see bf16())."""
    B = xn.shape[0]
    h1, h2, mu, v = forward(P, xn, lowp)
    v = v[:, 0]
    logstd = mu * F(0) + P["sigma"]
    sigma = np.exp(logstd).astype(F)
    z = (act - mu) / sigma
    nlp = (F(0.5) * (z ** 2).sum(-1) + LOG2PI + logstd.sum(-1)).astype(F)
    ratio = np.exp(old_nlp - nlp).astype(F)
    lo, hi = F(1 - cfg.e_clip), F(1 + cfg.e_clip)
    rc = np.clip(ratio, lo, hi)
    s1, s2 = -(adv * ratio), -(adv * rc)
    a_loss = np.maximum(s1, s2)
    inr = ((ratio >= lo) & (ratio <= hi)).astype(F)
    g1, g2 = -adv, -adv * inr
    g_r = np.where(s1 > s2, g1, np.where(s1 < s2, g2, F(0.5) * (g1 + g2)))
    dnlp = (g_r * (-ratio) / F(B)).astype(F)
    if cfg.clip_value:
        dvr = v - old_val
        vc = old_val + np.clip(dvr, F(-cfg.e_clip), F(cfg.e_clip))
        l1, l2 = (v - ret) ** 2, (vc - ret) ** 2
        c_loss = np.maximum(l1, l2)
        d1 = F(2) * (v - ret)
        d2 = F(2) * (vc - ret) * ((dvr >= -cfg.e_clip) & (dvr <= cfg.e_clip)).astype(F)
        dv = np.where(l1 > l2, d1, np.where(l1 < l2, d2, F(0.5) * (d1 + d2)))
    else:
        c_loss = (ret - v) ** 2
        dv = F(2) * (v - ret)
    dv = (dv * F(0.5 * cfg.critic_coef) / F(B)).astype(F)
    bh, bl = np.maximum(mu - F(1.1), 0), np.minimum(mu + F(1.1), 0)
    b_loss = (bl ** 2 + bh ** 2).sum(-1)
    dmu = dnlp[:, None] * (-z / sigma) + F(cfg.bounds_loss_coef / B) * F(2) * (bh + bl)
    # loss - entropy_coef * mean(entropy) (a2c_continuous.py:159): d entropy / d logstd = 1 per row
    dsig = (dnlp[:, None] * (F(1) - z * z) + F(-cfg.entropy_coef / B)).sum(0)
    ent = (F(0.5) + F(0.5 * math.log(2 * math.pi)) + logstd).sum(-1)
    kl = (np.log(old_sigma / sigma + F(1e-5)) + (sigma ** 2 + (old_mu - mu) ** 2) /
          (F(2) * (old_sigma ** 2 + F(1e-5))) - F(0.5)).sum(-1).mean()
    G = {"sigma": dsig}
    G["Wmu"] = dmu.T @ h2
    G["bmu"] = dmu.sum(0)
    G["Wv"] = (dv[:, None].T @ h2)
    G["bv"] = np.array([dv.sum()], F)
    dh2 = dmu @ P["Wmu"] + dv[:, None] @ P["Wv"]
    dz2 = dh2 * (F(1) - h2 * h2)
    G["W2"] = _mm(dz2.T, h1, lowp)
    G["b2"] = dz2.sum(0)
    dh1 = _mm(dz2, P["W2"], lowp)
    dz1 = dh1 * (F(1) - h1 * h1)
    G["W1"] = dz1.T @ xn
    G["b1"] = dz1.sum(0)
    losses = (float(a_loss.mean()), float(c_loss.mean()), float(ent.mean()), float(b_loss.mean()))
    return flatten(G), losses, float(kl), mu, sigma


def prepare_dataset(values_hn, rewards_hn, dones_hn, last_values, last_dones, cfg: PPOConfig, vrms: RMS,
                    normalize_value=True, normalize_advantage=True):
    """discount_values + returns (a2c_common.py:525-540, :763) and ContinuousA2CBase.prepare_dataset
    (:1257-1290): value RMS trained on the values then on the returns, both normalised, advantages
    (returns - values) normalised by their unbiased std.  Inputs [H, N] (values / rewards / dones of the
    rollout slots), last_values / last_dones [N]; outputs env-major [N*H] (swap_and_flatten01), vrms updated."""
    H, N = rewards_hn.shape
    advs = discount_values(cfg.gamma, cfg.tau, np.asarray(last_dones, F), np.asarray(last_values, F)[:, None],
                           np.asarray(dones_hn, F), np.asarray(values_hn, F)[:, :, None],
                           np.asarray(rewards_hn, F)[:, :, None])
    rets = (advs + np.asarray(values_hn, F)[:, :, None]).astype(F)
    flat = lambda a: np.ascontiguousarray(np.swapaxes(a, 0, 1).reshape(N * H))
    values, returns = flat(np.asarray(values_hn, F)), flat(rets[:, :, 0])
    adv = (returns - values).astype(F)
    if normalize_value:
        vrms.update(values[:, None])
        values = vrms.norm(values)
        vrms.update(returns[:, None])
        returns = vrms.norm(returns)
    if normalize_advantage:
        a64 = adv.astype(np.float64)
        adv = ((adv - F(a64.mean())) / (F(a64.std(ddof=1)) + F(1e-8))).astype(F)
    return values, returns, adv


PHILOX_M = (0xD2511F53, 0xCD9E8D57)
PHILOX_W = (0x9E3779B9, 0xBB67AE85)


def philox4x32_10(ctr, key):
    """Philox4x32-10 (Salmon et al. SC'11) over numpy arrays: ctr = 4 uint32 arrays (broadcast), key = 2
    ints; the generator of every in-kernel draw (csrc/usv_device.h philox4x32_10), restated vectorised
    and pinned against the C oracle's Random123 known-answer vectors (tests/test_oracle_golden.py)."""
    mask = np.uint64(0xFFFFFFFF)
    c = [np.asarray(x, np.uint64) & mask for x in np.broadcast_arrays(*ctr)]
    k0, k1 = np.uint64(key[0] & 0xFFFFFFFF), np.uint64(key[1] & 0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(PHILOX_M[0]) * c[0]
        p1 = np.uint64(PHILOX_M[1]) * c[2]
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ k0, p1 & mask, (p0 >> np.uint64(32)) ^ c[3] ^ k1, p0 & mask]
        k0 = (k0 + np.uint64(PHILOX_W[0])) & mask
        k1 = (k1 + np.uint64(PHILOX_W[1])) & mask
    return [x.astype(np.uint32) for x in c]


def u01(x):
    return ((np.asarray(x, np.uint32) >> np.uint32(8)).astype(F) * F(1.0 / 16777216.0)).astype(F)


def policy_normals(seed: int, step: int, n: int, site: int = 0x200):
    """The rollout kernel's Normal.sample draws (models.py:372-386 replaced by Box-Muller on
    Philox(key = seed, ctr = {env, step_lo, step_hi, site}), csrc/ppo.hip k_policy_step): [n, 2] fp32."""
    e = np.arange(n, dtype=np.uint64)
    r = philox4x32_10((e, step & 0xFFFFFFFF, (step >> 32) & 0xFFFFFFFF, site), (seed & 0xFFFFFFFF, seed >> 32))
    u = [u01(x) for x in r]
    two_pi = F(6.28318530717958647692)
    z0 = np.sqrt(F(-2.0) * np.log(F(1.0) - u[0])) * np.cos(two_pi * u[1])
    z1 = np.sqrt(F(-2.0) * np.log(F(1.0) - u[2])) * np.cos(two_pi * u[3])
    return np.stack([z0, z1], 1).astype(F)


def clip_grad(g: np.ndarray, max_norm: float):
    parts = unflatten(g)
    norms = np.array([np.linalg.norm(parts[k].astype(np.float64)) for k, _ in SHAPES], np.float64)
    total = float(np.linalg.norm(norms))
    coef = min(max_norm / (total + 1e-6), 1.0)
    return (g * F(coef)).astype(F), total


def adaptive_lr(lr, kl, thr, lo=1e-6, hi=1e-2):
    if kl > 2.0 * thr:
        lr = max(lr / 1.5, lo)
    if kl < 0.5 * thr:
        lr = min(lr * 1.5, hi)
    return lr


def train_epoch_update(P: dict, adam: Adam, lr: float, obs_rms: RMS, ds: dict, cfg: PPOConfig):
    """The mini-epoch / minibatch loop of ContinuousA2CBase.train_epoch (a2c_common.py:1190-1245)."""
    pvec = flatten(P)
    B = ds["obs"].shape[0]
    nmb = B // cfg.minibatch
    mu_ds, sig_ds = ds["mu"].copy(), ds["sigma"].copy()
    log = {"lr": [], "kl": [], "losses": []}
    for mini_ep in range(cfg.mini_epochs):
        for i in range(nmb):
            sl = slice(i * cfg.minibatch, (i + 1) * cfg.minibatch)
            if mini_ep == 0:
                obs_rms.update(ds["obs"][sl])
            xn = obs_rms.norm(ds["obs"][sl])
            g, losses, kl, mu, sigma = minibatch_grad(unflatten(pvec), xn, ds["actions"][sl], ds["old_logp"][sl],
                                                      ds["old_values"][sl], ds["returns"][sl], ds["advantages"][sl],
                                                      mu_ds[sl], sig_ds[sl], cfg)
            if cfg.truncate_grads:
                g, _ = clip_grad(g, cfg.grad_norm)
            pvec = adam.apply(pvec, g, lr, cfg)
            mu_ds[sl], sig_ds[sl] = mu, sigma
            lr = adaptive_lr(lr, kl, cfg.kl_threshold)
            log["lr"].append(lr)
            log["kl"].append(kl)
            log["losses"].append(losses)
    return unflatten(pvec), lr, log
