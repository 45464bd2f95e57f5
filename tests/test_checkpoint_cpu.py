"""rl_games checkpoint layout with a narrower observation (priv_dim 4 -> obs_dim 29).

The device network always has PPO_NIN inputs; a 29-input reference network maps onto it with
zero W1 columns (and RMS slots) past column 29, so a checkpoint round trip is exact and the
padded forward equals the reference's 29-input forward (a2c_common.py:590-621 layout).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from omniisaacgymenvs_loop_amd.rl_games import checkpoint as C


def _reference_shaped(obs_dim, seed=0):
    g = torch.Generator().manual_seed(seed)
    sd = {}
    for k, s in C.PARAM_LAYOUT:
        shape = (C.NH, obs_dim) if k == C.W1_KEY else s
        sd[k] = torch.randn(*shape, generator=g)
    sd["value_mean_std.running_mean"] = torch.randn(1, generator=g).double()
    sd["value_mean_std.running_var"] = torch.rand(1, generator=g).double() + 0.5
    sd["value_mean_std.count"] = torch.tensor(123.0, dtype=torch.float64)
    sd["running_mean_std.running_mean_std.state.running_mean"] = torch.randn(obs_dim, generator=g).double()
    sd["running_mean_std.running_mean_std.state.running_var"] = torch.rand(obs_dim, generator=g).double() + 0.5
    sd["running_mean_std.running_mean_std.state.count"] = torch.tensor(456.0, dtype=torch.float64)
    return sd


@pytest.mark.parametrize("obs_dim", [29, C.NIN])
def test_model_round_trip(obs_dim):
    sd = _reference_shaped(obs_dim)
    params = torch.full((C.NPARAM,), 7.0)
    obs_rms = torch.zeros(2 * C.NIN + 1, dtype=torch.float64)
    obs_rms[C.NIN:2 * C.NIN] = 1.0
    val_rms = torch.zeros(3, dtype=torch.float64)
    C.load_model_state_dict(sd, params, obs_rms, val_rms, obs_dim)
    w1 = C.split_flat(params)[C.W1_KEY]
    assert w1.shape == (C.NH, C.NIN)
    assert float(w1[:, obs_dim:].abs().sum()) == 0.0   # zero pad columns
    assert float(obs_rms[obs_dim:C.NIN].abs().sum()) == 0.0 and bool((obs_rms[C.NIN + obs_dim:2 * C.NIN] == 1).all())
    back = C.model_state_dict(params, obs_rms, val_rms, obs_dim)
    assert set(back) == set(sd)
    for k, t in sd.items():
        assert tuple(back[k].shape) == tuple(t.shape), k
        torch.testing.assert_close(back[k].double(), t.double(), rtol=0, atol=1e-6 if t.dtype == torch.float32 else 0)


def test_padded_forward_equals_narrow_forward():
    sd = _reference_shaped(29, seed=3)
    params = torch.zeros(C.NPARAM)
    C.load_model_state_dict(sd, params, torch.zeros(2 * C.NIN + 1, dtype=torch.float64),
                            torch.zeros(3, dtype=torch.float64), 29)
    w1 = C.split_flat(params)[C.W1_KEY]
    x = torch.randn(64, 29, dtype=torch.float64)
    xp = torch.cat([x, torch.zeros(64, C.NIN - 29, dtype=torch.float64)], 1)
    np.testing.assert_array_equal((xp @ w1.double().T).numpy(), (x @ sd[C.W1_KEY].double().T).numpy())


def test_optimizer_round_trip_narrow():
    g = torch.Generator().manual_seed(1)
    m = torch.randn(C.NPARAM, generator=g)
    v = torch.rand(C.NPARAM, generator=g)
    # pad columns of a narrow network never receive gradient: zero moments
    for t in (m, v):
        C.split_flat(t)[C.W1_KEY][:, 29:] = 0
    osd = C.optimizer_state_dict(m, v, 17, 3e-4, obs_dim=29)
    assert osd["state"][1]["exp_avg"].shape == (C.NH, 29)
    m2, v2 = torch.zeros_like(m), torch.zeros_like(v)
    step, lr = C.load_optimizer_state_dict(osd, m2, v2, obs_dim=29)
    assert step == 17 and lr == pytest.approx(3e-4)
    torch.testing.assert_close(m2, m, rtol=0, atol=0)
    torch.testing.assert_close(v2, v, rtol=0, atol=0)


def test_shape_mismatch_raises():
    sd = _reference_shaped(29)
    with pytest.raises(ValueError):
        C.load_model_state_dict(sd, torch.zeros(C.NPARAM), torch.zeros(2 * C.NIN + 1, dtype=torch.float64),
                                torch.zeros(3, dtype=torch.float64), C.NIN)


# ---- the reference's own checkpoint (811_3.5.../last_USV_ep_5450_rew_38.54975.pth, 13-input net) ----
import os  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF_CKPT = "/root/reference/811_3.5刹车_____（复件）/last_USV_ep_5450_rew_38.54975.pth"


def ckpt811_dict(d):
    """The reference's checkpoint dict rebuilt from the fixture arrays (a2c_common.py:590-606 layout)."""
    from collections import OrderedDict
    model = OrderedDict((str(k), torch.from_numpy(np.array(d["sd__" + str(k)]))) for k in d["keys"])
    state = {i: {"step": torch.tensor(float(d["opt_step"])), "exp_avg": torch.from_numpy(d[f"opt_m_{i}"]),
                 "exp_avg_sq": torch.from_numpy(d[f"opt_v_{i}"])} for i in range(len(C.PARAM_LAYOUT))}
    group = {"lr": float(d["opt_lr"]), "betas": (0.9, 0.999), "eps": 1e-08, "weight_decay": 0.0, "amsgrad": False,
             "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
             "params": list(range(len(C.PARAM_LAYOUT)))}
    return {"model": model, "epoch": int(d["epoch"]), "optimizer": {"state": state, "param_groups": [group]},
            "frame": int(d["frame"]), "last_mean_rewards": np.float32(d["last_mean_rewards"]), "env_state": None}


def test_reference_checkpoint_key_set_and_dtypes(golden):
    """The 811 checkpoint's key set, shapes and dtypes (pinned in the fixture), read by load_checkpoint with
    weights_only=True when the reference tree is present; its model maps onto the padded device vector and back
    bit for bit."""
    d = golden("ckpt811.npz")
    assert [str(k) for k in d["top_keys"]] == ["model", "epoch", "optimizer", "frame", "last_mean_rewards",
                                               "env_state"]
    keys = [str(k) for k in d["keys"]]
    assert keys[:6] == ["value_mean_std.running_mean", "value_mean_std.running_var", "value_mean_std.count",
                        "running_mean_std.running_mean_std.state.running_mean",
                        "running_mean_std.running_mean_std.state.running_var",
                        "running_mean_std.running_mean_std.state.count"]
    assert keys[6:] == [k for k, _ in C.PARAM_LAYOUT]
    assert d["sd__" + C.W1_KEY].shape == (C.NH, 13) and d["sd__" + C.W1_KEY].dtype == np.float32
    assert d["sd__value_mean_std.count"].dtype == np.float64 and d["sd__value_mean_std.count"].shape == ()
    if os.path.exists(REF_CKPT):
        ck = C.load_checkpoint(REF_CKPT)
        assert list(ck.keys()) == [str(k) for k in d["top_keys"]]
        assert list(ck["model"].keys()) == keys
        for k in keys:
            t = ck["model"][k]
            assert t.dtype == torch.from_numpy(np.array(d["sd__" + k])).dtype, k
            np.testing.assert_array_equal(t.numpy(), d["sd__" + k])
    sd = ckpt811_dict(d)["model"]
    params = torch.zeros(C.NPARAM)
    obs_rms = torch.zeros(2 * C.NIN + 1, dtype=torch.float64)
    obs_rms[C.NIN:2 * C.NIN] = 1.0
    val_rms = torch.zeros(3, dtype=torch.float64)
    C.load_model_state_dict(sd, params, obs_rms, val_rms, 13)
    back = C.model_state_dict(params, obs_rms, val_rms, 13)
    assert list(back.keys()) == keys
    for k in keys:
        assert back[k].dtype == sd[k].dtype and tuple(back[k].shape) == tuple(sd[k].shape), k
        torch.testing.assert_close(back[k], sd[k], rtol=0, atol=0)


def test_reference_checkpoint_optimizer_round_trip(golden):
    d = golden("ckpt811.npz")
    osd = ckpt811_dict(d)["optimizer"]
    m, v = torch.zeros(C.NPARAM), torch.zeros(C.NPARAM)
    step, lr = C.load_optimizer_state_dict(osd, m, v, 13)
    assert step == float(d["opt_step"]) and lr == pytest.approx(float(d["opt_lr"]))
    back = C.optimizer_state_dict(m, v, step, lr, 0.0, 13)
    for i in range(len(C.PARAM_LAYOUT)):
        torch.testing.assert_close(back["state"][i]["exp_avg"], osd["state"][i]["exp_avg"], rtol=0, atol=0)
        torch.testing.assert_close(back["state"][i]["exp_avg_sq"], osd["state"][i]["exp_avg_sq"], rtol=0, atol=0)


@pytest.mark.parametrize("steps", [0, 1999, 224_000, 2_100_000, 3_000_000])
def test_grad_scaler_state_stays_finite_and_loads(steps):
    """The mixed_precision checkpoint's 'scaler' entry stays a finite fp32 scale however long the run
    (a2c_continuous.get_full_state_weights at 3000 epochs x 1024 steps), and a reference GradScaler loads it."""
    import math
    import torch
    st = C.grad_scaler_state(steps)
    assert math.isfinite(st["scale"]) and torch.isfinite(torch.tensor(st["scale"], dtype=torch.float32))
    assert 65536.0 <= st["scale"] <= C.GRAD_SCALE_MAX and 0 <= st["_growth_tracker"] < 2000
    sc = torch.amp.GradScaler("cpu")
    sc.load_state_dict(st)
    assert sc.get_scale() == st["scale"] and sc.state_dict()["_growth_tracker"] == st["_growth_tracker"]
