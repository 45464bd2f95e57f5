"""The overlapped step (include/usv_hip.h: usv_field_stage + usv_env_step_part(.., 3) + usv_env_step_late;
USVVirtual.env_step(.., overlap=True); A2CAgent._play_steps_overlapped): the reset envs' potential fields
build on a side stream while every env steps and the next policy step runs; the reset envs' potential-
dependent reward (static_obs.py:335-657) finishes after their fields.  It must give exactly the plain
sequential step's results (same kernels, same inputs, same operation order)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _snap(task):
    torch.cuda.synchronize()
    return {"state": task.state.cpu().numpy(), "obs": task.obs_buf_t.cpu().numpy(), "rew": task.rew_buf.cpu().numpy(),
            "dones": task.dones.cpu().numpy(), "hist": task.hist.cpu().numpy(), "stats": task.stats.cpu().numpy(),
            "ibuf": task.ibuf.cpu().numpy(), "obst": task.obst.cpu().numpy(), "extras": task.extras_buf.cpu().numpy(),
            "sdf": task.field.cpu().numpy(), "cost": task.sdf.cpu().numpy(), "fnorm": task.fnorm.cpu().numpy()}


@pytest.mark.parametrize("half", ["0", "1"])
@pytest.mark.parametrize("n", [1024, 8192])
def test_overlapped_env_step_equals_plain_step(monkeypatch, n, half):
    """Eight steps from the first (every env reset: the 8,192-env case runs k_field_place's grid stride and
    several rounds of the sweep grid on the side stream), random actions, Philox draws: state, obs, reward,
    dones, history, episode sums, obstacles, extras and every field bit-identical after each step.  half: the
    side stream's sweeps as the packed 10 x 10-tile kernel ("0") or the small-batch 10 x 5-tile kernel ("1",
    USV_FIELD_HALF) against the plain step's 10 x 10-tile k_field_wave."""
    monkeypatch.setenv("USV_FIELD_HALF", half)
    from omniisaacgymenvs_loop_amd.tasks.usv_config import load_yaml
    from tests.test_oracle_golden import TEST_YAML
    from omniisaacgymenvs_loop_amd.tasks.usv_virtual import USVVirtual
    cfg = load_yaml(TEST_YAML)
    plain = USVVirtual(cfg, num_envs=n, device=DEV, seed=7)
    over = USVVirtual(cfg, num_envs=n, device=DEV, seed=7)
    rng = np.random.default_rng(3)
    for t in range(8):
        a = torch.tensor(rng.uniform(-1, 1, (n, 2)).astype(np.float32), device=DEV)
        plain.env_step(a)
        over.env_step(a, overlap=True)
        over.join_step()
        sp, so = _snap(plain), _snap(over)
        for k in sp:
            np.testing.assert_array_equal(so[k], sp[k], err_msg=f"{k} step {t}")


@pytest.mark.parametrize("reset_on_side,late_on_join,store_defer,fold_late",
                         [("0", "0", "1", "1"), ("1", "0", "1", "1"), ("0", "1", "1", "1"), ("0", "1", "0", "0")])
def test_overlapped_rollout_equals_sequential(monkeypatch, reset_on_side, late_on_join, store_defer, fold_late):
    """A2CAgent.play_steps with the overlapped env step (policy n+1 beside step n's field kernels) vs the
    sequential loop: every experience buffer, the meters and the env state bit-identical after two epochs
    of rollouts (the first from the all-env reset); also with the chained steps' reset and obstacle placement
    on the side stream (USV_RESET_ON_SIDE=1, usv_reset_part), and with step n's reward store inside step n + 1
    after its fork (USV_STORE_DEFER, the default) or after each join, the episode-extras fold after the fork
    (USV_FOLD_AFTER_FORK, the default) or inside usv_reset."""
    import os
    from tests.test_train_gpu import _agent_env
    monkeypatch.setenv("USV_RESET_ON_SIDE", reset_on_side)
    monkeypatch.setenv("USV_LATE_ON_JOIN", late_on_join)
    monkeypatch.setenv("USV_STORE_DEFER", store_defer)
    monkeypatch.setenv("USV_FOLD_AFTER_FORK", fold_late)
    runs = []
    for ov in ("0", "1"):
        os.environ["USV_STEP_OVERLAP"] = ov
        try:
            env, task, ag = _agent_env(1024, 4096, False)
            ag.obs = ag.env_reset()
            for _ in range(2):
                ag.play_steps()
            torch.cuda.synchronize()
            runs.append({k: getattr(ag, k).cpu().numpy() for k in
                         ("exp_obs", "exp_act", "exp_nlp", "exp_val", "exp_mu", "exp_sigma", "exp_done", "exp_rew",
                          "meter", "cur_rew", "cur_len")} | {"state": task.state.cpu().numpy()})
        finally:
            os.environ.pop("USV_STEP_OVERLAP", None)
    for k in runs[0]:
        np.testing.assert_array_equal(runs[1][k], runs[0][k], err_msg=k)
