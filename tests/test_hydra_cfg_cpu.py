"""Config composition (utils/hydra_cfg.py): the OmegaConf interpolation features the USV yamls use and
the reference's own unmodified train / task yamls composed like Hydra does
(scripts/rlgames_train111.py:113-124, utils/hydra_cfg/hydra_utils.py:36-41)."""
import os

import pytest

from omniisaacgymenvs_loop_amd.tasks.usv_config import build_usv_cfg
from omniisaacgymenvs_loop_amd.utils import hydra_cfg as HC

REF_CFG = "/root/reference/omniisaacgymenvs/cfg"
CFG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "omniisaacgymenvs_loop_amd", "cfg")


def test_relative_absolute_and_resolvers():
    cfg = {
        "seed": 42, "num_envs": "", "experiment": "", "checkpoint": "", "sim_device": "gpu", "rl_device": "cuda:3",
        "task": {"name": "USVVirtual", "env": {"numEnvs": "${resolve_default:512,${...num_envs}}"},
                 "sim": {"use_gpu": '${eq:${...sim_device},"GPU"}', "tag": "${task.name}-x",
                         "inner": {"deep": "${....seed}", "sib": "${.peer}", "peer": 7}}},
        "train": {"params": {"seed": "${...seed}", "load": "${if:${...checkpoint},True,False}",
                             "config": {"name": "${resolve_default:USV,${....experiment}}",
                                        "full": "${.name}", "dev": "${....rl_device}",
                                        "n": "${....task.env.numEnvs}", "has": "${contains:usv,${....task.name}}",
                                        "lst": [1, "${.....seed}"]}}},
    }
    r = HC.resolve(cfg)
    assert r["task"]["env"]["numEnvs"] == 512
    assert r["task"]["sim"]["use_gpu"] is True
    assert r["task"]["sim"]["tag"] == "USVVirtual-x"
    assert r["task"]["sim"]["inner"]["deep"] == 42 and r["task"]["sim"]["inner"]["sib"] == 7
    p = r["train"]["params"]
    assert p["seed"] == 42 and p["load"] is False
    assert p["config"]["name"] == "USV" and p["config"]["full"] == "USV" and p["config"]["dev"] == "cuda:3"
    assert p["config"]["n"] == 512 and p["config"]["has"] is True and p["config"]["lst"] == [1, 42]
    cfg["num_envs"], cfg["experiment"], cfg["checkpoint"] = 64, "run7", "a.pth"
    r = HC.resolve(cfg)
    assert r["train"]["params"]["config"]["n"] == 64 and r["train"]["params"]["config"]["name"] == "run7"
    assert r["train"]["params"]["load"] is True


def test_omegaconf_float_rule(tmp_path):
    f = tmp_path / "a.yaml"
    f.write_text("lr: 1e-4\nb: 3e-4\nc: 1.5\nd: '1e-4'\ne: 12\n")
    d = HC.load_yaml(str(f))
    assert d["lr"] == 1e-4 and isinstance(d["lr"], float) and d["b"] == 3e-4 and d["c"] == 1.5
    assert d["d"] == "1e-4" and d["e"] == 12


def test_cycle_is_an_error():
    with pytest.raises(KeyError):
        HC.resolve({"a": "${b}", "b": "${a}"})


@pytest.mark.skipif(not os.path.isdir(REF_CFG), reason="reference cfg tree not present")
def test_reference_yamls_unmodified():
    """The reference's own USV_PPOcontinuous_MLP.yaml and TEST task yaml, composed and resolved, give the
    packaged configs' values on every key the hot path reads (the packaged task yaml only turns scene
    replay off: the reference's NPZ path is a file on its author's machine)."""
    from omniisaacgymenvs_loop_amd.scripts.rlgames_train import build_config
    ref = build_config({"cfg_dir": REF_CFG, "num_envs": 1024, "seed": 7, "max_iterations": 11})
    ours = build_config({"num_envs": 1024, "seed": 7, "max_iterations": 11})
    pr, po = ref["train"]["params"], ours["train"]["params"]
    assert pr["seed"] == 7 and pr["load_checkpoint"] is False and pr["load_path"] == ""
    assert pr["config"]["name"] == "USV" and pr["config"]["full_experiment_name"] == "USV"
    assert pr["config"]["num_actors"] == 1024 and pr["config"]["max_epochs"] == 11
    for k in ("gamma", "tau", "learning_rate", "lr_schedule", "kl_threshold", "grad_norm", "entropy_coef",
              "truncate_grads", "e_clip", "horizon_length", "minibatch_size", "mini_epochs", "critic_coef",
              "clip_value", "bounds_loss_coef", "normalize_input", "normalize_value", "normalize_advantage",
              "reward_shaper", "env_name", "save_best_after", "save_frequency", "score_to_win"):
        assert pr["config"][k] == po["config"][k], k
    assert pr["network"] == po["network"] and pr["model"] == po["model"] and pr["algo"] == po["algo"]
    assert ref["task"]["env"]["numEnvs"] == 1024 and ref["task_name"] == "USVVirtual"
    assert ref["task"]["sim"]["use_gpu_pipeline"] is True
    assert ref["task"]["env"]["scene_replay"]["enabled"] is True
    ref["task"]["env"]["scene_replay"]["enabled"] = False
    a, b = build_usv_cfg(ref["task"]), build_usv_cfg(ours["task"])
    for name, _ in a._fields_:
        assert getattr(a, name) == getattr(b, name) or (
            hasattr(getattr(a, name), "__len__") and list(getattr(a, name)) == list(getattr(b, name))), name


def test_gotopose_curriculum_defaults_are_gotopose_parameters():
    """spawn_curriculum=True with no other curriculum key takes GoToPoseParameters' defaults
    (USV_task_parameters.py:107-113: 0.5 / 2.5 / 3.0 / 250 / 750), not GoToXYParameters' (:70-76)."""
    from omniisaacgymenvs_loop_amd.tasks.usv_config import build_usv_cfg, load_yaml
    y = load_yaml(os.path.join(CFG, "task", "USV", "USV_Virtual_GoToPose.yaml"))
    tp = y["env"]["task_parameters"]
    for k in list(tp):
        if k.startswith("spawn_curriculum"):
            del tp[k]
    tp["spawn_curriculum"] = True
    c = build_usv_cfg(y)
    assert c.curriculum_on == 1
    assert (c.cur_min_dist, c.cur_max_dist, c.cur_kill_dist, c.cur_warmup, c.cur_end) == \
        pytest.approx((0.5, 2.5, 3.0, 250.0, 750.0))
