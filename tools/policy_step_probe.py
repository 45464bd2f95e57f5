"""Standalone k_policy_step timing at N envs: median of 40 launches (HIP events on the launching stream), the
rollout's 16 slots in turn, Philox draws.   python3 tools/policy_step_probe.py 131072 [label]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from omniisaacgymenvs_loop_amd import _capi as c  # noqa: E402
from tests.test_ppo_gpu import _agent  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
label = sys.argv[2] if len(sys.argv) > 2 else ""
ag = _agent(n, 8192)
rng = np.random.default_rng(3)
obs = torch.tensor(rng.normal(0, 1, (n, 33)).astype(np.float32), device="cuda:0")
dprev = torch.zeros(n, device="cuda:0", dtype=torch.int64)
s = torch.cuda.current_stream()
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(40)]
for it in range(50):
    t = it % 16
    k = it - 10
    if k >= 0:
        ev[k][0].record(s)
    c.call("ppo_policy_step", c.byref(ag.cfg), c.ptr(ag.model_params), c.ptr(ag.obs_rms), c.ptr(ag.val_rms),
           c.ptr(obs), t, c.ptr(ag.exp_obs), c.ptr(ag.exp_act), c.ptr(ag.exp_nlp), c.ptr(ag.exp_val), c.ptr(ag.exp_mu),
           c.ptr(ag.exp_sigma), c.ptr(ag.exp_done), c.ptr(dprev), c.ptr(ag.actions), 7, it, None, None, s.cuda_stream)
    if k >= 0:
        ev[k][1].record(s)
torch.cuda.synchronize()
us = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
flop = 41984.0 * n
print(f"{label} envs {n}: k_policy_step median {us[len(us) // 2]:.2f} us (min {us[0]:.2f}), "
      f"{flop / (us[len(us) // 2] * 1e-6) / 1e12:.1f} TFLOP/s")
