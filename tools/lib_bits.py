"""Bits of a short training run under the library USV_HIP_LIB names (run once per library, then compare):
    python tools/lib_bits.py OUT.npz [epochs]      -> params, Adam moments, env state, experience, meters
    python tools/lib_bits.py --compare A.npz B.npz  -> every array bit-identical?"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]
    for k in a.files:
        print("%-10s %s" % (k, "same bits" if k not in bad else
                            "DIFFERS (max abs %.3g)" % float(np.abs(a[k].astype(np.float64) - b[k]).max())))
    sys.exit(1 if bad else 0)

import torch  # noqa: E402
from tests.test_train_gpu import _agent_env  # noqa: E402

epochs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
env, task, ag = _agent_env(4096, 8192, True)
ag.obs = ag.env_reset()
for _ in range(epochs):
    ag.train_epoch()
torch.cuda.synchronize()
np.savez(sys.argv[1], params=ag.model_params.cpu().numpy(), m=ag.adam_m.cpu().numpy(), v=ag.adam_v.cpu().numpy(),
         state=task.state.cpu().numpy(), exp_nlp=ag.exp_nlp.cpu().numpy(), exp_mu=ag.exp_mu.cpu().numpy(),
         kls=ag.kls.cpu().numpy(), meter=ag.meter.cpu().numpy())
print("saved", sys.argv[1])
