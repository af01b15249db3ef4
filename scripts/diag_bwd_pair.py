"""Per-parameter gradient difference between the one-chain-wave BPTT (MQ_BWD_PAIR=1) and the fused BPTT on the
same first step (diagnostic for gru_bwd_pair.hpp). Usage: python scripts/diag_bwd_pair.py [case]"""
import os
import sys

import numpy as np
import torch as th

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pymarl_amd import _lib  # noqa: E402
from tests.gpu_helpers import build, flat_grads  # noqa: E402
from tests.test_gpu_parity import Case  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "cfg2_qmix"
case = Case(name)
out = {}
for v in ("0", "1"):
    os.environ["MQ_BWD_PAIR"] = v
    args, buf, mac, learner, logger = build(case)
    np.random.seed(case.sampler_seed)
    batch = buf.sample(case.B)
    learner.train(batch[:, :batch.max_t_filled()], 0, case.episodes[0])
    th.cuda.synchronize()
    out[v] = (flat_grads(learner), learner.last_plan())
print("plans", out["0"][1]["fused_bwd"], out["1"][1]["fused_bwd"])
g0, g1 = out["0"][0], out["1"][0]
off = [int(x) for x in learner._handle.offsets]
names = _lib.PARAM_NAMES
if off is None:
    print("no offsets; total rel", np.abs(g0 - g1).max() / np.abs(g0).max())
else:
    for i, nm in enumerate(names):
        a, b = off[i], off[i + 1]
        if b <= a:
            continue
        x, y = g0[a:b], g1[a:b]
        print("%-14s n=%6d  max|d|=%.3e  max|g|=%.3e  rel=%.3e" % (nm, b - a, np.abs(x - y).max(), np.abs(x).max(),
                                                                np.abs(x - y).max() / max(np.abs(x).max(), 1e-30)))
a, b = off[0], off[1]
I = (b - a) // 64
x, y = g0[a:b].reshape(64, I), g1[a:b].reshape(64, I)
bad = np.abs(x - y) > 1e-3 * np.abs(x).max()
print("fc1.weight bad rows (units):", np.where(bad.any(1))[0].tolist()[:64])
print("fc1.weight bad cols (inputs):", np.where(bad.any(0))[0].tolist()[:112])
r = y[bad] / np.where(x[bad] == 0, 1, x[bad])
print("ratio new/old on bad: median %.3f min %.3f max %.3f" % (np.median(r), r.min(), r.max()) if r.size else "none")
print("unit 0 old", np.round(x[0, :8], 5).tolist(), "new", np.round(y[0, :8], 5).tolist())
