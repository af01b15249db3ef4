"""Compare the fused agent forward with the unfused GEMM path on a golden case: mac_out per step (debug aid)."""
import os
import sys

import numpy as np
import torch as th

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.golden_utils import Case  # noqa: E402
from tests.gpu_helpers import build, flat_grads  # noqa: E402


def run(case, unfused):
    if unfused:
        os.environ["MQ_PLAN"] = "unfused_fwd"
    else:
        os.environ.pop("MQ_PLAN", None)
    args, buf, mac, learner, logger = build(case)
    np.random.seed(case.sampler_seed)
    batch = buf.sample(case.B)
    batch = batch[:, :batch.max_t_filled()]
    learner.train(batch, 0, case.episodes[0])
    th.cuda.synchronize()
    return [learner.last_intermediate(w).cpu().numpy() for w in (0, 1)] + [flat_grads(learner)], learner.last_stats()


case = Case(sys.argv[1] if len(sys.argv) > 1 else "cfg2_qmix")
(a0, a1, ga), sa = run(case, False)
(b0, b1, gb), sb = run(case, True)
print("stats fused", sa)
print("stats unfused", sb)
for name, a, b in (("online", a0, b0), ("target", a1, b1)):
    d = np.abs(a - b).max(axis=(0, 2, 3))   # per t
    bad = np.nonzero(d > 1e-4)[0]
    print(name, "max|diff|", float(np.abs(a - b).max()), "bad steps", bad[:40].tolist())
    if len(bad):
        t = bad[0]
        e = np.abs(a[:, t] - b[:, t])
        print("  first bad t", t, "per-episode max", e.max(axis=(1, 2))[:8], "per-agent", e.max(axis=(0, 2)))

off = learner_offsets = None
d = np.abs(ga - gb)
print("grad max|diff|", float(d.max()), "rel", float(np.linalg.norm(ga - gb) / np.linalg.norm(gb)))
idx = np.argsort(-d)[:10]
print("worst idx", idx.tolist(), ga[idx].tolist(), gb[idx].tolist())
