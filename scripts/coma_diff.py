"""Diagnostic: how far the persistent critic chain, the three-launch critic path and the numpy oracle drift apart over
one coma_cfg5 train() (T = 180 dependent RMSprop steps) from the same state. Prints max |dP| of the critic params for
each pair and how many elements differ by more than 1e-3. Run once per library (MQ_LEARNER_LIB) on a GPU box.
Usage: python scripts/coma_diff.py [case]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.coma_np import OracleCOMALearner  # noqa: E402
from tests.golden_utils import ComaCase  # noqa: E402
from tests.gpu_helpers import build_coma  # noqa: E402
from tests.test_gpu_coma import load_state  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "coma_cfg5"
c = ComaCase(name)
out = {}
for path, env in (("chain", None), ("three_launch", "coma_chain=0")):
    if env:
        os.environ["MQ_PLAN"] = env
    else:
        os.environ.pop("MQ_PLAN", None)
    o = OracleCOMALearner(c.agent_params, c.critic_params, c.cfg())
    args, buf, mac, learner, logger = build_coma(c)
    np.random.seed(c.sampler_seed)
    batch = buf.sample(c.B)
    batch = batch[:, :batch.max_t_filled()]
    nb, _ = c.batch(0)
    load_state(learner, o)
    mac.action_selector.epsilon = c.epsilon[0]
    learner.train(batch, 1000, 0)
    assert learner.critic_path() == path
    out[path] = learner._critic.cpu().numpy().copy()
    if path == "chain":
        o.train(nb, 1000, 0, c.epsilon[0])
        out["oracle"] = o.flat("critic").copy()
for a, b in (("chain", "three_launch"), ("chain", "oracle"), ("three_launch", "oracle")):
    d = np.abs(out[a] - out[b])
    print(f"{name} {a} vs {b}: max {d.max():.3e}, > 1e-3: {(d > 1e-3).sum()}, > 3e-4: {(d > 3e-4).sum()} of {d.size}")
