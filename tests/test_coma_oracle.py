"""Pin the numpy COMA oracle (oracle/coma_np.py) to the golden vectors of the reference COMALearner.

The fixtures come from tests/golden/make_golden_coma.py, which runs the reference COMALearner.train
(coma_learner.py:32-148) in this container. Every train() is T sequential critic RMSprop steps followed by one agent
step, so the per-step stats get 1e-4 relative; parameters after each step 1e-4 of the tensor max.

At the cfg5 shape (T = 180 critic RMSprop steps per train) fp32 summation-order noise (numpy/OpenBLAS vs
torch/oneDNN) is amplified by RMSprop's per-element normalisation along the critic chain, as it is along QMIX
trajectories (DESIGN.md "Parity"): step 0's critic stats still agree to ~5e-6, but advantage_mean and coma_loss are
means of advantages that cancel to ~1e-4 of their own scale, so they are held to an absolute 2e-5 there, and later
steps (a different valid trajectory) to a 2 % band.
"""
import numpy as np
import pytest

from oracle.coma_np import OracleCOMALearner
from tests.golden_utils import COMA_STATS, ComaCase, rel_err


@pytest.fixture(scope="module")
def coma_cases():
    return {}


def get(cases, name):
    if name not in cases:
        cases[name] = ComaCase(name)
    return cases[name]


@pytest.mark.parametrize("name", ["coma_tiny", "coma_tiny_masked", "coma_cfg5"])
def test_coma_oracle_vs_reference(coma_cases, name):
    c = get(coma_cases, name)
    o = OracleCOMALearner(c.agent_params, c.critic_params, c.cfg())
    for k in range(c.steps):
        b, _ = c.batch(k)
        st = o.train(b, 1000 * (k + 1), 8 * k, c.epsilon[k])
        long_chain = c.T > 50
        for s in COMA_STATS:
            ref = c.z["stat_" + s][k]
            if not long_chain:
                tol = 1e-4 * abs(ref) + 1e-6
            elif k == 0:
                tol = 2e-5 if s in ("advantage_mean", "coma_loss") else 1e-4 * abs(ref)
            else:
                tol = 2e-2 * abs(ref) + (2e-4 if s in ("advantage_mean", "coma_loss") else 0.0)
            assert abs(st[s] - ref) <= tol, (name, k, s, st[s], ref)
        if k == 0 and "step0_agent_grads" in c.z:
            g = np.concatenate([v.ravel() for v in o.last["agent_grads"].values()])
            assert rel_err(g, c.z["step0_agent_grads"]) < 1e-4
            gc = np.concatenate([v.ravel() for v in o.last["critic_grads"][-1].values()])
            assert rel_err(gc, c.z["step0_critic_grads_last"]) < 1e-4
        if "step_agent" in c.z:
            assert rel_err(o.flat("agent"), c.z["step_agent"][k]) < 1e-4, (name, k)
            assert rel_err(o.flat("critic"), c.z["step_critic"][k]) < 1e-4, (name, k)
            assert rel_err(o.flat("target_critic"), c.z["step_target_critic"][k]) < 1e-4, (name, k)
            assert rel_err(o.flat("sq"), c.z["step_sq"][k]) < 1e-4, (name, k)
            assert rel_err(o.flat("critic_sq"), c.z["step_critic_sq"][k]) < 1e-4, (name, k)
    assert o.critic_training_steps == int(c.z["critic_training_steps"])
