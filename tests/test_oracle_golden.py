"""Pin the numpy oracle (oracle/qlearner_np.py) to the golden vectors produced by the reference learner.

The fixtures come from tests/golden/make_golden.py, which runs the reference QLearner.train (q_learner.py:37-116)
in this container. Tolerances: fp32 reduction order differs between numpy/OpenBLAS and torch/oneDNN, so
intermediates agree to ~1e-6 relative; the multi-step loss trajectory agrees to 1e-4 relative for the steps
before the training dynamics amplify that rounding (see DESIGN.md "Parity"), and the greedy actions agree
exactly wherever the reference's top-2 margin exceeds MARGIN_EPS.
"""
import numpy as np
import pytest

from oracle.qlearner_np import OracleQLearner, max_t_filled, sample_ids
from tests.golden_utils import rel_err

STATS = ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]
MARGIN_EPS = 1e-5
# steps whose loss/stats must match to 1e-4 rel; later steps of the 20-step cfg2 QMIX run drift chaotically
# (measured oracle-vs-reference: 4e-6 at step 10, 6e-5 at step 13, 1.2e-3 at step 16) and get 1e-2.
TIGHT_STEPS = 12


@pytest.mark.parametrize("name", ["tiny_qmix", "tiny_vdn", "tiny_qmix_full", "cfg2_qmix_ragged", "tiny_iql",
                                  "tiny_qmix_nodq", "tiny_qmix_nola", "tiny_vdn_noid", "tiny_qmix_bare"])
def test_intermediates_and_params(golden_cases, name):
    c = golden_cases[name]
    o = OracleQLearner(c.agent_params, c.mixer_params, c.cfg())
    for k in range(c.steps):
        b, _ = c.batch(k)
        if k == 0 and "step0_mac_out" in c.z:
            fw = o.forward(b)
            for key in ["mac_out", "target_mac_out", "chosen", "target_max", "q_tot", "targets", "td", "mask"]:
                assert rel_err(fw[key], c.z["step0_" + key]) < 2e-6, key
            assert np.array_equal(fw["cur_max_actions"], c.z["step0_cur_max_actions"])
        st = o.train(b, 1000 * k, c.episodes[k])
        for s in STATS:
            assert abs(st[s] - c.z["stat_" + s][k]) <= 1e-5 * abs(c.z["stat_" + s][k]) + 1e-7, (k, s)
        if k == 0 and "step0_grads_clipped" in c.z:
            g = np.concatenate([v.ravel() for v in o.last["grads"].values()])
            assert rel_err(g, c.z["step0_grads_clipped"]) < 2e-6
        if "step_params" in c.z:
            assert rel_err(o.flat(), c.z["step_params"][k]) < 5e-5
    if "sqavg_final" in c.z:
        assert rel_err(o.flat("sq"), c.z["sqavg_final"]) < 2e-6
    assert rel_err(o.flat("targets"), c.z["targets_final"]) < 5e-5


@pytest.mark.parametrize("name", ["cfg2_qmix", "cfg2_vdn", "cfg3_vdn", "cfg3_qmix", "cfg4_qmix", "cfg2_iql", "rw2_qmix",
                                  "rw4_vdn", "wide_qmix", "cfg3_vdn_b128", "cfg2_qmix_nodq", "cfg1_qmix", "cfg1_vdn"])
def test_cfg2_trajectory(golden_cases, name):
    c = golden_cases[name]
    o = OracleQLearner(c.agent_params, c.mixer_params, c.cfg())
    for k in range(c.steps):
        b, _ = c.batch(k)
        if k < c.z["cur_max_actions"].shape[0]:
            fw = o.forward(b)
            Tk = fw["cur_max_actions"].shape[1]   # ragged fixtures pad the time axis
            ref = c.z["cur_max_actions"][k][:, :Tk]
            clear = c.z["margin"][k][:, :Tk] > MARGIN_EPS
            assert np.array_equal(fw["cur_max_actions"][clear], ref[clear].astype(np.int64))
        st = o.train(b, 1000 * k, c.episodes[k])
        tol = 1e-4 if k < TIGHT_STEPS else 1e-2
        for s in STATS:
            assert abs(st[s] - c.z["stat_" + s][k]) <= tol * abs(c.z["stat_" + s][k]) + 1e-6, (k, s)


def test_sampler_ids_match_reference(golden_cases):
    for name in ["tiny_qmix", "cfg2_qmix"]:
        c = golden_cases[name]
        np.random.seed(c.sampler_seed)
        for k in range(c.steps):
            assert np.array_equal(sample_ids(c.n_episodes, c.B), c.z["ids"][k])


def test_max_t_filled_ragged(golden_cases):
    c = golden_cases["cfg2_qmix_ragged"]
    for k in range(c.steps):
        ids = c.z["ids"][k]
        b, _ = c.batch(k)
        assert b["filled"].shape[1] == max_t_filled(c.data["filled"][ids])
