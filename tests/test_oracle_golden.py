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


@pytest.mark.parametrize("name", ["tiny_qmix", "tiny_vdn", "tiny_iql"])
def test_huber_head_matches_torch(golden_cases, name, monkeypatch):
    """The oracle's opt-in Huber head (no reference counterpart; the L2 head above is pinned to the reference): its
    loss and d loss / d Q_tot equal torch's huber_loss(td * mask, 0, delta, sum) / mask.sum() and its autograd."""
    import torch as th
    import oracle.qlearner_np as onp
    c = golden_cases[name]
    delta = 1.0
    o = OracleQLearner(c.agent_params, c.mixer_params, dict(c.cfg(), huber_delta=delta))
    b, _ = c.batch(0)
    fw = o.forward(b, keep_cache=True)
    seen = {}
    real_qb = onp.qmix_backward
    monkeypatch.setattr(onp, "qmix_backward", lambda mp, cache, dy: (seen.setdefault("dy", dy), real_qb(mp, cache, dy))[1])
    real_ab = onp.agent_backward
    monkeypatch.setattr(onp, "agent_backward", lambda p, cache, dmac: (seen.setdefault("dmac", dmac), real_ab(p, cache, dmac))[1])
    o.gradients(b, fw=fw)
    q = th.tensor(np.asarray(fw["q_tot"], np.float64), requires_grad=True)
    m = th.tensor(np.asarray(fw["mask"], np.float64))
    tgt = th.tensor(np.asarray(fw["targets"], np.float64))
    loss = th.nn.functional.huber_loss((q - tgt) * m, th.zeros_like(q), reduction="sum", delta=delta) / m.sum()
    loss.backward()
    ax = np.abs(fw["td"] * fw["mask"])[fw["mask"] > 0]
    assert (ax <= delta).any() and (ax > delta).any()   # both regimes
    assert abs(fw["loss"] - loss.item()) <= 1e-5 * abs(loss.item())
    g = q.grad.numpy()
    if c.cfg()["mixer"] == "qmix":
        got = seen["dy"].reshape(g.shape)
    else:   # vdn / iql: the Q_tot gradient lands on the chosen actions' Q (one per agent)
        d = seen["dmac"][:, :-1]
        got = d.sum(-1) if c.cfg()["mixer"] == "none" else d.sum(-1)[..., :1]
    assert rel_err(got, g) < 1e-5
