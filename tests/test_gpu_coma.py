"""GPU parity of the HIP COMA learner (include/mc_coma.h) against the numpy oracle and the reference's goldens.

Runs through the product path: COMALearner.train -> libmq_learner.so (mc_train_step) on an MI355X.

* teacher-forced steps: before every train() the GPU learner is loaded with the oracle's agent / critic /
  target-critic parameters and both RMSprop states, so each step starts from the same state. Checked per step: the
  critic's Q values the actor used and the TD(lambda) targets, the policy, the nine stats, the agent's clipped
  gradient, and the agent update as RMSprop of the GPU's own gradient (exact up to rounding, as in the QMIX test).
  One train() is T dependent critic optimiser steps: fp32 summation-order noise grows along that chain as it does
  between the oracle and the reference (tests/test_coma_oracle.py), so the critic-side tolerances scale with T.
* free-running step 0 vs the reference golden run, at the oracle test's tolerances.
"""
import numpy as np
import pytest
import torch as th

from tests.golden_utils import COMA_STATS, ComaCase
from tests.gpu_helpers import set_switch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def coma_cases():
    return {}


def get(cases, name):
    if name not in cases:
        cases[name] = ComaCase(name)
    return cases[name]


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(1e-30, np.abs(b).max()))


def load_state(learner, o):
    with th.no_grad():
        learner._agent.copy_(th.from_numpy(o.flat("agent")))
        learner._critic.copy_(th.from_numpy(o.flat("critic")))
        learner._tcritic.copy_(th.from_numpy(o.flat("target_critic")))
        learner._asq.copy_(th.from_numpy(o.flat("sq")))
        learner._csq.copy_(th.from_numpy(o.flat("critic_sq")))
    learner.critic_training_steps = o.critic_training_steps
    learner.last_target_update_step = o.last_target_update_step


@pytest.mark.parametrize("name,steps", [("coma_tiny", 4), ("coma_tiny_masked", 3), ("coma_cfg5", 2)])
def test_coma_teacher_forced(coma_cases, name, steps):
    from oracle.coma_np import OracleCOMALearner
    from tests.gpu_helpers import build_coma
    c = get(coma_cases, name)
    args, buf, mac, learner, logger = build_coma(c)
    o = OracleCOMALearner(c.agent_params, c.critic_params, c.cfg())
    long_chain = c.T > 50
    np.random.seed(c.sampler_seed)
    for k in range(steps):
        batch = buf.sample(c.B)
        assert np.array_equal(batch.ep_ids_np, c.z["ids"][k])
        batch = batch[:, :batch.max_t_filled()]
        nb, _ = c.batch(k)
        load_state(learner, o)
        pa, asq = o.flat("agent").astype(np.float64), o.flat("sq").astype(np.float64)
        mac.action_selector.epsilon = c.epsilon[k]
        learner.train(batch, 1000 * (k + 1), 8 * k)
        st = learner.last_stats()
        so = o.train(nb, 1000 * (k + 1), 8 * k, c.epsilon[k])
        assert int(round(st["critic_steps"])) == len(o.last["critic_grads"])
        # the critic's per-step Q values (what the baseline used) and the TD(lambda) targets
        tq_tol = 1e-3 if long_chain else 1e-5
        assert rel(learner.last_intermediate(1).cpu().numpy(), o.last["targets"]) < 1e-5, (name, k)
        assert rel(learner.last_intermediate(0).cpu().numpy(), o.last["q_vals"]) < tq_tol, (name, k)
        assert rel(learner.last_intermediate(2).cpu().numpy(), o.last["pi"]) < (1e-3 if long_chain else 1e-5)
        for s in COMA_STATS:
            ref = so[s]
            if not long_chain:
                tol = 1e-4 * abs(ref) + 1e-6
            else:
                tol = 2e-5 if s in ("advantage_mean", "coma_loss") else 2e-3 * abs(ref)
            assert abs(st[s] - ref) <= tol, (name, k, s, st[s], ref)
        # agent: clipped gradient vs the oracle's, and RMSprop of the GPU's own gradient exactly
        g = learner._agrad[:learner.n_agent_params].cpu().numpy()
        g_or = np.concatenate([v.ravel() for v in o.last["agent_grads"].values()])
        assert rel(g, g_or) < (5e-2 if long_chain else 1e-4), (name, k)
        g64 = g.astype(np.float64)
        sq_exp = 0.99 * asq + 0.01 * g64 * g64
        p_exp = pa - 5e-4 * g64 / (np.sqrt(sq_exp) + 1e-5)
        assert rel(learner._agent.cpu().numpy(), p_exp) < 1e-6, (name, k)
        assert rel(learner._asq.cpu().numpy(), sq_exp) < 1e-5, (name, k)
        # critic after T RMSprop steps: an O(lr)-per-step band (per-element 1/(sqrt(v)+eps) normalisation)
        dc = np.abs(learner._critic.cpu().numpy() - o.flat("critic")).max()
        assert dc <= (5e-4 * 20 if not long_chain else 5e-4 * c.T), (name, k, dc)
        assert rel(learner._tcritic.cpu().numpy(), o.flat("target_critic")) < (1e-4 if not long_chain else 1e-1)


@pytest.mark.parametrize("name", ["coma_tiny", "coma_cfg5"])
def test_coma_vs_reference_step0(coma_cases, name):
    from tests.gpu_helpers import build_coma
    c = get(coma_cases, name)
    args, buf, mac, learner, logger = build_coma(c)
    np.random.seed(c.sampler_seed)
    batch = buf.sample(c.B)
    batch = batch[:, :batch.max_t_filled()]
    mac.action_selector.epsilon = c.epsilon[0]
    learner.train(batch, 1000, 0)
    st = learner.last_stats()
    for s in COMA_STATS:
        ref = c.z["stat_" + s][0]
        if c.T > 50:
            tol = 4e-5 if s in ("advantage_mean", "coma_loss") else (1e-3 if s == "agent_grad_norm" else 2e-4) * abs(ref)
        else:
            tol = 1e-4 * abs(ref) + 1e-6
        assert abs(st[s] - ref) <= tol, (name, s, st[s], ref)
        assert logger is not None
    if "step_agent" in c.z:
        assert rel(learner._agent.cpu().numpy(), c.z["step_agent"][0]) < 1e-4


def test_mac_pi_logits_policy(coma_cases):
    """BasicMAC.forward with pi_logits (HIP mac step + mc_policy) equals softmax / epsilon floor of the logits."""
    from tests.gpu_helpers import build_coma
    from pymarl_amd.components.episode_buffer import SampledBatch
    from oracle.qlearner_np import agent_unroll
    c = get(coma_cases, "coma_tiny_masked")
    args, buf, mac, learner, logger = build_coma(c)
    ids = c.z["ids"][0]
    batch = SampledBatch(buf, ids)
    nb, _ = c.batch(0)
    logits, _ = agent_unroll(c.agent_params, nb["obs"], nb["actions_onehot"])
    mac.init_hidden(c.B)
    mac.action_selector.epsilon = 0.3
    for t in range(3):
        got = mac.forward(batch, t).cpu().numpy()
        lg = logits[:, t].astype(np.float64).copy()
        av = nb["avail_actions"][:, t]
        lg[av == 0] = -1e10
        e = np.exp(lg - lg.max(-1, keepdims=True))
        sm = e / e.sum(-1, keepdims=True)
        nact = av.sum(-1, keepdims=True)
        with np.errstate(divide="ignore", invalid="ignore"):
            exp = 0.7 * sm + 0.3 / nact
        exp[av == 0] = 0.0
        assert np.abs(got - exp).max() < 1e-5, t


@pytest.mark.parametrize("name", ["coma_tiny_masked", "coma_cfg5"])
def test_coma_chain_matches_three_launch(coma_cases, name, monkeypatch):
    """The persistent critic chain (coma_chain.hpp, default) against the three-launch path (MQ_PLAN coma_chain=0) from
    the same state on the same batches: same products, other fixed summation orders for the bias gradients and
    the norm, so agreement to float rounding amplified along the T-step chain (tolerances as the oracle's)."""
    from oracle.coma_np import OracleCOMALearner
    from tests.gpu_helpers import build_coma
    c = get(coma_cases, name)
    o = OracleCOMALearner(c.agent_params, c.critic_params, c.cfg())
    runs = {}
    for path, env in (("chain", None), ("three_launch", "0")):
        set_switch(monkeypatch, "coma_chain", env)
        args, buf, mac, learner, logger = build_coma(c)
        np.random.seed(c.sampler_seed)
        out = []
        for k in range(2):
            batch = buf.sample(c.B)
            batch = batch[:, :batch.max_t_filled()]
            load_state(learner, o)
            mac.action_selector.epsilon = c.epsilon[k]
            learner.train(batch, 1000 * (k + 1), 8 * k)
            assert learner.critic_path() == path, (name, path)
            out.append((learner.last_stats(), learner._critic.cpu().numpy().copy(), learner._csq.cpu().numpy().copy(),
                        learner.last_intermediate(0).cpu().numpy(), learner._agent.cpu().numpy().copy()))
        runs[path] = out
    long_chain = c.T > 50
    for k in range(2):
        (sa, ca, qa, va, aa), (sb, cb, qb, vb, ab) = runs["chain"][k], runs["three_launch"][k]
        # T = 180 at cfg5: RMSprop's 1 / (sqrt(v) + eps) turns last-bit differences in near-zero gradients into
        # lr-sized steps, so two summation orders drift apart like either does from the oracle. Measured over one
        # coma_cfg5 train() (scripts/coma_diff.py, round 6): chain vs oracle 1.9e-3, three-launch vs oracle 3.5e-3,
        # chain vs three-launch 3.1e-3 (the oracle band of test_coma_teacher_forced is 5e-4 T = 0.09)
        assert np.abs(ca - cb).max() <= (5e-3 if long_chain else 1e-5), (name, k)
        assert rel(va, vb) < (1e-3 if long_chain else 1e-5), (name, k)
        assert rel(qa, qb) < (1e-2 if long_chain else 1e-4), (name, k)
        assert sa["critic_steps"] == sb["critic_steps"]
        for s in COMA_STATS:
            assert np.isfinite(sa[s]), (name, k, s)
            # the oracle test's bands: the actor-side means of small Q differences get an absolute one
            tol = (2e-3 if long_chain else 1e-4) * abs(sb[s]) + 1e-5
            if long_chain and s in ("advantage_mean", "coma_loss"):
                tol = max(tol, 2e-5)
            assert abs(sa[s] - sb[s]) <= tol, (name, k, s, sa[s], sb[s])


@pytest.mark.parametrize("path,env", [("chain", None), ("three_launch", "0")])
def test_coma_skipped_critic_steps(path, env, monkeypatch):
    """Steps whose mask is empty for every episode are skipped (coma_learner.py:121-122): slot 2 and slot 5 are
    made unwritten (filled = 0, no action) in every episode of the masked tiny case. Teacher-forced against the
    oracle through both critic paths; critic_steps counts the live steps only."""
    from oracle.coma_np import OracleCOMALearner
    from tests.gpu_helpers import build_coma
    set_switch(monkeypatch, "coma_chain", env)
    c = ComaCase("coma_tiny_masked")
    for h in (2, 5):
        c.data["filled"][:, h] = 0
        c.data["actions"][:, h] = 0
        c.data["actions_onehot"][:, h] = 0.0
    args, buf, mac, learner, logger = build_coma(c)
    o = OracleCOMALearner(c.agent_params, c.critic_params, c.cfg())
    np.random.seed(c.sampler_seed)
    batch = buf.sample(c.B)
    batch = batch[:, :batch.max_t_filled()]
    nb, _ = c.batch(0)
    load_state(learner, o)
    mac.action_selector.epsilon = c.epsilon[0]
    learner.train(batch, 1000, 0)
    assert learner.critic_path() == path
    st = learner.last_stats()
    so = o.train(nb, 1000, 0, c.epsilon[0])
    live = len(o.last["critic_grads"])
    T = nb["filled"].shape[1] - 1
    assert live <= T - 2, (live, T)   # the two holes were skipped
    assert int(round(st["critic_steps"])) == live
    assert rel(learner.last_intermediate(0).cpu().numpy(), o.last["q_vals"]) < 1e-5
    for s in COMA_STATS:
        assert abs(st[s] - so[s]) <= 1e-4 * abs(so[s]) + 1e-6, (path, s, st[s], so[s])
    dc = np.abs(learner._critic.cpu().numpy() - o.flat("critic")).max()
    assert dc <= 5e-4 * 20, dc


def test_coma_chain_failure_is_loud(monkeypatch):
    """A persistent-chain workgroup that stops flagging (MQ_DIAG coma_fault test hook) makes every workgroup leave
    within the bounded spin: the launch ends, the stats come out NaN with critic_steps = -1 and train() raises.
    The failed train() is rolled back: critic params / square_avg are restored and the actor update is skipped, so
    every parameter and optimiser buffer is bitwise its pre-train value, and the next train() equals a clean
    learner's first train() on the same batch bit for bit."""
    from tests.gpu_helpers import build_coma
    from pymarl_amd._lib import MQError
    set_switch(monkeypatch, "coma_chain", None)
    c = get({}, "coma_tiny")
    args, buf, mac, learner, logger = build_coma(c)
    np.random.seed(c.sampler_seed)
    batch = buf.sample(c.B)
    batch = batch[:, :batch.max_t_filled()]
    mac.action_selector.epsilon = c.epsilon[0]
    snap = lambda l: [t.cpu().numpy().copy() for t in (l._critic, l._csq, l._agent, l._asq, l._tcritic)]  # noqa
    before = snap(learner)
    set_switch(monkeypatch, "coma_fault", "1")
    with pytest.raises(MQError):
        learner.train(batch, 1000, 0)
    assert learner.critic_path() == "chain"
    assert np.isnan(learner._stats[0].item())
    for a, b in zip(before, snap(learner)):
        assert np.array_equal(a, b)
    assert learner.critic_training_steps == 0
    set_switch(monkeypatch, "coma_fault", None)
    learner.train(batch, 2000, 8)
    st = learner.last_stats()
    assert st["critic_steps"] > 0 and np.isfinite(st["critic_loss"])
    _, _, mac2, clean, _ = build_coma(c)
    mac2.action_selector.epsilon = c.epsilon[0]
    clean.train(batch, 2000, 8)
    for a, b in zip(snap(learner), snap(clean)):
        assert np.array_equal(a, b)
    assert learner.last_stats() == clean.last_stats()


def test_coma_chain_bitwise_deterministic(coma_cases, monkeypatch):
    """The persistent chain has no data atomics and sums every reduction in a fixed order: two train() calls from
    the same state on the same batch give bitwise-identical critic parameters, square_avg and stats."""
    from oracle.coma_np import OracleCOMALearner
    from tests.gpu_helpers import build_coma
    set_switch(monkeypatch, "coma_chain", None)
    c = get(coma_cases, "coma_cfg5")
    args, buf, mac, learner, logger = build_coma(c)
    o = OracleCOMALearner(c.agent_params, c.critic_params, c.cfg())
    np.random.seed(c.sampler_seed)
    batch = buf.sample(c.B)
    batch = batch[:, :batch.max_t_filled()]
    outs = []
    for _ in range(2):
        load_state(learner, o)
        mac.action_selector.epsilon = c.epsilon[0]
        learner.train(batch, 1000, 0)
        assert learner.critic_path() == "chain"
        outs.append((learner._critic.cpu().numpy().copy(), learner._csq.cpu().numpy().copy(),
                     learner._stats.cpu().numpy().copy()))
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b)
