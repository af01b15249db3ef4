"""Standalone module forwards on the GPU (the module API outside train()): QMixer.forward (qmix.py:28-47, HIP
mq_qmix_forward) and COMACritic.forward (coma.py:22-58, HIP mc_critic_forward), against outputs the REFERENCE
modules produced on the golden cases (tests/golden/make_golden.py, make_golden_coma.py) and against the oracle at
the cfg2 / cfg3 mixer shapes."""
import numpy as np
import pytest
import torch as th

from tests.golden_utils import Case, ComaCase

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(1e-30, np.abs(b).max()))


def test_qmixer_forward_vs_reference():
    from tests.gpu_helpers import build
    case = Case("tiny_qmix")
    args, buf, mac, learner, logger = build(case)
    ids = case.z["ids"][0]
    max_t = int(case.z["step0_max_t"])
    state = th.as_tensor(case.data["state"][ids][:, :max_t], device="cuda")
    chosen = th.as_tensor(case.z["step0_chosen"], device="cuda")
    q_tot = learner.mixer(chosen, state[:, :-1])
    assert q_tot.shape == (case.B, max_t - 1, 1)
    assert rel(q_tot.cpu().numpy(), case.z["step0_q_tot"]) < 1e-5
    tmax = th.as_tensor(case.z["step0_target_max"], device="cuda")
    tq = learner.target_mixer(tmax, state[:, 1:])
    assert rel(tq.cpu().numpy(), case.z["step0_target_q_tot"]) < 1e-5


@pytest.mark.parametrize("name", ["cfg2_qmix", "cfg3_qmix"])
def test_qmixer_forward_vs_oracle(name):
    from oracle.qlearner_np import qmix_forward
    from tests.gpu_helpers import build
    case = Case(name)
    args, buf, mac, learner, logger = build(case)
    rng = np.random.default_rng(0)
    B, T = case.B, case.T
    qs = rng.standard_normal((B, T, case.n)).astype(np.float32)
    st = case.data["state"][case.z["ids"][0]][:, :T]
    got = learner.mixer(th.as_tensor(qs, device="cuda"), th.as_tensor(st, device="cuda")).cpu().numpy()
    ref, _ = qmix_forward(learner_mixer_params(case), qs, st, case.n)
    assert rel(got, ref) < 1e-5


def learner_mixer_params(case):
    return {k: np.asarray(v, np.float32) for k, v in case.mixer_params.items()}


@pytest.mark.parametrize("name", ["coma_tiny", "coma_tiny_masked"])
def test_coma_critic_forward_vs_reference(name):
    from pymarl_amd.components.episode_buffer import SampledBatch
    from tests.gpu_helpers import build_coma
    case = ComaCase(name)
    args, buf, mac, learner, logger = build_coma(case)
    batch = SampledBatch(buf, case.z["ids"][0])
    batch = batch[:, :batch.max_t_filled()]
    q_all = learner.critic(batch)
    assert tuple(q_all.shape) == case.z["step0_critic_q_all"].shape
    assert rel(q_all.cpu().numpy(), case.z["step0_critic_q_all"]) < 1e-5
    for t in (0, 2):
        q = learner.critic(batch, t=t)
        assert rel(q.cpu().numpy(), case.z["step0_critic_q_t{}".format(t)]) < 1e-5
    q_tgt = learner.target_critic(batch)   # same initial weights
    assert rel(q_tgt.cpu().numpy(), case.z["step0_critic_q_all"]) < 1e-5
