"""Edge shapes of the QMIX / VDN learner on the GPU, teacher-forced against the numpy oracle (no reference
fixture exists for them, so they are pinned through the oracle, which the fixture shapes pin to the reference).

Each case sits on a boundary of a kernel's eligibility or layout:
* O = 128, A = 16: the fused forward with 8 gather slots per producer thread and the widest fused action set;
* n = 16: the widest fast mixer (one lane per agent, 16 agents);
* B = 1, n = 1: a single row (R = 1) and a one-agent mixer;
* A = 17: one action past the fused kernels (the unfused path) and the 32-action fast mixer;
* T = 1: a single transition per episode;
* min_len = 1: episodes as short as one step, terminated at t = 0, next to full-length ones.
"""
import pytest

from tests.golden_utils import SynthCase
from tests.test_gpu_parity import run_teacher_forced

pytestmark = pytest.mark.gpu

EDGE = {
    "edge_O128_A16": dict(n=4, A=16, O=128, S=64, T=20, B=8, n_episodes=24, steps=2),
    "edge_n16": dict(n=16, A=9, O=40, S=100, T=18, B=4, n_episodes=12, steps=2),
    "edge_B1_n1": dict(n=1, A=2, O=5, S=7, T=5, B=1, n_episodes=3, steps=3),
    "edge_B1_n1_vdn": dict(n=1, A=2, O=5, S=7, T=5, B=1, n_episodes=3, steps=2, mixer="vdn"),
    "edge_A17": dict(n=3, A=17, O=20, S=30, T=12, B=6, n_episodes=16, steps=2),
    "edge_T1": dict(n=2, A=4, O=6, S=9, T=1, B=5, n_episodes=9, steps=2),
    "edge_short": dict(n=3, A=5, O=30, S=48, T=40, B=16, n_episodes=40, steps=2, min_len=1),
}


@pytest.mark.parametrize("name", sorted(EDGE))
def test_edge_teacher_forced(name, monkeypatch):
    run_teacher_forced(SynthCase(name, **EDGE[name]), EDGE[name]["steps"], False, monkeypatch)
