"""Native RCCL data parallelism through the C-ABI (include/mq_learner.h mq_comm_attach, include/mc_coma.h
mc_comm_attach; SURVEY.md §8b's mq_allreduce_attach). One GPU here, so world = 1: the all-reduce is the identity
and everything else of the data-parallel step runs for real (the RCCL communicator, the in-stream ncclAllReduce of
the [grads | sums] buffer inside mq_forward_backward, the norm recomputed from the summed buffer in mq_apply; for
COMA the per-critic-step exchanges of the three-launch path). Each result must equal the same step without a
communicator to float rounding (the norm is summed in another order). Multi-rank correctness of the algebra is
tests/test_dp_gloo.py and tests/test_gpu_dp.py."""
import ctypes

import numpy as np
import pytest
import torch as th

from tests.golden_utils import COMA_STATS, Case, ComaCase
from tests.gpu_helpers import set_switch

pytestmark = pytest.mark.gpu

STATS = ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(1e-30, np.abs(b).max()))


def _unique_id(lib):
    buf = (ctypes.c_uint8 * 128)()
    assert lib.mq_comm_unique_id(buf) == 0, lib.mq_last_error()
    return buf


def test_qlearner_step_over_native_rccl(monkeypatch):
    from pymarl_amd.components.episode_buffer import SampledBatch
    from tests.gpu_helpers import build, flat_params
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    case = Case("tiny_qmix")
    runs = []
    for native in (True, False):
        args, buf, mac, learner, logger = build(case)
        gb = SampledBatch(buf, case.z["ids"][0])
        gb = gb[:, :gb.max_t_filled()]
        h = learner._get_handle(gb)
        if native:
            idb = _unique_id(h.lib)
            assert h.lib.mq_comm_attach(h.h, idb, 0, 1) == 0, h.lib.mq_last_error()
            assert h.lib.mq_comm_world(h.h) == 1
        learner.train(gb, 1000, case.episodes[0])
        st = learner.last_stats()
        runs.append((flat_params(learner), [st[s] for s in STATS]))
        if native:
            assert h.lib.mq_comm_detach(h.h) == 0
            assert h.lib.mq_comm_world(h.h) == 0
    (pa, sa), (pb, sb) = runs
    assert _rel(pa, pb) < 1e-6
    for x, y, name in zip(sa, sb, STATS):
        assert abs(x - y) <= 1e-5 * abs(y) + 1e-7, (name, x, y)


def test_coma_step_over_native_rccl(monkeypatch):
    from tests.gpu_helpers import build_coma
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    set_switch(monkeypatch, "coma_chain", "0")   # the reference path for the comparison: three launches, no exchange
    c = ComaCase("coma_tiny")
    runs = []
    for native in (True, False):
        args, buf, mac, learner, logger = build_coma(c)
        np.random.seed(c.sampler_seed)
        batch = buf.sample(c.B)
        batch = batch[:, :batch.max_t_filled()]
        if native:
            h = learner._get_handle(batch)
            idb = _unique_id(h.lib)
            assert h.lib.mc_comm_attach(h.h, idb, 0, 1) == 0, h.lib.mq_last_error()
        mac.action_selector.epsilon = c.epsilon[0]
        learner.train(batch, 1000, 0)
        assert learner.critic_path() == "three_launch"
        st = learner.last_stats()
        runs.append((learner._critic.cpu().numpy().copy(), learner._agent.cpu().numpy().copy(),
                     [st[s] for s in COMA_STATS], st["critic_steps"]))
    (ca, aa, sa, na), (cb, ab, sb, nb) = runs
    assert na == nb
    assert np.abs(ca - cb).max() <= 1e-5
    assert _rel(aa, ab) < 1e-5
    for x, y, name in zip(sa, sb, COMA_STATS):
        assert abs(x - y) <= 1e-4 * abs(y) + 1e-6, (name, x, y)


def test_caller_owned_communicator_shared_by_two_learners(monkeypatch):
    """SURVEY §8b's mq_allreduce_attach(handle, ncclComm_t): one communicator the caller owns (mq_comm_create),
    borrowed by a QMIX handle (mq_comm_use) and a COMA handle (mc_comm_use) of the same process. Each step equals
    the step without a communicator; detaching and destroying the handles leave it alive until mq_comm_free."""
    from pymarl_amd import _lib
    from pymarl_amd.components.episode_buffer import SampledBatch
    from tests.gpu_helpers import build, build_coma, flat_params
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    lib = _lib.load()
    comm = ctypes.c_void_p()
    assert lib.mq_comm_create(_unique_id(lib), 0, 1, ctypes.byref(comm)) == 0, lib.mq_last_error()
    try:
        case = Case("tiny_qmix")
        out = []
        for use in (True, False):
            args, buf, mac, learner, logger = build(case)
            gb = SampledBatch(buf, case.z["ids"][0])
            gb = gb[:, :gb.max_t_filled()]
            h = learner._get_handle(gb)
            if use:
                assert h.lib.mq_comm_use(h.h, comm) == 0, h.lib.mq_last_error()
                assert h.lib.mq_comm_world(h.h) == 1
            learner.train(gb, 1000, case.episodes[0])
            out.append(flat_params(learner))
            if use:
                assert h.lib.mq_comm_detach(h.h) == 0   # borrowed: the communicator stays alive
        assert _rel(out[0], out[1]) < 1e-6

        set_switch(monkeypatch, "coma_chain", "0")
        c = ComaCase("coma_tiny")
        runs = []
        for use in (True, False):
            args, cbuf, cmac, cl, _ = build_coma(c)
            np.random.seed(c.sampler_seed)
            batch = cbuf.sample(c.B)
            batch = batch[:, :batch.max_t_filled()]
            if use:
                hc = cl._get_handle(batch)
                assert hc.lib.mc_comm_use(hc.h, comm) == 0, hc.lib.mq_last_error()
            cmac.action_selector.epsilon = c.epsilon[0]
            cl.train(batch, 1000, 0)
            runs.append(cl._critic.cpu().numpy().copy())
            del cl   # handle destroyed: must not free the borrowed communicator
        assert np.abs(runs[0] - runs[1]).max() <= 1e-5
        # still usable after both handles let go of it
        args, buf, mac, learner, logger = build(case)
        gb = SampledBatch(buf, case.z["ids"][0])
        gb = gb[:, :gb.max_t_filled()]
        h = learner._get_handle(gb)
        assert h.lib.mq_comm_use(h.h, comm) == 0, h.lib.mq_last_error()
        learner.train(gb, 1000, case.episodes[0])
        assert h.lib.mq_comm_detach(h.h) == 0
    finally:
        th.cuda.synchronize()
        assert lib.mq_comm_free(comm) == 0


def test_coma_replicated_critic_world1(monkeypatch):
    """mc_set_actor_shard at world 1 over the native communicator: the whole batch is the only shard, the critic
    runs through the persistent chain with no exchange (bitwise the plain run's critic) and the actor's one
    all-reduce is the identity (agent parameters equal to rounding: the norm is recomputed from the summed buffer)."""
    from tests.gpu_helpers import build_coma
    monkeypatch.setenv("NCCL_SOCKET_IFNAME", "lo")
    set_switch(monkeypatch, "coma_chain", None)
    c = ComaCase("coma_cfg5")
    runs = []
    for repl in (True, False):
        args, buf, mac, learner, logger = build_coma(c)
        np.random.seed(c.sampler_seed)
        batch = buf.sample(c.B)
        batch = batch[:, :batch.max_t_filled()]
        h = learner._get_handle(batch)
        if repl:
            assert h.lib.mc_comm_attach(h.h, _unique_id(h.lib), 0, 1) == 0, h.lib.mq_last_error()
            assert h.lib.mc_set_actor_shard(h.h, 0, c.B) == 0, h.lib.mq_last_error()
        mac.action_selector.epsilon = c.epsilon[0]
        learner.train(batch, 1000, 0)
        assert learner.critic_path() == "chain"
        runs.append((learner._critic.cpu().numpy().copy(), learner._agent.cpu().numpy().copy(), learner.last_stats()))
    (ca, aa, sa), (cb, ab, sb) = runs
    assert np.array_equal(ca, cb)
    assert _rel(aa, ab) < 1e-6
    for k in ("critic_loss", "critic_grad_norm", "coma_loss", "agent_grad_norm", "pi_max"):
        assert abs(sa[k] - sb[k]) <= 1e-5 * abs(sb[k]) + 1e-7, (k, sa[k], sb[k])
