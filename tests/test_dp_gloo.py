"""Multi-rank learner math on CPU (gloo, world_size 2): per-rank UNNORMALISED gradients + loss/mask sums in one
buffer, one all-reduce (pymarl_amd.learners.dp.allreduce_grad_buffer, the call QLearner.train makes over RCCL),
then division by the global mask sum == the single-process gradient of the whole batch (q_learner.py:97).
The per-rank gradients come from the numpy oracle (test infrastructure) on each rank's shard of the golden
cfg2 / ragged batches, so unequal mask sums per shard are exercised."""
import json
import os
import socket

import numpy as np
import pytest
import torch as th
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _flat_grads(o, fw):
    ag, mg, _ = o.gradients(None, fw)
    return np.concatenate([v.ravel() for v in list(ag.values()) + list(mg.values())]).astype(np.float64)


def _worker(rank, world, port, name, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle.qlearner_np import OracleQLearner
        from pymarl_amd.learners.dp import allreduce_grad_buffer, shard_bounds
        from tests.golden_utils import Case
        c = Case(name)
        o = OracleQLearner(c.agent_params, c.mixer_params, c.cfg())
        batch, _ = c.batch(0)
        lo, hi = shard_bounds(c.B, rank, world)
        shard = {k: v[lo:hi] for k, v in batch.items()}
        fw = o.forward(shard, keep_cache=True)
        msum = float(fw["mask_sum"])
        g_unnorm = _flat_grads(o, fw) * msum                     # d sum (td*m)^2 / d theta on this shard
        m, td = fw["mask"], fw["td"]
        sums = [float(((td * m) ** 2).sum()), msum, float(np.abs(td * m).sum()),
                float((fw["q_tot"] * m).sum()), float((fw["targets"] * m).sum()), 0, 0, 0]
        buf = th.tensor(np.concatenate([g_unnorm, sums]), dtype=th.float64)
        allreduce_grad_buffer(buf)
        if rank == 0:
            np.save(out_path, buf.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", ["cfg2_qmix_ragged", "tiny_vdn"])
def test_two_rank_gradient_equals_single_process(tmp_path, name):
    out = str(tmp_path / "buf.npy")
    mp.spawn(_worker, args=(2, _free_port(), name, out), nprocs=2, join=True)
    buf = np.load(out)
    from oracle.qlearner_np import OracleQLearner
    from tests.golden_utils import Case
    c = Case(name)
    o = OracleQLearner(c.agent_params, c.mixer_params, c.cfg())
    batch, _ = c.batch(0)
    fw = o.forward(batch, keep_cache=True)
    g_full = _flat_grads(o, fw)
    P = g_full.size
    msum = buf[P + 1]
    assert msum == pytest.approx(float(fw["mask_sum"]))
    g_dp = buf[:P] / msum
    assert np.abs(g_dp - g_full).max() <= 1e-5 * np.abs(g_full).max()
    assert buf[P] / msum == pytest.approx(fw["loss"], rel=1e-5)


# ------------------------------------------------------------------------------------------------------------------
# The data-parallel train() contract (learners/dp.py): every rank passes the SAME GLOBAL sample, exactly as run.py:207-219
# does; the learner shards it itself, checks once that the ranks agree, and rejects an already-sharded batch. The
# plumbing runs on CPU here (QLearner built on the host; train() itself needs the GPU).

def _contract_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    try:
        from pymarl_amd import _lib
        from pymarl_amd.components.episode_buffer import SampledBatch
        from pymarl_amd.learners.dp import DPCheck, local_shard, shard_bounds
        from tests.golden_utils import Case
        from tests.gpu_helpers import build
        case = Case("cfg2_qmix_ragged")
        args, buf, mac, learner, logger = build(case, device="cpu", learner_dp=True)
        ids = case.z["ids"][0]
        gb = SampledBatch(buf, ids)
        gb = gb[:, :gb.max_t_filled()]
        # the learner's own sharding of the global sample (QLearner.train's first step)
        loc = learner._local_batch(gb)
        lo, hi = shard_bounds(len(ids), rank, world)
        res["ids_ok"] = bool(np.array_equal(loc.ep_ids_np, ids[lo:hi]) and loc.t_len == gb.t_len)
        res["checked"] = learner.dp_check.done == 1
        # an already-sharded batch (the old caller-shards contract) is rejected, never sharded twice
        try:
            learner._local_batch(gb.shard(rank, world))
            res["reshard"] = "accepted"
        except ValueError:
            res["reshard"] = "rejected"
        try:   # time-truncated shard keeps its tag
            learner._local_batch(gb.shard(rank, world)[:, :gb.t_len - 1])
            res["reshard_t"] = "accepted"
        except ValueError:
            res["reshard_t"] = "rejected"
        # a dense batch (the buffer_cpu_only flow's .to()) shards the same episodes
        dense = SampledBatch(buf, ids)[:, :gb.t_len]
        dense.dense = True
        dense.data = dense.materialize().data
        dl = local_shard(dense, rank, world, check=True)
        res["dense_ok"] = bool(dl.batch_size == hi - lo and th.equal(dl["obs"], dense["obs"][lo:hi]))
        # ranks that pass different samples: every rank raises (the check is collective)
        bad = SampledBatch(buf, ids if rank == 0 else ids[::-1].copy())
        try:
            local_shard(bad, rank, world, check=True)
            res["mismatch"] = "accepted"
        except _lib.MQError:
            res["mismatch"] = "raised"
        # equal ids over DIFFERENT replay contents (ranks whose rollouts diverged): every rank raises
        rew = buf.data.transition_data["reward"]
        saved = rew[ids[1], 2].clone()
        if rank == 1:
            rew[ids[1], 2] += 0.5
        try:
            local_shard(SampledBatch(buf, ids)[:, :gb.t_len], rank, world, check=True)
            res["contents"] = "accepted"
        except _lib.MQError:
            res["contents"] = "raised"
        rew[ids[1], 2] = saved
        # the schedule is a call count, the same on every rank: rank-local shape differences never make one rank
        # enter the check's collective alone; the next scheduled call catches them on every rank
        learner.dp_check = DPCheck(2)
        sched = []
        for call in range(4):
            t_len = gb.t_len - (call % 2) * rank    # rank 1 truncates differently on the unchecked calls
            try:
                learner._local_batch(SampledBatch(buf, ids)[:, :t_len])
                sched.append("ok")
            except _lib.MQError:
                sched.append("raised")
        res["schedule"] = sched
        learner.dp_check = DPCheck("always")
        try:
            learner._local_batch(SampledBatch(buf, ids if rank == 0 else ids[::-1].copy())[:, :gb.t_len])
            res["always"] = "accepted"
        except _lib.MQError:
            res["always"] = "raised"
        try:   # fewer episodes than ranks
            local_shard(SampledBatch(buf, ids[:1]), rank, world, check=False)
            res["tiny"] = "accepted"
        except ValueError:
            res["tiny"] = "rejected"
        # train() still has no CPU path
        try:
            learner.train(gb, 0, 0)
            res["cpu_train"] = "ran"
        except _lib.MQError:
            res["cpu_train"] = "raised"
    finally:
        dist.barrier()   # no rank tears gloo down while its peer is still in the last collective
        dist.destroy_process_group()
    np.save(out_path.format(rank), np.array([json.dumps(res)]))


def test_dp_train_contract_global_sample(tmp_path):
    out = str(tmp_path / "res{}.npy")
    mp.spawn(_contract_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    for r in range(2):
        res = json.loads(str(np.load(out.format(r))[0]))
        assert res == {"ids_ok": True, "checked": True, "reshard": "rejected", "reshard_t": "rejected",
                       "dense_ok": True, "mismatch": "raised", "contents": "raised",
                       "schedule": ["ok", "ok", "ok", "ok"], "always": "raised", "tiny": "rejected",
                       "cpu_train": "raised"}, (r, res)


def test_dp_check_schedule():
    from pymarl_amd.learners.dp import DPCheck
    c = DPCheck(None)
    assert [c.due() for _ in range(201)].count(True) == 3          # calls 0, 100, 200
    c = DPCheck(3)
    assert [c.due() for _ in range(7)] == [True, False, False, True, False, False, True]
    c = DPCheck("first")
    assert [c.due() for _ in range(3)] == [True, False, False]
    assert [DPCheck("off").due() for _ in range(2)] == [False, False]
    assert DPCheck("5").mode == 5
    with pytest.raises(ValueError):
        DPCheck("sometimes")


def test_content_digest_sees_contents():
    from pymarl_amd.components.episode_buffer import SampledBatch
    from pymarl_amd.learners.dp import batch_fingerprint, content_digest
    from tests.golden_utils import Case
    from tests.gpu_helpers import build
    case = Case("tiny_qmix")
    _, buf, _, _, _ = build(case, device="cpu")
    ids = case.z["ids"][0]
    a = SampledBatch(buf, ids)
    d0, f0 = content_digest(a), batch_fingerprint(a)
    assert d0 == content_digest(SampledBatch(buf, ids)) and f0 == batch_fingerprint(SampledBatch(buf, ids))
    obs = buf.data.transition_data["obs"]
    obs[ids[0], 1, 0, 0] = th.nextafter(obs[ids[0], 1, 0, 0], th.tensor(1e9))   # one ulp in one element
    assert content_digest(a) != d0 and batch_fingerprint(a) != f0
    # the dense (materialised) batch of the same rows has the same digest
    assert content_digest(a.materialize()) == content_digest(a)


def test_shared_comm_free_detaches_borrowers():
    import ctypes
    from pymarl_amd.learners.dp import SharedComm

    class _Lib:
        def __init__(self):
            self.calls = []

        def mq_comm_detach(self, h):
            self.calls.append(("mq", h.value))
            return 0

        def mc_comm_detach(self, h):
            self.calls.append(("mc", h.value))
            return 0

    class _H:
        def __init__(self, lib, v):
            self.lib, self.h, self.native = lib, ctypes.c_void_p(v), True

    lib = _Lib()
    a, b = _H(lib, 16), _H(lib, 32)
    gen = SharedComm.generation
    SharedComm._comm = ctypes.c_void_p(None)    # mq_comm_free(NULL) is a no-op
    SharedComm._borrowers = []
    import weakref
    SharedComm._borrowers += [(weakref.ref(a), "mq_comm_detach"), (weakref.ref(b), "mc_comm_detach")]
    SharedComm.free()
    assert lib.calls == [("mq", 16), ("mc", 32)]
    assert not a.native and not b.native and SharedComm._comm is None and SharedComm.generation == gen + 1


def test_learner_rebuilds_handle_after_shared_comm_free(monkeypatch):
    """after SharedComm.free() detached a borrowed communicator, the learner's next _get_handle must
    build a new handle that borrows the new communicator (data parallelism still on), not train on with the detached
    one. free() clears `native`, so the rebuild must not depend on it (SharedComm.stale keys on the generation)."""
    import ctypes
    from types import SimpleNamespace as SN
    from pymarl_amd import _lib
    from pymarl_amd.learners import q_learner as ql
    from pymarl_amd.learners.dp import SharedComm

    class _Lib:
        def mq_bind(self, *a):
            return 0

        def mq_comm_detach(self, h):
            return 0

        def mq_comm_free(self, c):
            return 0

    built = []

    class _FakeHandle:
        def __init__(self, cfg):
            self.lib, self.h, self.n_params = _Lib(), ctypes.c_void_p(len(built) + 1), 10
            built.append(self)

    lent = []

    def _lend(handle, use, detach, device):
        import weakref
        SharedComm._comm = ctypes.c_void_p(None)
        SharedComm._borrowers.append((weakref.ref(handle), detach))
        handle.native, handle.comm_gen = True, SharedComm.generation
        lent.append(handle)

    monkeypatch.setattr(ql._lib, "Handle", _FakeHandle)
    monkeypatch.setattr(ql, "native_comm_wanted", lambda dev: True)
    monkeypatch.setattr(SharedComm, "lend", staticmethod(_lend))
    monkeypatch.setattr(_lib, "load", lambda: _Lib())
    monkeypatch.setattr(SharedComm, "_borrowers", [])
    args = SN(batch_size=4, n_agents=2, n_actions=3, obs_shape=5, state_shape=4, rnn_hidden_dim=64,
              mixing_embed_dim=8, mixer="qmix", obs_last_action=True, obs_agent_id=True)
    fake = SN(args=args, mac=SN(agent=SN(input_dim=10)), _online=th.zeros(11), _target=th.zeros(11),
              _grad=th.zeros(11), _sq=th.zeros(10), _stats=th.zeros(8), n_params=10, _handle=None,
              _handle_key=None, _dp_active=lambda: True)
    monkeypatch.setattr(ql, "dp_world", lambda: (0, 2))
    batch = SN(batch_size=2, max_seq_length=6)
    h1 = ql.QLearner._get_handle(fake, batch)
    assert ql.QLearner._get_handle(fake, batch) is h1 and h1.native
    SharedComm.free()
    assert not h1.native and SharedComm.stale(h1)
    h2 = ql.QLearner._get_handle(fake, batch)
    assert h2 is not h1 and h2.native and not SharedComm.stale(h2) and lent == [h1, h2]
    assert not SharedComm.stale(None) and not SharedComm.stale(SN(native=False))
