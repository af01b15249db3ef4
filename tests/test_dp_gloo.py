"""Multi-rank learner math on CPU (gloo, world_size 2): per-rank UNNORMALISED gradients + loss/mask sums in one
buffer, one all-reduce (pymarl_amd.learners.dp.allreduce_grad_buffer, the call QLearner.train makes over RCCL),
then division by the global mask sum == the single-process gradient of the whole batch (q_learner.py:97).
The per-rank gradients come from the numpy oracle (test infrastructure) on each rank's shard of the golden
cfg2 / ragged batches, so unequal mask sums per shard are exercised."""
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
