"""Data-parallel QLearner end to end on the GPU: two ranks share cuda:0, each trains its shard of
the same global sample through the product path (QLearner.train -> libmq_learner.so with mq_set_data_parallel,
all-reduce of the fused [grads | sums] buffer between mq_forward_backward and mq_apply), and the result must equal
one process training the whole batch (q_learner.py:97's global normalisation).

The collective here is gloo on device tensors (two ranks cannot share one GPU under RCCL); the bench's N>1 path
makes the same call over RCCL. Ragged episodes give the two shards unequal mask sums.
"""
import os
import socket

import numpy as np
import pytest
import torch as th
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

CASE = "cfg2_qmix_ragged"
STEPS = 3
STATS = ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _train(learner, buf, case, rank, world, record):
    from pymarl_amd.components.episode_buffer import SampledBatch
    from tests.gpu_helpers import flat_grads, flat_params
    for k in range(STEPS):
        gb = SampledBatch(buf, case.z["ids"][k])
        gb = gb[:, :gb.max_t_filled()]
        batch = gb.shard(rank, world) if world > 1 else gb
        learner.train(batch, 1000 * k, case.episodes[k])
        st = learner.last_stats()
        record["stats"].append([st[s] for s in STATS])
        record["grads"].append(flat_grads(learner))
        record["params"].append(flat_params(learner))


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    th.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from tests.golden_utils import Case
        from tests.gpu_helpers import build
        case = Case(CASE)
        args, buf, mac, learner, logger = build(case, learner_dp=True)
        rec = {"stats": [], "grads": [], "params": []}
        _train(learner, buf, case, rank, world, rec)
        th.cuda.synchronize()
        if rank == 0:
            np.savez(out_path, **{k: np.asarray(v) for k, v in rec.items()})
    finally:
        dist.destroy_process_group()


def test_two_rank_dp_equals_single_process(tmp_path):
    from tests.golden_utils import Case
    from tests.gpu_helpers import build, rel
    out = str(tmp_path / "dp.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    dp = np.load(out)

    case = Case(CASE)
    args, buf, mac, learner, logger = build(case)
    ref = {"stats": [], "grads": [], "params": []}
    _train(learner, buf, case, 0, 1, ref)

    # step 0 starts from identical state: the only difference is the order the two shards' partial sums are
    # added in, so gradients and stats agree to fp32 rounding
    assert rel(dp["grads"][0], ref["grads"][0]) < 1e-5
    assert rel(dp["stats"][0], ref["stats"][0]) < 1e-5
    # later steps: a gradient element near 0 can flip sign between the two summation orders and RMSprop's
    # per-parameter normalisation turns that into an O(lr) parameter difference, so stats get a band, the DP run's
    # step-0 update is checked exactly against RMSprop of its own all-reduced gradient, and the end state is
    # bounded by O(lr) per element
    for k in range(STEPS):
        assert rel(dp["stats"][k], ref["stats"][k]) < 1e-3, (k, dp["stats"][k], ref["stats"][k])
    g = dp["grads"][0].astype(np.float64)
    p0 = np.concatenate([v.ravel() for v in list(case.agent_params.values()) + list(case.mixer_params.values())])
    assert rel(dp["params"][0], p0 - 5e-4 * g / (np.sqrt(0.01 * g * g) + 1e-5)) < 1e-6
    assert np.abs(dp["params"][-1] - ref["params"][-1]).max() <= 20 * 5e-4
