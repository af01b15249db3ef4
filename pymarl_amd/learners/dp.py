"""Data-parallel learner step: episodes shard across ranks, ONE all-reduce per train step.

Contract (the same for QLearner and COMALearner): every rank calls `learner.train(batch, ...)` with the SAME GLOBAL
sample, exactly as the reference's run loop does (run.py:207-219: `buffer.sample(batch_size)`, `[:, :max_t]`,
`.to(device)`). Ranks run with the same seed, so `ReplayBuffer.sample`'s `np.random.choice` draws the same episode
ids on every rank. The learner keeps its own contiguous shard of the episodes (`local_shard`), checks once that the
ranks really passed the same sample (`check_same_batch`: a fingerprint of the ids, batch size and t_len, compared with
one MAX all-reduce), and rejects a batch that was already sharded (it would be sharded twice).

Every rank backpropagates the UNNORMALISED loss sum (td*m)^2 of its shard; the gradient buffer carries the
mask / stats sums in its tail (include/mq_learner.h, MQ_NSUMS). Summing that single buffer across ranks and
dividing by the global sum(mask) afterwards reproduces the reference's global normalisation
loss = sum (td*m)^2 / sum(m) (q_learner.py:97) exactly — averaging per-rank losses would not.

On a GPU the collective is issued on a dedicated communication stream: it waits on an event recorded after the
reduction kernels on the compute stream, and the compute stream waits on an event recorded after it, before
mq_apply. Nothing on the compute stream is serialised behind RCCL's own stream beyond that one dependency, and the
host never blocks.
"""
import ctypes
import hashlib
import os

import numpy as np
import torch
import torch.distributed as dist

_COMM = {}


def dp_world():
    """(rank, world) of the default process group, or (0, 1) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def native_comm_wanted(device):
    """The library's own RCCL communicator replaces torch.distributed's collective when the process group is RCCL
    (backend "nccl" on ROCm), the learner lives on a GPU and MQ_NATIVE_COMM is not "0": the all-reduce then runs
    in stream order inside libmq_learner (mq_comm_attach / mc_comm_attach), with no Python between the kernels."""
    if os.environ.get("MQ_NATIVE_COMM", "1") == "0":
        return False
    return (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
            and dist.get_backend() == "nccl" and torch.device(device).type == "cuda")


def broadcast_comm_id(lib, device):
    """Rank 0's RCCL unique id (mq_comm_unique_id), shipped to every rank over the process group."""
    from .. import _lib
    raw = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
    if dist.get_rank() == 0:
        _lib.check(lib.mq_comm_unique_id(raw))
    t = torch.tensor(list(bytes(raw)), dtype=torch.uint8, device=device)
    dist.broadcast(t, 0)
    return (ctypes.c_uint8 * _lib.COMM_ID_BYTES)(*t.cpu().tolist())


def shard_batch(batch, rank, world):
    """Episodes [rank*B/world, (rank+1)*B/world) of a sampled or dense batch, tagged `dp_shard = (rank, world)`."""
    if hasattr(batch, "shard"):
        return batch.shard(rank, world)
    lo, hi = shard_bounds(batch.batch_size, rank, world)
    out = batch[lo:hi]
    out.dp_shard = (rank, world)
    return out


def _t_len(batch):
    return int(getattr(batch, "t_len", batch.max_seq_length))


def batch_fingerprint(batch):
    """63-bit fingerprint of what a rank is about to train on: batch size, t_len and the sampled episode ids (a
    SampledBatch, dense or not, keeps them; a plain EpisodeBatch contributes its shape only)."""
    h = hashlib.blake2b(digest_size=8)
    h.update(np.asarray([batch.batch_size, _t_len(batch)], dtype=np.int64).tobytes())
    ids = getattr(batch, "ep_ids_np", None)
    if ids is not None:
        h.update(np.ascontiguousarray(ids, dtype=np.int64).tobytes())
    return int.from_bytes(h.digest(), "little") >> 1


def check_same_batch(batch, device, group=None):
    """Raise unless every rank passes the same global sample (one MAX all-reduce of [fp, -fp]; synchronises)."""
    from .. import _lib
    fp = batch_fingerprint(batch)
    dev = device if (torch.device(device).type == "cuda" and dist.get_backend(group) == "nccl") else "cpu"
    t = torch.tensor([fp, -fp], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    hi, lo = int(t[0].item()), -int(t[1].item())
    if hi != fp or lo != fp:
        raise _lib.MQError(
            "data-parallel learner: the ranks passed different batches to train() (batch {} episodes, t_len {}). "
            "Every rank must pass the same GLOBAL sample (same seed, so ReplayBuffer.sample draws the same ids); "
            "the learner shards it itself".format(batch.batch_size, _t_len(batch)))


def local_shard(batch, rank, world, check=True, device="cpu", group=None):
    """This rank's part of the GLOBAL sample `batch` (the data-parallel train() contract above). A batch that is
    already a shard (`SampledBatch.shard`, `shard_batch`) is rejected: it would be sharded twice."""
    if getattr(batch, "dp_shard", None) is not None:
        raise ValueError("data-parallel learner: train() takes the global sample on every rank and shards it "
                         "itself; this batch is already shard {} of {}".format(*batch.dp_shard))
    if batch.batch_size < world:
        raise ValueError("data-parallel learner: {} episodes cannot be shared by {} ranks".format(batch.batch_size,
                                                                                                 world))
    if check:
        check_same_batch(batch, device, group)
    return shard_batch(batch, rank, world)


class SharedComm:
    """One RCCL communicator per process (mq_comm_create), created once on first use (rank 0's id broadcast over
    torch.distributed) and lent to every learner handle with mq_comm_use / mc_comm_use. Handles never free it, so a
    handle rebuilt mid-run (larger batch or episode) re-attaches without a collective."""
    _comm = None
    _key = None

    @classmethod
    def get(cls, lib, device):
        from .. import _lib
        key = (torch.device(device).index, dist.get_world_size(), id(dist.group.WORLD))
        if cls._comm is None or cls._key != key:
            uid = broadcast_comm_id(lib, device)
            comm = ctypes.c_void_p()
            _lib.check(lib.mq_comm_create(uid, dist.get_rank(), dist.get_world_size(), ctypes.byref(comm)))
            cls._comm, cls._key = comm, key
        return cls._comm

    @classmethod
    def free(cls):
        """Release the communicator (call after the last train() and before destroy_process_group)."""
        if cls._comm is not None:
            from .. import _lib
            _lib.load().mq_comm_free(cls._comm)
            cls._comm = cls._key = None


def shard_bounds(batch_size, rank, world):
    """Contiguous episode slice [lo, hi) of `rank`."""
    return rank * batch_size // world, (rank + 1) * batch_size // world


def comm_stream(device):
    """The per-device communication stream (created once, highest priority: it gates mq_apply)."""
    key = torch.device(device).index
    if key not in _COMM:
        lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
        _COMM[key] = torch.cuda.Stream(device=device, priority=min(lo, hi))
    return _COMM[key]


def allreduce_grad_buffer(buf, group=None):
    """Sum the fused [grads | sums] buffer over the process group (RCCL over xGMI on MI355X; gloo on CPU).
    GPU buffers: on the communication stream, event-joined both ways with the current (compute) stream."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1):
        return buf
    if buf.is_cuda and dist.get_backend(group) == "nccl":
        compute = torch.cuda.current_stream(buf.device)
        comm = comm_stream(buf.device)
        ready = torch.cuda.Event()
        ready.record(compute)
        comm.wait_event(ready)
        with torch.cuda.stream(comm):
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
            done = torch.cuda.Event()
            done.record(comm)
        buf.record_stream(comm)
        compute.wait_event(done)
    else:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf
