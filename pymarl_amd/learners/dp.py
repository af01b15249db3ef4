"""Data-parallel learner step: episodes shard across ranks, ONE all-reduce per train step.

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
import os

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
    """Episodes [rank*B/world, (rank+1)*B/world) of a sampled or dense batch."""
    if hasattr(batch, "shard"):
        return batch.shard(rank, world)
    lo, hi = shard_bounds(batch.batch_size, rank, world)
    return batch[lo:hi]


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
