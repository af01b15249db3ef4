"""Data-parallel learner step: episodes shard across ranks, ONE all-reduce per train step.

Contract (the same for QLearner and COMALearner): every rank calls `learner.train(batch, ...)` with the SAME GLOBAL
sample, exactly as the reference's run loop does (run.py:207-219: `buffer.sample(batch_size)`, `[:, :max_t]`,
`.to(device)`). Ranks run with the same seed, so `ReplayBuffer.sample`'s `np.random.choice` draws the same episode
ids on every rank. The learner keeps its own contiguous shard of the episodes (`local_shard`), checks on a call-count
schedule that is the same on every rank (`DPCheck`) that the ranks really passed the same sample (`check_same_batch`: a
fingerprint of the batch size, t_len, episode ids and a digest of the sampled rows' contents, compared with one MAX
all-reduce), and rejects a batch that was already sharded (it would be sharded twice).

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
import weakref

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


# fields whose sampled rows are digested: what the loss reads (q_learner.py:39-44, 58-86; coma_learner.py:32-46)
DIGEST_FIELDS = ("reward", "actions", "terminated", "filled", "avail_actions", "obs", "state")
_MIX = -7046029254386353131   # 0x9E3779B97F4A7C15 as int64 (golden-ratio multiplier); products wrap mod 2^64
DIGEST_CHUNK = 1 << 22        # elements per hashing pass (5 int64 temporaries of 32 MB each)


def content_digest(batch):
    """64-bit digest of the CONTENTS of the sampled transitions (the fields the learner reads, DIGEST_FIELDS), computed
    where the batch lives (device kernels for a GPU replay, one host read-back). Every element's bit pattern is mixed
    with its position and the sum wraps in int64, so the result does not depend on the summation order: two ranks get
    the same digest exactly when their sampled rows are bitwise equal (up to hash collisions). Each field is hashed
    in chunks of DIGEST_CHUNK elements, so the int64 temporaries stay a few hundred MB whatever the batch size; the
    chunk sums add up modulo 2^64 to the whole field's sum."""
    acc = 0
    for k in DIGEST_FIELDS:
        try:
            v = batch[k]
        except (KeyError, TypeError):
            continue
        if v.dtype == torch.float32:
            v = v.contiguous().view(torch.int32)
        v = v.reshape(-1)
        s = 0
        for lo in range(0, v.numel(), DIGEST_CHUNK):
            c = v[lo:lo + DIGEST_CHUNK].to(torch.int64)
            pos = torch.arange(lo + 1, lo + c.numel() + 1, dtype=torch.int64, device=c.device)
            x = (c + pos) * _MIX
            x = x ^ (x >> 29)          # arithmetic shift: deterministic for negative values too
            s += int((x * _MIX).sum().item())
        acc = (acc * 31 + s) & 0xFFFFFFFFFFFFFFFF
    return acc


def batch_fingerprint(batch):
    """63-bit fingerprint of what a rank is about to train on: batch size, t_len, the sampled episode ids (a
    SampledBatch, dense or not, keeps them) and the digest of the sampled rows' contents (content_digest), so ranks
    that draw the same ids from replay buffers whose contents differ (diverged rollouts, run.py:203-204) disagree."""
    h = hashlib.blake2b(digest_size=8)
    h.update(np.asarray([batch.batch_size, _t_len(batch)], dtype=np.int64).tobytes())
    ids = getattr(batch, "ep_ids_np", None)
    if ids is not None:
        h.update(np.ascontiguousarray(ids, dtype=np.int64).tobytes())
    h.update(np.asarray([content_digest(batch)], dtype=np.uint64).tobytes())
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
            "data-parallel learner: the ranks passed different batches to train() (batch {} episodes, t_len {}; "
            "the sampled ids or the contents of the sampled episodes differ). Every rank must pass the same GLOBAL "
            "sample from the same replay contents (same seed, so ReplayBuffer.sample draws the same ids); the "
            "learner shards it itself".format(batch.batch_size, _t_len(batch)))


class DPCheck:
    """When a data-parallel train() runs check_same_batch. The decision depends only on the call count, which is the
    same on every rank (ranks that made different numbers of train() calls would already disagree on the gradient
    all-reduce), so every rank enters the check's collective together — never one rank alone. `learner_dp_check`:
    "first" (the first call only), "always", "off", or an int N (calls 0, N, 2N, ...; the default is 100, which costs
    one small all-reduce and a digest every 100 steps)."""
    DEFAULT_EVERY = 100

    def __init__(self, mode):
        if mode is None:
            mode = self.DEFAULT_EVERY
        if isinstance(mode, str) and mode.isdigit():
            mode = int(mode)
        if not (mode in ("first", "always", "off") or (isinstance(mode, int) and mode > 0)):
            raise ValueError("learner_dp_check must be 'first', 'always', 'off' or a positive int, not {!r}"
                             .format(mode))
        self.mode = mode
        self.calls = 0
        self.done = 0

    def due(self):
        """Whether this call checks; advances the call counter."""
        c, self.calls = self.calls, self.calls + 1
        if self.mode == "always":
            return True
        if self.mode == "off":
            return False
        if self.mode == "first":
            return c == 0
        return c % self.mode == 0


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
    handle rebuilt mid-run (larger batch or episode) re-attaches without a collective. The handles that borrowed it
    are tracked: free() detaches them first (mq_comm_detach / mc_comm_detach), so none is left holding a destroyed
    communicator; a learner that trains again afterwards re-attaches to a new one (`generation` changed)."""
    _comm = None
    _key = None
    generation = 0
    _borrowers = []   # (weakref to the Handle / ComaHandle, detach function name)

    @classmethod
    def get(cls, lib, device):
        from .. import _lib
        key = (torch.device(device).index, dist.get_world_size(), id(dist.group.WORLD))
        if cls._comm is None or cls._key != key:
            if cls._comm is not None:
                cls.free()
            uid = broadcast_comm_id(lib, device)
            comm = ctypes.c_void_p()
            _lib.check(lib.mq_comm_create(uid, dist.get_rank(), dist.get_world_size(), ctypes.byref(comm)))
            cls._comm, cls._key = comm, key
        return cls._comm

    @classmethod
    def lend(cls, handle, use, detach, device):
        """Attach the process communicator to `handle` (a _lib.Handle / ComaHandle) with `use` (mq_comm_use /
        mc_comm_use) and remember to detach it (`detach`) before the communicator is freed."""
        from .. import _lib
        comm = cls.get(handle.lib, device)
        _lib.check(getattr(handle.lib, use)(handle.h, comm))
        cls._borrowers = [(r, d) for r, d in cls._borrowers if r() is not None]
        cls._borrowers.append((weakref.ref(handle), detach))
        handle.native = True
        handle.comm_gen = cls.generation

    @classmethod
    def stale(cls, handle):
        """True when `handle` borrowed a communicator that has since been freed (free() detached it and moved the
        generation on). Independent of `handle.native`, which free() clears: the learner must rebuild such a handle
        so the next train() re-attaches, instead of training on with no cross-rank sum."""
        gen = getattr(handle, "comm_gen", None) if handle is not None else None
        return gen is not None and gen != cls.generation

    @classmethod
    def free(cls):
        """Release the communicator (call after the last train() and before destroy_process_group). Every handle
        that still borrows it is detached first and falls back to `native = False`; the learner rebuilds it on its
        next train() (stale()), which re-attaches a new communicator."""
        if cls._comm is not None:
            from .. import _lib
            for ref, detach in cls._borrowers:
                h = ref()
                if h is not None and getattr(h, "h", None) and h.h.value:
                    getattr(h.lib, detach)(h.h)
                    h.native = False
            cls._borrowers = []
            _lib.load().mq_comm_free(cls._comm)
            cls._comm = cls._key = None
            cls.generation += 1


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
