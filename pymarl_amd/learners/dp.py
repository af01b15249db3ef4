"""Data-parallel learner step: episodes shard across ranks, ONE all-reduce per train step.

Every rank backpropagates the UNNORMALISED loss sum (td*m)^2 of its shard; the gradient buffer carries the
mask / stats sums in its tail (include/mq_learner.h, MQ_NSUMS). Summing that single buffer across ranks and
dividing by the global sum(mask) afterwards reproduces the reference's global normalisation
loss = sum (td*m)^2 / sum(m) (q_learner.py:97) exactly — averaging per-rank losses would not.
"""
import torch.distributed as dist


def shard_bounds(batch_size, rank, world):
    """Contiguous episode slice [lo, hi) of `rank`."""
    return rank * batch_size // world, (rank + 1) * batch_size // world


def allreduce_grad_buffer(buf, group=None):
    """Sum the fused [grads | sums] buffer over the process group (RCCL over xGMI on MI355X; gloo on CPU)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf
