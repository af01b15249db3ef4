"""Replay preprocessing transforms (reference: src/components/transforms.py:4-22)."""
import torch as th


class Transform:
    def transform(self, tensor):
        raise NotImplementedError

    def infer_output_info(self, vshape_in, dtype_in):
        raise NotImplementedError


class OneHot(Transform):
    """actions (..., 1) int -> actions_onehot (..., out_dim) float32 (transforms.py:12-22)."""

    def __init__(self, out_dim):
        self.out_dim = out_dim

    def transform(self, tensor):
        out = th.zeros(*tensor.shape[:-1], self.out_dim, dtype=th.float32, device=tensor.device)
        return out.scatter_(-1, tensor.long(), 1.0)

    def infer_output_info(self, vshape_in, dtype_in):
        return (self.out_dim,), th.float32
