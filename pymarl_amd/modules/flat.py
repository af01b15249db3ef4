"""Flat-parameter packing: module parameters as views into one contiguous fp32 buffer.

The HIP learner addresses every parameter by offset into a single device buffer (include/mq_learner.h,
MQ_P_*). nn.Module parameters stay ordinary `nn.Parameter`s with the reference's names, so `state_dict()`,
`load_state_dict()`, `parameters()` and the agent.th / mixer.th / opt.th checkpoint files are unchanged
(reference: q_learner.py:131-143, basic_controller.py:91-92).
"""
import torch as th


def pack(modules, flat=None, device=None):
    """Copy the parameters of `modules` (in order) into `flat` (allocated if None) and re-point them at it."""
    params = [p for m in modules for p in m.parameters()]
    total = sum(p.numel() for p in params)
    if flat is None:
        dev = device if device is not None else (params[0].device if params else "cpu")
        flat = th.empty(total, dtype=th.float32, device=dev)
    assert flat.numel() >= total and flat.dtype == th.float32
    o = 0
    with th.no_grad():
        for p in params:
            n = p.numel()
            view = flat[o:o + n].view_as(p)
            view.copy_(p.data)
            p.data = view
            o += n
    return flat, total


def rebind(modules, flat):
    """Re-point parameters at `flat` without copying (after the buffer moved devices)."""
    o = 0
    for m in modules:
        for p in m.parameters():
            n = p.numel()
            p.data = flat[o:o + n].view_as(p)
            o += n
    return o


class FlatModule(th.nn.Module):
    """nn.Module whose parameters live in `self._flat`; device moves keep the flat layout."""

    def _init_flat(self):
        self._flat, _ = pack([self])

    def flat_params(self):
        return self._flat

    def _apply(self, fn, recurse=True):
        flat = getattr(self, "_flat", None)
        if flat is None:
            return super()._apply(fn, recurse)
        new = fn(flat)
        if new is not flat:
            self._flat = new
        rebind([self], self._flat)
        return self

    def __deepcopy__(self, memo):
        cls = self.__class__
        new = cls.__new__(cls)
        memo[id(self)] = new
        for k, v in self.__dict__.items():
            if k == "_flat":
                continue
            import copy
            setattr(new, k, copy.deepcopy(v, memo))
        new._flat, _ = pack([new], device=self._flat.device)
        return new
