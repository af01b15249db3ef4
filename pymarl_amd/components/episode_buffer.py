"""EpisodeBatch / ReplayBuffer with the reference API, laid out for an HBM-resident replay.

Reference: src/components/episode_buffer.py (EpisodeBatch :8-262, ReplayBuffer :264-304). Same constructor
signatures, scheme/groups/preprocess semantics, `update`, `__getitem__` (key, key tuple, (batch, time) slices),
`max_t_filled`, `to`, `insert_episode_batch`, `can_sample`, `sample`.

MI355X-first differences (behaviour-preserving for the learner):
* `ReplayBuffer.sample(B)` draws the episode ids exactly like the reference (np.random.choice on numpy's global
  RNG, :291-298) but returns a `SampledBatch`: a zero-copy view (storage + device id vector + t_len). The learner
  kernels gather the rows by id straight from HBM, so the reference's 16 MB fancy-index copy and host->device
  transfer disappear. Indexing a key of a SampledBatch still materialises the gathered tensor, as the reference's
  would.
* Episode lengths are tracked on the host at insert time, so `SampledBatch.max_t_filled()` is a host max (no
  device sync); the result equals the reference's `sum(filled, 1).max(0)`.
* A host-resident buffer (`buffer_cpu_only: True`, run.py:137-139) keeps the reference's flow: `sample` ->
  `[:, :max_t]` -> `.to(args.device)` in place (run.py:208-215). `SampledBatch.to` then gathers the sampled episodes
  on the host and copies each field to the device once; the batch is dense from then on (`dense`), and the learner
  reads it through the dense (no episode id) kernel path.
"""
from __future__ import annotations

from functools import reduce
from types import SimpleNamespace as SN

import numpy as np
import torch as th


def _prod(shape):
    return reduce(lambda a, b: a * b, shape, 1)


class EpisodeBatch:
    dp_shard = None   # (rank, world) when this batch is one rank's shard of a global sample (learners/dp.py)

    def __init__(self, scheme, groups, batch_size, max_seq_length, data=None, preprocess=None, device="cpu"):
        self.scheme = scheme.copy()
        self.groups = groups
        self.batch_size = batch_size
        self.max_seq_length = max_seq_length
        self.preprocess = {} if preprocess is None else preprocess
        self.device = device
        if data is not None:
            self.data = data
        else:
            self.data = SN(transition_data={}, episode_data={})
            self._setup_data(self.scheme, self.groups, batch_size, max_seq_length, self.preprocess)

    # -- storage -------------------------------------------------------------------------------------------
    def _setup_data(self, scheme, groups, batch_size, max_seq_length, preprocess):
        for k, (new_k, transforms) in (preprocess or {}).items():
            assert k in scheme
            vshape, dtype = scheme[k]["vshape"], scheme[k].get("dtype", th.float32)
            for tr in transforms:
                vshape, dtype = tr.infer_output_info(vshape, dtype)
            self.scheme[new_k] = {"vshape": vshape, "dtype": dtype}
            for extra in ("group", "episode_const"):
                if extra in scheme[k]:
                    self.scheme[new_k][extra] = scheme[k][extra]
        assert "filled" not in scheme, '"filled" is a reserved key for masking.'
        scheme.update({"filled": {"vshape": (1,), "dtype": th.long}})
        for key, info in scheme.items():
            assert "vshape" in info, "Scheme must define vshape for {}".format(key)
            vshape = info["vshape"]
            vshape = (vshape,) if isinstance(vshape, int) else tuple(vshape)
            dtype = info.get("dtype", th.float32)
            group = info.get("group")
            if group:
                assert group in groups, "Group {} must have its number of members defined in _groups_".format(group)
                shape = (groups[group], *vshape)
            else:
                shape = vshape
            if info.get("episode_const", False):
                self.data.episode_data[key] = th.zeros((batch_size, *shape), dtype=dtype, device=self.device)
            else:
                self.data.transition_data[key] = th.zeros((batch_size, max_seq_length, *shape), dtype=dtype,
                                                          device=self.device)

    def extend(self, scheme, groups=None):
        self._setup_data(scheme, self.groups if groups is None else groups, self.batch_size, self.max_seq_length,
                         None)

    def to(self, device):
        for store in (self.data.transition_data, self.data.episode_data):
            for k, v in store.items():
                store[k] = v.to(device)
        self.device = device
        return self

    def update(self, data, bs=slice(None), ts=slice(None), mark_filled=True):
        slices = self._parse_slices((bs, ts))
        for k, v in data.items():
            if k in self.data.transition_data:
                target = self.data.transition_data
                if mark_filled:
                    target["filled"][tuple(slices)] = 1
                    mark_filled = False
                _slices = tuple(slices)
            elif k in self.data.episode_data:
                target = self.data.episode_data
                _slices = slices[0]
            else:
                raise KeyError("{} not found in transition or episode data".format(k))
            dtype = self.scheme[k].get("dtype", th.float32)
            if not th.is_tensor(v):
                v = np.asarray(v)   # one host array, one host-to-device copy per field
            v = th.as_tensor(v, dtype=dtype, device=self.device)
            dest = target[k][_slices]
            self._check_safe_view(v, dest)
            target[k][_slices] = v.view_as(dest)
            if k in self.preprocess:
                new_k, transforms = self.preprocess[k]
                v = target[k][_slices]
                for tr in transforms:
                    v = tr.transform(v)
                target[new_k][_slices] = v.view_as(target[new_k][_slices])

    @staticmethod
    def _check_safe_view(v, dest):
        idx = len(v.shape) - 1
        for s in dest.shape[::-1]:
            if idx >= 0 and v.shape[idx] == s:
                idx -= 1
            elif s != 1:
                raise ValueError("Unsafe reshape of {} to {}".format(v.shape, dest.shape))

    # -- indexing ------------------------------------------------------------------------------------------
    def __getitem__(self, item):
        if isinstance(item, str):
            if item in self.data.episode_data:
                return self.data.episode_data[item]
            if item in self.data.transition_data:
                return self.data.transition_data[item]
            raise ValueError(item)
        if isinstance(item, tuple) and all(isinstance(it, str) for it in item):
            new_data = SN(transition_data={}, episode_data={})
            for key in item:
                if key in self.data.transition_data:
                    new_data.transition_data[key] = self.data.transition_data[key]
                elif key in self.data.episode_data:
                    new_data.episode_data[key] = self.data.episode_data[key]
                else:
                    raise KeyError("Unrecognised key {}".format(key))
            new_scheme = {key: self.scheme[key] for key in item}
            new_groups = {self.scheme[key]["group"]: self.groups[self.scheme[key]["group"]]
                          for key in item if "group" in self.scheme[key]}
            return EpisodeBatch(new_scheme, new_groups, self.batch_size, self.max_seq_length, data=new_data,
                                device=self.device)
        item = self._parse_slices(item)
        new_data = SN(transition_data={}, episode_data={})
        for k, v in self.data.transition_data.items():
            new_data.transition_data[k] = v[tuple(item)]
        for k, v in self.data.episode_data.items():
            new_data.episode_data[k] = v[item[0]]
        ret_bs = self._get_num_items(item[0], self.batch_size)
        ret_max_t = self._get_num_items(item[1], self.max_seq_length)
        out = EpisodeBatch(self.scheme, self.groups, ret_bs, ret_max_t, data=new_data, device=self.device)
        # a time slice of a shard is still that shard
        if self.dp_shard is not None and isinstance(item[0], slice) and item[0] == slice(None):
            out.dp_shard = self.dp_shard
        return out

    @staticmethod
    def _get_num_items(indexing_item, max_size):
        if isinstance(indexing_item, (list, np.ndarray)):
            return len(indexing_item)
        if isinstance(indexing_item, th.Tensor):
            return int(indexing_item.numel())
        if isinstance(indexing_item, slice):
            rng = indexing_item.indices(max_size)
            return 1 + (rng[1] - rng[0] - 1) // rng[2]
        raise TypeError(indexing_item)

    @staticmethod
    def _parse_slices(items):
        if isinstance(items, (slice, int, list, np.ndarray, th.Tensor)):
            items = (items, slice(None))
        if isinstance(items[1], list):
            raise IndexError("Indexing across Time must be contiguous")
        parsed = []
        for it in items:
            if isinstance(it, (int, np.integer)):
                parsed.append(slice(int(it), int(it) + 1))
            elif isinstance(it, slice):
                parsed.append(slice(*(int(x) if x is not None else None for x in (it.start, it.stop, it.step))))
            else:
                parsed.append(it)
        return parsed

    def max_t_filled(self):
        return th.sum(self.data.transition_data["filled"], 1).max(0)[0]

    def __repr__(self):
        return "EpisodeBatch. Batch Size:{} Max_seq_len:{} Keys:{} Groups:{}".format(
            self.batch_size, self.max_seq_length, self.scheme.keys(), self.groups.keys())


def _same_device(a, b):
    a, b = th.device(a), th.device(b)
    if a.type != b.type:
        return False
    if a.type != "cuda" or a.index == b.index:
        return True
    cur = th.cuda.current_device() if th.cuda.is_available() else 0
    return (cur if a.index is None else a.index) == (cur if b.index is None else b.index)


def is_replay_view(batch):
    """True for a SampledBatch that still reads its replay buffer's storage through episode ids."""
    return isinstance(batch, SampledBatch) and not batch.dense


class SampledBatch(EpisodeBatch):
    """A sampled view of a ReplayBuffer: (storage, episode ids, t_len). Zero-copy; gathered on access.
    After `.to(<another device>)` it is a dense EpisodeBatch on that device (`dense` = True)."""

    dense = False

    def __init__(self, source, ep_ids, t_len=None):
        self.source = source
        self.ep_ids_np = np.asarray(ep_ids, dtype=np.int64)
        self._ep_ids_dev = None
        self.t_len = source.max_seq_length if t_len is None else int(t_len)
        super().__init__(source.scheme, source.groups, len(self.ep_ids_np), self.t_len,
                         data=SN(transition_data=_LazyGather(self, True), episode_data=_LazyGather(self, False)),
                         preprocess=None, device=source.device)

    def __getitem__(self, item):
        if self.dense:
            return EpisodeBatch.__getitem__(self, item)
        if isinstance(item, tuple) and len(item) == 2 and isinstance(item[0], slice) and item[0] == slice(None) \
                and isinstance(item[1], slice) and item[1].start in (None, 0) and item[1].step in (None, 1):
            stop = self.t_len if item[1].stop is None else min(int(item[1].stop), self.t_len)
            return SampledBatch._view(self, stop)
        if isinstance(item, str):
            return self.data.episode_data[item] if item in self.source.data.episode_data \
                else self.data.transition_data[item]
        return self.materialize()[item]

    @property
    def ep_ids(self):
        """Device copy of the ids, uploaded on first use (the learner passes small id sets in kernel arguments)."""
        if self._ep_ids_dev is None:
            host = th.from_numpy(self.ep_ids_np)
            if th.device(self.source.device).type == "cuda":
                # pinned + async: the id upload is stream-ordered and never stalls the host on earlier kernels
                self._ep_ids_dev = host.pin_memory().to(self.source.device, non_blocking=True)
            else:
                self._ep_ids_dev = host.to(self.source.device)
        return self._ep_ids_dev

    @classmethod
    def _view(cls, other, t_len):
        new = cls.__new__(cls)
        new.source, new.ep_ids_np, new.t_len = other.source, other.ep_ids_np, int(t_len)
        new._ep_ids_dev = other._ep_ids_dev
        new.dp_shard = other.dp_shard
        EpisodeBatch.__init__(new, other.source.scheme, other.source.groups, len(other.ep_ids_np), new.t_len,
                              data=SN(transition_data=_LazyGather(new, True), episode_data=_LazyGather(new, False)),
                              preprocess=None, device=other.source.device)
        return new

    def materialize(self):
        """The reference's EpisodeBatch for these ids (episode_buffer.py:205-217 gather + time truncation)."""
        td = {k: v[self.ep_ids][:, :self.t_len] for k, v in self.source.data.transition_data.items()}
        ed = {k: v[self.ep_ids] for k, v in self.source.data.episode_data.items()}
        return EpisodeBatch(self.scheme, self.groups, self.batch_size, self.t_len,
                            data=SN(transition_data=td, episode_data=ed), device=self.device)

    def max_t_filled(self):
        lens = self.source.episode_lengths
        if lens is not None:   # host lengths: valid for the dense copy too (same episodes, same t_len)
            return int(min(lens[self.ep_ids_np].max(), self.t_len))
        return int(self.materialize().max_t_filled())

    def shard(self, rank, world):
        """Contiguous slice [rank*B/world, (rank+1)*B/world) of the episodes. The data-parallel learners
        take the GLOBAL sample and call this themselves (learners/dp.py local_shard); the result is tagged so that
        passing it to a data-parallel train() is an error rather than a second sharding."""
        from ..learners.dp import shard_bounds
        lo, hi = shard_bounds(len(self.ep_ids_np), rank, world)
        if self.dense:
            out = EpisodeBatch.__getitem__(self, slice(lo, hi))
        else:
            out = SampledBatch(self.source, self.ep_ids_np[lo:hi], self.t_len)
        out.dp_shard = (rank, world)   # a data-parallel learner rejects it: train() takes the global sample
        return out

    def to(self, device):
        """EpisodeBatch.to (episode_buffer.py:91-96), in place as run.py:214-215 calls it. On the buffer's own device
        it is a no-op (the kernels gather by id from the buffer). Otherwise — a host-resident buffer
        (buffer_cpu_only) moving to the GPU — the sampled episodes are gathered on the host, truncated to t_len
        (the reference's fancy index + `[:, :max_t]`, :205-217), and each field is copied to `device` once, from
        pinned memory on the current stream. The batch is dense from then on."""
        if _same_device(device, self.device):
            return self
        mat = self.materialize()
        to_gpu = th.device(device).type == "cuda"
        moved = SN(transition_data={}, episode_data={})
        for src, dst in ((mat.data.transition_data, moved.transition_data),
                         (mat.data.episode_data, moved.episode_data)):
            for k, v in src.items():
                v = v.contiguous()
                if to_gpu and v.device.type == "cpu":
                    v = v.pin_memory()
                dst[k] = v.to(device, non_blocking=to_gpu)
        self.data = moved
        self.device = device
        self.dense = True
        return self


class _LazyGather(dict):
    def __init__(self, batch, transition):
        super().__init__()
        self._b, self._t = batch, transition

    def _src(self):
        s = self._b.source.data
        return s.transition_data if self._t else s.episode_data

    def __getitem__(self, k):
        v = self._src()[k][self._b.ep_ids]
        return v[:, :self._b.t_len] if self._t else v

    def __contains__(self, k):
        return k in self._src()

    def keys(self):
        return self._src().keys()

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def __iter__(self):
        return iter(self.keys())


class ReplayBuffer(EpisodeBatch):
    def __init__(self, scheme, groups, buffer_size, max_seq_length, preprocess=None, device="cpu"):
        super().__init__(scheme, groups, buffer_size, max_seq_length, preprocess=preprocess, device=device)
        self.buffer_size = buffer_size
        self.buffer_index = 0
        self.episodes_in_buffer = 0
        self.episode_lengths = np.zeros(buffer_size, dtype=np.int64)   # sum(filled) per episode, host side
        # A bitmask view of avail_actions ([N][T][agents] int64, bit a = action a available); the learner's mixer
        # reads 8 bytes per agent row from it instead of 4 n_actions (mq_replay.avail_bits). It is a derived cache, so
        # it remembers which storage it was built from: (the avail_actions tensor's data pointer, its in-place write
        # counter `_version`, which every write bumps, through views and indexing included). avail_bits_current()
        # rebuilds it whenever that stamp moved, so a write that bypasses update() (e.g.
        # `transition_data["avail_actions"][...] = x`, or a replaced tensor) can never leave the mixer reading stale
        # bits; the write paths below keep it current cheaply, rebuilding only the rows they wrote.
        av = self.data.transition_data.get("avail_actions")
        self.avail_bits = None
        self._bits_at = None
        if av is not None and av.dim() >= 3 and 0 < av.shape[-1] <= 64:
            self.avail_bits = th.zeros(av.shape[:-1], dtype=th.int64, device=av.device)
            self._bits_at = self._avail_stamp()   # zero storage, zero bits

    def _avail_stamp(self):
        av = self.data.transition_data.get("avail_actions")
        return None if av is None else (av.data_ptr(), av._version)

    def _bits_fresh(self):
        return self.avail_bits is not None and self._bits_at == self._avail_stamp()

    def refresh_avail_bits(self, bs=slice(None)):
        if self.avail_bits is None:
            return
        av = self.data.transition_data["avail_actions"][bs]
        w = th.ones(av.shape[-1], dtype=th.int64, device=av.device) << th.arange(av.shape[-1], device=av.device)
        self.avail_bits[bs] = ((av != 0).to(th.int64) * w).sum(-1)   # distinct bits: the sum is the OR
        self._bits_at = self._avail_stamp()

    def avail_bits_current(self):
        """The avail bitmask, rebuilt first if avail_actions was written since it was last built (None when the
        buffer has no bitmask: no avail_actions, or more than 64 actions)."""
        if self.avail_bits is None:
            return None
        if not self._bits_fresh():
            self.refresh_avail_bits()
        return self.avail_bits

    def update(self, data, bs=slice(None), ts=slice(None), mark_filled=True):
        fresh = self._bits_fresh()   # before this write: were the bits current?
        super().update(data, bs, ts, mark_filled)
        if "avail_actions" in data:
            # only the written rows, unless something else wrote the storage since the last rebuild
            self.refresh_avail_bits(self._parse_slices((bs, ts))[0] if fresh else slice(None))

    def to(self, device):
        fresh = self._bits_fresh()
        super().to(device)
        if self.avail_bits is not None:
            self.avail_bits = self.avail_bits.to(device)
            if fresh:
                self._bits_at = self._avail_stamp()
        return self

    def insert_episode_batch(self, ep_batch):
        if self.buffer_index + ep_batch.batch_size <= self.buffer_size:
            sl = slice(self.buffer_index, self.buffer_index + ep_batch.batch_size)
            self.update(ep_batch.data.transition_data, sl, slice(0, ep_batch.max_seq_length), mark_filled=False)
            self.update(ep_batch.data.episode_data, sl)
            filled = ep_batch.data.transition_data["filled"]
            self.episode_lengths[sl] = filled.sum(1).reshape(-1).cpu().numpy()
            self.buffer_index += ep_batch.batch_size
            self.episodes_in_buffer = max(self.episodes_in_buffer, self.buffer_index)
            self.buffer_index = self.buffer_index % self.buffer_size
            assert self.buffer_index < self.buffer_size
        else:
            left = self.buffer_size - self.buffer_index
            self.insert_episode_batch(ep_batch[0:left, :])
            self.insert_episode_batch(ep_batch[left:, :])

    def load_arrays(self, arrays, n_episodes=None):
        """Bulk-fill the storage from numpy/torch arrays in the scheme layout (synthetic replay, checkpoints)."""
        n = n_episodes if n_episodes is not None else len(next(iter(arrays.values())))
        fresh = self._bits_fresh()
        for k, v in arrays.items():
            if k in self.data.transition_data:
                self.data.transition_data[k][:n] = th.as_tensor(v, device=self.device)
            elif k in self.data.episode_data:
                self.data.episode_data[k][:n] = th.as_tensor(v, device=self.device)
        self.episode_lengths[:n] = self.data.transition_data["filled"][:n].sum(1).reshape(-1).cpu().numpy()
        self.refresh_avail_bits(slice(0, n) if fresh else slice(None))
        self.episodes_in_buffer = max(self.episodes_in_buffer, n)
        self.buffer_index = n % self.buffer_size

    def can_sample(self, batch_size):
        return self.episodes_in_buffer >= batch_size

    def sample(self, batch_size):
        assert self.can_sample(batch_size)
        if self.episodes_in_buffer == batch_size:
            ids = np.arange(batch_size)
        else:
            ids = np.random.choice(self.episodes_in_buffer, batch_size, replace=False)
        return SampledBatch(self, ids)

    def __repr__(self):
        return "ReplayBuffer. {}/{} episodes. Keys:{} Groups:{}".format(
            self.episodes_in_buffer, self.buffer_size, self.scheme.keys(), self.groups.keys())
