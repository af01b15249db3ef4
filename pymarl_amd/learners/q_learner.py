"""QLearner: QMIX / VDN / IQL learner (reference: src/learners/q_learner.py:9-143), MI355X-native.

Same constructor, `train(batch, t_env, episode_num)`, `_update_targets`, `cuda`, `save_models`, `load_models`,
the five logged stats and the episode-counted hard target update. The whole of train() — replay gather,
both GRU unrolls, double-Q selection, mixer, masked L2 TD loss, BPTT, clip_grad_norm_, RMSprop — is one
launch sequence of hand-written HIP kernels in libmq_learner.so (include/mq_learner.h); torch only owns the
device buffers. There is no CPU path: a learner that is not on a HIP device raises.

Data parallel: with `args.learner_dp = True` and torch.distributed initialised (RCCL, one process
per GPU), every rank calls train() with the SAME GLOBAL sample, as run.py:207-219 does unchanged (ranks share the
seed, so the sampled ids agree; ids and contents checked on a call-count schedule, `args.learner_dp_check`); the
learner trains its own contiguous shard
of the episodes (dp.local_shard), the unnormalised gradient buffer (+ the loss/mask sums in its tail) is summed with
ONE all_reduce, and every rank then applies the identical normalised update. Under an RCCL process group the learner
borrows the process's library communicator (dp.SharedComm: mq_comm_create once, mq_comm_use per handle): the
all-reduce is then issued inside mq_forward_backward, in stream order, and a train step makes no Python call between
its kernels. Other backends (gloo) all-reduce from Python (dp.py).
"""
from __future__ import annotations

import copy
import ctypes

import numpy as np

import torch as th
from torch.optim import RMSprop

from .. import _lib
from ..components.episode_buffer import is_replay_view
from ..modules.flat import pack, rebind
from .dp import DPCheck, SharedComm, allreduce_grad_buffer, dp_world, local_shard, native_comm_wanted
from ..modules.mixers.qmix import QMixer
from ..modules.mixers.vdn import VDNMixer

MIXER_IDS = {None: _lib.MIXER_NONE, "vdn": _lib.MIXER_VDN, "qmix": _lib.MIXER_QMIX}
_FIELDS = [("obs", th.float32), ("state", th.float32), ("actions", th.int64), ("avail_actions", th.int32),
           ("reward", th.float32), ("terminated", th.uint8), ("filled", th.int64)]


def make_config(args, mixer, input_dim=None, max_batch=1, max_seq=2):
    cfg = _lib.MQConfig()
    cfg.n_agents = args.n_agents
    cfg.n_actions = args.n_actions
    obs = getattr(args, "obs_shape", None)
    if obs is None and input_dim is not None:
        obs = input_dim - (args.n_actions if args.obs_last_action else 0) - (args.n_agents if args.obs_agent_id else 0)
    cfg.obs_dim = int(obs)
    st = getattr(args, "state_shape", 1)
    cfg.state_dim = int(st if isinstance(st, int) else th.Size(st).numel())
    cfg.rnn_hidden_dim = args.rnn_hidden_dim
    cfg.mixing_embed_dim = getattr(args, "mixing_embed_dim", 32)
    cfg.mixer = mixer
    cfg.double_q = int(bool(getattr(args, "double_q", True)))
    cfg.obs_last_action = int(bool(args.obs_last_action))
    cfg.obs_agent_id = int(bool(args.obs_agent_id))
    cfg.gamma = getattr(args, "gamma", 0.99)
    cfg.lr = getattr(args, "lr", 5e-4)
    cfg.optim_alpha = getattr(args, "optim_alpha", 0.99)
    cfg.optim_eps = getattr(args, "optim_eps", 1e-5)
    cfg.grad_norm_clip = getattr(args, "grad_norm_clip", 10.0)
    cfg.max_batch = int(max_batch)
    cfg.max_seq = int(max_seq)
    # opt-in masked Huber TD loss (north_star; the reference has L2 only, q_learner.py:96-97): td_loss: huber,
    # huber_delta (default 1.0); anything else keeps L2
    cfg.huber_delta = float(getattr(args, "huber_delta", 1.0)) if getattr(args, "td_loss", "l2") == "huber" else 0.0
    return cfg


def _field_view(t, dtype):
    """(tensor usable by the kernels, t_stride): [B][T][...] with trailing dims contiguous and the right dtype."""
    if t.dtype != dtype:
        t = t.to(dtype)
    inner = 1
    for s in t.shape[2:]:
        inner *= s
    ok = t.stride(1) == inner and t.stride(0) % max(1, inner) == 0 and t[0, 0].is_contiguous()
    if not ok:
        t = t.contiguous()
    return t, t.stride(0) // max(1, inner)


def replay_view(batch, avail_bits=True):
    """MQReplay for an EpisodeBatch (episode-major storage) or a SampledBatch (storage + device ids).
    Returns (struct, keepalive) — keep the second alive until the kernels that read it have been queued.
    avail_bits: hand the kernels the buffer's avail bitmask (ReplayBuffer.avail_bits_current: rebuilt first if the
    storage was written behind its back), else they read the int32 avail_actions rows."""
    keep = []
    rep = _lib.MQReplay()
    if is_replay_view(batch):
        src = batch.source.data.transition_data
        tstride = batch.source.max_seq_length
        if len(batch.ep_ids_np) <= _lib.INLINE_IDS:
            # ids travel in the kernel arguments: no host-to-device copy on the step's stream
            host = np.ascontiguousarray(batch.ep_ids_np, dtype=np.int64)
            keep.append(host)
            rep.ep_ids_host = host.ctypes.data
            rep.ep_ids = None
        else:
            ids = batch.ep_ids
            keep.append(ids)
            rep.ep_ids = ids.data_ptr()
        rep.n_episodes = batch.source.batch_size
        rep.t_len = batch.t_len
        tensors = {}
        for k, dt in _FIELDS:
            if k not in src:
                continue
            t = src[k]
            if t.dtype != dt or not t.is_contiguous():
                raise _lib.MQError("replay field {} must be a contiguous {} tensor".format(k, dt))
            tensors[k] = t
        cur = getattr(batch.source, "avail_bits_current", None)
        bits = cur() if (avail_bits and cur is not None) else None
        if bits is not None:
            keep.append(bits)
            rep.avail_bits = bits.data_ptr()
    else:
        src = batch.data.transition_data
        tensors, strides = {}, set()
        for k, dt in _FIELDS:
            if k not in src:
                continue
            t, ts = _field_view(src[k], dt)
            tensors[k] = t
            strides.add(ts)
        if len(strides) != 1:
            tensors = {k: v.contiguous() for k, v in tensors.items()}
            strides = {batch.max_seq_length}
        tstride = strides.pop()
        rep.ep_ids = None
        rep.n_episodes = batch.batch_size
        rep.t_len = batch.max_seq_length
    for k, t in tensors.items():
        keep.append(t)
        setattr(rep, k, t.data_ptr())
    _lib.require_gpu(tensors["obs"])
    rep.batch_size = batch.batch_size
    rep.t_stride = int(tstride)
    return rep, keep


class QLearner:
    def __init__(self, mac, scheme, logger, args):
        self.args = args
        self.mac = mac
        self.logger = logger
        self.params = list(mac.parameters())
        self.last_target_update_episode = 0
        self.mixer = None
        if args.mixer is not None:
            if args.mixer == "vdn":
                self.mixer = VDNMixer()
            elif args.mixer == "qmix":
                self.mixer = QMixer(args)
            else:
                raise ValueError("Mixer {} not recognised.".format(args.mixer))
            self.params += list(self.mixer.parameters())
            self.target_mixer = copy.deepcopy(self.mixer)
        self.optimiser = RMSprop(params=self.params, lr=args.lr, alpha=args.optim_alpha, eps=args.optim_eps)
        self.target_mac = copy.deepcopy(mac)
        self.log_stats_t = -self.args.learner_log_interval - 1
        self.dp = bool(getattr(args, "learner_dp", False))
        # when to check that the ranks passed the same global sample (ids AND contents): a call-count schedule, the
        # same on every rank (dp.DPCheck: "first", "always", "off" or every N calls, default 100)
        self.dp_check = DPCheck(getattr(args, "learner_dp_check", None))
        # the mixer's double-Q selection reads the replay buffer's avail bitmask (False: the int32 avail_actions rows;
        # bitwise the same result, test_avail_bits_bitwise)
        self.use_avail_bits = bool(getattr(args, "learner_avail_bits", True))

        # flat device buffers: [agent params | mixer params] for online and target nets (MQ_P_* order)
        self._mods = [m for m in (self.mac.agent, self.mixer) if m is not None and len(list(m.parameters()))]
        self._tmods = [m for m in (self.target_mac.agent, getattr(self, "target_mixer", None))
                       if m is not None and len(list(m.parameters()))]
        dev = self.mac.agent.fc1.weight.device
        self._online, self.n_params = pack(self._mods, device=dev)
        self._target, _ = pack(self._tmods, device=dev)
        self._alloc_state(dev)
        self._handle = None
        self._handle_key = None
        self._opt_steps = 0

    # -- buffers ---------------------------------------------------------------------------------------------
    def _alloc_state(self, dev):
        P = self.n_params
        self._grad = th.zeros(P + _lib.NSUMS, dtype=th.float32, device=dev)
        self._sq = th.zeros(P, dtype=th.float32, device=dev)
        self._stats = th.zeros(_lib.NSTATS, dtype=th.float32, device=dev)
        self._curmax = None
        self._relink()

    def _relink(self):
        """Point module params, .grad and the optimiser's square_avg at the flat buffers."""
        Pa = sum(p.numel() for p in self.mac.agent.parameters())
        rebind(self._mods, self._online)
        rebind(self._tmods, self._target)
        self.mac.agent._flat = self._online[:Pa]
        self.target_mac.agent._flat = self._target[:Pa]
        if self.mixer is not None and hasattr(self.mixer, "_flat"):
            self.mixer._flat = self._online[Pa:self.n_params]
            self.target_mixer._flat = self._target[Pa:self.n_params]
        self._step_t = th.tensor(float(getattr(self, "_opt_steps", 0)))
        o = 0
        for p in self.params:
            n = p.numel()
            p.grad = self._grad[o:o + n].view_as(p)
            st = self.optimiser.state[p]
            st["square_avg"] = self._sq[o:o + n].view_as(p)
            st["step"] = self._step_t   # one shared counter: train() increments it once, not once per parameter
            o += n
        self._handle = None

    def _dp_active(self):
        if not self.dp:
            return False
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1

    def _local_batch(self, batch):
        """Data parallel: this rank's shard of the global sample (dp.local_shard), the ranks' agreement checked per
        `self.dp_check`."""
        rank, world = dp_world()
        check = self.dp_check.due()
        out = local_shard(batch, rank, world, check=check, device=self._online.device)
        self.dp_check.done += int(check)
        return out

    def _get_handle(self, batch):
        T = batch.source.max_seq_length if is_replay_view(batch) else batch.max_seq_length
        world = dp_world()[1] if self._dp_active() else 1
        need_b = max(batch.batch_size, -(-getattr(self.args, "batch_size", 1) // world))
        key = (need_b, T)
        if SharedComm.stale(self._handle):
            self._handle = None   # its communicator was freed (SharedComm.free detached it): rebuild and re-attach
        if self._handle is None or self._handle_key[0] < need_b or self._handle_key[1] < T:
            cfg = make_config(self.args, MIXER_IDS[self.args.mixer], input_dim=self.mac.agent.input_dim,
                              max_batch=need_b, max_seq=T)
            h = _lib.Handle(cfg)
            Tmax = T
            self._curmax = th.zeros(Tmax * need_b * self.args.n_agents, dtype=th.int32, device=self._online.device)
            _lib.check(h.lib.mq_bind(h.h, _lib.ptr(self._online), _lib.ptr(self._target), _lib.ptr(self._grad),
                                     _lib.ptr(self._sq), _lib.ptr(self._stats), _lib.ptr(self._curmax)))
            h.dp_on = False
            h.native = False
            if self._dp_active() and native_comm_wanted(self._online.device):
                # the process's communicator, created once (a handle rebuilt later needs no collective to attach)
                SharedComm.lend(h, "mq_comm_use", "mq_comm_detach", self._online.device)
            if h.n_params != self.n_params:
                raise _lib.MQError("parameter layout mismatch: library {} vs modules {}".format(h.n_params,
                                                                                              self.n_params))
            self._handle, self._handle_key = h, key
        return self._handle

    # -- reference API ---------------------------------------------------------------------------------------
    def train(self, batch, t_env: int, episode_num: int):
        _lib.require_gpu(self._online)
        # decided per call: torch.distributed may be initialised after the handle was created; mq_apply must then
        # recompute the gradient norm from the all-reduced buffer
        dp = self._dp_active()
        if dp:
            batch = self._local_batch(batch)
        h = self._get_handle(batch)
        want = dp or getattr(self, "force_dp_norm", False)
        if want != h.dp_on:
            _lib.check(h.lib.mq_set_data_parallel(h.h, int(want)))
            h.dp_on = want
        rep, keep = replay_view(batch, self.use_avail_bits)
        lib, s = h.lib, _lib.stream_ptr()
        if dp and not h.native:
            _lib.check(lib.mq_forward_backward(h.h, ctypes.byref(rep), s))
            allreduce_grad_buffer(self._grad)
            _lib.check(lib.mq_apply(h.h, s))
        else:
            # one call: mq_forward_backward (+ the native all-reduce when attached) and mq_apply
            _lib.check(lib.mq_train_step(h.h, ctypes.byref(rep), s))
        self._opt_steps += 1
        self._step_t += 1   # every parameter's optimiser state holds this tensor (see save_models)
        self._last_batch = (batch.batch_size, rep.t_len)
        del keep

        if (episode_num - self.last_target_update_episode) / self.args.target_update_interval >= 1.0:
            self._update_targets()
            self.last_target_update_episode = episode_num

        if t_env - self.log_stats_t >= self.args.learner_log_interval:
            st = self._stats.tolist()
            self.logger.log_stat("loss", st[0], t_env)
            self.logger.log_stat("grad_norm", st[1], t_env)
            self.logger.log_stat("td_error_abs", st[2], t_env)
            self.logger.log_stat("q_taken_mean", st[3], t_env)
            self.logger.log_stat("target_mean", st[4], t_env)
            self.log_stats_t = t_env

    def _update_targets(self):
        if self._online.is_cuda and self._handle is not None:
            _lib.check(self._handle.lib.mq_update_targets(self._handle.h, _lib.stream_ptr()))
        else:
            with th.no_grad():
                self._target.copy_(self._online)
        self.logger.console_logger.info("Updated target network")

    def cuda(self):
        dev = th.device("cuda", th.cuda.current_device())
        self._online = self._online.to(dev)
        self._target = self._target.to(dev)
        self._grad = self._grad.to(dev)
        self._sq = self._sq.to(dev)
        self._stats = self._stats.to(dev)
        self._relink()

    def save_models(self, path):
        self.mac.save_models(path)
        if self.mixer is not None:
            th.save(self.mixer.state_dict(), "{}/mixer.th".format(path))
        # per-parameter step tensors in the file, as torch's RMSprop writes them: the live state shares one counter,
        # and a loader that kept it shared would count every parameter's update into it
        sd = self.optimiser.state_dict()
        sd["state"] = {i: dict(v, step=v["step"].clone()) if "step" in v else v for i, v in sd["state"].items()}
        th.save(sd, "{}/opt.th".format(path))

    def load_models(self, path):
        self.mac.load_models(path)
        # Not quite right but I don't want to save target networks (reference comment, q_learner.py:139)
        self.target_mac.load_models(path)
        ml = lambda s, loc: s  # noqa: E731
        if self.mixer is not None:
            self.mixer.load_state_dict(th.load("{}/mixer.th".format(path), map_location=ml, weights_only=True))
        sd = th.load("{}/opt.th".format(path), map_location=ml, weights_only=True)
        self.optimiser.load_state_dict(sd)
        o = 0
        for p in self.params:   # load_state_dict replaced the state tensors: copy back into the flat buffer
            n = p.numel()
            st = self.optimiser.state.get(p, {})
            if "square_avg" in st:
                self._sq[o:o + n].copy_(st["square_avg"].reshape(-1))
            o += n
        steps = [float(self.optimiser.state[p]["step"]) for p in self.params if "step" in self.optimiser.state[p]]
        self._opt_steps = int(steps[0]) if steps else 0
        self._relink()

    # -- extras (parity / diagnostics) -----------------------------------------------------------------------
    def collective(self):
        """How a data-parallel step sums the gradient buffer: "rccl-native" (the library's communicator),
        "torch.distributed", or None (not data parallel)."""
        if not self._dp_active():
            return None
        return "rccl-native" if (self._handle is not None and self._handle.native) else "torch.distributed"

    def last_stats(self):
        """dict of the last step's stats (loss, grad_norm, td_error_abs, q_taken_mean, target_mean, mask_sum)."""
        st = self._stats.tolist()
        return dict(loss=st[0], grad_norm=st[1], td_error_abs=st[2], q_taken_mean=st[3], target_mean=st[4],
                    mask_sum=st[5])

    def last_plan(self):
        """Kernel variants the last train() launched (mq_last_plan): rows, fused_fwd, rw_fwd, fused_bwd, rw_bwd,
        inline_ids, hyper, mix, tiles, dwh (where QMIX's dW_hyper ran: "red1" or "bptt_grid")."""
        pl = _lib.MQPlan()
        _lib.check(self._handle.lib.mq_last_plan(self._handle.h, ctypes.byref(pl)))
        d = pl.as_dict()
        d["hyper"] = _lib.HYP_NAMES[d["hyper"]]
        d["mix"] = _lib.MIX_NAMES[d["mix"]]
        d["dwh"] = ("red1", "bptt_grid")[d["dwh"]]
        return d

    def last_cur_max_actions(self):
        """Double-Q greedy actions of the last step as (B, T, n) int64 (q_learner.py:75)."""
        B, Tp = self._last_batch
        n = self.args.n_agents
        a = self._curmax[:(Tp - 1) * B * n].view(Tp - 1, B, n)
        return a.permute(1, 0, 2).long()

    def last_intermediate(self, which):
        """0 / 1: online / target mac_out as (B, T+1, n, A); 2: dLoss_num/dchosen as (B, T, n);
        3: online relu(fc1(inputs)) as (B, T+1, n, 64)."""
        B, Tp = self._last_batch
        n, A = self.args.n_agents, self.args.n_actions
        cnt = ctypes.c_int64()
        h = self._handle
        _lib.check(h.lib.mq_copy_intermediate(h.h, which, None, ctypes.byref(cnt), None))
        out = th.empty(cnt.value, dtype=th.float32, device=self._online.device)
        _lib.check(h.lib.mq_copy_intermediate(h.h, which, _lib.ptr(out), ctypes.byref(cnt), _lib.stream_ptr()))
        if which in (0, 1):
            return out.view(Tp, B, n, A).permute(1, 0, 2, 3)
        if which == 3:
            return out.view(Tp, B, n, -1).permute(1, 0, 2, 3)
        return out.view(Tp - 1, B, n).permute(1, 0, 2)

    def set_timing(self, slots=1, phases=None):
        """Record HIP events around the named phases (None = all) for the next `slots` steps (0 = off)."""
        h = self._handle
        names = h.lib.mq_phase_names().decode().split(";")
        mask = 0xFFFFFFFF if phases is None else sum(1 << names.index(p) for p in phases)
        _lib.check(h.lib.mq_set_timing(h.h, int(slots), mask))

    def phase_times(self):
        h = self._handle
        ms = (ctypes.c_float * 32)()
        n = ctypes.c_int32()
        _lib.check(h.lib.mq_phase_times(h.h, ms, 32, ctypes.byref(n)))
        names = h.lib.mq_phase_names().decode().split(";")
        return {names[i]: ms[i] for i in range(n.value)}

    def phase_names(self):
        return _lib.load().mq_phase_names().decode().split(";")
