"""COMALearner: counterfactual multi-agent policy gradients (reference: src/learners/coma_learner.py:9-171),
MI355X-native.

Same constructor, `train(batch, t_env, episode_num)`, `_update_targets`, `cuda`, `save_models`, `load_models`, the
nine logged stats and the critic-step-counted hard target update. All of train() — the critic's all-steps target
pass, TD(lambda), the T sequential critic RMSprop steps, the actor's GRU unroll, the pi_logits policy, the
counterfactual baseline and the policy-gradient BPTT, both clips and both RMSprop steps — is one launch sequence of
hand-written HIP kernels (include/mc_coma.h, pymarl_amd/csrc/coma_kernels.hpp); torch only owns the buffers.
There is no CPU path. One synchronisation per train(): the stats read-back the target update needs.

Data parallel (not in the reference): with `args.learner_dp = True` and torch.distributed initialised,
every rank passes the SAME global sample to train() and trains its share of it, in one of two modes
(`args.coma_dp_mode`, default "auto"):
* "replicated" (auto when B * n_agents <= 80, the persistent critic chain's limit; coma_smac's B = 8 at MMM2's 10
  agents): every rank runs the critic's T steps on the whole batch — identical on every rank, so no per-step
  exchange — and the actor on its own episodes, with ONE all-reduce of the agent gradient (mc_set_actor_shard);
* "exchange": every rank trains its shard, and the library sums the global per-step mask sums, each live critic
  step's gradient, the critic stat sums and the agent gradient across ranks (T + 3 all-reduces per train;
  include/mc_coma.h, mc_set_data_parallel).
The ranks' agreement on the global sample (ids and contents) is checked on a call-count schedule that is the same on
every rank (`args.learner_dp_check`, dp.DPCheck / dp.check_same_batch): in
"replicated" mode every rank's critic must see the same batch or the critics drift apart silently. A batch that is
already a shard is rejected. Under an RCCL process group the exchanges run on the process's library communicator
(dp.SharedComm: mq_comm_create once, mc_comm_use per handle), in stream order with no Python callback; other backends
call back into `dist.all_reduce`. A critic-chain timeout on any rank is all-reduced with the agent gradient, so every
rank rolls the train() back and raises together.

Reference quirk kept on purpose: the actor reads `mac.action_selector.epsilon`, the value the last rollout call of
select_actions left there (basic_controller.py:64-67).
"""
from __future__ import annotations

import copy
import ctypes

import torch as th
from torch.optim import RMSprop

from .. import _lib
from ..modules.critics.coma import COMACritic
from ..modules.flat import pack, rebind
from .dp import DPCheck, SharedComm, dp_world, local_shard, native_comm_wanted, shard_bounds
from .q_learner import replay_view
from ..components.episode_buffer import is_replay_view

CC_MAXR = 80   # coma_chain.hpp: most critic rows (B * n_agents) the persistent chain takes


def make_coma_config(args, input_dim, max_batch, max_seq):
    cfg = _lib.MCConfig()
    cfg.n_agents = args.n_agents
    cfg.n_actions = args.n_actions
    cfg.obs_dim = int(input_dim - (args.n_actions if args.obs_last_action else 0) -
                      (args.n_agents if args.obs_agent_id else 0))
    st = getattr(args, "state_shape", 1)
    cfg.state_dim = int(st if isinstance(st, int) else th.Size(st).numel())
    cfg.rnn_hidden_dim = args.rnn_hidden_dim
    cfg.obs_last_action = int(bool(args.obs_last_action))
    cfg.obs_agent_id = int(bool(args.obs_agent_id))
    cfg.mask_before_softmax = int(bool(getattr(args, "mask_before_softmax", True)))
    cfg.gamma = args.gamma
    cfg.td_lambda = args.td_lambda
    cfg.lr = args.lr
    cfg.critic_lr = args.critic_lr
    cfg.optim_alpha = args.optim_alpha
    cfg.optim_eps = args.optim_eps
    cfg.grad_norm_clip = args.grad_norm_clip
    cfg.max_batch = int(max_batch)
    cfg.max_seq = int(max_seq)
    return cfg


class COMALearner:
    def __init__(self, mac, scheme, logger, args):
        self.args = args
        self.n_agents = args.n_agents
        self.n_actions = args.n_actions
        self.mac = mac
        self.logger = logger
        self.last_target_update_step = 0
        self.critic_training_steps = 0
        self.log_stats_t = -self.args.learner_log_interval - 1
        self.critic = COMACritic(scheme, args)
        self.target_critic = copy.deepcopy(self.critic)
        self.agent_params = list(mac.parameters())
        self.critic_params = list(self.critic.parameters())
        self.params = self.agent_params + self.critic_params
        self.agent_optimiser = RMSprop(params=self.agent_params, lr=args.lr, alpha=args.optim_alpha,
                                       eps=args.optim_eps)
        self.critic_optimiser = RMSprop(params=self.critic_params, lr=args.critic_lr, alpha=args.optim_alpha,
                                        eps=args.optim_eps)
        dev = self.mac.agent.fc1.weight.device
        self._agent, self.n_agent_params = pack([self.mac.agent], device=dev)
        self._critic, self.n_critic_params = pack([self.critic], device=dev)
        self._tcritic, _ = pack([self.target_critic], device=dev)
        self._alloc_state(dev)
        self._handle = None
        self._handle_key = None
        self._steps = 0
        self.dp = bool(getattr(args, "learner_dp", False))
        self.dp_check = DPCheck(getattr(args, "learner_dp_check", None))   # call-count schedule (see QLearner)
        self._dp_cb = None
        self._dp_scratch = None

    # -- buffers ---------------------------------------------------------------------------------------------
    def _alloc_state(self, dev):
        Pa, Pc = self.n_agent_params, self.n_critic_params
        self._agrad = th.zeros(Pa + _lib.NSUMS, dtype=th.float32, device=dev)
        self._asq = th.zeros(Pa, dtype=th.float32, device=dev)
        self._cgrad = th.zeros(Pc + _lib.MC_NTAIL, dtype=th.float32, device=dev)
        self._csq = th.zeros(Pc, dtype=th.float32, device=dev)
        self._stats = th.zeros(_lib.MC_NSTATS, dtype=th.float32, device=dev)
        self._relink()

    def _relink(self):
        """Point module params, .grad and both optimisers' square_avg at the flat buffers."""
        rebind([self.mac.agent], self._agent)
        rebind([self.critic], self._critic)
        rebind([self.target_critic], self._tcritic)
        self.mac.agent._flat = self._agent
        self.critic._flat = self._critic
        self.target_critic._flat = self._tcritic
        for params, grad, sq, opt in ((self.agent_params, self._agrad, self._asq, self.agent_optimiser),
                                      (self.critic_params, self._cgrad, self._csq, self.critic_optimiser)):
            o = 0
            for p in params:
                n = p.numel()
                p.grad = grad[o:o + n].view_as(p)
                st = opt.state[p]
                st["square_avg"] = sq[o:o + n].view_as(p)
                st.setdefault("step", th.tensor(0.0))
                o += n
        self._handle = None

    def _get_handle(self, batch):
        T = batch.source.max_seq_length if is_replay_view(batch) else batch.max_seq_length
        need_b = max(batch.batch_size, getattr(self.args, "batch_size", 1))
        if SharedComm.stale(self._handle):
            self._handle = None   # its communicator was freed (SharedComm.free detached it): rebuild and re-attach
        if self._handle is None or self._handle_key[0] < need_b or self._handle_key[1] < T:
            cfg = make_coma_config(self.args, self.mac.agent.input_dim, need_b, T)
            h = _lib.ComaHandle(cfg)
            if h.agent_offsets[-1] != self.n_agent_params or h.critic_offsets[-1] != self.n_critic_params:
                raise _lib.MQError("parameter layout mismatch: library ({}, {}) vs modules ({}, {})".format(
                    h.agent_offsets[-1], h.critic_offsets[-1], self.n_agent_params, self.n_critic_params))
            P = _lib.ptr
            _lib.check(h.lib.mc_bind(h.h, P(self._agent), P(self._agrad), P(self._asq), P(self._critic),
                                     P(self._tcritic), P(self._cgrad), P(self._csq), P(self._stats)))
            h.native = False
            if self._dp_active():
                rank, world = dp_world()
                if native_comm_wanted(self._critic.device):
                    SharedComm.lend(h, "mc_comm_use", "mc_comm_detach", self._critic.device)
                else:
                    self._dp_scratch = th.zeros(8 * T, dtype=th.float32, device=self._critic.device)
                    self._dp_cb = _lib.MC_ALLREDUCE_FN(self._allreduce)
                    _lib.check(h.lib.mc_set_data_parallel(h.h, self._dp_cb, None, rank, P(self._dp_scratch),
                                                          self._dp_scratch.numel()))
            self._handle, self._handle_key = h, (need_b, T)
        return self._handle

    def _dp_active(self):
        if not self.dp:
            return False
        import torch.distributed as dist
        return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1

    def dp_mode(self, batch_size):
        """None (not data parallel), "replicated" or "exchange" for a global batch of `batch_size` episodes."""
        if not self._dp_active():
            return None
        mode = getattr(self.args, "coma_dp_mode", "auto")
        if mode == "auto":
            mode = "replicated" if batch_size * self.n_agents <= CC_MAXR else "exchange"
        if mode not in ("replicated", "exchange"):
            raise ValueError("coma_dp_mode {!r} not recognised".format(mode))
        return mode

    def collective(self):
        """"rccl-native", "torch.distributed" (callbacks) or None, for the last handle."""
        if not self._dp_active():
            return None
        return "rccl-native" if (self._handle is not None and self._handle.native) else "torch.distributed"

    def _allreduce(self, ptr, count, stream, ctx):
        """mc_allreduce_fn: sum `count` floats of one of our own device buffers over the ranks, in stream order."""
        try:
            from .dp import allreduce_grad_buffer
            for base in (self._cgrad, self._agrad, self._dp_scratch):
                if base is not None and base.data_ptr() == ptr and count <= base.numel():
                    allreduce_grad_buffer(base[:count])
                    return 0
            return 1
        except Exception as e:   # an exception must not unwind through the C frames
            self.logger.console_logger.error("COMA data-parallel all-reduce failed: %r", e)
            return 1

    # -- reference API ---------------------------------------------------------------------------------------
    def train(self, batch, t_env: int, episode_num: int):
        _lib.require_gpu(self._agent)
        mode = self.dp_mode(batch.batch_size)
        if mode is not None:
            rank, world = dp_world()
            check = self.dp_check.due()
            local = local_shard(batch, rank, world, check=check, device=self._critic.device)   # validates too
            self.dp_check.done += int(check)
            if mode == "exchange":     # this rank's shard through every step, summed in the library
                batch = local
        h = self._get_handle(batch)
        if mode == "replicated":       # the critic on the whole global batch, the actor on this rank's episodes
            lo, hi = shard_bounds(batch.batch_size, rank, world)
            _lib.check(h.lib.mc_set_actor_shard(h.h, lo, hi))
        elif mode == "exchange":
            _lib.check(h.lib.mc_set_actor_shard(h.h, 0, 0))
        rep, keep = replay_view(batch)
        eps = float(self.mac.action_selector.epsilon)
        _lib.check(h.lib.mc_train_step(h.h, ctypes.byref(rep), ctypes.c_float(eps), _lib.stream_ptr()))
        del keep
        st = self._stats.tolist()   # the one synchronisation per train(): stats + critic step count
        steps = int(round(st[9]))
        if steps < 0:
            # the library put the critic back to its pre-train version and skipped the actor update: the learner's
            # state is this call's starting state (no step counted), so a retry or MQ_PLAN=coma_chain=0 can follow. Under
            # data parallelism the failure word travels with the agent gradient's all-reduce, so every rank rolled
            # back and raises here together and a retry keeps the ranks' collective sequence in step
            raise _lib.MQError("COMA critic chain: a workgroup hand-off timed out; this train() was rolled back "
                               "(critic and agent unchanged; MQ_PLAN=coma_chain=0 selects the three-launch critic)")
        self.critic_training_steps += steps
        self._steps += 1
        for p in self.agent_params:
            self.agent_optimiser.state[p]["step"] += 1
        for p in self.critic_params:
            self.critic_optimiser.state[p]["step"] += steps
        self._last = dict(zip(_lib.COMA_STATS, st))
        self._last_batch = (batch.batch_size, rep.t_len)

        if (self.critic_training_steps - self.last_target_update_step) / self.args.target_update_interval >= 1.0:
            self._update_targets()
            self.last_target_update_step = self.critic_training_steps

        if t_env - self.log_stats_t >= self.args.learner_log_interval:
            for key in ["critic_loss", "critic_grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]:
                self.logger.log_stat(key, self._last[key], t_env)
            self.logger.log_stat("advantage_mean", self._last["advantage_mean"], t_env)
            self.logger.log_stat("coma_loss", self._last["coma_loss"], t_env)
            self.logger.log_stat("agent_grad_norm", self._last["agent_grad_norm"], t_env)
            self.logger.log_stat("pi_max", self._last["pi_max"], t_env)
            self.log_stats_t = t_env

    def _update_targets(self):
        if self._critic.is_cuda and self._handle is not None:
            _lib.check(self._handle.lib.mc_update_targets(self._handle.h, _lib.stream_ptr()))
        else:
            with th.no_grad():
                self._tcritic.copy_(self._critic)
        self.logger.console_logger.info("Updated target network")

    def cuda(self):
        dev = th.device("cuda", th.cuda.current_device())
        for name in ("_agent", "_critic", "_tcritic", "_agrad", "_asq", "_cgrad", "_csq", "_stats"):
            setattr(self, name, getattr(self, name).to(dev))
        self._relink()

    def save_models(self, path):
        self.mac.save_models(path)
        th.save(self.critic.state_dict(), "{}/critic.th".format(path))
        th.save(self.agent_optimiser.state_dict(), "{}/agent_opt.th".format(path))
        th.save(self.critic_optimiser.state_dict(), "{}/critic_opt.th".format(path))

    def load_models(self, path):
        ml = lambda s, loc: s  # noqa: E731
        self.mac.load_models(path)
        self.critic.load_state_dict(th.load("{}/critic.th".format(path), map_location=ml, weights_only=True))
        # Not quite right but I don't want to save target networks (reference comment, coma_learner.py:167)
        self.target_critic.load_state_dict(self.critic.state_dict())
        for fname, opt, params, sq in (("agent_opt.th", self.agent_optimiser, self.agent_params, self._asq),
                                       ("critic_opt.th", self.critic_optimiser, self.critic_params, self._csq)):
            opt.load_state_dict(th.load("{}/{}".format(path, fname), map_location=ml, weights_only=True))
            o = 0
            for p in params:
                n = p.numel()
                st = opt.state.get(p, {})
                if "square_avg" in st:
                    sq[o:o + n].copy_(st["square_avg"].reshape(-1))
                o += n
        self._relink()

    # -- extras (parity / diagnostics) -----------------------------------------------------------------------
    def last_stats(self):
        return dict(self._last)

    def last_intermediate(self, which):
        """0: the critic Q values the actor used, (B, T, n, A); 1: TD(lambda) targets (B, T, n); 2: pi (B, T, n, A)."""
        B, Tp = self._last_batch
        T, n, A = Tp - 1, self.n_agents, self.n_actions
        cnt = ctypes.c_int64()
        h = self._handle
        _lib.check(h.lib.mc_copy_intermediate(h.h, which, None, ctypes.byref(cnt), None))
        out = th.empty(cnt.value, dtype=th.float32, device=self._agent.device)
        _lib.check(h.lib.mc_copy_intermediate(h.h, which, _lib.ptr(out), ctypes.byref(cnt), _lib.stream_ptr()))
        B = cnt.value // (T * n * (1 if which == 1 else A))   # pi has the actor's episodes (its shard when replicated)
        if which == 1:
            return out.view(T, B, n).permute(1, 0, 2)
        return out.view(T, B, n, A).permute(1, 0, 2, 3)

    def set_timing(self, on=True):
        """HIP events around the critic prologue, the T-step critic chain and the actor of the following steps."""
        _lib.check(self._handle.lib.mc_set_timing(self._handle.h, int(bool(on))))

    def phase_times(self):
        """{prologue, critic_chain, actor} ms of the last train() (synchronises)."""
        ms = (ctypes.c_float * 3)()
        _lib.check(self._handle.lib.mc_phase_times(self._handle.h, ms))
        return {"prologue": ms[0], "critic_chain": ms[1], "actor": ms[2]}

    def critic_path(self):
        """"chain" (one persistent launch for the T critic steps), "three_launch", or None before train()."""
        return {1: "chain", 0: "three_launch"}.get(int(self._handle.lib.mc_last_critic_path(self._handle.h)))
