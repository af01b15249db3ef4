"""COMACritic: fc1 -> ReLU -> fc2 -> ReLU -> fc3 over [state | obs | joint actions (own masked) | last joint
actions | agent id] (reference: src/modules/critics/coma.py:6-70).

Same submodule / parameter names and shapes, so state_dicts and critic.th interchange with the reference. Inside
COMALearner.train the critic (its all-steps target pass and its T per-step optimiser steps) runs as HIP kernels on
this module's flat parameter buffer (include/mc_coma.h). `forward(batch, t=None)` is the standalone HIP path
`mc_critic_forward` (critic inputs built in-kernel from the replay rows, three fp32 MFMA linear layers) for callers
outside train(); it returns values, not an autograd graph.
"""
import torch as th
import torch.nn as nn

from ... import _lib
from ..flat import FlatModule

CRITIC_HIDDEN = 128   # coma.py:17-19


def critic_input_dim(scheme, n_agents):
    """coma.py:61-70, reading an int or 1-tuple vshape (the reference breaks on the tuple)."""
    def width(v):
        return v if isinstance(v, int) else int(v[0])
    return (width(scheme["state"]["vshape"]) + width(scheme["obs"]["vshape"]) +
            width(scheme["actions_onehot"]["vshape"]) * n_agents * 2 + n_agents)


class COMACritic(FlatModule):
    def __init__(self, scheme, args):
        super().__init__()
        self.args = args
        self.n_actions = args.n_actions
        self.n_agents = args.n_agents
        self.input_dim = critic_input_dim(scheme, self.n_agents)
        self.output_type = "q"
        self.fc1 = nn.Linear(self.input_dim, CRITIC_HIDDEN)
        self.fc2 = nn.Linear(CRITIC_HIDDEN, CRITIC_HIDDEN)
        self.fc3 = nn.Linear(CRITIC_HIDDEN, self.n_actions)
        self._init_flat()

        def width(v):
            return v if isinstance(v, int) else int(v[0])
        self.state_dim = width(scheme["state"]["vshape"])
        self.obs_dim = width(scheme["obs"]["vshape"])

    def _config(self):
        cfg = _lib.MCConfig()
        cfg.n_agents, cfg.n_actions = self.n_agents, self.n_actions
        cfg.obs_dim, cfg.state_dim = self.obs_dim, self.state_dim
        cfg.rnn_hidden_dim = getattr(self.args, "rnn_hidden_dim", 64)
        return cfg

    def forward(self, batch, t=None):
        """coma.py:22-27: q (bs, max_t, n_agents, n_actions) for every stored step (t=None) or step t (max_t=1)."""
        from ...learners.q_learner import replay_view
        rep, keep = replay_view(batch)
        _lib.require_gpu(self._flat)
        tq = rep.t_len if t is None else 1
        if t is not None and not (0 <= int(t) < rep.t_len):
            raise IndexError("t={} outside the batch's {} steps".format(t, rep.t_len))
        cfg = self._config()
        lib = _lib.load()
        n_ws = lib.mc_critic_forward_workspace(cfg, batch.batch_size, tq)
        ws = th.empty(max(int(n_ws), 1), dtype=th.float32, device=self._flat.device)
        q = th.empty(batch.batch_size, tq, self.n_agents, self.n_actions, dtype=th.float32, device=self._flat.device)
        _lib.check(lib.mc_critic_forward(_lib.ptr(self._flat), cfg, rep, -1 if t is None else int(t), _lib.ptr(q),
                                         _lib.ptr(ws), _lib.stream_ptr()))
        del keep
        return q
