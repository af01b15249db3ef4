"""QMixer: state-conditioned monotonic mixing (reference: src/modules/mixers/qmix.py:7-47).

Holds the hypernetwork parameters under the reference's names (hyper_w_1, hyper_w_final, hyper_b_1, V.0, V.2)
so mixer.th interchanges. Inside QLearner.train the forward/backward run fused into the HIP train step (hypernet
contraction on fp32 MFMA, mixing + TD + backward in `mix_kernel`); `forward(agent_qs, states)` is the standalone
HIP kernel `mq_qmix_forward` (include/mq_learner.h) for callers outside train(). It returns values, not an
autograd graph (the learner computes the mixer's gradients itself).
"""
import numpy as np
import torch as th
import torch.nn as nn

from ... import _lib
from ..flat import FlatModule


class QMixer(FlatModule):
    def __init__(self, args):
        super().__init__()
        self.args = args
        self.n_agents = args.n_agents
        self.state_dim = int(np.prod(args.state_shape))
        self.embed_dim = args.mixing_embed_dim
        self.hyper_w_1 = nn.Linear(self.state_dim, self.embed_dim * self.n_agents)
        self.hyper_w_final = nn.Linear(self.state_dim, self.embed_dim)
        self.hyper_b_1 = nn.Linear(self.state_dim, self.embed_dim)
        self.V = nn.Sequential(nn.Linear(self.state_dim, self.embed_dim), nn.ReLU(), nn.Linear(self.embed_dim, 1))
        self._init_flat()

    def forward(self, agent_qs, states):
        """qmix.py:28-47: agent_qs (bs, T, n_agents), states (bs, T, state_dim) -> q_tot (bs, T, 1)."""
        bs = agent_qs.size(0)
        qs = agent_qs.detach().reshape(-1, self.n_agents).float().contiguous()
        st = states.detach().reshape(-1, self.state_dim).float().contiguous()
        _lib.require_gpu(qs)
        _lib.require_gpu(self._flat)
        rows = qs.shape[0]
        if st.shape[0] != rows:
            raise ValueError("agent_qs has {} rows but states has {}".format(rows, st.shape[0]))
        out = th.empty(rows, dtype=th.float32, device=qs.device)
        lib = _lib.load()
        _lib.check(lib.mq_qmix_forward(_lib.ptr(self._flat), self.n_agents, self.state_dim, self.embed_dim,
                                       _lib.ptr(qs), _lib.ptr(st), _lib.ptr(out), rows, _lib.stream_ptr()))
        return out.view(bs, -1, 1)
