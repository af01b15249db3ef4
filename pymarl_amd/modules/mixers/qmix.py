"""QMixer: state-conditioned monotonic mixing (reference: src/modules/mixers/qmix.py:7-47).

Holds the hypernetwork parameters under the reference's names (hyper_w_1, hyper_w_final, hyper_b_1, V.0, V.2)
so mixer.th interchanges. Its forward/backward run fused inside the learner's HIP train step (hypernet
contraction on fp32 MFMA, mixing + TD + backward in `mix_kernel`); a standalone forward is not exposed.
"""
import numpy as np
import torch.nn as nn

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
        raise NotImplementedError("QMixer runs fused inside QLearner.train (mix_kernel); no standalone forward")
