"""COMACritic: fc1 -> ReLU -> fc2 -> ReLU -> fc3 over [state | obs | joint actions (own masked) | last joint
actions | agent id] (reference: src/modules/critics/coma.py:6-70).

Same submodule / parameter names and shapes, so state_dicts and critic.th interchange with the reference. Inside
COMALearner.train the critic (its all-steps target pass and its T per-step optimiser steps) runs as HIP kernels on
this module's flat parameter buffer (include/mc_coma.h); this module only holds the parameters.
"""
import torch.nn as nn

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

    def forward(self, batch, t=None):
        raise NotImplementedError("COMACritic runs inside COMALearner.train (mc_train_step); there is no standalone "
                                  "torch forward on the MI355X path")
