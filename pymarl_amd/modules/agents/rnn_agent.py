"""RNNAgent: fc1 -> ReLU -> GRUCell -> fc2 (reference: src/modules/agents/rnn_agent.py:7-36).

Same submodules and parameter names (fc1, rnn, fc2), so state_dicts interchange with the reference. `forward`
runs the HIP `mq_agent_forward` kernel; inside the learner the whole unroll is fused into the train step.
"""
from collections import OrderedDict

import torch as th
import torch.nn as nn

from ... import _lib
from ..flat import FlatModule


def input_dim(input_shape):
    if isinstance(input_shape, (dict, OrderedDict)):
        return int(input_shape["1d"][0])
    if isinstance(input_shape, tuple):
        assert len(input_shape) == 1, "Input shape has unsupported dimensionality: {}".format(input_shape)
        return int(input_shape[0])
    return int(input_shape)


class RNNAgent(FlatModule):
    def __init__(self, input_shape, args):
        super().__init__()
        self.args = args
        self.input_shape = input_shape
        self.input_dim = input_dim(input_shape)
        self.fc1 = nn.Linear(self.input_dim, args.rnn_hidden_dim)
        self.rnn = nn.GRUCell(args.rnn_hidden_dim, args.rnn_hidden_dim)
        self.fc2 = nn.Linear(args.rnn_hidden_dim, args.n_actions)
        self._init_flat()
        self._handle = None

    def init_hidden(self):
        return self.fc1.weight.new_zeros(1, self.args.rnn_hidden_dim)

    def handle(self):
        """Inference handle (agent-only layout) bound to this module's flat parameters."""
        from ...learners.q_learner import make_config
        if self._handle is None or self._handle[1] != self._flat.data_ptr():
            cfg = make_config(self.args, mixer=_lib.MIXER_NONE, input_dim=self.input_dim, max_batch=1, max_seq=2)
            h = _lib.Handle(cfg)
            _lib.check(h.lib.mq_bind(h.h, _lib.ptr(self._flat), None, None, None, None, None))
            self._handle = (h, self._flat.data_ptr())
        return self._handle[0]

    def forward(self, inputs, hidden_state):
        if isinstance(inputs, (dict, OrderedDict)):
            inputs = inputs["1d"]
        _lib.require_gpu(inputs)
        x = inputs.reshape(-1, self.input_dim).float().contiguous()
        h_in = hidden_state.reshape(-1, self.args.rnn_hidden_dim).float().contiguous()
        h_out = th.empty_like(h_in)
        q = th.empty(x.shape[0], self.args.n_actions, dtype=th.float32, device=x.device)
        hd = self.handle()
        _lib.check(hd.lib.mq_agent_forward(hd.h, _lib.ptr(x), x.shape[0], _lib.ptr(h_in), _lib.ptr(h_out),
                                           _lib.ptr(q), 0, _lib.stream_ptr()))
        return q, h_out

    def __getstate__(self):
        d = self.__dict__.copy()
        d["_handle"] = None
        return d
