from .rnn_agent import RNNAgent

REGISTRY = {}
REGISTRY["rnn"] = RNNAgent
