from .q_learner import QLearner

REGISTRY = {}
REGISTRY["q_learner"] = QLearner
