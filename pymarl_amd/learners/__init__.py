from .coma_learner import COMALearner
from .q_learner import QLearner

REGISTRY = {}
REGISTRY["q_learner"] = QLearner
REGISTRY["coma_learner"] = COMALearner
