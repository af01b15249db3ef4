from .coma import COMACritic

REGISTRY = {"coma": COMACritic}
