"""Environments (reference: src/envs/__init__.py). SC2/SMAC is out of scope (host-side rollout);
`FakeEnv` implements the MultiAgentEnv contract so the runner -> replay -> learner loop runs without it."""
from .multiagentenv import MultiAgentEnv
from .fake_env import FakeEnv

REGISTRY = {"fake": FakeEnv}
