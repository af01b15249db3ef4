"""Golden episodes of the REFERENCE EpisodeRunner (src/runners/episode_runner.py) and ParallelRunner
(src/runners/parallel_runner.py) on the synthetic FakeEnv.

    python tests/golden/make_golden_runner.py        # writes tests/golden/runner_fake.npz, runner_parallel_fake.npz

Not part of the product and never run on the GPU box. The reference runner cannot import its SC2 environment here
(pysc2 / absl absent), so a stub `envs` module registering pymarl_amd's FakeEnv under "fake" is
injected before the import (the SURVEY's documented workaround). The MAC is a seeded stub that picks a uniformly
random AVAILABLE action from the avail_actions the runner stored for that step, so the episode depends on the
runner storing every field at the right slot. Recorded: every transition field of 4 episodes, and the runner's
logged stats.
"""
import os
import sys
import types
from types import SimpleNamespace as SN

sys.dont_write_bytecode = True   # /root/reference is read-only: no __pycache__ there

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference/src")
import torch as th  # noqa: E402

from pymarl_amd.envs.fake_env import FakeEnv  # noqa: E402

envs_stub = types.ModuleType("envs")
envs_stub.REGISTRY = {"fake": FakeEnv}
sys.modules["envs"] = envs_stub

from components.transforms import OneHot  # noqa: E402  (reference)
from runners.episode_runner import EpisodeRunner  # noqa: E402  (reference)
from runners.parallel_runner import ParallelRunner  # noqa: E402  (reference)

N_AGENTS, N_ACTIONS, OBS, STATE, LIMIT = 3, 9, 30, 48, 20
EPISODES = 4
FIELDS = ["obs", "state", "actions", "avail_actions", "reward", "terminated", "filled", "actions_onehot"]


class StubMAC:
    """Seeded uniform choice among the avail_actions stored in the batch at t_ep."""

    def __init__(self, seed=5):
        self.rng = np.random.Generator(np.random.PCG64(seed))
        self.action_selector = SN(epsilon=0.25)

    def init_hidden(self, batch_size):
        pass

    def select_actions(self, ep_batch, t_ep, t_env, bs=slice(None), test_mode=False):
        avail = ep_batch["avail_actions"][:, t_ep].cpu().numpy()
        keys = self.rng.random(avail.shape)
        keys[avail == 0] = -1.0
        return th.as_tensor(keys.argmax(-1), dtype=th.long)


class StubBatchMAC(StubMAC):
    """The same seeded choice over the envs `bs` selects (the parallel runner passes the running envs)."""

    def select_actions(self, ep_batch, t_ep, t_env, bs=slice(None), test_mode=False):
        avail = ep_batch["avail_actions"][bs, t_ep].cpu().numpy()
        keys = self.rng.random(avail.shape)
        keys[avail == 0] = -1.0
        return th.as_tensor(keys.argmax(-1), dtype=th.long)


class Logger:
    def __init__(self):
        self.stats = []

    def log_stat(self, key, value, t):
        self.stats.append((key, float(value), int(t)))


def scheme():
    return {
        "state": {"vshape": STATE},
        "obs": {"vshape": OBS, "group": "agents"},
        "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
        "avail_actions": {"vshape": (N_ACTIONS,), "group": "agents", "dtype": th.int},
        "reward": {"vshape": (1,)},
        "terminated": {"vshape": (1,), "dtype": th.uint8},
    }


def run_reference():
    args = SN(batch_size_run=1, env="fake", env_args=dict(n_agents=N_AGENTS, n_actions=N_ACTIONS, obs_dim=OBS,
                                                           state_dim=STATE, episode_limit=LIMIT, seed=3),
              device="cpu", test_nepisode=2, runner_log_interval=25)
    logger = Logger()
    runner = EpisodeRunner(args, logger)
    runner.setup(scheme(), {"agents": N_AGENTS}, {"actions": ("actions_onehot", [OneHot(out_dim=N_ACTIONS)])},
                 StubMAC())
    out = {}
    for e in range(EPISODES):
        b = runner.run(test_mode=(e == 3))
        for k in FIELDS:
            out["ep{}_{}".format(e, k)] = b[k].numpy().copy()
    out["t_env"] = np.array(runner.t_env)
    names = sorted({k for k, _, _ in logger.stats})
    out["stat_names"] = np.array(names)
    out["stats"] = np.array([[names.index(k), v, t] for k, v, t in logger.stats], dtype=np.float64)
    return out


PAR_ENVS, PAR_RUNS, END_THRESHOLD = 4, 6, -0.9


def run_reference_parallel():
    args = SN(batch_size_run=PAR_ENVS, env="fake", env_args=dict(n_agents=N_AGENTS, n_actions=N_ACTIONS, obs_dim=OBS,
                                                                  state_dim=STATE, episode_limit=LIMIT, seed=3,
                                                                  end_threshold=END_THRESHOLD),
              device="cpu", buffer_cpu_only=True, test_nepisode=4, runner_log_interval=25)
    logger = Logger()
    runner = ParallelRunner(args, logger)
    runner.setup(scheme(), {"agents": N_AGENTS}, {"actions": ("actions_onehot", [OneHot(out_dim=N_ACTIONS)])},
                 StubBatchMAC())
    out = {}
    for e in range(PAR_RUNS):
        b = runner.run(test_mode=(e == PAR_RUNS - 1))
        for k in FIELDS:
            out["run{}_{}".format(e, k)] = b[k].numpy().copy()
        out["run{}_t_env".format(e)] = np.array(runner.t_env)
    runner.close_env()
    names = sorted({k for k, _, _ in logger.stats})
    out["stat_names"] = np.array(names)
    out["stats"] = np.array([[names.index(k), v, t] for k, v, t in logger.stats], dtype=np.float64)
    return out


if __name__ == "__main__":
    outp = run_reference_parallel()
    path = os.path.join(HERE, "runner_parallel_fake.npz")
    np.savez_compressed(path, **outp)
    print("parallel runs: filled per env", [outp["run{}_filled".format(e)].sum((1, 2)).tolist() for e in range(PAR_RUNS)],
          "->", path, os.path.getsize(path) // 1024, "KB")
    out = run_reference()
    path = os.path.join(HERE, "runner_fake.npz")
    np.savez_compressed(path, **out)
    print("episode lengths", [int(out["ep{}_filled".format(e)].sum()) for e in range(EPISODES)], "t_env",
          int(out["t_env"]), "->", path, os.path.getsize(path) // 1024, "KB")
