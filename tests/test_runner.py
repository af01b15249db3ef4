"""Runner plumbing: pymarl_amd's EpisodeRunner on the synthetic FakeEnv writes exactly the episodes
the reference EpisodeRunner writes (tests/golden/runner_fake.npz, made by tests/golden/make_golden_runner.py with the
same env seed and the same seeded stub MAC): every transition field bit for bit, t_env and the logged stats. This
pins the replay-format contract the learner path reads (filled / terminated / final-slot conventions). CPU only."""
import os
from types import SimpleNamespace as SN

import numpy as np
import torch as th

from pymarl_amd.components.transforms import OneHot
from pymarl_amd.runners import REGISTRY as runner_REGISTRY

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "runner_fake.npz")
N_AGENTS, N_ACTIONS, OBS, STATE, LIMIT = 3, 9, 30, 48, 20
FIELDS = ["obs", "state", "actions", "avail_actions", "reward", "terminated", "filled", "actions_onehot"]


class StubMAC:
    """Seeded uniform choice among the avail_actions the runner stored at t_ep (same as the golden generator)."""

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


def test_episode_runner_matches_reference():
    z = np.load(GOLDEN, allow_pickle=False)
    args = SN(batch_size_run=1, env="fake", env_args=dict(n_agents=N_AGENTS, n_actions=N_ACTIONS, obs_dim=OBS,
                                                           state_dim=STATE, episode_limit=LIMIT, seed=3),
              device="cpu", test_nepisode=2, runner_log_interval=25)
    logger = Logger()
    runner = runner_REGISTRY["episode"](args, logger)
    assert runner.get_env_info() == {"state_shape": STATE, "obs_shape": OBS, "n_actions": N_ACTIONS,
                                     "n_agents": N_AGENTS, "episode_limit": LIMIT}
    runner.setup(scheme(), {"agents": N_AGENTS}, {"actions": ("actions_onehot", [OneHot(out_dim=N_ACTIONS)])},
                 StubMAC())
    for e in range(4):
        b = runner.run(test_mode=(e == 3))
        for k in FIELDS:
            got = b[k].numpy()
            ref = z["ep{}_{}".format(e, k)]
            assert got.shape == ref.shape and got.dtype == ref.dtype, (e, k, got.shape, ref.shape)
            assert np.array_equal(got, ref), (e, k)
    assert runner.t_env == int(z["t_env"])
    names = list(z["stat_names"])
    # compared as sorted (key, t) lists: the reference orders the per-key "_mean" stats by a Python set
    ref_stats = sorted((names[int(i)], int(t), v) for i, v, t in z["stats"])
    got_stats = sorted((k, t, v) for k, v, t in logger.stats)
    assert [(k, t) for k, t, _ in got_stats] == [(k, t) for k, t, _ in ref_stats]
    for (k, _, v), (_, _, rv) in zip(got_stats, ref_stats):
        assert abs(v - rv) <= 1e-6 * max(1.0, abs(rv)), (k, v, rv)


def test_fake_env_contract():
    from pymarl_amd.envs import REGISTRY
    env = REGISTRY["fake"](n_agents=2, n_actions=5, obs_dim=7, state_dim=11, episode_limit=6, seed=1)
    obs, state = env.reset()
    assert len(obs) == 2 and obs[0].shape == (7,) and state.shape == (11,)
    steps = 0
    while True:
        av = np.array(env.get_avail_actions())
        assert av.shape == (2, 5) and np.all(av[:, 1] == 1)
        r, term, info = env.step(np.argmax(av, 1))
        steps += 1
        if term:
            break
    assert steps <= 6
    assert info.get("episode_limit", False) == (steps == 6 and "battle_won" not in info)
