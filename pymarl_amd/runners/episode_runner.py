"""EpisodeRunner: batch_size_run = 1, the environment stepped in the learner's process
(reference: src/runners/episode_runner.py:8-127). The loop and the stats are the shared BatchRollout
(rollout.py); this class only binds a single in-process env to it."""
from functools import partial

from ..components.episode_buffer import EpisodeBatch
from ..envs import REGISTRY as env_REGISTRY
from .env_pool import InProcessEnvs
from .rollout import BatchRollout


class EpisodeRunner(BatchRollout):
    log_train_stats_t0 = -1000000

    def __init__(self, args, logger):
        assert args.batch_size_run == 1, "EpisodeRunner steps one environment; use the parallel runner for more"
        self.env = env_REGISTRY[args.env](**args.env_args)
        self._init_rollout(args, logger, InProcessEnvs(self.env))

    def setup(self, scheme, groups, preprocess, mac):
        self.new_batch = partial(EpisodeBatch, scheme, groups, self.batch_size, self.episode_limit + 1,
                                 preprocess=preprocess, device=self.args.device)
        self.mac = mac

    def n_test_episodes(self):
        return self.args.test_nepisode   # episode_runner.py:105 compares with test_nepisode exactly

    def save_replay(self):
        self.env.save_replay()
