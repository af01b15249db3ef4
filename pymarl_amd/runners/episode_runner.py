"""EpisodeRunner: one environment, one episode per run() (reference: src/runners/episode_runner.py:8-127).

The replay-format contract the learner path depends on: an episode of length L writes
slots 0..L of obs / state / avail_actions / actions (slot L: the final observation and the action chosen in it),
reward and terminated for slots 0..L-1, terminated[L-1] = 1 only when the env terminated for a reason other than
the episode limit, and `filled` for the slots written. The batch lives on args.device (the GPU for the MI355X
learner), so actions chosen by the HIP MAC step never leave the device until the env needs them.
"""
from functools import partial

import numpy as np

from ..components.episode_buffer import EpisodeBatch
from ..envs import REGISTRY as env_REGISTRY


class EpisodeRunner:
    def __init__(self, args, logger):
        self.args = args
        self.logger = logger
        self.batch_size = self.args.batch_size_run
        assert self.batch_size == 1
        self.env = env_REGISTRY[self.args.env](**self.args.env_args)
        self.episode_limit = self.env.episode_limit
        self.t = 0
        self.t_env = 0
        self.train_returns, self.test_returns = [], []
        self.train_stats, self.test_stats = {}, {}
        self.log_train_stats_t = -1000000

    def setup(self, scheme, groups, preprocess, mac):
        self.new_batch = partial(EpisodeBatch, scheme, groups, self.batch_size, self.episode_limit + 1,
                                 preprocess=preprocess, device=self.args.device)
        self.mac = mac

    def get_env_info(self):
        return self.env.get_env_info()

    def save_replay(self):
        self.env.save_replay()

    def close_env(self):
        self.env.close()

    def reset(self):
        self.batch = self.new_batch()
        self.env.reset()
        self.t = 0

    def _observe(self):
        return {"state": [self.env.get_state()], "avail_actions": [self.env.get_avail_actions()],
                "obs": [self.env.get_obs()]}

    def run(self, test_mode=False):
        self.reset()
        terminated = False
        episode_return = 0.0
        env_info = {}
        self.mac.init_hidden(batch_size=self.batch_size)
        while not terminated:
            self.batch.update(self._observe(), ts=self.t)
            actions = self.mac.select_actions(self.batch, t_ep=self.t, t_env=self.t_env, test_mode=test_mode)
            reward, terminated, env_info = self.env.step(actions[0])
            episode_return += reward
            # a cut at the episode limit is not a true termination (episode_runner.py:69-78)
            self.batch.update({"actions": actions, "reward": [(reward,)],
                               "terminated": [(terminated != env_info.get("episode_limit", False),)]}, ts=self.t)
            self.t += 1
        self.batch.update(self._observe(), ts=self.t)
        actions = self.mac.select_actions(self.batch, t_ep=self.t, t_env=self.t_env, test_mode=test_mode)
        self.batch.update({"actions": actions}, ts=self.t)

        cur_stats = self.test_stats if test_mode else self.train_stats
        cur_returns = self.test_returns if test_mode else self.train_returns
        prefix = "test_" if test_mode else ""
        for k in set(cur_stats) | set(env_info):
            cur_stats[k] = cur_stats.get(k, 0) + env_info.get(k, 0)
        cur_stats["n_episodes"] = 1 + cur_stats.get("n_episodes", 0)
        cur_stats["ep_length"] = self.t + cur_stats.get("ep_length", 0)
        if not test_mode:
            self.t_env += self.t
        cur_returns.append(episode_return)
        if test_mode and len(self.test_returns) == getattr(self.args, "test_nepisode", 1):
            self._log(cur_returns, cur_stats, prefix)
        elif self.t_env - self.log_train_stats_t >= getattr(self.args, "runner_log_interval", 0):
            self._log(cur_returns, cur_stats, prefix)
            if hasattr(self.mac.action_selector, "epsilon"):
                self.logger.log_stat("epsilon", self.mac.action_selector.epsilon, self.t_env)
            self.log_train_stats_t = self.t_env
        return self.batch

    def _log(self, returns, stats, prefix):
        self.logger.log_stat(prefix + "return_mean", float(np.mean(returns)), self.t_env)
        self.logger.log_stat(prefix + "return_std", float(np.std(returns)), self.t_env)
        returns.clear()
        for k, v in stats.items():
            if k != "n_episodes":
                self.logger.log_stat(prefix + k + "_mean", v / stats["n_episodes"], self.t_env)
        stats.clear()
