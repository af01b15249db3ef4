"""The batched rollout loop shared by EpisodeRunner and ParallelRunner.

One `run()` collects one episode per environment of the group into an EpisodeBatch of batch_size_run episodes
(max_seq_length = episode_limit + 1) living on args.device, so the HIP MAC step (BasicMAC.select_actions ->
mq_mac_forward + mq_greedy_actions) reads its inputs where the runner wrote them and only the chosen actions cross
to the host, where the envs need them.

Replay-format contract (reference episode_runner.py:48-123 and parallel_runner.py:88-204,
which write the same layout): an episode of length L fills slots 0..L of state / obs / avail_actions / actions
(slot L holds the final observation and the action the MAC picked in it), reward and terminated for 0..L-1, with
terminated = 1 only for a termination that is not the episode-limit cut, and `filled` for every written slot.

Per iteration: pick actions for every env whose current slot needs one (`pick`: those still running when the
slot was written, i.e. including an env that just terminated, for its final slot), record them, step the envs that
are still running, write their reward / terminated at t and the next observation at t + 1. The loop ends once an
iteration finds no env running.
"""
from __future__ import annotations

import numpy as np

from .env_pool import stack_pre


class BatchRollout:
    log_train_stats_t0 = -100000

    def _init_rollout(self, args, logger, envs):
        self.args = args
        self.logger = logger
        self.envs = envs
        self.batch_size = envs.n
        self.env_info = envs.env_info()
        self.episode_limit = self.env_info["episode_limit"]
        self.t = 0
        self.t_env = 0
        self.train_returns, self.test_returns = [], []
        self.train_stats, self.test_stats = {}, {}
        self.log_train_stats_t = self.log_train_stats_t0

    def n_test_episodes(self):
        """Test returns collected before the test stats are logged: the reference ParallelRunner rounds
        test_nepisode to whole runs (parallel_runner.py:194-195); EpisodeRunner overrides it with test_nepisode
        itself (episode_runner.py:105)."""
        return max(1, self.args.test_nepisode // self.batch_size) * self.batch_size

    def get_env_info(self):
        return self.env_info

    def close_env(self):
        self.envs.close()

    def reset(self):
        self.batch = self.new_batch()
        self.batch.update(stack_pre(self.envs.reset()), ts=0)
        self.t = 0
        self.env_steps_this_run = 0

    def run(self, test_mode=False):
        self.reset()
        B = self.batch_size
        returns = [0.0] * B
        lengths = [0] * B
        done = [False] * B
        final_infos = []          # in termination order
        pick = list(range(B))
        self.mac.init_hidden(batch_size=B)
        while True:
            actions = self.mac.select_actions(self.batch, t_ep=self.t, t_env=self.t_env, bs=pick, test_mode=test_mode)
            self.batch.update({"actions": actions.unsqueeze(1).to(self.batch.device)}, bs=pick, ts=self.t,
                              mark_filled=False)
            running = [i for i in range(B) if not done[i]]
            if not running:
                break
            host = actions.to("cpu").numpy()
            row = {i: j for j, i in enumerate(pick)}
            replies = self.envs.step(running, [host[row[i]] for i in running])
            rewards, terms, nxt = [], [], []
            for i, (reward, terminated, info, state, avail, obs) in zip(running, replies):
                returns[i] += reward
                lengths[i] += 1
                if not test_mode:
                    self.env_steps_this_run += 1
                if terminated:
                    final_infos.append(info)
                done[i] = terminated
                rewards.append((reward,))
                # a cut at the episode limit is not a true termination
                terms.append((bool(terminated) and not info.get("episode_limit", False),))
                nxt.append((state, avail, obs))
            self.batch.update({"reward": rewards, "terminated": terms}, bs=running, ts=self.t, mark_filled=False)
            self.t += 1
            self.batch.update(stack_pre(nxt), bs=running, ts=self.t, mark_filled=True)
            pick = running
        if not test_mode:
            self.t_env += self.env_steps_this_run
        self.envs.stats()   # the env-side stats round trip of the reference's parallel runner (values unused there)
        self._account(test_mode, returns, lengths, final_infos)
        return self.batch

    def _account(self, test_mode, returns, lengths, final_infos):
        stats = self.test_stats if test_mode else self.train_stats
        rets = self.test_returns if test_mode else self.train_returns
        prefix = "test_" if test_mode else ""
        keys = set(stats)
        for d in final_infos:
            keys |= set(d)
        for k in keys:
            stats[k] = stats.get(k, 0) + sum(d.get(k, 0) for d in final_infos)
        stats["n_episodes"] = stats.get("n_episodes", 0) + self.batch_size
        stats["ep_length"] = stats.get("ep_length", 0) + sum(lengths)
        rets.extend(returns)
        if test_mode and len(self.test_returns) == self.n_test_episodes():
            self._log(rets, stats, prefix)
        elif self.t_env - self.log_train_stats_t >= self.args.runner_log_interval:
            self._log(rets, stats, prefix)
            if hasattr(self.mac.action_selector, "epsilon"):
                self.logger.log_stat("epsilon", self.mac.action_selector.epsilon, self.t_env)
            self.log_train_stats_t = self.t_env

    def _log(self, returns, stats, prefix):
        self.logger.log_stat(prefix + "return_mean", float(np.mean(returns)), self.t_env)
        self.logger.log_stat(prefix + "return_std", float(np.std(returns)), self.t_env)
        returns.clear()
        n = stats["n_episodes"]
        for k, v in stats.items():
            if k != "n_episodes":
                self.logger.log_stat(prefix + k + "_mean", v / n, self.t_env)
        stats.clear()
