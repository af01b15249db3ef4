"""A deterministic synthetic MultiAgentEnv (stand-in for SMAC, which cannot run here: no SC2 binary, no network).

State and observations follow a seeded random walk that the joint action feeds back into, so a runner that records
the wrong action or the wrong time slot produces a different episode. Action 1 is always available (as in the
synthetic replay of pymarl_amd/utils/synthetic.py); an episode terminates at a seeded length in
[episode_limit // 2, episode_limit] (or earlier, once the state crosses `end_threshold`, if given), or is cut at the
limit with info["episode_limit"] = True (episode_runner.py:69-78
turns that into terminated = False).
"""
import numpy as np

from .multiagentenv import MultiAgentEnv


class FakeEnv(MultiAgentEnv):
    def __init__(self, n_agents=3, n_actions=9, obs_dim=30, state_dim=48, episode_limit=60, seed=0, p_avail=0.7,
                 p_truncate=0.5, end_threshold=None, **kwargs):
        self.n_agents = int(n_agents)
        self.n_actions = int(n_actions)
        self.obs_dim = int(obs_dim)
        self.state_dim = int(state_dim)
        self.episode_limit = int(episode_limit)
        self.p_avail = float(p_avail)
        self.p_truncate = float(p_truncate)
        # optional action-dependent early end: the episode also terminates once state[2] exceeds this (from t = 3),
        # so identically seeded envs stepped with different actions end at different times
        self.end_threshold = None if end_threshold is None else float(end_threshold)
        self._rng = np.random.Generator(np.random.PCG64(seed))
        self._proj = self._rng.standard_normal((self.n_agents * self.n_actions, self.state_dim)).astype(np.float32)
        self._obs_proj = self._rng.standard_normal((self.n_agents, self.state_dim, self.obs_dim)).astype(np.float32)
        self.reset()

    def reset(self):
        self._t = 0
        self._state = self._rng.standard_normal(self.state_dim).astype(np.float32)
        if self._rng.random() < self.p_truncate:
            self._length = self.episode_limit + 1          # runs into the limit
        else:
            self._length = int(self._rng.integers(max(1, self.episode_limit // 2), self.episode_limit + 1))
        self._avail = self._draw_avail()
        return self.get_obs(), self.get_state()

    def _draw_avail(self):
        av = (self._rng.random((self.n_agents, self.n_actions)) < self.p_avail).astype(np.int32)
        av[:, 1] = 1
        return av

    def step(self, actions):
        a = np.asarray(actions.cpu() if hasattr(actions, "cpu") else actions, dtype=np.int64).reshape(-1)
        assert a.shape[0] == self.n_agents
        assert np.all(self._avail[np.arange(self.n_agents), a] == 1), "unavailable action taken"
        onehot = np.zeros(self.n_agents * self.n_actions, np.float32)
        onehot[np.arange(self.n_agents) * self.n_actions + a] = 1.0
        self._state = (0.9 * self._state + 0.1 * np.tanh(onehot @ self._proj) +
                       0.05 * self._rng.standard_normal(self.state_dim)).astype(np.float32)
        reward = float(np.mean(a == (self._t % self.n_actions)) + 0.01 * self._state[0])
        self._t += 1
        info = {}
        terminated = False
        early = self.end_threshold is not None and self._t >= 3 and self._state[2] > self.end_threshold
        if self._t >= self._length or early:
            terminated = True
            info["battle_won"] = bool(self._state[1] > 0)
        elif self._t >= self.episode_limit:
            terminated = True
            info["episode_limit"] = True
        self._avail = self._draw_avail()
        return reward, terminated, info

    def get_obs(self):
        return [self.get_obs_agent(i) for i in range(self.n_agents)]

    def get_obs_agent(self, agent_id):
        return np.tanh(self._state @ self._obs_proj[agent_id]).astype(np.float32)

    def get_obs_size(self):
        return self.obs_dim

    def get_state(self):
        return self._state.copy()

    def get_state_size(self):
        return self.state_dim

    def get_avail_actions(self):
        return [self._avail[i].tolist() for i in range(self.n_agents)]

    def get_avail_agent_actions(self, agent_id):
        return self._avail[agent_id].tolist()

    def get_total_actions(self):
        return self.n_actions

    def render(self):
        pass

    def close(self):
        pass

    def seed(self):
        return None

    def save_replay(self):
        pass

    def get_stats(self):
        """Env-side episode stats (SMAC's StarCraft2Env.get_stats; requested by the parallel runner)."""
        return {}
