"""Helpers shared by the parity tests: load a golden case, rebuild its replay and weights bit-exactly."""
from __future__ import annotations

import os
from collections import OrderedDict

import numpy as np

from pymarl_amd.utils.synthetic import agent_param_shapes, init_params, make_replay, qmix_param_shapes

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASE_NAMES = ["tiny_qmix", "tiny_vdn", "tiny_qmix_full", "cfg2_qmix", "cfg2_vdn", "cfg2_qmix_ragged",
              "cfg3_vdn", "cfg3_qmix", "cfg4_qmix", "tiny_iql", "cfg2_iql", "rw2_qmix", "rw4_vdn", "wide_qmix",
              "cfg3_vdn_b128", "tiny_qmix_nodq", "tiny_qmix_nola", "tiny_vdn_noid", "tiny_qmix_bare",
              "cfg2_qmix_nodq", "cfg1_qmix", "cfg1_vdn"]


class Case:
    def __init__(self, name):
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.z = {k: z[k] for k in z.files}
        g = lambda k: int(self.z[k])  # noqa: E731
        self.n, self.A, self.O, self.S, self.T = g("n"), g("A"), g("O"), g("S"), g("T")
        self.B, self.n_episodes, self.steps = g("B"), g("n_episodes"), g("steps")
        self.mixer = str(self.z["mixer"])
        self.ragged = bool(self.z["ragged"])
        self.episodes = [int(e) for e in self.z["episodes"]]
        self.data = make_replay(self.n_episodes, self.T, self.n, self.A, self.O, self.S,
                                seed=g("data_seed"), ragged=self.ragged)
        # learner flags the golden run used (absent in the older fixtures: the shipped configs' True / True / True)
        fl = lambda k: bool(self.z[k]) if k in self.z else True  # noqa: E731
        self.double_q, self.obs_last_action, self.obs_agent_id = fl("double_q"), fl("obs_last_action"), fl("obs_agent_id")
        self.I = self.O + (self.A if self.obs_last_action else 0) + (self.n if self.obs_agent_id else 0)
        self.agent_shapes = agent_param_shapes(self.I, 64, self.A)
        self.mixer_shapes = qmix_param_shapes(self.S, self.n, 32) if self.mixer == "qmix" else OrderedDict()
        self.agent_params = init_params(self.agent_shapes, seed=g("weight_seed"))
        self.mixer_params = (init_params(self.mixer_shapes, seed=g("weight_seed") + 100)
                             if self.mixer == "qmix" else OrderedDict())
        self.sampler_seed = g("sampler_seed")

    def cfg(self):
        return dict(n_agents=self.n, n_actions=self.A, obs_dim=self.O, state_dim=self.S, mixer=self.mixer,
                    gamma=0.99, lr=5e-4, optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10.0,
                    double_q=self.double_q, obs_last_action=self.obs_last_action, obs_agent_id=self.obs_agent_id,
                    target_update_interval=200, learner_log_interval=0, rnn_hidden_dim=64, mixing_embed_dim=32)

    def batch(self, step):
        """The (ids-gathered, max_t-truncated) numpy batch the reference trained on at `step`."""
        ids = self.z["ids"][step]
        b = OrderedDict((k, v[ids]) for k, v in self.data.items())
        max_t = int(b["filled"].sum(1).max())
        return OrderedDict((k, v[:, :max_t]) for k, v in b.items()), ids

    def unflatten(self, flat):
        out, o = OrderedDict(), 0
        for k, s in list(self.agent_shapes.items()) + list(self.mixer_shapes.items()):
            sz = int(np.prod(s))
            out[k] = flat[o:o + sz].reshape(s)
            o += sz
        return out


class SynthCase(Case):
    """A Case without a reference fixture: replay, weights and sampled ids from the same seeded generators, for
    shapes the reference goldens do not cover (edge cases: checked against the oracle only, "parity unpinned"
    against the reference itself; the oracle is pinned on the fixture shapes)."""

    def __init__(self, name, n, A, O, S, T, B, n_episodes, steps, mixer="qmix", ragged=True, min_len=1,
                 data_seed=11, weight_seed=12, sampler_seed=13):
        self.name = name
        self.double_q = self.obs_last_action = self.obs_agent_id = True
        self.n, self.A, self.O, self.S, self.T, self.B = n, A, O, S, T, B
        self.n_episodes, self.steps, self.mixer, self.ragged = n_episodes, steps, mixer, ragged
        self.episodes = [8 * k for k in range(steps)]
        self.data = make_replay(n_episodes, T, n, A, O, S, seed=data_seed, ragged=ragged, min_len=min_len)
        self.I = O + A + n
        self.agent_shapes = agent_param_shapes(self.I, 64, A)
        self.mixer_shapes = qmix_param_shapes(S, n, 32) if mixer == "qmix" else OrderedDict()
        self.agent_params = init_params(self.agent_shapes, seed=weight_seed)
        self.mixer_params = init_params(self.mixer_shapes, seed=weight_seed + 100) if mixer == "qmix" else OrderedDict()
        self.sampler_seed = sampler_seed
        state = np.random.get_state()   # the ids ReplayBuffer.sample draws after np.random.seed(sampler_seed)
        np.random.seed(sampler_seed)
        ids = [np.arange(B) if n_episodes == B else np.random.choice(n_episodes, B, replace=False)
               for _ in range(steps)]
        np.random.set_state(state)
        self.z = {"ids": np.stack(ids)}


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(1e-30, np.abs(b).max()))


COMA_CASE_NAMES = ["coma_tiny", "coma_tiny_masked", "coma_cfg5"]
COMA_STATS = ["critic_loss", "critic_grad_norm", "td_error_abs", "q_taken_mean", "target_mean", "advantage_mean",
              "coma_loss", "agent_grad_norm", "pi_max"]


class ComaCase:
    """A golden COMA case (tests/golden/make_golden_coma.py): replay, weights, sampler ids, per-step epsilon."""

    def __init__(self, name):
        from oracle.coma_np import critic_input_dim, critic_param_shapes
        self.name = name
        z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
        self.z = {k: z[k] for k in z.files}
        g = lambda k: int(self.z[k])  # noqa: E731
        self.n, self.A, self.O, self.S, self.T = g("n"), g("A"), g("O"), g("S"), g("T")
        self.B, self.n_episodes, self.steps = g("B"), g("n_episodes"), g("steps")
        self.ragged = bool(self.z["ragged"])
        self.mask_before_softmax = bool(self.z["mask_before_softmax"])
        self.target_update_interval = g("target_update_interval")
        self.data = make_replay(self.n_episodes, self.T, self.n, self.A, self.O, self.S, seed=g("data_seed"),
                                ragged=self.ragged)
        self.I = self.O + self.A + self.n
        self.K = critic_input_dim(self.n, self.A, self.O, self.S)
        self.agent_shapes = agent_param_shapes(self.I, 64, self.A)
        self.critic_shapes = critic_param_shapes(self.K, self.A)
        self.agent_params = init_params(self.agent_shapes, seed=g("weight_seed"))
        self.critic_params = init_params(self.critic_shapes, seed=g("weight_seed") + 200)
        self.sampler_seed = g("sampler_seed")
        self.epsilon = [float(e) for e in self.z["epsilon"]]

    def cfg(self):
        return dict(n_agents=self.n, n_actions=self.A, gamma=0.99, td_lambda=0.8, lr=5e-4, critic_lr=5e-4,
                    optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10.0,
                    target_update_interval=self.target_update_interval,
                    mask_before_softmax=self.mask_before_softmax)

    def batch(self, step):
        ids = self.z["ids"][step]
        b = OrderedDict((k, v[ids]) for k, v in self.data.items())
        max_t = int(b["filled"].sum(1).max())
        return OrderedDict((k, v[:, :max_t]) for k, v in b.items()), ids
