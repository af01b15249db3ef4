"""Seeded synthetic replay and parameter initialisation (numpy only).

The reference has no fixtures; its learner is fed by SC2 rollouts (src/run.py:200-220) that cannot run offline.
SURVEY.md §8d fixes a synthetic-replay recipe instead, and everything here follows it so that the golden
generator (tests/golden/make_golden.py), the parity tests and bench.py see bit-identical inputs:

* obs, state ~ N(0, 1) f32; avail ~ Bernoulli(0.7) with action 1 always available;
  actions uniform over the available set; reward ~ U(0, 1).
* filled / terminated obey the replay contract of the reference runner (src/runners/episode_runner.py:48-113):
  an episode of length L writes slots 0..L (slot L = the last obs/state/avail/action, no reward), sets
  terminated[L-1] when the env terminated, and leaves every later slot zero. An episode that did not terminate
  has L == episode_limit.
* actions_onehot is the reference's OneHot preprocess (src/components/transforms.py:16-19) applied only to filled
  slots, i.e. zero on padding, as the runner leaves it.

Field dtypes and layouts are the reference scheme's (src/run.py:122-135): obs (N,T+1,n,O) f32, state (N,T+1,S) f32,
actions (N,T+1,n,1) i64, avail_actions (N,T+1,n,A) i32, reward (N,T+1,1) f32, terminated (N,T+1,1) u8,
filled (N,T+1,1) i64, actions_onehot (N,T+1,n,A) f32.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import numpy as np


def make_replay(n_episodes, episode_limit, n_agents, n_actions, obs_dim, state_dim, seed=0, ragged=False,
                min_len=None):
    """Return an OrderedDict of numpy arrays in the reference scheme layout (see module docstring).

    ragged: episode lengths uniform in [min_len, T] (min_len defaults to T // 2, the fixtures' recipe)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    N, T, n, A = int(n_episodes), int(episode_limit), int(n_agents), int(n_actions)
    Tp = T + 1
    obs = rng.standard_normal((N, Tp, n, obs_dim), dtype=np.float32)
    state = rng.standard_normal((N, Tp, state_dim), dtype=np.float32)
    avail = (rng.random((N, Tp, n, A)) < 0.7).astype(np.int32)
    avail[..., 1] = 1
    keys = rng.random((N, Tp, n, A))
    keys[avail == 0] = -1.0
    actions = keys.argmax(-1).astype(np.int64)[..., None]
    reward = rng.random((N, Tp, 1), dtype=np.float32)
    terminated = np.zeros((N, Tp, 1), dtype=np.uint8)
    filled = np.ones((N, Tp, 1), dtype=np.int64)

    if ragged:
        lengths = rng.integers(max(1, T // 2) if min_len is None else max(1, int(min_len)), T + 1, size=N)
    else:
        lengths = np.full(N, T, dtype=np.int64)
    for e in range(N):
        L = int(lengths[e])
        if L < T or e % 2 == 0:
            terminated[e, L - 1, 0] = 1
        # slot L holds the final obs/state/avail/action only; later slots are never written
        reward[e, L:] = 0.0
        if L + 1 < Tp:
            filled[e, L + 1:] = 0
            obs[e, L + 1:] = 0.0
            state[e, L + 1:] = 0.0
            avail[e, L + 1:] = 0
            actions[e, L + 1:] = 0

    onehot = np.zeros((N, Tp, n, A), dtype=np.float32)
    np.put_along_axis(onehot, actions, 1.0, axis=-1)
    onehot *= filled[:, :, None, :].astype(np.float32)

    return OrderedDict(
        state=state, obs=obs, actions=actions, avail_actions=avail, reward=reward,
        terminated=terminated, filled=filled, actions_onehot=onehot,
    )


def agent_param_shapes(input_dim, hidden_dim, n_actions):
    """RNNAgent parameters in `state_dict` / `parameters()` order (src/modules/agents/rnn_agent.py:19-21)."""
    H = hidden_dim
    return OrderedDict([
        ("fc1.weight", (H, input_dim)), ("fc1.bias", (H,)),
        ("rnn.weight_ih", (3 * H, H)), ("rnn.weight_hh", (3 * H, H)),
        ("rnn.bias_ih", (3 * H,)), ("rnn.bias_hh", (3 * H,)),
        ("fc2.weight", (n_actions, H)), ("fc2.bias", (n_actions,)),
    ])


def qmix_param_shapes(state_dim, n_agents, embed_dim):
    """QMixer parameters in `state_dict` / `parameters()` order (src/modules/mixers/qmix.py:14-23)."""
    S, E = state_dim, embed_dim
    return OrderedDict([
        ("hyper_w_1.weight", (E * n_agents, S)), ("hyper_w_1.bias", (E * n_agents,)),
        ("hyper_w_final.weight", (E, S)), ("hyper_w_final.bias", (E,)),
        ("hyper_b_1.weight", (E, S)), ("hyper_b_1.bias", (E,)),
        ("V.0.weight", (E, S)), ("V.0.bias", (E,)),
        ("V.2.weight", (1, E)), ("V.2.bias", (1,)),
    ])


def init_params(shapes, seed):
    """Uniform(-1/sqrt(fan_in), 1/sqrt(fan_in)) per tensor (torch nn.Linear / GRUCell default scale), PCG64-seeded.

    Weights come from numpy so the fixtures never depend on torch's RNG; a bias takes the fan-in
    of the weight it follows.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    out = OrderedDict()
    fan_in = 1
    for name, shape in shapes.items():
        if len(shape) == 2:
            fan_in = shape[1]
        bound = 1.0 / math.sqrt(fan_in)
        if name.startswith("rnn."):
            bound = 1.0 / math.sqrt(shape[-1] if len(shape) == 2 else shape[0] // 3)
        out[name] = rng.uniform(-bound, bound, size=shape).astype(np.float32)
    return out
