"""The rollout side on the GPU: EpisodeRunner or ParallelRunner (FakeEnv; 4 worker processes)
-> HBM ReplayBuffer -> QLearner.train,
with the HIP MAC step choosing the actions. Checks that the greedy (test-mode) actions the runner recorded are the
oracle's masked argmax of the agent's Q on the recorded episode (clear margins; basic_controller.py:30-38,
action_selectors.py:44-62), that every episode obeys the replay contract, and that training on runner-made episodes
gives finite stats."""
import logging
from types import SimpleNamespace as SN

import numpy as np
import pytest
import torch as th

pytestmark = pytest.mark.gpu

# BASELINE configs[0]'s shape (SMAC 3m, upstream obs / state sizes): episode_limit 60
N, A, O, S, LIMIT = 3, 9, 30, 48, 60
MARGIN_EPS = 1e-5   # argmax-equal wherever the top-2 gap exceeds 1e-5 * max(1, |Q|)


def build(kind="episode", bsr=1, cpu_only=False):
    from pymarl_amd.components.episode_buffer import ReplayBuffer
    from pymarl_amd.components.transforms import OneHot
    from pymarl_amd.controllers import REGISTRY as mac_REGISTRY
    from pymarl_amd.learners import REGISTRY as le_REGISTRY
    from pymarl_amd.runners import REGISTRY as r_REGISTRY
    from pymarl_amd.utils.logging import Logger
    args = SN(n_agents=N, n_actions=A, state_shape=S, obs_shape=O, rnn_hidden_dim=64, mixing_embed_dim=32,
              mixer="qmix", lr=5e-4, optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10.0, gamma=0.99, double_q=True,
              target_update_interval=200, learner_log_interval=0, obs_last_action=True, obs_agent_id=True,
              agent="rnn", mac="basic_mac", agent_output_type="q", action_selector="epsilon_greedy",
              epsilon_start=1.0, epsilon_finish=0.05, epsilon_anneal_time=500, batch_size=8, batch_size_run=bsr,
              env="fake", env_args=dict(n_agents=N, n_actions=A, obs_dim=O, state_dim=S, episode_limit=LIMIT, seed=4,
                                        end_threshold=None if kind == "episode" else -0.9),
              device="cuda", use_cuda=True, test_nepisode=1, runner_log_interval=10 ** 9, learner="q_learner",
              buffer_cpu_only=cpu_only)
    logger = Logger(logging.getLogger("runner-test"))
    runner = r_REGISTRY[kind](args, logger)
    scheme = {"state": {"vshape": S}, "obs": {"vshape": O, "group": "agents"},
              "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
              "avail_actions": {"vshape": (A,), "group": "agents", "dtype": th.int},
              "reward": {"vshape": (1,)}, "terminated": {"vshape": (1,), "dtype": th.uint8}}
    groups = {"agents": N}
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=A)])}
    # run.py:137-139: the replay lives on the host under buffer_cpu_only
    buf = ReplayBuffer(scheme, groups, 64, LIMIT + 1, preprocess=preprocess, device="cpu" if cpu_only else "cuda")
    mac = mac_REGISTRY["basic_mac"](buf.scheme, groups, args)
    runner.setup(scheme=scheme, groups=groups, preprocess=preprocess, mac=mac)
    learner = le_REGISTRY["q_learner"](mac, buf.scheme, logger, args)
    learner.cuda()
    return args, runner, buf, mac, learner


def check_contract(b, i=0):
    filled = b["filled"][i, :, 0].cpu().numpy()
    term = b["terminated"][i, :, 0].cpu().numpy()
    L = int(filled.sum()) - 1
    assert np.all(filled[:L + 1] == 1) and np.all(filled[L + 1:] == 0)
    assert term[L:].sum() == 0 and term[:max(0, L - 1)].sum() == 0
    assert L == LIMIT or term[L - 1] == 1   # cut at the limit, or a true termination at L-1
    av = b["avail_actions"][i, :L + 1].cpu().numpy()
    act = b["actions"][i, :L + 1, :, 0].cpu().numpy()
    assert np.all(np.take_along_axis(av, act[..., None], 2) == 1)
    return L


@pytest.mark.parametrize("kind,bsr,cpu_only", [("episode", 1, False), ("parallel", 4, False), ("parallel", 4, True)])
def test_runner_greedy_actions_and_training(kind, bsr, cpu_only):
    """cpu_only: the reference's buffer_cpu_only layout — the ParallelRunner writes a host batch
    (parallel_runner.py:45), the MAC moves each step's rows to the device, the host replay is sampled, truncated and
    moved with `.to(args.device)` before train (run.py:208-219)."""
    from oracle.qlearner_np import agent_unroll
    args, runner, buf, mac, learner = build(kind, bsr, cpu_only)
    np.random.seed(0)
    th.manual_seed(0)
    try:
        for ep in range(10 // bsr):
            b = runner.run(test_mode=False)
            for i in range(bsr):
                check_contract(b, i)
            buf.insert_episode_batch(b)
        # greedy test-mode episodes: recorded actions = masked argmax of the agent's Q (clear margins)
        b = runner.run(test_mode=True)
    finally:
        runner.close_env()
    assert b.device == ("cpu" if cpu_only else "cuda")
    p = {k: v.detach().cpu().numpy() for k, v in mac.agent.state_dict().items()}
    decisions = ties = tie_flips = 0
    for i in range(bsr):
        L = check_contract(b, i)
        obs = b["obs"][i:i + 1, :L + 1].cpu().numpy()
        oh = b["actions_onehot"][i:i + 1, :L + 1].cpu().numpy()
        q, _ = agent_unroll(p, obs, oh)
        av = b["avail_actions"][i:i + 1, :L + 1].cpu().numpy()
        qm = np.where(av == 0, -np.inf, q)
        greedy = qm.argmax(-1)
        top2 = -np.sort(-qm, -1)[..., :2]
        tie = (top2[..., 0] - top2[..., 1]) <= MARGIN_EPS * np.maximum(1.0, np.abs(top2[..., 0]))
        rec = b["actions"][i:i + 1, :L + 1, :, 0].cpu().numpy()
        # every greedy decision equals the oracle's masked argmax except near-ties, which are counted
        assert np.array_equal(rec[~tie], greedy[~tie])
        decisions += int(tie.size)
        ties += int(tie.sum())
        tie_flips += int((rec != greedy)[tie].sum())
    print("greedy decisions {} near-ties {} near-tie flips {}".format(decisions, ties, tie_flips))
    assert ties <= max(2, decisions // 100), (decisions, ties)   # near-ties are rare: a sanity bound
    # training on runner-made episodes, sampled the way run.py:207-219 does
    for k in range(3):
        s = buf.sample(8)
        s = s[:, :s.max_t_filled()]
        if s.device != args.device:
            s.to(args.device)
        learner.train(s, runner.t_env, 10 + k)
        st = learner.last_stats()
        assert all(np.isfinite(v) for v in st.values()), st
