"""Build the MI355X learner on a golden case (same data, weights and sampler seed as the reference run)."""
from __future__ import annotations

import logging
from types import SimpleNamespace as SN

import numpy as np
import torch as th

from pymarl_amd.components.episode_buffer import ReplayBuffer
from pymarl_amd.components.transforms import OneHot
from pymarl_amd.controllers import REGISTRY as mac_REGISTRY
from pymarl_amd.learners import REGISTRY as le_REGISTRY
from pymarl_amd.utils.logging import Logger


CKPT = {name: "ckpt_{}_step2".format(name) for name in ("tiny_qmix", "tiny_vdn")}


def make_args(case, **over):
    a = SN(n_agents=case.n, n_actions=case.A, state_shape=case.S, obs_shape=case.O, rnn_hidden_dim=64,
           mixing_embed_dim=32, mixer=None if case.mixer == "none" else case.mixer, lr=5e-4, optim_alpha=0.99,
           optim_eps=1e-5, grad_norm_clip=10.0, gamma=0.99, double_q=case.double_q, target_update_interval=200,
           learner_log_interval=0, obs_last_action=case.obs_last_action, obs_agent_id=case.obs_agent_id,
           agent="rnn", mac="basic_mac",
           agent_output_type="q", action_selector="epsilon_greedy", epsilon_start=1.0, epsilon_finish=0.05,
           epsilon_anneal_time=50000, batch_size=case.B, learner="q_learner", device="cuda", use_cuda=True)
    for k, v in over.items():
        setattr(a, k, v)
    return a


def make_scheme(case):
    return {
        "state": {"vshape": case.S},
        "obs": {"vshape": case.O, "group": "agents"},
        "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
        "avail_actions": {"vshape": (case.A,), "group": "agents", "dtype": th.int},
        "reward": {"vshape": (1,)},
        "terminated": {"vshape": (1,), "dtype": th.uint8},
    }


def build(case, device="cuda", buffer_device=None, **over):
    """buffer_device: where the ReplayBuffer lives (default: with the learner); "cpu" is the reference's
    buffer_cpu_only layout (run.py:137-139)."""
    args = make_args(case, **over)
    groups = {"agents": case.n}
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=case.A)])}
    buf = ReplayBuffer(make_scheme(case), groups, case.n_episodes, case.T + 1, preprocess=preprocess,
                       device=buffer_device or device)
    buf.load_arrays(case.data)
    mac = mac_REGISTRY["basic_mac"](buf.scheme, groups, args)
    logger = Logger(logging.getLogger("mq-test"))
    learner = le_REGISTRY["q_learner"](mac, buf.scheme, logger, args)
    if device != "cpu":
        learner.cuda()
    sd = {k: th.from_numpy(v) for k, v in case.agent_params.items()}
    mac.agent.load_state_dict(sd)
    learner.target_mac.agent.load_state_dict(sd)
    if case.mixer == "qmix":
        md = {k: th.from_numpy(v) for k, v in case.mixer_params.items()}
        learner.mixer.load_state_dict(md)
        learner.target_mixer.load_state_dict(md)
    return args, buf, mac, learner, logger


def flat_params(learner):
    return learner._online[:learner.n_params].detach().cpu().numpy().copy()


def flat_targets(learner):
    return learner._target[:learner.n_params].detach().cpu().numpy().copy()


def flat_grads(learner):
    return learner._grad[:learner.n_params].detach().cpu().numpy().copy()


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(1e-30, np.abs(b).max()))


def make_coma_args(case, **over):
    a = SN(n_agents=case.n, n_actions=case.A, state_shape=case.S, obs_shape=case.O, rnn_hidden_dim=64, lr=5e-4,
           critic_lr=5e-4, optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10.0, gamma=0.99, td_lambda=0.8,
           target_update_interval=case.target_update_interval, learner_log_interval=0, obs_last_action=True,
           obs_agent_id=True, agent="rnn", mac="basic_mac", agent_output_type="pi_logits",
           action_selector="multinomial", epsilon_start=0.5, epsilon_finish=0.01, epsilon_anneal_time=100000,
           mask_before_softmax=case.mask_before_softmax, batch_size=case.B, learner="coma_learner", device="cuda",
           use_cuda=True)
    for k, v in over.items():
        setattr(a, k, v)
    return a


def build_coma(case, device="cuda", **over):
    args = make_coma_args(case, **over)
    groups = {"agents": case.n}
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=case.A)])}
    buf = ReplayBuffer(make_scheme(case), groups, case.n_episodes, case.T + 1, preprocess=preprocess, device=device)
    buf.load_arrays(case.data)
    mac = mac_REGISTRY["basic_mac"](buf.scheme, groups, args)
    logger = Logger(logging.getLogger("mc-test"))
    learner = le_REGISTRY["coma_learner"](mac, buf.scheme, logger, args)
    learner.cuda()
    mac.agent.load_state_dict({k: th.from_numpy(v) for k, v in case.agent_params.items()})
    cd = {k: th.from_numpy(v) for k, v in case.critic_params.items()}
    learner.critic.load_state_dict(cd)
    learner.target_critic.load_state_dict(cd)
    return args, buf, mac, learner, logger


# The library's two switch variables (pymarl_amd/csrc/switches.hpp): MQ_PLAN for plan overrides, MQ_DIAG for
# diagnostics and test hooks, each a comma-separated list of `key` / `key=value` items.
DIAG_KEYS = ("pair_stamp", "hyp_sched", "coma_trace", "coma_fault")


def switch_value(env, key, value):
    """`env`'s MQ_PLAN / MQ_DIAG string with item `key` set (value True: a bare key; str / int: key=value) or
    removed (value None)."""
    var = "MQ_DIAG" if key in DIAG_KEYS else "MQ_PLAN"
    items = [i for i in env.get(var, "").split(",") if i and i.split("=", 1)[0] != key]
    if value is not None:
        items.append(key if value is True else "{}={}".format(key, value))
    return var, ",".join(items)


def set_switch(monkeypatch, key, value=True):
    """monkeypatch-scoped set_switch: restored after the test."""
    import os
    var, v = switch_value(os.environ, key, value)
    if v:
        monkeypatch.setenv(var, v)
    else:
        monkeypatch.delenv(var, raising=False)
