"""Generate the COMA golden fixtures by running the REFERENCE COMALearner (nicholasburden/pymarl) in this container.

    python tests/golden/make_golden_coma.py            # writes tests/golden/coma_*.npz

Not part of the product and never run on the GPU box (it needs /root/reference). Same recipe as make_golden.py:
the reference hot path is imported from /root/reference/src, fed the seeded synthetic replay of
pymarl_amd/utils/synthetic.py with numpy-seeded weights loaded via load_state_dict, and recorded:

* per-step values of the nine stats COMALearner.train logs (coma_learner.py:85-96),
* the sampled episode ids of ReplayBuffer.sample under np.random.seed(2) (episode_buffer.py:291-298),
* the epsilon each step's policy used (the MAC's action_selector.epsilon, read at basic_controller.py:64-67),
* for the small shape, the clipped agent gradients and the last critic step's clipped gradients of step 0, and
  agent / critic / target-critic parameters and both RMSprop states after every step.

Workarounds: default.yaml is missing, so `args` is built explicitly (coma_smac.yaml
values: lr = critic_lr = 5e-4, td_lambda 0.8, mask_before_softmax False, multinomial selector); BasicMAC mutates
scheme["obs"]["vshape"] into a tuple, which breaks COMACritic._get_input_shape, so the critic is given an
unmutated copy of the scheme.
"""
from __future__ import annotations

import copy
import os
import sys
from types import SimpleNamespace as SN

sys.dont_write_bytecode = True   # /root/reference is read-only: no __pycache__ there

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, "/root/reference/src")

import torch as th  # noqa: E402

from oracle.coma_np import critic_input_dim, critic_param_shapes  # noqa: E402
from pymarl_amd.utils.synthetic import agent_param_shapes, init_params, make_replay  # noqa: E402

from components.episode_buffer import ReplayBuffer  # noqa: E402  (reference)
from components.transforms import OneHot  # noqa: E402  (reference)
from controllers.basic_controller import BasicMAC  # noqa: E402  (reference)
from learners.coma_learner import COMALearner  # noqa: E402  (reference)


class _Console:
    def info(self, *a, **k):
        pass


class _Logger:
    def __init__(self):
        self.console_logger = _Console()
        self.stats = {}

    def log_stat(self, key, value, t):
        if isinstance(value, th.Tensor):
            value = value.item()
        self.stats.setdefault(key, []).append(float(value))


STATS = ["critic_loss", "critic_grad_norm", "td_error_abs", "q_taken_mean", "target_mean", "advantage_mean",
         "coma_loss", "agent_grad_norm", "pi_max"]


def make_args(case):
    return SN(n_agents=case["n"], n_actions=case["A"], state_shape=case["S"], obs_shape=case["O"], rnn_hidden_dim=64,
              lr=5e-4, critic_lr=5e-4, optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10.0, gamma=0.99,
              td_lambda=0.8, target_update_interval=case["target_update_interval"], learner_log_interval=0,
              obs_last_action=True, obs_agent_id=True, agent="rnn", mac="basic_mac", agent_output_type="pi_logits",
              action_selector="multinomial", epsilon_start=0.5, epsilon_finish=0.01, epsilon_anneal_time=100000,
              mask_before_softmax=case["mask_before_softmax"], action_input_representation=None, obs_decoder=None,
              avail_actions_encoder=None, device="cpu", use_cuda=False)


def make_scheme(n, A, O, S):
    return {
        "state": {"vshape": S},
        "obs": {"vshape": O, "group": "agents", "vshape_decoded": O},
        "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
        "avail_actions": {"vshape": (A,), "group": "agents", "dtype": th.int},
        "reward": {"vshape": (1,)},
        "terminated": {"vshape": (1,), "dtype": th.uint8},
    }


def flat(params):
    return np.concatenate([p.detach().cpu().numpy().ravel() for p in params]).astype(np.float32)


def flat_grads(params):
    return np.concatenate([p.grad.detach().cpu().numpy().ravel() for p in params]).astype(np.float32)


def flat_sq(opt, params):
    return np.concatenate([opt.state[p]["square_avg"].cpu().numpy().ravel() for p in params]).astype(np.float32)


def run_case(name, case):
    th.set_num_threads(8)
    n, A, O, S, T = case["n"], case["A"], case["O"], case["S"], case["T"]
    args = make_args(case)
    scheme = make_scheme(n, A, O, S)
    groups = {"agents": n}
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=A)])}
    buf = ReplayBuffer(scheme, groups, case["n_episodes"], T + 1, preprocess=preprocess, device="cpu")
    data = make_replay(case["n_episodes"], T, n, A, O, S, seed=case["data_seed"], ragged=case["ragged"])
    for k, v in data.items():
        buf.data.transition_data[k][:] = th.from_numpy(v)
    buf.episodes_in_buffer = case["n_episodes"]
    buf.buffer_index = 0

    critic_scheme = copy.deepcopy(buf.scheme)   # BasicMAC mutates scheme["obs"]["vshape"]
    mac = BasicMAC(buf.scheme, groups, args)
    logger = _Logger()
    learner = COMALearner(mac, critic_scheme, logger, args)
    I = O + A + n
    w_agent = init_params(agent_param_shapes(I, 64, A), seed=case["weight_seed"])
    mac.agent.load_state_dict({k: th.from_numpy(v) for k, v in w_agent.items()})
    K = critic_input_dim(n, A, O, S)
    w_critic = init_params(critic_param_shapes(K, A), seed=case["weight_seed"] + 200)
    learner.critic.load_state_dict({k: th.from_numpy(v) for k, v in w_critic.items()})
    learner.target_critic.load_state_dict({k: th.from_numpy(v) for k, v in w_critic.items()})

    out = {k: np.array(v) for k, v in case.items() if not isinstance(v, (str, bool))}
    for kb in ("mask_before_softmax", "ragged", "full"):
        out[kb] = np.array(int(case[kb]))
    np.random.seed(case["sampler_seed"])
    ids_all, eps_all = [], []
    per = {"agent": [], "critic": [], "target_critic": [], "sq": [], "critic_sq": []}
    for k in range(case["steps"]):
        st = np.random.get_state()
        batch = buf.sample(case["B"])
        after = np.random.get_state()
        np.random.set_state(st)
        ids = np.random.choice(buf.episodes_in_buffer, case["B"], replace=False)
        np.random.set_state(after)
        assert np.array_equal(batch["obs"].numpy(), buf["obs"][ids].numpy())
        ids_all.append(ids.astype(np.int64))
        batch = batch[:, :batch.max_t_filled()]
        t_env = 1000 * (k + 1)
        eps = float(learner.mac.action_selector.schedule.eval(t_env))
        learner.mac.action_selector.epsilon = eps
        eps_all.append(eps)
        if case["full"] and k == 0:
            # the reference COMACritic.forward (coma.py:22-27) on its own, all steps and single steps
            with th.no_grad():
                out["step0_critic_q_all"] = learner.critic(batch).numpy().copy()
                out["step0_critic_q_t0"] = learner.critic(batch, t=0).numpy().copy()
                out["step0_critic_q_t2"] = learner.critic(batch, t=2).numpy().copy()
        learner.train(batch, t_env=t_env, episode_num=8 * k)
        if case["full"]:
            if k == 0:
                out["step0_agent_grads"] = flat_grads(learner.agent_params)
                out["step0_critic_grads_last"] = flat_grads(learner.critic_params)
            per["agent"].append(flat(learner.agent_params))
            per["critic"].append(flat(learner.critic_params))
            per["target_critic"].append(flat(learner.target_critic.parameters()))
            per["sq"].append(flat_sq(learner.agent_optimiser, learner.agent_params))
            per["critic_sq"].append(flat_sq(learner.critic_optimiser, learner.critic_params))
    out["ids"] = np.stack(ids_all)
    out["epsilon"] = np.array(eps_all, np.float64)
    out["critic_training_steps"] = np.array(learner.critic_training_steps)
    for key in STATS:
        out["stat_" + key] = np.array(logger.stats[key], dtype=np.float64)
    if case["full"]:
        for kk, v in per.items():
            out["step_" + kk] = np.stack(v)
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print(name, "steps", case["steps"], "critic_loss", np.round(out["stat_critic_loss"], 5), "coma_loss",
          np.round(out["stat_coma_loss"], 6), "->", path, os.path.getsize(path) // 1024, "KB")


TINY = dict(n=3, A=5, O=12, S=20, T=10, B=4, n_episodes=6, data_seed=0, weight_seed=1, sampler_seed=2, ragged=True,
            steps=4, full=True, target_update_interval=15, mask_before_softmax=False)
CFG5 = dict(n=10, A=18, O=176, S=322, T=180, B=8, n_episodes=16, data_seed=0, weight_seed=1, sampler_seed=2,
            ragged=True, steps=3, full=False, target_update_interval=200, mask_before_softmax=False)

CASES = {
    "coma_tiny": TINY,
    "coma_tiny_masked": dict(TINY, mask_before_softmax=True, steps=3),
    # BASELINE configs[4] shape (MMM2: n=10, A=18), coma_smac.yaml batch_size 8
    "coma_cfg5": CFG5,
}

if __name__ == "__main__":
    only = sys.argv[1:]
    for nm, cs in CASES.items():
        if only and nm not in only:
            continue
        run_case(nm, cs)
