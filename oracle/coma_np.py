"""ORACLE — test infrastructure only. CPU restatement of the reference COMA learner step in numpy float32.

Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may import this module, and only as the
checker / the timed CPU baseline. The product path (pymarl_amd) never imports it and has no CPU fallback.

What it restates (reference = nicholasburden/pymarl @ /root/reference, cited file:line):
* COMACritic._build_inputs ........ src/modules/critics/coma.py:30-58 (state | obs | joint actions_onehot with the
                                    agent's own block zeroed | last joint actions (0 at t=0) | agent-id onehot)
* COMACritic.forward .............. src/modules/critics/coma.py:22-27 (fc1 -> relu -> fc2 -> relu -> fc3)
* build_td_lambda_targets ......... src/utils/rl_utils.py:4-14
* COMALearner._train_critic ....... src/learners/coma_learner.py:100-148 (one critic RMSprop step per t, reversed,
                                    each with its own masked L2 loss, clip_grad_norm_ and stats)
* BasicMAC.forward pi_logits ...... src/controllers/basic_controller.py:53-73 (softmax, optional -1e10 mask
                                    before it, epsilon floor, optional zeroing)
* COMALearner.train ............... src/learners/coma_learner.py:32-98 (renormalised masked policy, counterfactual
                                    baseline sum(pi * Q), advantage * log pi loss, agent clip + RMSprop, target
                                    critic update by critic training steps, the nine logged stats)
The backward passes are derived by hand (autograd in the reference). The agent recurrence reuses
qlearner_np.agent_unroll / agent_backward (rnn_agent.py:27-36).

Parity pinning: tests/test_coma_oracle.py checks this module against tests/golden/coma_*.npz, which
tests/golden/make_golden_coma.py produced by running the reference COMALearner itself (torch 2.10 CPU).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

from .qlearner_np import F32, agent_backward, agent_unroll, clip_grad_norm, rmsprop_step

CRITIC_HIDDEN = 128   # coma.py:17-19


def critic_param_shapes(input_dim, n_actions, hidden=CRITIC_HIDDEN):
    """COMACritic parameters in parameters() order (coma.py:17-19)."""
    return OrderedDict([
        ("fc1.weight", (hidden, input_dim)), ("fc1.bias", (hidden,)),
        ("fc2.weight", (hidden, hidden)), ("fc2.bias", (hidden,)),
        ("fc3.weight", (n_actions, hidden)), ("fc3.bias", (n_actions,)),
    ])


def critic_input_dim(n_agents, n_actions, obs_dim, state_dim):
    """coma.py:61-70."""
    return state_dim + obs_dim + 2 * n_agents * n_actions + n_agents


def critic_inputs(state, obs, actions_onehot, n_agents):
    """coma.py:30-58 with t=None: (B, Tp, n, S + O + 2 n A + n)."""
    B, Tp, n, _ = obs.shape
    A = actions_onehot.shape[-1]
    st = np.repeat(state[:, :, None, :], n, axis=2)
    joint = np.repeat(actions_onehot.reshape(B, Tp, 1, n * A), n, axis=2)
    agent_mask = np.repeat((F32(1.0) - np.eye(n, dtype=F32)).reshape(-1, 1), A, axis=1).reshape(n, n * A)
    acts = joint * agent_mask[None, None]
    last = np.concatenate([np.zeros_like(actions_onehot[:, :1]), actions_onehot[:, :-1]], 1)
    last = np.repeat(last.reshape(B, Tp, 1, n * A), n, axis=2)
    eye = np.broadcast_to(np.eye(n, dtype=F32), (B, Tp, n, n))
    return np.concatenate([st, obs, acts, last, eye], -1).astype(F32)


def critic_forward(cp, x):
    """coma.py:22-27 on rows x (..., K) -> (h1, h2, q)."""
    h1 = np.maximum(x @ cp["fc1.weight"].T + cp["fc1.bias"], F32(0.0)).astype(F32)
    h2 = np.maximum(h1 @ cp["fc2.weight"].T + cp["fc2.bias"], F32(0.0)).astype(F32)
    q = (h2 @ cp["fc3.weight"].T + cp["fc3.bias"]).astype(F32)
    return h1, h2, q


def critic_backward(cp, x, h1, h2, dq):
    """Hand-derived backward of critic_forward over rows (M, .): grads in parameters() order."""
    g = OrderedDict()
    g["fc3.weight"] = dq.T @ h2
    g["fc3.bias"] = dq.sum(0)
    dh2 = (dq @ cp["fc3.weight"]) * (h2 > 0)
    g["fc2.weight"] = dh2.T @ h1
    g["fc2.bias"] = dh2.sum(0)
    dh1 = (dh2 @ cp["fc2.weight"]) * (h1 > 0)
    g["fc1.weight"] = dh1.T @ x
    g["fc1.bias"] = dh1.sum(0)
    order = ["fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias", "fc3.weight", "fc3.bias"]
    return OrderedDict((k, g[k].astype(F32)) for k in order)


def td_lambda_targets(rewards, terminated, mask, target_qs, gamma, td_lambda):
    """rl_utils.py:4-14. rewards/terminated/mask (B, T, 1), target_qs (B, T+1, n) -> (B, T, n)."""
    ret = np.zeros_like(target_qs)
    ret[:, -1] = target_qs[:, -1] * (F32(1.0) - terminated.sum(1))
    lg = F32(td_lambda * gamma)
    og = F32((1 - td_lambda) * gamma)
    for t in range(ret.shape[1] - 2, -1, -1):
        ret[:, t] = lg * ret[:, t + 1] + mask[:, t] * (rewards[:, t] + og * target_qs[:, t + 1] *
                                                      (F32(1.0) - terminated[:, t]))
    return ret[:, :-1].astype(F32)


def policy_from_logits(logits, avail, epsilon, mask_before_softmax):
    """basic_controller.py:53-73 (test_mode=False) followed by coma_learner.py:59-62. Returns (pi, cache)."""
    A = logits.shape[-1]
    lg = logits.copy()
    if mask_before_softmax:
        lg[avail == 0] = F32(-1e10)
    mx = lg.max(-1, keepdims=True)
    e = np.exp(lg - mx).astype(F32)
    sm = (e / e.sum(-1, keepdims=True)).astype(F32)
    if mask_before_softmax:
        nact = avail.sum(-1, keepdims=True).astype(F32)
    else:
        nact = F32(A)
    with np.errstate(divide="ignore", invalid="ignore"):   # rows with no available action: zeroed below
        out = (F32(1.0 - epsilon) * sm + (np.ones_like(sm) * F32(epsilon)) / nact).astype(F32)
    if mask_before_softmax:
        out[avail == 0] = 0.0
    out[avail == 0] = 0.0
    s = out.sum(-1, keepdims=True).astype(F32)
    with np.errstate(invalid="ignore", divide="ignore"):
        pi = (out / s).astype(F32)
    pi[avail == 0] = 0.0
    return pi, (sm, out, s)


def policy_backward(dpi, pi, cache, avail, epsilon, mask_before_softmax):
    """Backward of policy_from_logits (rows whose available set is empty get zero gradient)."""
    sm, out, s = cache
    dpi = np.where(avail == 0, F32(0.0), dpi).astype(F32)
    with np.errstate(invalid="ignore", divide="ignore"):
        dout = ((dpi - (dpi * pi).sum(-1, keepdims=True)) / s).astype(F32)
    dout = np.where((avail == 0) | (s == 0), F32(0.0), dout).astype(F32)
    dsm = (F32(1.0 - epsilon) * dout).astype(F32)
    dl = (sm * (dsm - (sm * dsm).sum(-1, keepdims=True))).astype(F32)
    if mask_before_softmax:
        dl[avail == 0] = 0.0
    return dl


class OracleCOMALearner:
    """numpy COMALearner (coma_learner.py:9-171) over numpy EpisodeBatch dicts."""

    def __init__(self, agent_params, critic_params, cfg):
        self.cfg = dict(cfg)
        self.p = OrderedDict((k, np.array(v, F32)) for k, v in agent_params.items())
        self.cp = OrderedDict((k, np.array(v, F32)) for k, v in critic_params.items())
        self.ctp = OrderedDict((k, v.copy()) for k, v in self.cp.items())
        self.sq = OrderedDict((k, np.zeros_like(v)) for k, v in self.p.items())
        self.csq = OrderedDict((k, np.zeros_like(v)) for k, v in self.cp.items())
        self.critic_training_steps = 0
        self.last_target_update_step = 0
        self.last = {}

    def train(self, batch, t_env, episode_num, epsilon):
        """coma_learner.py:32-98; `epsilon` is the MAC's action_selector.epsilon the reference reads (:56 via
        basic_controller.py:64-67). Returns the stats dict it would log."""
        c = self.cfg
        n, A = c["n_agents"], c["n_actions"]
        rewards = batch["reward"][:, :-1].astype(F32)
        actions_all = batch["actions"]
        terminated = batch["terminated"][:, :-1].astype(F32)
        mask = batch["filled"][:, :-1].astype(F32).copy()
        mask[:, 1:] = mask[:, 1:] * (F32(1.0) - terminated[:, :-1])
        avail = batch["avail_actions"][:, :-1]
        B, Tp = batch["filled"].shape[:2]
        T = Tp - 1

        # ---- critic (coma_learner.py:100-148)
        X = critic_inputs(batch["state"], batch["obs"], batch["actions_onehot"], n)
        _, _, tq = critic_forward(self.ctp, X)
        targets_taken = np.take_along_axis(tq, actions_all, axis=3)[..., 0]
        targets = td_lambda_targets(rewards, terminated, mask, targets_taken, c["gamma"], c["td_lambda"])
        q_vals = np.zeros((B, T, n, A), F32)
        log = {k: [] for k in ["critic_loss", "critic_grad_norm", "td_error_abs", "target_mean", "q_taken_mean"]}
        critic_grads = []
        for t in reversed(range(T)):
            mask_t = np.broadcast_to(mask[:, t], (B, n)).astype(F32)
            if mask_t.sum() == 0:
                continue
            x = X[:, t].reshape(B * n, -1)
            h1, h2, q = critic_forward(self.cp, x)
            q_vals[:, t] = q.reshape(B, n, A)
            a_t = actions_all[:, t].reshape(B * n)
            q_taken = q[np.arange(B * n), a_t].reshape(B, n)
            targets_t = targets[:, t]
            td = q_taken - targets_t
            mtd = (td * mask_t).astype(F32)
            msum = F32(mask_t.sum())
            loss = F32((mtd * mtd).sum()) / msum
            dq = np.zeros((B * n, A), F32)
            dq[np.arange(B * n), a_t] = ((F32(2.0) * mtd) / msum * mask_t).reshape(-1)
            grads = critic_backward(self.cp, x, h1, h2, dq)
            gn = clip_grad_norm(grads, c["grad_norm_clip"])
            critic_grads.append(grads)
            rmsprop_step(self.cp, grads, self.csq, c["critic_lr"], c["optim_alpha"], c["optim_eps"])
            self.critic_training_steps += 1
            mel = float(mask_t.sum())
            log["critic_loss"].append(float(loss))
            log["critic_grad_norm"].append(gn)
            log["td_error_abs"].append(float(np.abs(mtd).sum()) / mel)
            log["q_taken_mean"].append(float((q_taken * mask_t).sum()) / mel)
            log["target_mean"].append(float((targets_t * mask_t).sum()) / mel)

        # ---- actor (coma_learner.py:50-83)
        actions = actions_all[:, :-1]
        logits, acache = agent_unroll(self.p, batch["obs"][:, :T], batch["actions_onehot"][:, :T], keep_cache=True)
        mbs = bool(c.get("mask_before_softmax", True))
        pi, pcache = policy_from_logits(logits, avail, epsilon, mbs)
        baseline = (pi * q_vals).sum(-1).astype(F32)
        q_taken = np.take_along_axis(q_vals, actions, axis=3)[..., 0]
        pi_taken = np.take_along_axis(pi, actions, axis=3)[..., 0].copy()
        m = np.broadcast_to(mask, (B, T, n)).astype(F32)
        pi_taken[m == 0] = 1.0
        log_pi = np.log(pi_taken).astype(F32)
        adv = (q_taken - baseline).astype(F32)
        msum = F32(m.sum())
        coma_loss = -F32(((adv * log_pi) * m).sum()) / msum
        dlogpi = (-(adv * m) / msum).astype(F32)
        dpt = np.where(m == 0, F32(0.0), dlogpi / pi_taken).astype(F32)
        dpi = np.zeros_like(pi)
        np.put_along_axis(dpi, actions, dpt[..., None], axis=3)
        dl = policy_backward(dpi, pi, pcache, avail, epsilon, mbs)
        ag = agent_backward(self.p, acache, dl)
        agent_gn = clip_grad_norm(ag, c["grad_norm_clip"])
        rmsprop_step(self.p, ag, self.sq, c["lr"], c["optim_alpha"], c["optim_eps"])

        if (self.critic_training_steps - self.last_target_update_step) / c["target_update_interval"] >= 1.0:
            self.ctp = OrderedDict((k, v.copy()) for k, v in self.cp.items())
            self.last_target_update_step = self.critic_training_steps

        nl = len(log["critic_loss"])
        stats = {k: sum(v) / nl for k, v in log.items()}
        stats["advantage_mean"] = float((adv * m).sum()) / float(msum)
        stats["coma_loss"] = float(coma_loss)
        stats["agent_grad_norm"] = agent_gn
        stats["pi_max"] = float((pi.max(-1) * m).sum()) / float(msum)
        self.last = dict(q_vals=q_vals, targets=targets, pi=pi, logits=logits, adv=adv, agent_grads=ag,
                         critic_grads=critic_grads, stats=stats, targets_taken=targets_taken)
        return stats

    def flat(self, which="agent"):
        d = {"agent": self.p, "critic": self.cp, "target_critic": self.ctp, "sq": self.sq, "critic_sq": self.csq}[which]
        return np.concatenate([v.ravel() for v in d.values()]).astype(F32)
