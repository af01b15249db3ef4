"""ORACLE — test infrastructure only. CPU restatement of the reference QMIX/VDN learner step in numpy float32.

Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may import this module, and only as the
checker / the timed CPU baseline. The product path (pymarl_amd) never imports it and has no CPU fallback.

What it restates (reference = nicholasburden/pymarl @ /root/reference, cited file:line):
* ReplayBuffer.sample id draw ............ src/components/episode_buffer.py:291-298
* EpisodeBatch.max_t_filled .............. src/components/episode_buffer.py:255-256
* BasicMAC._build_inputs ................. src/controllers/basic_controller.py:100-135 (obs | last-action onehot
                                           (zeros at t=0) | agent-id onehot)
* RNNAgent.forward ....................... src/modules/agents/rnn_agent.py:27-36 (fc1 -> relu -> GRUCell -> fc2)
* QMixer.forward / VDNMixer.forward ...... src/modules/mixers/qmix.py:28-47, src/modules/mixers/vdn.py:9-10
* QLearner.train ......................... src/learners/q_learner.py:37-116 (double-Q, -9999999 masks, masked L2,
                                           clip_grad_norm_, RMSprop, target update by episodes, the five stats)
The backward pass is derived by hand (autograd in the reference); GRUCell follows ATen's CPU gru_cell:
r = s(gi_r + gh_r), z = s(gi_z + gh_z), n = tanh(gi_n + r*gh_n), h' = (h - n)*z + n.

Parity pinning: tests/test_oracle_golden.py checks this module against tests/golden/*.npz, which
tests/golden/make_golden.py produced by running the reference learner itself (torch 2.10 CPU).
"""
from __future__ import annotations

from collections import OrderedDict

import numpy as np

F32 = np.float32
NEG = F32(-9999999.0)   # q_learner.py:68,74


def sample_ids(episodes_in_buffer, batch_size):
    """episode_buffer.py:291-298 — uniform without replacement on numpy's global legacy RNG."""
    if episodes_in_buffer == batch_size:
        return np.arange(batch_size)
    return np.random.choice(episodes_in_buffer, batch_size, replace=False)


def max_t_filled(filled):
    """episode_buffer.py:255-256 on a (B, T+1, 1) filled array."""
    return int(filled.sum(1).max())


def _sigmoid(x):
    return (F32(1.0) / (F32(1.0) + np.exp(-x))).astype(F32)


def _relu(x):
    return np.maximum(x, F32(0.0))


def _elu(x):
    return np.where(x > 0, x, np.expm1(np.minimum(x, F32(0.0)))).astype(F32)


def build_inputs(obs_t, onehot_prev, n_agents, flags=(True, True)):
    """basic_controller.py:100-135: cat[obs_t, onehot(a_{t-1}) (0 at t=0) if obs_last_action (:111-116),
    eye(n) if obs_agent_id (:118-120)] -> (B*n, I). flags = (obs_last_action, obs_agent_id)."""
    B = obs_t.shape[0]
    parts = [obs_t]
    if flags[0]:
        parts.append(onehot_prev)
    if flags[1]:
        parts.append(np.broadcast_to(np.eye(n_agents, dtype=F32), (B, n_agents, n_agents)))
    return np.concatenate(parts, -1).reshape(B * n_agents, -1).astype(F32)


def agent_unroll(p, obs, actions_onehot, keep_cache=False, relu_mask=None, pre_out=None, flags=(True, True)):
    """BasicMAC.forward over t = 0..T (q_learner.py:47-52 / 58-62) with RNNAgent (rnn_agent.py:27-36).

    obs (B,Tp,n,O), actions_onehot (B,Tp,n,A) -> mac_out (B,Tp,n,A) [+ cache for the backward pass].
    relu_mask (B,Tp,n,H) bool: take the fc1 relu's on/off decisions from another implementation (a parity test
    following it through fc1 pre-activations that round to the other side of 0). pre_out: list receiving the
    fc1 pre-activations per step. flags: (obs_last_action, obs_agent_id), basic_controller.py:111-120.
    """
    B, Tp, n, _ = obs.shape
    A = actions_onehot.shape[-1]
    H = p["rnn.weight_hh"].shape[1]
    h = np.zeros((B * n, H), F32)                                   # init_hidden, basic_controller.py:77-81
    outs, cache = [], []
    for t in range(Tp):
        prev = np.zeros((B, n, A), F32) if t == 0 else actions_onehot[:, t - 1]
        x = build_inputs(obs[:, t], prev, n, flags)
        pre = x @ p["fc1.weight"].T + p["fc1.bias"]
        if pre_out is not None:
            pre_out.append(pre.reshape(B, n, -1))
        on = pre > 0 if relu_mask is None else relu_mask[:, t].reshape(B * n, -1)
        x1 = np.where(on, pre, F32(0.0)).astype(F32)
        gi = x1 @ p["rnn.weight_ih"].T + p["rnn.bias_ih"]
        gh = h @ p["rnn.weight_hh"].T + p["rnn.bias_hh"]
        r = _sigmoid(gh[:, :H] + gi[:, :H])
        z = _sigmoid(gh[:, H:2 * H] + gi[:, H:2 * H])
        nn_ = np.tanh(gi[:, 2 * H:] + gh[:, 2 * H:] * r).astype(F32)
        h_new = ((h - nn_) * z + nn_).astype(F32)
        q = h_new @ p["fc2.weight"].T + p["fc2.bias"]
        if keep_cache:
            cache.append((x, x1, on, h, r, z, nn_, gh[:, 2 * H:].copy(), h_new))
        h = h_new
        outs.append(q.reshape(B, n, A))
    return np.stack(outs, 1).astype(F32), cache


def fc1_preacts(p, obs, actions_onehot, flags=(True, True)):
    """fc1 pre-activations of every (b, t, agent) (rnn_agent.py:28 before the relu): (B,Tp,n,H)."""
    B, Tp, n, _ = obs.shape
    A = actions_onehot.shape[-1]
    out = []
    for t in range(Tp):
        prev = np.zeros((B, n, A), F32) if t == 0 else actions_onehot[:, t - 1]
        x = build_inputs(obs[:, t], prev, n, flags)
        out.append((x @ p["fc1.weight"].T + p["fc1.bias"]).reshape(B, n, -1))
    return np.stack(out, 1).astype(F32)


def qmix_forward(mp, agent_qs, states, n_agents, keep_cache=False):
    """QMixer.forward, qmix.py:28-47. agent_qs (B,T,n), states (B,T,S) -> (B,T,1)."""
    B, T = agent_qs.shape[:2]
    E = mp["hyper_b_1.weight"].shape[0]
    s = states.reshape(-1, states.shape[-1]).astype(F32)
    q = agent_qs.reshape(-1, n_agents).astype(F32)
    hw1 = s @ mp["hyper_w_1.weight"].T + mp["hyper_w_1.bias"]
    w1 = np.abs(hw1).reshape(-1, n_agents, E)
    hb1 = s @ mp["hyper_b_1.weight"].T + mp["hyper_b_1.bias"]
    pre = np.einsum("mn,mne->me", q, w1).astype(F32) + hb1
    hid = _elu(pre)
    hwf = s @ mp["hyper_w_final.weight"].T + mp["hyper_w_final.bias"]
    wf = np.abs(hwf)
    hv = s @ mp["V.0.weight"].T + mp["V.0.bias"]
    rv = _relu(hv)
    v = rv @ mp["V.2.weight"].T + mp["V.2.bias"]
    y = (hid * wf).sum(-1, keepdims=True).astype(F32) + v
    cache = (s, q, hw1, w1, hb1, pre, hid, hwf, wf, hv, rv) if keep_cache else None
    return y.reshape(B, T, 1).astype(F32), cache


def qmix_backward(mp, cache, dy):
    """Hand-derived backward of qmix_forward. dy (M,) -> (dq (M,n), grads in QMixer.parameters() order)."""
    s, q, hw1, w1, hb1, pre, hid, hwf, wf, hv, rv = cache
    M, n, E = w1.shape
    d_hid = dy[:, None] * wf
    d_hwf = (dy[:, None] * hid) * np.sign(hwf)
    d_pre = d_hid * np.where(pre > 0, F32(1.0), np.exp(np.minimum(pre, F32(0.0)))).astype(F32)
    d_hw1 = (q[:, :, None] * d_pre[:, None, :]).reshape(M, n * E) * np.sign(hw1)
    d_hw1 = d_hw1.astype(F32)
    dq = np.einsum("me,mne->mn", d_pre, w1).astype(F32)
    d_rv = dy[:, None] * mp["V.2.weight"][0][None, :]
    d_hv = d_rv * (hv > 0)
    g = OrderedDict()
    g["hyper_w_1.weight"] = d_hw1.T @ s
    g["hyper_w_1.bias"] = d_hw1.sum(0)
    g["hyper_w_final.weight"] = d_hwf.T @ s
    g["hyper_w_final.bias"] = d_hwf.sum(0)
    g["hyper_b_1.weight"] = d_pre.T @ s
    g["hyper_b_1.bias"] = d_pre.sum(0)
    g["V.0.weight"] = d_hv.T @ s
    g["V.0.bias"] = d_hv.sum(0)
    g["V.2.weight"] = (dy[None, :] @ rv)
    g["V.2.bias"] = np.array([dy.sum()], F32)
    return dq, OrderedDict((k, v.astype(F32)) for k, v in g.items())


def agent_backward(p, cache, dmac_out):
    """BPTT of agent_unroll. dmac_out (B,Tp,n,A) -> grads in RNNAgent.parameters() order."""
    H = p["rnn.weight_hh"].shape[1]
    B, Tp, n, A = dmac_out.shape
    g = OrderedDict((k, np.zeros_like(v)) for k, v in p.items())
    dh = np.zeros((B * n, H), F32)
    for t in range(Tp - 1, -1, -1):
        x, x1, on, h_prev, r, z, nn_, ghn, h_new = cache[t]
        dq = dmac_out[:, t].reshape(B * n, A)
        g["fc2.weight"] += dq.T @ h_new
        g["fc2.bias"] += dq.sum(0)
        dh = dh + dq @ p["fc2.weight"]
        dn = dh * (F32(1.0) - z)
        dz = dh * (h_prev - nn_)
        dan = dn * (F32(1.0) - nn_ * nn_)
        dar = (dan * ghn) * (r * (F32(1.0) - r))
        daz = dz * (z * (F32(1.0) - z))
        dgi = np.concatenate([dar, daz, dan], 1).astype(F32)
        dgh = np.concatenate([dar, daz, dan * r], 1).astype(F32)
        g["rnn.weight_ih"] += dgi.T @ x1
        g["rnn.bias_ih"] += dgi.sum(0)
        g["rnn.weight_hh"] += dgh.T @ h_prev
        g["rnn.bias_hh"] += dgh.sum(0)
        dx1 = (dgi @ p["rnn.weight_ih"]) * on
        g["fc1.weight"] += dx1.T @ x
        g["fc1.bias"] += dx1.sum(0)
        dh = (dh * z + dgh @ p["rnn.weight_hh"]).astype(F32)
    return g


def clip_grad_norm(grads, max_norm):
    """torch.nn.utils.clip_grad_norm_ (norm of per-tensor norms, clamp(max_norm/(norm+1e-6), max=1))."""
    norms = np.array([np.sqrt((g.astype(np.float64) ** 2).sum()) for g in grads.values()])
    total = F32(np.sqrt((norms ** 2).sum()))
    coef = min(F32(max_norm) / (total + F32(1e-6)), F32(1.0))
    for k in grads:
        grads[k] = (grads[k] * F32(coef)).astype(F32)
    return float(total)


def rmsprop_step(params, grads, sq, lr, alpha, eps):
    """torch.optim.RMSprop single-tensor step (no momentum, not centred): q_learner.py:30,103."""
    for k in params:
        sq[k] = (sq[k] * F32(alpha) + (grads[k] * grads[k]) * F32(1.0 - alpha)).astype(F32)
        avg = np.sqrt(sq[k]) + F32(eps)
        params[k] = (params[k] + F32(-lr) * (grads[k] / avg)).astype(F32)


class OracleQLearner:
    """numpy QLearner (q_learner.py:9-143) over numpy EpisodeBatch dicts (keys as in the reference scheme)."""

    def __init__(self, agent_params, mixer_params, cfg):
        self.cfg = dict(cfg)
        self.p = OrderedDict((k, np.array(v, F32)) for k, v in agent_params.items())
        self.mp = OrderedDict((k, np.array(v, F32)) for k, v in (mixer_params or {}).items())
        self.tp = OrderedDict((k, v.copy()) for k, v in self.p.items())
        self.tmp = OrderedDict((k, v.copy()) for k, v in self.mp.items())
        self.sq = OrderedDict((k, np.zeros_like(v)) for k, v in list(self.p.items()) + list(self.mp.items()))
        self.last_target_update_episode = 0
        self.log_stats_t = -self.cfg.get("learner_log_interval", 0) - 1
        self.last = {}

    @property
    def input_flags(self):
        """(obs_last_action, obs_agent_id): basic_controller.py:111,118 (True / True in every shipped config)."""
        return (bool(self.cfg.get("obs_last_action", True)), bool(self.cfg.get("obs_agent_id", True)))

    def forward(self, batch, keep_cache=False, cur_max_override=None, relu_override=None):
        """q_learner.py:39-97: returns dict of intermediates (+ caches).

        cur_max_override (B, T, n): use these double-Q argmax actions instead of recomputing them — lets a parity
        test follow the other implementation through near-tie argmax flips (both choices are correct fp32 ties).
        relu_override (B, T+1, n, H) bool: the online agent's fc1 relu decisions, likewise (see agent_unroll).
        """
        c = self.cfg
        n = c["n_agents"]
        rewards = batch["reward"][:, :-1].astype(F32)
        actions = batch["actions"][:, :-1]
        terminated = batch["terminated"][:, :-1].astype(F32)
        mask = batch["filled"][:, :-1].astype(F32).copy()
        mask[:, 1:] = mask[:, 1:] * (F32(1.0) - terminated[:, :-1])
        avail = batch["avail_actions"]
        fl = self.input_flags
        mac_out, acache = agent_unroll(self.p, batch["obs"], batch["actions_onehot"], keep_cache, relu_override,
                                       flags=fl)
        chosen = np.take_along_axis(mac_out[:, :-1], actions, axis=3)[..., 0]
        tmo_full, _ = agent_unroll(self.tp, batch["obs"], batch["actions_onehot"], flags=fl)
        tmo = tmo_full[:, 1:].copy()
        tmo[avail[:, 1:] == 0] = NEG
        if c.get("double_q", True):
            mod = mac_out.copy()
            mod[avail == 0] = NEG
            cur_max = mod[:, 1:].argmax(axis=3)
            if cur_max_override is not None:
                cur_max = np.asarray(cur_max_override, dtype=np.int64)
            target_max = np.take_along_axis(tmo, cur_max[..., None], axis=3)[..., 0]
        else:   # q_learner.py:77-78: target_mac_out.max(dim=3); argmax kept for the decision accounting
            cur_max = tmo.argmax(axis=3)
            if cur_max_override is not None:
                cur_max = np.asarray(cur_max_override, dtype=np.int64)
            target_max = tmo.max(axis=3)
        mcache = None
        if c["mixer"] == "qmix":
            q_tot, mcache = qmix_forward(self.mp, chosen, batch["state"][:, :-1], n, keep_cache)
            tq_tot, _ = qmix_forward(self.tmp, target_max, batch["state"][:, 1:], n)
        elif c["mixer"] == "vdn":
            q_tot = chosen.sum(2, keepdims=True).astype(F32)
            tq_tot = target_max.sum(2, keepdims=True).astype(F32)
        else:
            q_tot, tq_tot = chosen, target_max
        targets = (rewards + F32(c["gamma"]) * (F32(1.0) - terminated) * tq_tot).astype(F32)
        td = (q_tot - targets).astype(F32)
        m = np.broadcast_to(mask, td.shape).astype(F32)
        mtd = td * m
        msum = F32(m.sum())
        hd = F32(c.get("huber_delta", 0.0))
        if hd > 0:   # opt-in masked Huber (no reference counterpart: parity unpinned; L2 below is q_learner.py:96-97)
            ax = np.abs(mtd)
            loss = F32(np.where(ax <= hd, F32(0.5) * mtd * mtd, hd * (ax - F32(0.5) * hd)).astype(F32).sum()) / msum
        else:
            loss = F32((mtd * mtd).sum()) / msum
        return dict(mac_out=mac_out, target_mac_out=tmo, cur_max_actions=cur_max, chosen=chosen,
                    target_max=target_max, q_tot=q_tot, target_q_tot=tq_tot, targets=targets, td=td, mask=m,
                    mask_sum=msum, loss=float(loss), acache=acache, mcache=mcache, actions=actions)

    def gradients(self, batch, fw=None, cur_max_override=None, relu_override=None):
        """Unclipped gradients of the loss (agent params then mixer params, reference order)."""
        c = self.cfg
        fw = fw or self.forward(batch, keep_cache=True, cur_max_override=cur_max_override,
                                relu_override=relu_override)
        td, m, msum = fw["td"], fw["mask"], fw["mask_sum"]
        hd = F32(c.get("huber_delta", 0.0))
        if hd > 0:   # d/dQ_tot of sum(huber(td*m))/sum(m)
            dq_tot = (np.clip(td * m, -hd, hd) * m * (F32(1.0) / msum)).astype(F32)
        else:
            dq_tot = ((F32(2.0) * (td * m)) * (F32(1.0) / msum)) * m            # d/dQ_tot of sum((td*m)^2)/sum(m)
        B, T = td.shape[:2]
        n = c["n_agents"]
        mg = OrderedDict()
        if c["mixer"] == "qmix":
            dchosen, mg = qmix_backward(self.mp, fw["mcache"], dq_tot.reshape(-1).astype(F32))
            dchosen = dchosen.reshape(B, T, n)
        elif c["mixer"] == "vdn":
            dchosen = np.broadcast_to(dq_tot, (B, T, n)).astype(F32)
        else:
            dchosen = dq_tot.astype(F32)
        A = fw["mac_out"].shape[-1]
        dmac = np.zeros_like(fw["mac_out"])
        oh = np.zeros((B, T, n, A), F32)
        np.put_along_axis(oh, fw["actions"], 1.0, axis=3)
        dmac[:, :-1] = oh * dchosen[..., None]
        ag = agent_backward(self.p, fw["acache"], dmac)
        return ag, mg, fw

    def train(self, batch, t_env, episode_num, cur_max_override=None, relu_override=None):
        """q_learner.py:37-116; returns the stats dict it would log."""
        c = self.cfg
        ag, mg, fw = self.gradients(batch, cur_max_override=cur_max_override, relu_override=relu_override)
        grads = OrderedDict(list(ag.items()) + list(mg.items()))
        grad_norm = clip_grad_norm(grads, c["grad_norm_clip"])
        params = OrderedDict(list(self.p.items()) + list(self.mp.items()))
        rmsprop_step(params, grads, self.sq, c["lr"], c["optim_alpha"], c["optim_eps"])
        for k in self.p:
            self.p[k] = params[k]
        for k in self.mp:
            self.mp[k] = params[k]
        if (episode_num - self.last_target_update_episode) / c["target_update_interval"] >= 1.0:
            self.update_targets()
            self.last_target_update_episode = episode_num
        m, td = fw["mask"], fw["td"]
        msum = float(m.sum())
        stats = dict(loss=fw["loss"], grad_norm=grad_norm,
                     td_error_abs=float(np.abs(td * m).sum()) / msum,
                     q_taken_mean=float((fw["q_tot"] * m).sum()) / (msum * c["n_agents"]),
                     target_mean=float((fw["targets"] * m).sum()) / (msum * c["n_agents"]))
        self.last = dict(grads=grads, fw=fw, stats=stats)
        return stats

    def update_targets(self):
        """q_learner.py:118-122."""
        self.tp = OrderedDict((k, v.copy()) for k, v in self.p.items())
        self.tmp = OrderedDict((k, v.copy()) for k, v in self.mp.items())

    def flat(self, which="params"):
        if which == "params":
            d = list(self.p.values()) + list(self.mp.values())
        elif which == "targets":
            d = list(self.tp.values()) + list(self.tmp.values())
        else:
            d = list(self.sq.values())
        return np.concatenate([v.ravel() for v in d]).astype(F32)
