"""Generate the golden parity fixtures by running the REFERENCE learner (nicholasburden/pymarl) in this container.

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

Not part of the product and never run on the GPU box (it needs /root/reference). It imports the reference's hot
path from /root/reference/src (those modules import with torch + numpy only), feeds it the seeded
synthetic replay of pymarl_amd/utils/synthetic.py with numpy-seeded weights loaded via load_state_dict, and records:

* per-step loss and the five learner stats exactly as QLearner.train logs them (q_learner.py:109-116),
* the sampled episode ids of ReplayBuffer.sample under np.random.seed(2) (episode_buffer.py:291-298),
* the double-Q greedy actions and their top-2 margins (q_learner.py:71-76),
* for the small shapes, every intermediate of train() (mac_out ... td), the clipped gradients after step 0,
  and parameters + RMSprop state after each step,
* greedy BasicMAC.select_actions(test_mode=True) outputs (basic_controller.py:30-38).

Intermediates are produced by re-running lines 39-97 of q_learner.py on the reference's own MAC / mixer modules
(same weights, no grad) just before each train() call; that restatement is checked against the loss train()
itself logs.

Workarounds: default.yaml is missing, so `args` is built explicitly with upstream-PyMARL
values; `scheme["obs"]["vshape_decoded"]` is required by this fork's BasicMAC._get_input_shape.
"""
from __future__ import annotations

import os
import sys
from types import SimpleNamespace as SN

sys.dont_write_bytecode = True   # /root/reference is read-only: no __pycache__ there

import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_SRC = "/root/reference/src"
sys.path.insert(0, REPO)
sys.path.insert(0, REF_SRC)

import torch as th  # noqa: E402

from pymarl_amd.utils.synthetic import (agent_param_shapes, init_params, make_replay,  # noqa: E402
                                        qmix_param_shapes)

from components.episode_buffer import ReplayBuffer  # noqa: E402  (reference)
from components.transforms import OneHot  # noqa: E402  (reference)
from controllers.basic_controller import BasicMAC  # noqa: E402  (reference)
from learners.q_learner import QLearner  # noqa: E402  (reference)


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


def make_args(n, A, O, S, mixer, H=64, E=32, double_q=True, obs_last_action=True, obs_agent_id=True):
    return SN(n_agents=n, n_actions=A, state_shape=S, obs_shape=O, rnn_hidden_dim=H, mixing_embed_dim=E,
              mixer=mixer, lr=5e-4, optim_alpha=0.99, optim_eps=1e-5, grad_norm_clip=10.0, gamma=0.99,
              double_q=double_q, target_update_interval=200, learner_log_interval=0,
              obs_last_action=obs_last_action, obs_agent_id=obs_agent_id, agent="rnn", mac="basic_mac",
              agent_output_type="q",
              action_selector="epsilon_greedy", epsilon_start=1.0, epsilon_finish=0.05, epsilon_anneal_time=50000,
              action_input_representation=None, obs_decoder=None, avail_actions_encoder=None,
              device="cpu", use_cuda=False)


def make_scheme(n, A, O, S):
    return {
        "state": {"vshape": S},
        "obs": {"vshape": O, "group": "agents", "vshape_decoded": O},
        "actions": {"vshape": (1,), "group": "agents", "dtype": th.long},
        "avail_actions": {"vshape": (A,), "group": "agents", "dtype": th.int},
        "reward": {"vshape": (1,)},
        "terminated": {"vshape": (1,), "dtype": th.uint8},
    }


def build(case):
    n, A, O, S, T = case["n"], case["A"], case["O"], case["S"], case["T"]
    flags = {k: case[k] for k in ("double_q", "obs_last_action", "obs_agent_id") if k in case}
    args = make_args(n, A, O, S, case["mixer"], **flags)
    scheme = make_scheme(n, A, O, S)
    groups = {"agents": n}
    preprocess = {"actions": ("actions_onehot", [OneHot(out_dim=A)])}
    buf = ReplayBuffer(scheme, groups, case["n_episodes"], T + 1, preprocess=preprocess, device="cpu")
    data = make_replay(case["n_episodes"], T, n, A, O, S, seed=case["data_seed"], ragged=case["ragged"])
    for k, v in data.items():
        buf.data.transition_data[k][:] = th.from_numpy(v)
    buf.episodes_in_buffer = case["n_episodes"]
    buf.buffer_index = 0

    mac = BasicMAC(buf.scheme, groups, args)
    logger = _Logger()
    learner = QLearner(mac, buf.scheme, logger, args)
    I = O + (A if args.obs_last_action else 0) + (n if args.obs_agent_id else 0)   # basic_controller.py:150-153
    w_agent = init_params(agent_param_shapes(I, 64, A), seed=case["weight_seed"])
    mac.agent.load_state_dict({k: th.from_numpy(v) for k, v in w_agent.items()})
    learner.target_mac.agent.load_state_dict({k: th.from_numpy(v) for k, v in w_agent.items()})
    if case["mixer"] == "qmix":
        w_mix = init_params(qmix_param_shapes(S, n, 32), seed=case["weight_seed"] + 100)
        learner.mixer.load_state_dict({k: th.from_numpy(v) for k, v in w_mix.items()})
        learner.target_mixer.load_state_dict({k: th.from_numpy(v) for k, v in w_mix.items()})
    return args, buf, mac, learner, logger


@th.no_grad()
def intermediates(learner, batch):
    """q_learner.py:39-97 re-run on the reference's own modules (no grad); returns numpy copies."""
    args = learner.args
    rewards = batch["reward"][:, :-1]
    actions = batch["actions"][:, :-1]
    terminated = batch["terminated"][:, :-1].float()
    mask = batch["filled"][:, :-1].float()
    mask[:, 1:] = mask[:, 1:] * (1 - terminated[:, :-1])
    avail_actions = batch["avail_actions"]
    mac_out = []
    learner.mac.init_hidden(batch.batch_size)
    for t in range(batch.max_seq_length):
        mac_out.append(learner.mac.forward(batch, t=t))
    mac_out = th.stack(mac_out, dim=1)
    chosen = th.gather(mac_out[:, :-1], dim=3, index=actions).squeeze(3)
    tmo = []
    learner.target_mac.init_hidden(batch.batch_size)
    for t in range(batch.max_seq_length):
        tmo.append(learner.target_mac.forward(batch, t=t))
    tmo = th.stack(tmo[1:], dim=1)
    tmo[avail_actions[:, 1:] == 0] = -9999999
    if args.double_q:   # q_learner.py:71-76
        mod = mac_out.clone().detach()
        mod[avail_actions == 0] = -9999999
        cur_max = mod[:, 1:].max(dim=3, keepdim=True)[1]
        top2 = th.topk(mod[:, 1:], 2, dim=3)[0]
        target_max = th.gather(tmo, 3, cur_max).squeeze(3)
    else:               # q_learner.py:77-78; the argmax and margin recorded are the target net's
        cur_max = tmo.max(dim=3, keepdim=True)[1]
        top2 = th.topk(tmo, 2, dim=3)[0]
        target_max = tmo.max(dim=3)[0]
    margin = (top2[..., 0] - top2[..., 1])
    if learner.mixer is not None:
        q_tot = learner.mixer(chosen, batch["state"][:, :-1])
        tq_tot = learner.target_mixer(target_max, batch["state"][:, 1:])
    else:
        q_tot, tq_tot = chosen, target_max
    targets = rewards + args.gamma * (1 - terminated) * tq_tot
    td = q_tot - targets
    m = mask.expand_as(td)
    loss = ((td * m) ** 2).sum() / m.sum()
    f = lambda x: x.detach().cpu().numpy().copy()  # noqa: E731
    return dict(mac_out=f(mac_out), target_mac_out=f(tmo), cur_max_actions=f(cur_max.squeeze(3)).astype(np.int64),
                margin=f(margin), chosen=f(chosen), target_max=f(target_max), q_tot=f(q_tot),
                target_q_tot=f(tq_tot), targets=f(targets), td=f(td), mask=f(mask), loss=float(loss))


def flat_params(learner):
    ps = [p.detach().cpu().numpy().ravel() for p in learner.params]
    return np.concatenate(ps).astype(np.float32)


def flat_targets(learner):
    ps = [p.detach().cpu().numpy().ravel() for p in learner.target_mac.agent.parameters()]
    if learner.mixer is not None:
        ps += [p.detach().cpu().numpy().ravel() for p in learner.target_mixer.parameters()]
    return np.concatenate(ps).astype(np.float32)


def flat_grads(learner):
    return np.concatenate([p.grad.detach().cpu().numpy().ravel() for p in learner.params]).astype(np.float32)


def flat_sqavg(learner):
    st = learner.optimiser.state
    return np.concatenate([st[p]["square_avg"].cpu().numpy().ravel() for p in learner.params]).astype(np.float32)


def run_case(name, case):
    th.set_num_threads(8)
    args, buf, mac, learner, logger = build(case)
    np.random.seed(case["sampler_seed"])
    out = {k: np.array(v) for k, v in case.items() if not isinstance(v, str)}
    out["mixer"] = np.array(case["mixer"] or "none")   # IQL (mixer: None, iql_smac.yaml:21) is stored as "none"
    if case.get("store_params", True):
        out["params_init"] = flat_params(learner)
    ids_all, losses, full = [], [], case["full"]
    cur_max_steps, margin_steps = [], []
    per_step = {"params": [], "targets": [], "sqavg": []}
    episodes = case["episodes"]
    for k in range(case["steps"]):
        st = np.random.get_state()
        batch = buf.sample(case["B"])
        after = np.random.get_state()
        np.random.set_state(st)
        if buf.episodes_in_buffer == case["B"]:
            ids = np.arange(case["B"])
        else:
            ids = np.random.choice(buf.episodes_in_buffer, case["B"], replace=False)
        np.random.set_state(after)
        assert np.array_equal(batch["obs"].numpy(), buf["obs"][ids].numpy())
        ids_all.append(ids.astype(np.int64))
        max_t = int(batch.max_t_filled())
        batch = batch[:, :max_t]
        inter = intermediates(learner, batch)
        if k < case["record_actions_steps"]:
            cur_max_steps.append(inter["cur_max_actions"].astype(np.uint8))
            margin_steps.append(inter["margin"].astype(np.float32))
        if full and k == 0:
            for kk, vv in inter.items():
                out["step0_" + kk] = np.asarray(vv)
            out["step0_max_t"] = np.array(max_t)
            # greedy select_actions(test_mode=True) over the whole sampled batch, t = 0..max_t-1
            # (Categorical(avail) inside select_action raises on an all-zero avail row, so stop at the first
            #  padded slot of the shortest episode)
            t_all = int(batch["filled"].sum(1).min())
            mac.init_hidden(batch.batch_size)
            acts = [mac.select_actions(batch, t_ep=t, t_env=0, test_mode=True).numpy() for t in range(t_all)]
            out["greedy_actions"] = np.stack(acts, 1).astype(np.int64)
        learner.train(batch, t_env=1000 * k, episode_num=episodes[k])
        if k == case.get("ckpt_step", -1):
            # the reference's own checkpoint files (q_learner.py:131-135, basic_controller.py:91-92)
            ck = os.path.join(HERE, "ckpt_{}_step{}".format(name, k))
            os.makedirs(ck, exist_ok=True)
            learner.save_models(ck)
        losses.append(logger.stats["loss"][-1])
        assert abs(losses[-1] - inter["loss"]) <= 1e-6 * max(1.0, abs(losses[-1])), (losses[-1], inter["loss"])
        if full and k == 0:
            out["step0_grads_clipped"] = flat_grads(learner)
        if full:
            per_step["params"].append(flat_params(learner))
            per_step["targets"].append(flat_targets(learner))
            per_step["sqavg"].append(flat_sqavg(learner))
    out["ids"] = np.stack(ids_all)
    for key in ["loss", "grad_norm", "td_error_abs", "q_taken_mean", "target_mean"]:
        out["stat_" + key] = np.array(logger.stats[key], dtype=np.float64)
    if cur_max_steps:
        # ragged batches truncate to different max_t: pad the time axis to T (padded slots: action 0, margin -1, so
        # no test counts them as a clear decision; readers slice [:, :max_t - 1])
        Tm = max(a.shape[1] for a in cur_max_steps)
        pad = lambda a, v: np.pad(a, ((0, 0), (0, Tm - a.shape[1]), (0, 0)), constant_values=v)  # noqa: E731
        out["cur_max_actions"] = np.stack([pad(a, 0) for a in cur_max_steps])
        out["margin"] = np.stack([pad(m, -1.0) for m in margin_steps])
    if full:
        out["step_params"] = np.stack(per_step["params"])
        out["targets_final"] = per_step["targets"][-1]
        out["sqavg_final"] = per_step["sqavg"][-1]
    elif case.get("store_params", True):
        out["params_final"] = flat_params(learner)
        out["targets_final"] = flat_targets(learner)
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **out)
    print(name, "steps", case["steps"], "loss[0..]", np.round(out["stat_loss"][:4], 6), "->", path,
          os.path.getsize(path) // 1024, "KB")


TINY = dict(n=3, A=9, O=30, S=48, T=10, B=4, n_episodes=6, data_seed=0, weight_seed=1, sampler_seed=2,
            ragged=True, steps=4, episodes=[0, 8, 200, 208], full=True, record_actions_steps=4)
CFG2 = dict(n=8, A=14, O=80, S=168, T=120, B=32, n_episodes=64, data_seed=0, weight_seed=1, sampler_seed=2,
            ragged=False, steps=20, episodes=[8 * k for k in range(10)] + [200 + 8 * k for k in range(10)],
            full=False, record_actions_steps=3)

CFG3 = dict(n=27, A=36, O=285, S=1170, T=180, B=4, n_episodes=8, data_seed=0, weight_seed=1, sampler_seed=2,
            ragged=True, steps=4, episodes=[0, 8, 200, 208], full=False, record_actions_steps=2)
CFG4 = dict(n=5, A=11, O=80, S=120, T=120, B=64, n_episodes=96, data_seed=0, weight_seed=1, sampler_seed=2,
            ragged=False, steps=4, episodes=[0, 8, 200, 208], full=False, record_actions_steps=2)

CFG1 = dict(n=3, A=9, O=30, S=48, T=60, B=8, n_episodes=40, data_seed=6, weight_seed=7, sampler_seed=8,
            ragged=True, steps=10, episodes=[8 * k for k in range(5)] + [200 + 8 * k for k in range(5)],
            full=False, record_actions_steps=10)

# Batches past the fused kernels' row limits (R = B * n rows): R in (512, 1024] runs gru_fwd_kernel<2>, (1024, 2048]
# gru_fwd_kernel<4>, > 2048 gru_fwd_kernel<8>; B > 256 (MQ_INLINE_IDS) passes the episode ids as a device vector.
# Small O / S / T keep the reference's CPU run short.
WIDE = dict(data_seed=3, weight_seed=4, sampler_seed=5, ragged=True, steps=3, episodes=[0, 8, 200], full=False,
            record_actions_steps=3)

CASES = {
    "tiny_qmix": dict(TINY, mixer="qmix", ckpt_step=2),
    "tiny_vdn": dict(TINY, mixer="vdn", ckpt_step=2),
    # IQL (src/config/algs/iql_smac.yaml:21, mixer: None): the loss normaliser is n_agents * sum(mask)
    # (q_learner.py:89-97, mask.expand_as(td_error))
    "tiny_iql": dict(TINY, mixer=None),
    "cfg2_iql": dict(CFG2, mixer=None, steps=10, episodes=[8 * k for k in range(5)] + [200 + k for k in range(5)]),
    "rw2_qmix": dict(WIDE, n=8, A=6, O=12, S=20, T=12, B=72, n_episodes=96, mixer="qmix"),
    "rw4_vdn": dict(WIDE, n=16, A=7, O=10, S=16, T=10, B=80, n_episodes=100, mixer="vdn"),
    "wide_qmix": dict(WIDE, n=8, A=5, O=8, S=12, T=8, B=300, n_episodes=320, mixer="qmix"),
    # BASELINE configs[2] exactly (27m_vs_30m shape, VDN, B = 128): R = 3456 rows, the bench's kernel path
    # 6 steps with a target update at step 3 (episodes 16 -> 200): the row-tile kernels hold the reference's
    # free-running trajectory past an update
    "cfg3_vdn_b128": dict(CFG3, mixer="vdn", B=128, n_episodes=136, steps=6, episodes=[0, 8, 16, 200, 208, 216],
                          ragged=True, record_actions_steps=2),
    "tiny_qmix_full": dict(TINY, mixer="qmix", ragged=False, n_episodes=4, steps=3, episodes=[0, 200, 201]),
    "cfg2_qmix": dict(CFG2, mixer="qmix"),
    "cfg2_vdn": dict(CFG2, mixer="vdn", steps=10, episodes=[8 * k for k in range(5)] + [200 + k for k in range(5)]),
    "cfg2_qmix_ragged": dict(CFG2, mixer="qmix", ragged=True, steps=5, episodes=[0, 8, 200, 208, 216]),
    # BASELINE configs[2] shape (27m_vs_30m, VDN) at a reduced batch: A=36 > 16 and I=348 run the unfused kernels
    "cfg3_vdn": dict(CFG3, mixer="vdn"),
    # the same shape under QMIX: S=1170 exercises the hypernet / dW_hyper kernels at a long K
    "cfg3_qmix": dict(CFG3, mixer="qmix", steps=3, episodes=[0, 8, 200], store_params=False),
    # BASELINE configs[3] shape (2s3z, QMIX): one rank's shard of B=512 over 8 GPUs, R = 64*5 = 320 rows > 256
    "cfg4_qmix": dict(CFG4, mixer="qmix", steps=8, episodes=[0, 8, 16, 24, 200, 208, 216, 224]),
    # the reference branches no shipped config takes: double_q: False (q_learner.py:77-78), obs_last_action /
    # obs_agent_id: False (basic_controller.py:111-120, 150-153)
    "tiny_qmix_nodq": dict(TINY, mixer="qmix", double_q=False),
    "tiny_qmix_nola": dict(TINY, mixer="qmix", obs_last_action=False),
    "tiny_vdn_noid": dict(TINY, mixer="vdn", obs_agent_id=False),
    "tiny_qmix_bare": dict(TINY, mixer="qmix", obs_last_action=False, obs_agent_id=False, double_q=False),
    "cfg2_qmix_nodq": dict(CFG2, mixer="qmix", double_q=False, steps=5, episodes=[0, 8, 200, 208, 216]),
    # BASELINE configs[0]'s learner shape (QMIX on SMAC 3m, batch_size 8, upstream-SMAC obs / state: SURVEY §8a
    # cfg1): n = 3, A = 9, O = 30, S = 48, T = 60, B = 8; ragged like SMAC episodes, a target update at step 5
    "cfg1_qmix": dict(CFG1, mixer="qmix"),
    "cfg1_vdn": dict(CFG1, mixer="vdn", steps=5, episodes=[0, 8, 200, 208, 216]),
}

if __name__ == "__main__":
    only = sys.argv[1:]
    for name, case in CASES.items():
        if only and name not in only:
            continue
        run_case(name, case)
